// K5 — soft-argmin disparity and entropy confidence, left (softmax over k) and right
// (softmax over j), on arbitrary-stride volumes.
//
// Reference: estimate_left_disparity / estimate_right_disparity (utils.py:112-152):
//   D_L[j] = j - sum_k k p_k,  D_R[k] = sum_j j p_j - k,  p = softmax;
// estimate_left_confidence / estimate_right_confidence (utils.py:154-170):
//   C = 1 - (-sum p log2(p + 1e-6)) / log2(W).
// p is formed like ATen's CPU softmax: e = exp(x - max), p = e * (1 / sum e).
//
// Each output reduces one line of the volume, read from HBM once and held in registers
// while the max, the sum of exponentials and the p-weighted sum are formed:
//   sam_row_kernel — the line is contiguous (stride 1): one wave per line, up to 4
//     elements per lane (one float4 where aligned), wave shuffles for the reductions;
//   sam_col_kernel — the line is strided: a lane per line, consecutive lanes on
//     consecutive (contiguous) lines so each load is one coalesced row segment, and the
//     block's 4 waves split the line's length (partials combined through LDS).
// Lines longer than 256 take the generic kernels below them (re-read per pass).
#include <cmath>
#include <cstdint>

#include "sa_common.h"

namespace {

struct SGeo {
  int H, W1, W2;
  long sb, sh, sj, sk;
  long obs;  // output batch stride (elements)
  float log2W1, log2W2;  // math.log2(W) of the reference (double), rounded once to fp32
};

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Reduce along an axis of length n with element stride es, output index o of `nout`
// outputs along the other axis with element stride os.  LEFT: output is j, reduce k.
// `mode` 0: disparity volume (D = sign * (sum p*i) + base), 1: confidence volume.
struct LineJob {
  const float *vol;
  float *out;
  int mode;
};

constexpr int SAM_NMAX = 256;  // register-resident line length limit

__device__ __forceinline__ float sam_final(int mode, int left, int o, float acc, const SGeo &g) {
  if (mode == 0) return left ? ((float)o - acc) : (acc - (float)o);
  return 1.0f - (-acc) / (left ? g.log2W2 : g.log2W1);
}

// one wave per LPW contiguous lines of n <= 256 elements (all of its lines' loads issued
// before any reduction, so a wave has LPW x 2 KB in flight instead of 2 KB); V4: element
// 4*lane+i (float4 loads), else element lane+64*i
constexpr int SAM_LPW = 4;

template <bool V4>
__global__ __launch_bounds__(256) void sam_row_kernel(LineJob jd, LineJob jc, SGeo g, int left, long nlines) {
  const long line0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * SAM_LPW;
  if (line0 >= nlines) return;
  const int lane = threadIdx.x & 63;
  const int nout = left ? g.W1 : g.W2;
  const int n = left ? g.W2 : g.W1;
  const LineJob jobs[2] = {jd, jc};
  int idx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) idx[i] = V4 ? 4 * lane + i : lane + 64 * i;
  float v[SAM_LPW][2][4];
  long ob[SAM_LPW];
  int oo[SAM_LPW];
#pragma unroll
  for (int t = 0; t < SAM_LPW; ++t) {
    const long line = line0 + t < nlines ? line0 + t : nlines - 1;   // a ragged tail re-reads the last line
    const long bh = line / nout;
    const int o = (int)(line % nout);
    const long b = bh / g.H, h = bh % g.H;
    ob[t] = b * g.obs + h * nout;
    oo[t] = o;
    const long base = b * g.sb + h * g.sh + (long)o * (left ? g.sj : g.sk);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (!jobs[q].vol) continue;
      const float *src = jobs[q].vol + base;
      if (V4) {
        if (4 * lane < n) {
          const float4 x = *reinterpret_cast<const float4 *>(src + 4 * lane);
          v[t][q][0] = x.x, v[t][q][1] = x.y, v[t][q][2] = x.z, v[t][q][3] = x.w;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[t][q][i] = -INFINITY;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[t][q][i] = idx[i] < n ? src[idx[i]] : -INFINITY;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < SAM_LPW; ++t) {
    if (line0 + t >= nlines) break;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const LineJob &J = jobs[q];
      if (!J.vol) continue;
      const float m = wave_max(fmaxf(fmaxf(v[t][q][0], v[t][q][1]), fmaxf(v[t][q][2], v[t][q][3])));
      float e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = idx[i] < n ? expf(v[t][q][i] - m) : 0.f;
      const float inv = 1.0f / wave_sum((e[0] + e[1]) + (e[2] + e[3]));
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = e[i] * inv;
        if (idx[i] < n) acc += J.mode == 0 ? p * (float)idx[i] : p * log2f(p + 1e-6f);
      }
      acc = wave_sum(acc);
      if (lane == 0) J.out[ob[t] + oo[t]] = sam_final(J.mode, left, oo[t], acc, g);
    }
  }
}

// a lane per strided line of n <= 256 elements, 64 lines per block; wave w holds the
// line's elements [w*per, (w+1)*per), per = ceil(n/4) <= 64
__global__ __launch_bounds__(256) void sam_col_kernel(LineJob jd, LineJob jc, SGeo g, int left, long nlines) {
  __shared__ float red[3][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long line = (long)blockIdx.x * 64 + lane;
  const bool valid = line < nlines;
  const int nout = left ? g.W1 : g.W2;
  const int n = left ? g.W2 : g.W1;
  const long es = left ? g.sk : g.sj;
  const long bh = valid ? line / nout : 0;
  const int o = valid ? (int)(line % nout) : 0;
  const long b = bh / g.H, h = bh % g.H;
  const int per = (n + 3) >> 2, k0 = w * per;
  const int cnt = valid ? max(0, min(per, n - k0)) : 0;
  const long base = b * g.sb + h * g.sh + (long)o * (left ? g.sj : g.sk) + (long)k0 * es;
  const LineJob jobs[2] = {jd, jc};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const LineJob &J = jobs[q];
    if (!J.vol) continue;
    const float *src = J.vol + base;
    float v[64];
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      v[i] = i < cnt ? src[(long)i * es] : -INFINITY;
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) m = fmaxf(m, v[i]);
    red[0][w][lane] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0][lane], red[0][1][lane]), fmaxf(red[0][2][lane], red[0][3][lane]));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      v[i] = i < cnt ? expf(v[i] - m) : 0.f;
      s += v[i];
    }
    red[1][w][lane] = s;
    __syncthreads();
    const float inv = 1.0f / ((red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]));
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const float p = v[i] * inv;
      if (i < cnt) acc += J.mode == 0 ? p * (float)(k0 + i) : p * log2f(p + 1e-6f);
    }
    red[2][w][lane] = acc;
    __syncthreads();
    if (w == 0 && valid) {
      acc = (red[2][0][lane] + red[2][1][lane]) + (red[2][2][lane] + red[2][3][lane]);
      J.out[b * g.obs + h * nout + o] = sam_final(J.mode, left, o, acc, g);
    }
    __syncthreads();  // red is reused by the next volume
  }
}

// one wave per line (contiguous reduction axis)
__global__ __launch_bounds__(256) void sam_contig_kernel(LineJob jd, LineJob jc, SGeo g, int left,
                                                         long nlines) {
  const long line = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (line >= nlines) return;
  const int lane = threadIdx.x & 63;
  const int nout = left ? g.W1 : g.W2;  // outputs per (b,h)
  const int n = left ? g.W2 : g.W1;     // reduction length
  const long bh = line / nout;
  const int o = (int)(line % nout);
  const long b = bh / g.H, h = bh % g.H;
  const long base = b * g.sb + h * g.sh + (long)o * (left ? g.sj : g.sk);
  const LineJob jobs[2] = {jd, jc};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const LineJob &J = jobs[q];
    if (!J.vol) continue;
    const float *v = J.vol + base;
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, v[i]);
    m = wave_max(m);
    float s = 0.f;
    for (int i = lane; i < n; i += 64) s += expf(v[i] - m);
    s = wave_sum(s);
    const float inv = 1.0f / s;
    float acc = 0.f;
    if (J.mode == 0) {
      for (int i = lane; i < n; i += 64) acc += (expf(v[i] - m) * inv) * (float)i;
    } else {
      for (int i = lane; i < n; i += 64) {
        const float p = expf(v[i] - m) * inv;
        acc += p * log2f(p + 1e-6f);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) {
      float r;
      if (J.mode == 0) r = left ? ((float)o - acc) : (acc - (float)o);
      else r = 1.0f - (-acc) / (left ? g.log2W2 : g.log2W1);
      J.out[b * g.obs + h * nout + o] = r;
    }
  }
}

// one thread per line (strided reduction axis, contiguous output axis)
__global__ __launch_bounds__(256) void sam_strided_kernel(LineJob jd, LineJob jc, SGeo g, int left,
                                                          long nlines) {
  const long line = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (line >= nlines) return;
  const int nout = left ? g.W1 : g.W2;
  const int n = left ? g.W2 : g.W1;
  const long bh = line / nout;
  const int o = (int)(line % nout);
  const long b = bh / g.H, h = bh % g.H;
  const long es = left ? g.sk : g.sj;
  const long base = b * g.sb + h * g.sh + (long)o * (left ? g.sj : g.sk);
  const LineJob jobs[2] = {jd, jc};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const LineJob &J = jobs[q];
    if (!J.vol) continue;
    const float *v = J.vol + base;
    float m = -INFINITY;
    for (int i = 0; i < n; ++i) m = fmaxf(m, v[i * es]);
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += expf(v[i * es] - m);
    const float inv = 1.0f / s;
    float acc = 0.f;
    if (J.mode == 0) {
      for (int i = 0; i < n; ++i) acc += (expf(v[i * es] - m) * inv) * (float)i;
    } else {
      for (int i = 0; i < n; ++i) {
        const float p = expf(v[i * es] - m) * inv;
        acc += p * log2f(p + 1e-6f);
      }
    }
    float r;
    if (J.mode == 0) r = left ? ((float)o - acc) : (acc - (float)o);
    else r = 1.0f - (-acc) / (left ? g.log2W2 : g.log2W1);
    J.out[b * g.obs + h * nout + o] = r;
  }
}

int launch_side(LineJob jd, LineJob jc, const SGeo &g, int B, int left, hipStream_t s) {
  const long nlines = (long)B * g.H * (left ? g.W1 : g.W2);
  const long red_stride = left ? g.sk : g.sj;
  const int n = left ? g.W2 : g.W1;
  if (n <= SAM_NMAX) {
    if (red_stride == 1) {
      // float4 rows: every line start 16-byte aligned
      auto al = [](const float *p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
      const long os = left ? g.sj : g.sk;
      const bool v4 = n % 4 == 0 && g.sb % 4 == 0 && g.sh % 4 == 0 && os % 4 == 0 && al(jd.vol) && al(jc.vol);
      const unsigned nb = (unsigned)((nlines + 4 * SAM_LPW - 1) / (4 * SAM_LPW));
      if (v4) sam_row_kernel<true><<<nb, 256, 0, s>>>(jd, jc, g, left, nlines);
      else sam_row_kernel<false><<<nb, 256, 0, s>>>(jd, jc, g, left, nlines);
    } else {
      sam_col_kernel<<<(unsigned)((nlines + 63) / 64), 256, 0, s>>>(jd, jc, g, left, nlines);
    }
  } else if (red_stride == 1) {
    sam_contig_kernel<<<(unsigned)((nlines + 3) / 4), 256, 0, s>>>(jd, jc, g, left, nlines);
  } else {
    sam_strided_kernel<<<(unsigned)((nlines + 255) / 256), 256, 0, s>>>(jd, jc, g, left, nlines);
  }
  return sa::check_launch("sa_softargmin_conf");
}

}  // namespace

extern "C" int sa_softargmin_conf(const float *vol_disp, const float *vol_conf, int B, int H, int W1,
                                  int W2, long sb, long sh, long sj, long sk, float *dL, float *dR,
                                  float *cL, float *cR, long out_bs, void *stream) {
  SA_REQUIRE(vol_disp || vol_conf, "sa_softargmin_conf: no volume");
  SA_REQUIRE(!vol_disp || (dL && dR), "sa_softargmin_conf: dL/dR missing");
  SA_REQUIRE(!vol_conf || (cL && cR), "sa_softargmin_conf: cL/cR missing");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 1 && W2 > 1, "sa_softargmin_conf: bad shape");
  SA_REQUIRE(sj == 1 || sk == 1, "sa_softargmin_conf: one of sj/sk must be 1");
  SA_REQUIRE(out_bs >= (long)H * (W1 > W2 ? W1 : W2), "sa_softargmin_conf: out_bs too small");
  SGeo g{H, W1, W2, sb, sh, sj, sk, out_bs, (float)std::log2((double)W1), (float)std::log2((double)W2)};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_SOFTARGMIN, s);
  LineJob ld{vol_disp, dL, 0}, lc{vol_conf, cL, 1};
  LineJob rd{vol_disp, dR, 0}, rc{vol_conf, cR, 1};
  int rc1 = launch_side(ld, lc, g, B, 1, s);
  if (rc1) return rc1;
  return launch_side(rd, rc, g, B, 0, s);
}
