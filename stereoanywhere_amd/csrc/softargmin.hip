// K5 — soft-argmin disparity and entropy confidence, left (softmax over k) and right
// (softmax over j), on arbitrary-stride volumes.
//
// Reference: estimate_left_disparity / estimate_right_disparity (utils.py:112-152):
//   D_L[j] = j - sum_k k p_k,  D_R[k] = sum_j j p_j - k,  p = softmax;
// estimate_left_confidence / estimate_right_confidence (utils.py:154-170):
//   C = 1 - (-sum p log2(p + 1e-6)) / log2(W).
// p is formed like ATen's CPU softmax: e = exp(x - max), p = e * (1 / sum e).
//
// Each output reduces one line of the volume.  If that line is contiguous (stride 1)
// one wave owns it and the lanes stride along it (wave shuffles for the reductions);
// otherwise one thread owns it and consecutive threads own consecutive (contiguous)
// lines, so every load instruction of the wave is still one coalesced row segment.
// Two passes per line (max/sum, then p-weighted sums) — the second is an L2 hit.
#include <cmath>

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
  if (red_stride == 1) {
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
