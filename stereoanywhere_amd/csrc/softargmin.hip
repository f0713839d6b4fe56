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

// wave reductions on DPP (sa_common.h): __shfl_xor compiled to ds_bpermute, an LDS round trip
// per step, 18 dependent ones per row of the slice kernels (latency-bound: 156 -> 124 us at cfg2)
__device__ __forceinline__ float wave_max(float v) { return sa::wave_max_dpp(v); }
__device__ __forceinline__ float wave_sum(float v) { return sa::wave_sum_dpp(v); }

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

// exp(d) for d = x - max <= 0 and log2(y) for y = p + 1e-6 in [1e-6, 1 + 1e-6]: the hardware
// v_exp_f32 / v_log_f32 (one quarter-rate op each; relative error ~1e-7 here, against ~10 VALU
// operations of the library's range-reduced expf / log2f).  The slice kernel below is
// VALU-bound, not HBM-bound, with the library versions.
__device__ __forceinline__ float exp_le0(float d) { return __builtin_amdgcn_exp2f(d * 1.44269504088896341f); }
__device__ __forceinline__ float log2_pos(float y) { return __builtin_amdgcn_logf(y); }
// exp(x - m) as exp2(x log2e - m log2e) with the row's m log2e formed once (one FMA per cell
// instead of a subtract and a multiply; the rounding of m log2e is a common factor of the row,
// which the normalisation removes)
constexpr float SAM_L2E = 1.44269504088896341f;
__device__ __forceinline__ float exp_shift(float x, float ml2e) { return __builtin_amdgcn_exp2f(fmaf(x, SAM_L2E, -ml2e)); }

// One pass over each (b, h) slice: both reductions of a volume from one read.  A block of 1024
// threads holds the slice's n x n cells in registers, element (k, j) at wave k % 16, slot
// r = k / 16, lane j % 64, slot c = j / 64 (j is the contiguous axis, sj == 1).  The right
// side (softmax over j, per k) reduces within a wave as each row's loads land; the left side
// (softmax over k, per j) combines the 16 waves' column partials through LDS.  blockIdx.y
// picks the volume (0: disparity, 1: confidence).  The two launches of the line kernels above
// each read both volumes; this reads each once.
// A workgroup barrier for LDS exchanges only: the LDS operations complete, then s_barrier (a
// __syncthreads also waits for every outstanding global load, here the prefetch kernel's DMAs
// of the next slice)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The reductions of one slice held in registers (x: cell (k, j) at row slot r = (k - w) / 16,
// column slot c = (j - lane) / 64; cells outside the slice are masked here): the right side per row
// within a wave, the left side per column through the 16 waves' LDS partials (red, colv).  CONF:
// the confidence volume (entropy terms) or the disparity volume (index-weighted sums), a template
// argument so neither volume's blocks evaluate the other's terms (with a run-time flag the
// compiler formed both and selected: the log2 of every cell on the disparity volume too).
// RT: the kind from the run-time flag rconf instead (one body for both volumes: the 18 x 5 slot
// instance, whose two bodies would spill past its 128 VGPRs)
template <int NR, int NC, bool CONF, bool RT = false>
__device__ __forceinline__ void slice_reduce(float (&x)[NR][NC], float (&red)[16][NC * 64], float (&colv)[NC * 64],
                                             const int n, const SGeo &g, float *outL, float *outR,
                                             const long ob, const int w, const int lane, const int tid,
                                             const bool rconf = false) {
  const bool conf = RT ? rconf : CONF;
  // cells outside the slice -> -inf; only the column slots that can reach past n and the rows past
  // it (both wave-uniform tests) take the select
  auto mask_row = [&](int r) __attribute__((always_inline)) {
    const int k = w + 16 * r;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (k >= n || 64 * c + 63 >= n) x[r][c] = (k < n && lane + 64 * c < n) ? x[r][c] : -INFINITY;
  };
  // ---- right: per row k, softmax over j (estimate_right_*, utils.py:132-152, 162-170).  Rows in
  // groups of RG: each group's max / sum / accumulate reductions run as RG interleaved DPP chains
  // (one row at a time, the wave waited on one chain's latency after another: round 6, 4 rows per
  // group; the same operations per row, so the same bits)
  const float lw_r = g.log2W1;
  constexpr int RG = NR % 4 == 0 ? 4 : NR % 3 == 0 ? 3 : NR % 2 == 0 ? 2 : 1;
#pragma unroll
  for (int r0 = 0; r0 < NR; r0 += RG) {
    if (w + 16 * r0 >= n) continue;   // wave-uniform (rows k >= n of a group: all -inf, unused)
#pragma unroll
    for (int u = 0; u < RG; ++u) mask_row(r0 + u);
    float m[RG];
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      m[u] = x[r0 + u][0];
#pragma unroll
      for (int c = 1; c < NC; ++c) m[u] = fmaxf(m[u], x[r0 + u][c]);
    }
    sa::wave_reduce_bfly_n<true>(m);
    float e[RG][NC], se[RG];
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      se[u] = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        e[u][c] = exp_shift(x[r0 + u][c], m[u] * SAM_L2E);   // -inf (j >= n) -> 0
        se[u] += e[u][c];
      }
    }
    sa::wave_reduce_bfly_n<false>(se);
    float acc[RG];
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      const float inv = __builtin_amdgcn_rcpf(se[u]);   // (v_rcp_f32, 1 ulp; the IEEE division's 10 VALU)
      acc[u] = 0.f;
      // (no j < n test: a masked cell has e = 0, so p = 0 and the term is an exact 0, log2 of
      // 1e-6 being finite)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int j = lane + 64 * c;
        const float p = e[u][c] * inv;
        acc[u] = fmaf(p, conf ? log2_pos(p + 1e-6f) : (float)j, acc[u]);
      }
    }
    sa::wave_reduce_bfly_n<false>(acc);
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      const int k = w + 16 * (r0 + u);
      if (lane == 0 && k < n) outR[ob + k] = conf ? 1.0f - (-acc[u]) / lw_r : acc[u] - (float)k;
    }
  }
  // ---- left: per column j, softmax over k (estimate_left_*, utils.py:112-130, 154-161)
  auto column_total = [&](float *part, bool is_max) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < NC; ++c) red[w][lane + 64 * c] = part[c];
    lds_barrier();
    if (tid < n) {
      float t = red[0][tid];
#pragma unroll
      for (int i = 1; i < 16; ++i) t = is_max ? fmaxf(t, red[i][tid]) : t + red[i][tid];
      colv[tid] = t;
    }
    lds_barrier();
#pragma unroll
    for (int c = 0; c < NC; ++c) part[c] = colv[lane + 64 * c < n ? lane + 64 * c : 0];
    lds_barrier();   // red / colv are reused by the next total
  };
  // the rows of the groups the right side skipped (wave-uniform: none when 16 NR == n)
#pragma unroll
  for (int r0 = 0; r0 < NR; r0 += RG)
    if (w + 16 * r0 >= n) {
#pragma unroll
      for (int u = 0; u < RG; ++u) mask_row(r0 + u);
    }
  float q[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    q[c] = x[0][c];
#pragma unroll
    for (int r = 1; r < NR; ++r) q[c] = fmaxf(q[c], x[r][c]);
  }
  column_total(q, true);   // q = column max
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float se = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      x[r][c] = exp_shift(x[r][c], q[c] * SAM_L2E);   // rows k >= n: -inf -> 0
      se += x[r][c];
    }
    q[c] = se;
  }
  column_total(q, false);   // q = column sum of exponentials
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float inv = __builtin_amdgcn_rcpf(q[c]);
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) {   // (rows k >= n: p = 0, as above)
      const int k = w + 16 * r;
      const float p = x[r][c] * inv;
      acc = fmaf(p, conf ? log2_pos(p + 1e-6f) : (float)k, acc);
    }
    q[c] = acc;
  }
  // the column totals of the accumulated terms, written by the threads that own column tid
#pragma unroll
  for (int c = 0; c < NC; ++c) red[w][lane + 64 * c] = q[c];
  lds_barrier();
  if (tid < n) {
    float acc = red[0][tid];
#pragma unroll
    for (int i = 1; i < 16; ++i) acc += red[i][tid];
    outL[ob + tid] = conf ? 1.0f - (-acc) / g.log2W2 : (float)tid - acc;
  }
}

// loads of one slice + slice_reduce, per volume kind (the kernel branches once, before the loads:
// with the branch after them the compiler shared values across both inlined bodies and spilled)
template <int NR, int NC, bool CONF, bool RT = false>
__device__ __forceinline__ void slice_one(const float *__restrict__ src, float (&red)[16][NC * 64],
                                          float (&colv)[NC * 64], const int n, const SGeo &g, float *outL,
                                          float *outR, const long ob, const int w, const int lane, const int tid,
                                          const bool rconf = false) {
  float x[NR][NC];
  // unconditional loads of clamped cells, all issued before any arithmetic; the cells outside the
  // slice become -inf only where they are first used (a load under the (k < n && j < n) predicate
  // compiled to a branch around each load; a select right after the load, to a branch on the
  // wave-uniform k < n with an immediate vmcnt(0) per load)
  // (buffer loads: the row offset wave-uniform in an SGPR, the column offset per lane; 64-bit
  // addresses cost a VALU add per load)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int kc = min(w + 16 * r, n - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c)
      x[r][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, min(lane + 64 * c, n - 1) * 4,
                                                                               kc * (int)g.sk * 4, 0));
  }
  slice_reduce<NR, NC, CONF, RT>(x, red, colv, n, g, outL, outR, ob, w, lane, tid, rconf);
}

#ifndef SA_SAM_CONF_FIRST
#define SA_SAM_CONF_FIRST 1   // 0: the disparity blocks first (the order before round 6's last change)
#endif

template <int NR, int NC>
__global__ __launch_bounds__(1024) void sam_slice_kernel(const float *__restrict__ vd, const float *__restrict__ vc,
                                                         SGeo g, int n, float *dL, float *dR, float *cL, float *cR,
                                                         int y0) {
  __shared__ float red[16][NC * 64];
  __shared__ float colv[NC * 64];
  // with both volumes the confidence blocks (the costlier kind: a log2 per cell and side) take
  // grid row 0, which the dispatcher issues first: the cheaper disparity blocks fill the last
  // partial round of one-block-per-CU waves (1088 blocks at cfg2 = 4.25 rounds of 256 CUs)
  const int conf = gridDim.y == 2 ? SA_SAM_CONF_FIRST ^ (int)blockIdx.y : y0 + (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / g.H, h = bh % g.H;
  const long so = (long)b * g.sb + (long)h * g.sh;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long ob = (long)b * g.obs + (long)h * n;
  if constexpr (NR * NC > 64)
    slice_one<NR, NC, false, true>(conf ? vc + so : vd + so, red, colv, n, g, conf ? cL : dL, conf ? cR : dR, ob, w,
                                   lane, tid, conf != 0);
  else if (conf)
    slice_one<NR, NC, true>(vc + so, red, colv, n, g, cL, cR, ob, w, lane, tid);
  else
    slice_one<NR, NC, false>(vd + so, red, colv, n, g, dL, dR, ob, w, lane, tid);
}

#ifndef SA_SAM_DIAG
#define SA_SAM_DIAG 0   // timing diagnostics (wrong results): 1 loads only, 2 no loads (synthetic cells)
#endif

// sam_slice_kernel with 16-byte rows (n % 4 == 0, n <= 256, rows 16-byte aligned): lane L holds
// columns 4L .. 4L + 3 of each of its wave's rows (one dwordx4 load per row instead of four
// dword loads), wave w rows k = w + 16 r.  The row sums add a lane's four terms first, then
// across the wave; the column partials go through LDS as in sam_slice_kernel.
template <int NR>
__global__ __launch_bounds__(1024) void sam_slice4_kernel(const float *__restrict__ vd, const float *__restrict__ vc,
                                                          SGeo g, int n, float *dL, float *dR, float *cL, float *cR,
                                                          int y0) {
  using f4 = __attribute__((ext_vector_type(4))) float;
  __shared__ __attribute__((aligned(16))) float red[16][256];
  __shared__ float colv[256];
  const int conf = y0 + (int)blockIdx.y;
  const float *vol = conf ? vc : vd;
  float *outL = conf ? cL : dL, *outR = conf ? cR : dR;
  const int bh = blockIdx.x, b = bh / g.H, h = bh % g.H;
  const float *src = vol + (long)b * g.sb + (long)h * g.sh;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long ob = (long)b * g.obs + (long)h * n;
  const bool lv = 4 * lane < n;
  f4 x[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int k = w + 16 * r;
    if (SA_SAM_DIAG == 2)
      x[r] = (k < n && lv) ? f4{(float)(k ^ lane), (float)(k + lane), (float)(k - lane), (float)(k * 3 % 7)} : f4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    else
      x[r] = (k < n && lv) ? *reinterpret_cast<const f4 *>(src + (long)k * g.sk + 4 * lane)
                           : f4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
  if (SA_SAM_DIAG == 1) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) t += x[r].x + x[r].y + x[r].z + x[r].w;
    if (t == 1.2345f) outL[ob + lane] = t;
    return;
  }
  // ---- right: per row k, softmax over j
  const float lw_r = g.log2W1;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int k = w + 16 * r;
    if (k >= n) continue;   // wave-uniform
    float m = fmaxf(fmaxf(x[r].x, x[r].y), fmaxf(x[r].z, x[r].w));
    m = wave_max(m);
    f4 e;
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = exp_le0(x[r][i] - m);   // -inf (j >= n) -> 0
    const float inv = 1.0f / wave_sum((e.x + e.y) + (e.z + e.w));
    float acc = 0.f;
    if (lv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = e[i] * inv;
        acc += conf ? p * log2_pos(p + 1e-6f) : p * (float)(4 * lane + i);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) outR[ob + k] = conf ? 1.0f - (-acc) / lw_r : acc - (float)k;
  }
  // ---- left: per column j, softmax over k
  auto column_total = [&](f4 &part, bool is_max) __attribute__((always_inline)) {
    *reinterpret_cast<f4 *>(&red[w][4 * lane]) = part;
    __syncthreads();
    if (tid < n) {
      float t = red[0][tid];
#pragma unroll
      for (int i = 1; i < 16; ++i) t = is_max ? fmaxf(t, red[i][tid]) : t + red[i][tid];
      colv[tid] = t;
    }
    __syncthreads();
    if (lv) part = *reinterpret_cast<const f4 *>(&colv[4 * lane]);
    __syncthreads();   // red / colv are reused by the next total
  };
  f4 q = x[0];
#pragma unroll
  for (int r = 1; r < NR; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = fmaxf(q[i], x[r][i]);
  column_total(q, true);   // q = column max
  f4 se = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[r][i] = exp_le0(x[r][i] - q[i]);   // rows k >= n: -inf -> 0
      se[i] += x[r][i];
    }
  column_total(se, false);   // column sum of exponentials
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float inv = 1.0f / se[i];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int k = w + 16 * r;
      const float p = x[r][i] * inv;
      if (k < n) acc[i] += conf ? p * log2_pos(p + 1e-6f) : p * (float)k;
    }
  }
  *reinterpret_cast<f4 *>(&red[w][4 * lane]) = acc;
  __syncthreads();
  if (tid < n) {
    float t = red[0][tid];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][tid];
    outL[ob + tid] = conf ? 1.0f - (-t) / g.log2W2 : (float)tid - t;
  }
}

// sam_slice_kernel for a slice of side n (sj == 1, W1 == W2); false if no instantiation fits
int sa_softargmin_v4 = 0;
bool launch_slices(const float *vd, const float *vc, const SGeo &g, int B, int n, float *dL, float *dR, float *cL,
                   float *cR, hipStream_t s) {
  // grid.y: the volumes present (a confidence-only call starts at y0 = 1)
  const dim3 grid((unsigned)(B * g.H), vd && vc ? 2u : 1u);
  const int y0 = vd ? 0 : 1;
  auto al = [](const float *p) { return !p || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (sa_softargmin_v4 && n % 4 == 0 && n <= 256 && g.sb % 4 == 0 && g.sh % 4 == 0 && g.sk % 4 == 0 && al(vd) && al(vc)) {
    if (n <= 240)
      sam_slice4_kernel<15><<<grid, 1024, 0, s>>>(vd, vc, g, n, dL, dR, cL, cR, y0);
    else
      sam_slice4_kernel<16><<<grid, 1024, 0, s>>>(vd, vc, g, n, dL, dR, cL, cR, y0);
    return true;
  }
#define SA_SLICE(NR_, NC_)                                                                          \
  if (n <= 16 * NR_ && n <= 64 * NC_ && (long)(n - 1) * g.sk * 4 + (long)n * 4 < 0x7fffffffL) {     \
    sam_slice_kernel<NR_, NC_><<<grid, 1024, 0, s>>>(vd, vc, g, n, dL, dR, cL, cR, y0);           \
    return true;                                                                                    \
  }
  SA_SLICE(8, 2)
  SA_SLICE(12, 3)
  SA_SLICE(15, 4)   // (n = 240, the model's 1/4 width: no all-padding row per thread)
  SA_SLICE(16, 4)
  SA_SLICE(18, 5)
#undef SA_SLICE
  return false;
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

// 1: the one-pass slice kernel where it applies (default); 0: the two line-kernel launches
// (sa_softargmin_set_one_pass, for A/B runs and tests)
static int sa_softargmin_one_pass = 1;
extern "C" void sa_softargmin_set_one_pass(int on) {
  // 0: the two line-kernel launches; 1 (default): the one-pass slice kernel; 2: the one-pass
  // slice kernel with 16-byte rows where they apply (cfg2: 128 against 119 us, so not default).
  // (Round 6 measured a persistent form that prefetches the next slice's first 144 rows into LDS
  // by LDS-DMA while reducing the current one: 136.6 against 118.7 us.  The slice reductions, not
  // the loads, bound this kernel: ~24 us of arithmetic per slice and volume, one block per CU.)
  sa_softargmin_one_pass = on ? 1 : 0;
  sa_softargmin_v4 = on == 2 ? 1 : 0;
}
extern "C" int sa_softargmin_get_one_pass() { return sa_softargmin_one_pass ? (sa_softargmin_v4 ? 2 : 1) : 0; }

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
  // one read of each volume: a block per (b, h) slice (the model's layout: j contiguous, square)
  if (sj == 1 && W1 == W2 && sa_softargmin_one_pass && launch_slices(vol_disp, vol_conf, g, B, W1, dL, dR, cL, cR, s))
    return sa::check_launch("sa_softargmin_conf");
  LineJob ld{vol_disp, dL, 0}, lc{vol_conf, cL, 1};
  LineJob rd{vol_disp, dR, 0}, rc{vol_conf, cR, 1};
  int rc1 = launch_side(ld, lc, g, B, 1, s);
  if (rc1) return rc1;
  return launch_side(rd, rc, g, B, 0, s);
}
