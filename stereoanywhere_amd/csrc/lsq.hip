// Mono-scale alignment: softLRC, weighted LSQ with exact quantile band, mirror
// detector and initial coordinates.
//
// Reference: softlrc + disp_warping (utils.py:172-198), fuzzy_and (240-241),
// weighted_lsq (345-384), scaled mono maps (stereoanywhere.py:191-199),
// handcrafted_mirror_detector (utils.py:255-269), coords init (stereoanywhere.py:261-262).
//
// The reference's weighted_lsq runs torch.quantile + boolean indexing +
// torch.linalg.lstsq per sample: host syncs and a CPU-side LAPACK call on GPU.  Here
// one workgroup per sample finds the four order statistics the two linear quantiles
// need by an 8-bit-per-pass radix select on the float bits (relu'd values are
// non-negative, so their bit patterns order like the values), then accumulates the
// 2x2 weighted normal equations in float64 and solves them — no host round trip.
#include <cmath>
#include <cstdint>

#include "sa_common.h"

namespace {

// ------------------------------------------------------------------ softLRC
__device__ __forceinline__ float softplus_ref(float x) {
  // torch softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}

// grid_sample(bilinear, zeros, align_corners=True) of one [H,W] plane at the grid
// point (gx, gy) already normalised to [-1, 1] (ATen CPU ApplyGridSample order).
__device__ __forceinline__ float sample_zero_ac(const float *__restrict__ img, int H, int W, float gx,
                                                float gy) {
  const float ix = (gx + 1.0f) * ((float)(W - 1) / 2.0f);
  const float iy = (gy + 1.0f) * ((float)(H - 1) / 2.0f);
  float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, e = 1.0f - w;
  const float n = iy - yn, s = 1.0f - n;
  const float nw = s * e, ne = s * w, sw = n * e, se = n * w;
  xw = fminf(fmaxf(xw, -2.0f), (float)W + 1.0f);
  yn = fminf(fmaxf(yn, -2.0f), (float)H + 1.0f);
  const int xi = (int)xw, yi = (int)yn;
  auto at = [&](int y, int x) {
    return (x >= 0 && x <= W - 1 && y >= 0 && y <= H - 1) ? img[(long)y * W + x] : 0.0f;
  };
  return at(yi, xi) * nw + at(yi, xi + 1) * ne + at(yi + 1, xi) * sw + at(yi + 1, xi + 1) * se;
}

// softlrc of pixel (y, x): compare d_self with d_other warped by relu(d_src)
// sign = -1: left map (sample at x - relu(d2)), +1: right map (x + relu(d3)).
__device__ __forceinline__ float softlrc_px(const float *__restrict__ dself, const float *__restrict__ dother,
                                            int H, int W, int y, int x, float sign, float th,
                                            float div) {
  const float dsrc = fmaxf(dself[(long)y * W + x], 0.0f);
  const float xn = sign < 0 ? ((float)x - dsrc) : ((float)x + dsrc);
  const float gx = 2.0f * (xn / (float)W) - 1.0f;
  const float gy = 2.0f * ((float)y / (float)H) - 1.0f;
  const float warped = sample_zero_ac(dother, H, W, gx, gy);
  const float d = dself[(long)y * W + x];
  return softplus_ref(-fabsf(d - warped) + th) / div;
}

__global__ __launch_bounds__(256) void softlrc_kernel(const float *__restrict__ d2, const float *__restrict__ d3,
                                                      const float *__restrict__ c2, const float *__restrict__ c3,
                                                      int H, int W, long bs, float th, float div, long npix,
                                                      float *__restrict__ s2, float *__restrict__ s3) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long b = p / hw, r = p % hw;
  const int y = (int)(r / W), x = (int)(r % W);
  const float *a = d2 + b * bs, *c = d3 + b * bs;
  // softlrc_disp2 uses warped_disp3 = disp_warping(relu(disp2), disp3, right_disp=False)
  float v2 = softlrc_px(a, c, H, W, y, x, -1.0f, th, div);
  float v3 = softlrc_px(c, a, H, W, y, x, +1.0f, th, div);
  if (c2) v2 = c2[b * bs + r] * v2;
  if (c3) v3 = c3[b * bs + r] * v3;
  s2[b * bs + r] = v2;
  s3[b * bs + r] = v3;
}

// ------------------------------------------------------------------ weighted LSQ
constexpr int LSQ_THREADS = 1024;

__device__ __forceinline__ unsigned key_of(float d) {
  d = fmaxf(d, 0.0f);  // F.relu (utils.py:352)
  if (d == 0.0f) d = 0.0f;  // -0 -> +0 so bit order == value order
  return __float_as_uint(d);
}

__device__ __forceinline__ float lerp_ref(float a, float b, float w) {
  // at::lerp CPU: |w| < 0.5 ? a + w (b - a) : b - (b - a)(1 - w)
  return fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < LSQ_THREADS / 64; ++i) t += red[i];  // fixed order: deterministic
  return t;
}

// LDS histogram add of one key per lane.  Keys of a wave often share a few bins (the
// high digits: sign and exponent; clustered values): the lanes of each of the first few
// distinct bins are counted with one atomic of their number instead of a many-way
// same-address conflict; lanes left after that add one each.
__device__ __forceinline__ void hist_add(unsigned *h, unsigned bin, bool count) {
  unsigned long long act = __ballot(count);
  const unsigned long long me = 1ull << (threadIdx.x & 63);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    if (!act) return;
    const int leader = __ffsll((long long)act) - 1;
    const unsigned lb = __shfl(bin, leader);
    const unsigned long long same = __ballot((act & me) && bin == lb);
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(&h[lb], (unsigned)__popcll(same));
    act &= ~same;
  }
  if (act & me) atomicAdd(&h[bin], 1u);
}

// KPT > 0: the sample's keys (n <= KPT * LSQ_THREADS) stay in registers over the four
// radix passes; KPT == 0: they are re-read from memory each pass.
template <int KPT>
__global__ __launch_bounds__(LSQ_THREADS) void lsq_kernel(const float *__restrict__ mde, const float *__restrict__ disp,
                                                          const float *__restrict__ conf, int n, float q_lo,
                                                          float q_hi, float *__restrict__ scale,
                                                          float *__restrict__ shift) {
  __shared__ unsigned hist[4][256];
  __shared__ unsigned prefix[4];
  __shared__ unsigned remain[4];
  __shared__ double red[LSQ_THREADS / 64];
  __shared__ float qv[2];
  const int b = blockIdx.x;
  const float *md = mde + (long)b * n, *dd = disp + (long)b * n, *cd = conf + (long)b * n;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;

  unsigned keys[KPT > 0 ? KPT : 1];
  if (KPT > 0) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int j = t + i * LSQ_THREADS;
      keys[i] = j < n ? key_of(dd[j]) : 0u;
    }
  }

  // ranks of torch.quantile(linear): rank = q * (n - 1) in fp32
  const float r_lo = q_lo * (float)(n - 1), r_hi = q_hi * (float)(n - 1);
  if (t < 4) {
    const float r = (t < 2) ? r_lo : r_hi;
    const float idx = (t & 1) ? ceilf(r) : truncf(r);
    remain[t] = (unsigned)idx;
    prefix[t] = 0u;
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift_ = 24 - 8 * pass;
    for (int i = t; i < 4 * 256; i += LSQ_THREADS) (&hist[0][0])[i] = 0u;
    __syncthreads();
    // ranks whose selected prefix so far equals an earlier rank's share its histogram
    unsigned pre[4];
    int src[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pre[r] = prefix[r];
      src[r] = r;
      for (int q = r - 1; q >= 0; --q)
        if (pre[q] == pre[r]) src[r] = q;
    }
    auto count = [&](unsigned k, bool valid) {
      const unsigned bin = (k >> shift_) & 255u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (src[r] != r) continue;  // uniform
        const bool match = valid && (pass == 0 || ((k ^ pre[r]) >> (shift_ + 8)) == 0u);
        hist_add(hist[r], bin, match);
      }
    };
    if (KPT > 0) {
#pragma unroll
      for (int i = 0; i < KPT; ++i) count(keys[i], t + i * LSQ_THREADS < n);
    } else {
      for (int i0 = 0; i0 < n; i0 += LSQ_THREADS) {
        const int i = i0 + t;
        count(i < n ? key_of(dd[i]) : 0u, i < n);
      }
    }
    __syncthreads();
    if (wv < 4) {
      // wave wv selects rank wv's digit: lane l owns bins 4l..4l+3; inclusive scan of the
      // lane totals, the first lane whose running count passes the rank holds the digit
      const unsigned *hr = hist[src[wv]];
      const unsigned rem = remain[wv];
      const unsigned c0 = hr[4 * lane], c1 = hr[4 * lane + 1], c2 = hr[4 * lane + 2], c3 = hr[4 * lane + 3];
      unsigned inc = c0 + c1 + c2 + c3;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
      }
      const unsigned long long past = __ballot(inc > rem);
      const int L = past ? __ffsll((long long)past) - 1 : 63;
      if (lane == L) {
        unsigned acc = inc - (c0 + c1 + c2 + c3), sel = 4u * L + 3u;
        const unsigned cs[4] = {c0, c1, c2, c3};
        for (int k = 0; k < 4; ++k) {
          if (acc + cs[k] > rem) {
            sel = 4u * L + k;
            break;
          }
          acc += cs[k];
        }
        remain[wv] = rem - acc;
        prefix[wv] = pre[wv] | (sel << shift_);
      }
    }
    __syncthreads();
  }
  if (t < 2) {
    const float r = t == 0 ? r_lo : r_hi;
    const float lo = __uint_as_float(prefix[2 * t]), hi = __uint_as_float(prefix[2 * t + 1]);
    qv[t] = lerp_ref(lo, hi, r - truncf(r));
  }
  __syncthreads();
  const float qlo = qv[0], qhi = qv[1];
  double s11 = 0, s12 = 0, s22 = 0, t1 = 0, t2 = 0;
  auto accum = [&](int i, unsigned k) {
    const float d = __uint_as_float(k);
    if (qlo <= d && d <= qhi) {
      const float m = fabsf(md[i]);
      const float c = fabsf(cd[i]) * 0.9f + 0.1f;
      const float w = sqrtf(c);
      const float a1 = m * w, y = fabsf(d) * w;
      s11 += (double)a1 * a1;
      s12 += (double)a1 * w;
      s22 += (double)w * w;
      t1 += (double)a1 * y;
      t2 += (double)w * y;
    }
  };
  if (KPT > 0) {
#pragma unroll
    for (int u = 0; u < KPT; ++u)
      if (t + u * LSQ_THREADS < n) accum(t + u * LSQ_THREADS, keys[u]);
  } else {
    for (int i = t; i < n; i += LSQ_THREADS) accum(i, key_of(dd[i]));
  }
  s11 = block_sum(s11, red);
  s12 = block_sum(s12, red);
  s22 = block_sum(s22, red);
  t1 = block_sum(t1, red);
  t2 = block_sum(t2, red);
  if (t == 0) {
    const double det = s11 * s22 - s12 * s12;
    double sc, sh;
    if (s22 > 0 && fabs(det) > 1e-12 * s11 * s22) {
      sc = (s22 * t1 - s12 * t2) / det;
      sh = (s11 * t2 - s12 * t1) / det;
    } else if (s22 > 0) {
      // rank-deficient (all kept mono values equal): minimum-norm solution like gelsy
      const double m0 = s12 / s22, c0 = t2 / s22;
      sc = c0 * m0 / (m0 * m0 + 1.0);
      sh = c0 / (m0 * m0 + 1.0);
    } else {
      sc = 0.0;
      sh = 0.0;
    }
    scale[b] = (float)sc;
    shift[b] = (float)sh;
  }
}

// ---------------------------------------------------- weighted LSQ, grid-wide variant
// The same radix select and normal equations spread over LSQ_NB(n) blocks per sample:
// one launch per 8-bit digit, each block histograms its slice in LDS and adds the
// non-zero bins to the sample's global histogram; the block that finishes last (an
// arrival counter) selects the digit for the next launch and clears the histogram.  The
// final launch forms per-block float64 partials that the last block sums in block order
// (deterministic) before solving.  Workspace per sample, zeroed before the first launch:
//   LsqState (64 B) | hist[4][256] u32 | part[nb][5] f64.
constexpr int LSQ_BT = 256, LSQ_EPT = 8, LSQ_CH = LSQ_BT * LSQ_EPT;

struct LsqState {
  unsigned prefix[4], remain[4], count, pad[7];
};

inline int lsq_nb(int n) { return (n + LSQ_CH - 1) / LSQ_CH; }
inline long lsq_ws_stride(int n) { return ((64 + 4096 + (long)lsq_nb(n) * 40) + 255) / 256 * 256; }

__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lsq_initial_ranks(int n, float q_lo, float q_hi, int r, unsigned &rem) {
  const float rk = (r < 2 ? q_lo : q_hi) * (float)(n - 1);
  rem = (unsigned)((r & 1) ? ceilf(rk) : truncf(rk));
}

__global__ __launch_bounds__(LSQ_BT) void lsq_hist_kernel(const float *__restrict__ disp, int n, int nb, float q_lo,
                                                          float q_hi, int pass, char *__restrict__ ws, long wss) {
  __shared__ unsigned hist[4][256];
  __shared__ unsigned s_pre[4], s_rem[4];
  __shared__ int s_last;
  const int b = blockIdx.x / nb, j = blockIdx.x % nb;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  LsqState *st = reinterpret_cast<LsqState *>(ws + b * wss);
  unsigned *gh = reinterpret_cast<unsigned *>(ws + b * wss + 64);
  if (t < 4) {
    if (pass == 0) {
      lsq_initial_ranks(n, q_lo, q_hi, t, s_rem[t]);
      s_pre[t] = 0u;
    } else {
      s_pre[t] = st->prefix[t];
      s_rem[t] = st->remain[t];
    }
  }
  for (int i = t; i < 4 * 256; i += LSQ_BT) (&hist[0][0])[i] = 0u;
  __syncthreads();
  const int shift_ = 24 - 8 * pass;
  unsigned pre[4];
  int src[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    pre[r] = s_pre[r];
    src[r] = r;
    for (int q = r - 1; q >= 0; --q)
      if (pre[q] == pre[r]) src[r] = q;
  }
  const float *dd = disp + (long)b * n + (long)j * LSQ_CH;
  const int cnt = min(LSQ_CH, n - j * LSQ_CH);
  unsigned keys[LSQ_EPT];
#pragma unroll
  for (int i = 0; i < LSQ_EPT; ++i) keys[i] = t + i * LSQ_BT < cnt ? key_of(dd[t + i * LSQ_BT]) : 0u;
#pragma unroll
  for (int i = 0; i < LSQ_EPT; ++i) {
    const bool valid = t + i * LSQ_BT < cnt;
    const unsigned bin = (keys[i] >> shift_) & 255u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (src[r] != r) continue;
      const bool match = valid && (pass == 0 || ((keys[i] ^ pre[r]) >> (shift_ + 8)) == 0u);
      hist_add(hist[r], bin, match);
    }
  }
  __syncthreads();
  for (int i = t; i < 4 * 256; i += LSQ_BT) {
    const unsigned c = (&hist[0][0])[i];
    if (c && src[i >> 8] == (i >> 8)) atomicAdd(&gh[i], c);
  }
  __threadfence();
  __syncthreads();
  if (t == 0) s_last = atomicAdd(&st->count, 1u) == (unsigned)(nb - 1);
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  if (wv < 4) {
    const unsigned *hr = gh + 256 * src[wv];
    const unsigned rem = s_rem[wv];
    const unsigned c0 = ld_agent(hr + 4 * lane), c1 = ld_agent(hr + 4 * lane + 1);
    const unsigned c2 = ld_agent(hr + 4 * lane + 2), c3 = ld_agent(hr + 4 * lane + 3);
    unsigned inc = c0 + c1 + c2 + c3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    const unsigned long long past = __ballot(inc > rem);
    const int L = past ? __ffsll((long long)past) - 1 : 63;
    if (lane == L) {
      unsigned acc = inc - (c0 + c1 + c2 + c3), sel = 4u * L + 3u;
      const unsigned cs[4] = {c0, c1, c2, c3};
      for (int k = 0; k < 4; ++k) {
        if (acc + cs[k] > rem) {
          sel = 4u * L + k;
          break;
        }
        acc += cs[k];
      }
      st->remain[wv] = rem - acc;
      st->prefix[wv] = pre[wv] | (sel << shift_);
    }
  }
  __syncthreads();
  for (int i = t; i < 4 * 256; i += LSQ_BT) gh[i] = 0u;
  if (t == 0) st->count = 0u;
}

__global__ __launch_bounds__(LSQ_BT) void lsq_solve_kernel(const float *__restrict__ mde, const float *__restrict__ disp,
                                                           const float *__restrict__ conf, int n, int nb, float q_lo,
                                                           float q_hi, char *__restrict__ ws, long wss,
                                                           float *__restrict__ scale, float *__restrict__ shift) {
  __shared__ double red[5][LSQ_BT / 64];
  __shared__ int s_last;
  const int b = blockIdx.x / nb, j = blockIdx.x % nb;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  LsqState *st = reinterpret_cast<LsqState *>(ws + b * wss);
  double *part = reinterpret_cast<double *>(ws + b * wss + 64 + 4096);
  const float r_lo = q_lo * (float)(n - 1), r_hi = q_hi * (float)(n - 1);
  const float qlo = lerp_ref(__uint_as_float(st->prefix[0]), __uint_as_float(st->prefix[1]), r_lo - truncf(r_lo));
  const float qhi = lerp_ref(__uint_as_float(st->prefix[2]), __uint_as_float(st->prefix[3]), r_hi - truncf(r_hi));
  const long off = (long)b * n + (long)j * LSQ_CH;
  const int cnt = min(LSQ_CH, n - j * LSQ_CH);
  double acc[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < LSQ_EPT; ++i) {
    const int e = t + i * LSQ_BT;
    if (e >= cnt) continue;
    const float d = __uint_as_float(key_of(disp[off + e]));
    if (qlo <= d && d <= qhi) {
      const float m = fabsf(mde[off + e]);
      const float c = fabsf(conf[off + e]) * 0.9f + 0.1f;
      const float w = sqrtf(c);
      const float a1 = m * w, y = fabsf(d) * w;
      acc[0] += (double)a1 * a1;
      acc[1] += (double)a1 * w;
      acc[2] += (double)w * w;
      acc[3] += (double)a1 * y;
      acc[4] += (double)w * y;
    }
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    double v = acc[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[q][wv] = v;
  }
  __syncthreads();
  if (t < 5) part[j * 5 + t] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
  __threadfence();
  __syncthreads();
  if (t == 0) s_last = atomicAdd(&st->count, 1u) == (unsigned)(nb - 1);
  __syncthreads();
  if (!s_last || t != 0) return;
  __threadfence();
  double s[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < nb; ++k)
    for (int q = 0; q < 5; ++q)
      s[q] += __hip_atomic_load(part + k * 5 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  st->count = 0u;
  const double s11 = s[0], s12 = s[1], s22 = s[2], t1 = s[3], t2 = s[4];
  const double det = s11 * s22 - s12 * s12;
  double sc, sh;
  if (s22 > 0 && fabs(det) > 1e-12 * s11 * s22) {
    sc = (s22 * t1 - s12 * t2) / det;
    sh = (s11 * t2 - s12 * t1) / det;
  } else if (s22 > 0) {
    const double m0 = s12 / s22, c0 = t2 / s22;
    sc = c0 * m0 / (m0 * m0 + 1.0);
    sh = c0 / (m0 * m0 + 1.0);
  } else {
    sc = 0.0;
    sh = 0.0;
  }
  scale[b] = (float)sc;
  shift[b] = (float)sh;
}

// ------------------------------------------------------------------ scaled mono + mirror
__global__ __launch_bounds__(256) void scale_maps_kernel(const float *__restrict__ m2, const float *__restrict__ m3,
                                                         const float *__restrict__ scale,
                                                         const float *__restrict__ shift, long hw, long in_bs,
                                                         long npix, float *__restrict__ sm2,
                                                         float *__restrict__ sm3) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long b = p / hw, r = p % hw;
  const float s = scale[b], t = shift[b];
  sm2[p] = s * m2[b * in_bs + r] + t;
  sm3[p] = s * m3[b * in_bs + r] + t;
}

__global__ __launch_bounds__(256) void mirror_kernel(const float *__restrict__ sm2, const float *__restrict__ sm3,
                                                     const float *__restrict__ dL, const float *__restrict__ confl,
                                                     int H, int W, long in_bs, float th, float div,
                                                     float conf_th, long npix, float *__restrict__ mirror,
                                                     float *__restrict__ coords_x) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long b = p / hw, r = p % hw;
  const int y = (int)(r / W), x = (int)(r % W);
  const float lrc = softlrc_px(sm2 + b * hw, sm3 + b * hw, H, W, y, x, -1.0f, th, div);
  const float sc = confl[b * in_bs + r], md = sm2[p], sd = dL[b * in_bs + r];
  const float both = sc * lrc;
  const float near_ = sa::sigmoidf_ref(20.0f * (md - sd));
  const float a = both * near_;
  const float bb = (1.0f - sc) * lrc;
  const float better = a + bb - a * bb;
  mirror[p] = sa::sigmoidf_ref(20.0f * (better - conf_th));
  coords_x[p] = (float)x - md;
}

}  // namespace

extern "C" int sa_softlrc(const float *d2, const float *d3, const float *conf2, const float *conf3, int B,
                          int H, int W, long map_bs, float lrc_th, float *s2, float *s3, void *stream) {
  SA_REQUIRE(d2 && d3 && s2 && s3, "sa_softlrc: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_softlrc: empty shape");
  SA_REQUIRE(map_bs >= (long)H * W, "sa_softlrc: map_bs too small");
  const long npix = (long)B * H * W;
  const float div = (float)std::log(1.0 + std::exp((double)lrc_th));
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  softlrc_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(d2, d3, conf2, conf3, H, W, map_bs, lrc_th,
                                                                div, npix, s2, s3);
  return sa::check_launch("sa_softlrc");
}

extern "C" int sa_weighted_lsq(const float *mde, const float *disp, const float *conf, int B, int n_per_b,
                               float q_lo, float q_hi, float *scale, float *shift, void *stream) {
  SA_REQUIRE(mde && disp && conf && scale && shift, "sa_weighted_lsq: null pointer");
  SA_REQUIRE(B > 0 && n_per_b > 0, "sa_weighted_lsq: empty input");
  SA_REQUIRE(q_lo >= 0.f && q_lo <= q_hi && q_hi <= 1.f, "sa_weighted_lsq: quantiles out of order");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LSQ, s);
  if (n_per_b <= 32 * LSQ_THREADS)
    lsq_kernel<32><<<B, LSQ_THREADS, 0, s>>>(mde, disp, conf, n_per_b, q_lo, q_hi, scale, shift);
  else
    lsq_kernel<0><<<B, LSQ_THREADS, 0, s>>>(mde, disp, conf, n_per_b, q_lo, q_hi, scale, shift);
  return sa::check_launch("sa_weighted_lsq");
}

extern "C" long sa_weighted_lsq_ws_size(int B, int n_per_b) {
  if (B <= 0 || n_per_b <= 0) return -1;
  return (long)B * lsq_ws_stride(n_per_b);
}

extern "C" int sa_weighted_lsq_ws(const float *mde, const float *disp, const float *conf, int B, int n_per_b,
                                  float q_lo, float q_hi, float *scale, float *shift, void *ws, void *stream) {
  SA_REQUIRE(mde && disp && conf && scale && shift && ws, "sa_weighted_lsq_ws: null pointer");
  SA_REQUIRE(B > 0 && n_per_b > 0, "sa_weighted_lsq_ws: empty input");
  SA_REQUIRE(q_lo >= 0.f && q_lo <= q_hi && q_hi <= 1.f, "sa_weighted_lsq_ws: quantiles out of order");
  SA_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, "sa_weighted_lsq_ws: workspace not 16-byte aligned");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LSQ, s);
  const int nb = lsq_nb(n_per_b);
  const long wss = lsq_ws_stride(n_per_b);
  char *w = static_cast<char *>(ws);
  for (int pass = 0; pass < 4; ++pass) {
    lsq_hist_kernel<<<(unsigned)(B * nb), LSQ_BT, 0, s>>>(disp, n_per_b, nb, q_lo, q_hi, pass, w, wss);
    const int rc = sa::check_launch("sa_weighted_lsq_ws/hist");
    if (rc) return rc;
  }
  lsq_solve_kernel<<<(unsigned)(B * nb), LSQ_BT, 0, s>>>(mde, disp, conf, n_per_b, nb, q_lo, q_hi, w, wss, scale,
                                                         shift);
  return sa::check_launch("sa_weighted_lsq_ws/solve");
}

extern "C" int sa_mono_scale_mirror(const float *m2, const float *m3, const float *scale, const float *shift,
                                    const float *dL, const float *conf_l, int B, int H, int W, long in_bs,
                                    float lrc_th, float conf_th, float *sm2, float *sm3, float *mirror,
                                    float *coords_x, void *stream) {
  SA_REQUIRE(m2 && m3 && scale && shift && dL && conf_l && sm2 && sm3 && mirror && coords_x,
             "sa_mono_scale_mirror: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_mono_scale_mirror: empty shape");
  SA_REQUIRE(in_bs >= (long)H * W, "sa_mono_scale_mirror: in_bs too small");
  const long npix = (long)B * H * W;
  const float div = (float)std::log(1.0 + std::exp((double)lrc_th));
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  const unsigned nb = (unsigned)((npix + 255) / 256);
  scale_maps_kernel<<<nb, 256, 0, s>>>(m2, m3, scale, shift, (long)H * W, in_bs, npix, sm2, sm3);
  int rc = sa::check_launch("sa_mono_scale_mirror/scale");
  if (rc) return rc;
  mirror_kernel<<<nb, 256, 0, s>>>(sm2, sm3, dL, conf_l, H, W, in_bs, lrc_th, div, conf_th, npix, mirror, coords_x);
  return sa::check_launch("sa_mono_scale_mirror/mirror");
}
