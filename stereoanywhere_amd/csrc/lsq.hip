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
    const int leader = __ffsll((long long)act) - 1;   // (wave-uniform: a v_readlane, not an LDS round trip)
    const unsigned lb = (unsigned)__builtin_amdgcn_readlane((int)bin, leader);
    const unsigned long long same = __ballot((act & me) && bin == lb);
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(&h[lb], (unsigned)__popcll(same));
    act &= ~same;
  }
  if (act & me) atomicAdd(&h[bin], 1u);
}

// ------------------------------------------------- weighted LSQ, one launch (round 6)
// One workgroup of 1024 threads per sample, one launch for the whole batch.  The four order
// statistics (floor / ceil ranks of the two linear quantiles) come from one pass over the keys
// instead of four radix passes:
//   A. a histogram of the top 15 bits of every key (relu'd values: sign 0, so 16384 bins of
//      relative width 2^-6) in LDS; a wave per rank finds the rank's bin and the count below it
//      (per-thread sums of 8 bins, then the bins of the one segment);
//   B. the keys of the (at most 4, usually 2) selected bins and their indices are copied into an LDS
//      pool at offsets known from the histogram (the pool holds 16384 keys: 25 % of a model sample);
//      the same pass accumulates the normal equations of every key in a bin strictly between the
//      lower and the upper quantile's bins (inside the band whatever the exact quantiles);
//   C. a 9-bit and an 8-bit radix pass over each rank's bin (its pool slice) give the exact key;
//      then the pooled keys inside the band add their terms (their mono / confidence values
//      gathered by index).
// A sample whose selected bins hold more keys than the pool (e.g. a quarter of the pixels at
// one value) takes the four full 8-bit radix passes instead (lsq_select_radix below, the round-5
// single-block algorithm) and a separate pass for the normal equations, in the same launch.
// Every pass streams the sample's keys from memory (L2-resident after the first) in chunks of
// L1_CH keys per thread whose loads are all in flight together: one load at a time, the pass
// would wait a round trip per key.
#ifdef SA_LSQ_CLOCK   // phase timestamps of block 0 (diagnostic builds)
__device__ long long g_lsq_clock[8];
#define LSQ_STAMP(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_lsq_clock[i] = __builtin_amdgcn_s_memrealtime()
#else
#define LSQ_STAMP(i)
#endif
constexpr int L1_BINS = 16384, L1_SHIFT = 17, L1_POOL = 16384, L1_SEG = 8, L1_CH = 16;
// Bin 0 holds the exact zeros alone, bin b >= 1 the positive keys whose top bits are b - 1: the
// relu'd zeros can be half of a sample (the model's synthetic-weight disparities; an edge's
// out-of-view pixels), and a quantile among them is exactly 0 without pooling or a radix pass (in
// one shared bin with the smallest positive keys they overflowed the pool: the four-pass fallback,
// 177 against ~75 us).  The largest key (NaN 0x7fc00000) maps to bin 16353 < L1_BINS.
__device__ __forceinline__ unsigned bin_of(unsigned k) { return k ? (k >> L1_SHIFT) + 1u : 0u; }

// f(key, index, valid) over this thread's keys of dd[0 .. n), in chunks of L1_CH loads in flight
template <class Fn>
__device__ __forceinline__ void lsq_stream_keys(const float *__restrict__ dd, int n, Fn f) {
  const int t = threadIdx.x;
  for (int base = 0; base < n; base += L1_CH * LSQ_THREADS) {
    unsigned k[L1_CH];
#pragma unroll
    for (int c = 0; c < L1_CH; ++c)   // (clamped, not predicated: a load under a branch waits at once)
      k[c] = key_of(dd[min(base + c * LSQ_THREADS + t, n - 1)]);
#pragma unroll
    for (int c = 0; c < L1_CH; ++c) {
      const int j = base + c * LSQ_THREADS + t;
      f(k[c], j, j < n);
    }
  }
}

// a[i] of a 4-entry register array for a wave-uniform i < 4 (no dynamic indexing: that goes to scratch)
template <class T>
__device__ __forceinline__ T pick4(const T (&a)[4], int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// the first index i of cnt[0 .. 64 * PER) (LDS) whose inclusive prefix count exceeds rem, and the
// count of the entries before it; every lane of the calling wave gets both
template <int PER>
__device__ __forceinline__ void wave_find(const unsigned *cnt, unsigned rem, int &idx, unsigned &below) {
  const int lane = threadIdx.x & 63;
  unsigned c[PER], tot = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    c[k] = cnt[lane * PER + k];
    tot += c[k];
  }
  unsigned inc = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  const unsigned long long past = __ballot(inc > rem);
  const int L = past ? __ffsll((long long)past) - 1 : 63;
  unsigned acc = inc - tot;
  int sel = PER - 1;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (acc + c[k] > rem) {
      sel = k;
      break;
    }
    acc += c[k];
  }
  idx = __shfl(L * PER + sel, L);
  below = __shfl(acc, L);
}

// The round-5 single-block selection: four 8-bit radix passes over all n keys (re-read from
// memory), ranks sharing a prefix share a histogram.  hist: LDS [4][256]; pre / rem: LDS [4]
// (rem holds the ranks on entry, the keys' prefixes in pre on exit).
__device__ __forceinline__ void lsq_select_radix(const float *__restrict__ dd, int n, unsigned *hist, unsigned *prefix,
                                 unsigned *remain) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < 4) prefix[t] = 0u;
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift_ = 24 - 8 * pass;
    for (int i = t; i < 4 * 256; i += LSQ_THREADS) hist[i] = 0u;
    __syncthreads();
    unsigned pre[4];
    int src[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pre[r] = prefix[r];
      src[r] = r;
      for (int q = r - 1; q >= 0; --q)
        if (pre[q] == pre[r]) src[r] = q;
    }
    lsq_stream_keys(dd, n, [&](unsigned k, int, bool valid) {
      const unsigned bin = (k >> shift_) & 255u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (src[r] != r) continue;
        const bool match = valid && (pass == 0 || ((k ^ pre[r]) >> (shift_ + 8)) == 0u);
        hist_add(hist + 256 * r, bin, match);
      }
    });
    __syncthreads();
    if (wv < 4) {
      int d;
      unsigned below;
      wave_find<4>(hist + 256 * pick4(src, wv), remain[wv], d, below);
      if (lane == 0) {
        remain[wv] -= below;
        prefix[wv] = pick4(pre, wv) | ((unsigned)d << shift_);
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(LSQ_THREADS) void lsq1_kernel(const float *__restrict__ mde, const float *__restrict__ disp,
                                                           const float *__restrict__ conf, int n, float q_lo,
                                                           float q_hi, float *__restrict__ scale,
                                                           float *__restrict__ shift) {
  __shared__ unsigned hist[L1_BINS];           // pass A; then the pooled keys' indices
  __shared__ unsigned pool[L1_POOL];           // the selected bins' keys
  __shared__ unsigned seg[L1_BINS / L1_SEG];   // 8-bin sums; then [4][512] digit histograms
  static_assert(L1_BINS / L1_SEG >= 4 * 512 && L1_BINS >= L1_POOL, "LDS reuse");
  __shared__ unsigned s_bin[4], s_rem[4], s_off[4], s_cnt[4], s_pre[4], s_total;
  __shared__ int s_list[4], s_fall;
  __shared__ double red[LSQ_THREADS / 64];
  __shared__ float qv[2];
  const int b = blockIdx.x;
  const float *md = mde + (long)b * n, *dd = disp + (long)b * n, *cd = conf + (long)b * n;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  LSQ_STAMP(7);

  // ranks of torch.quantile(linear): rank = q * (n - 1) in fp32
  const float r_lo = q_lo * (float)(n - 1), r_hi = q_hi * (float)(n - 1);
  if (t < 4) {
    const float r = (t < 2) ? r_lo : r_hi;
    s_rem[t] = (unsigned)((t & 1) ? ceilf(r) : truncf(r));
  }
  for (int i = t; i < L1_BINS; i += LSQ_THREADS) hist[i] = 0u;
  __syncthreads();
  LSQ_STAMP(0);
  // A: histogram of the top bits
  lsq_stream_keys(dd, n, [&](unsigned k, int, bool v) { hist_add(hist, bin_of(k), v); });
  __syncthreads();
  LSQ_STAMP(1);
  {
    unsigned sacc = 0;
#pragma unroll
    for (int k = 0; k < L1_SEG; ++k) sacc += hist[t * L1_SEG + k];
    for (int q = t + LSQ_THREADS; q < L1_BINS / L1_SEG; q += LSQ_THREADS) {   // (L1_BINS / L1_SEG > LSQ_THREADS)
      unsigned a2 = 0;
#pragma unroll
      for (int k = 0; k < L1_SEG; ++k) a2 += hist[q * L1_SEG + k];
      seg[q] = a2;
    }
    seg[t] = sacc;
  }
  __syncthreads();
  if (wv < 4) {   // wave r: rank r's bin and the keys below it
    int sg;
    unsigned below;
    wave_find<L1_BINS / L1_SEG / 64>(seg, s_rem[wv], sg, below);
    if (lane == 0) {
      unsigned acc = below, rem = s_rem[wv];
      int bin = sg * L1_SEG + L1_SEG - 1;
      for (int k = 0; k < L1_SEG; ++k) {
        const unsigned c = hist[sg * L1_SEG + k];
        if (acc + c > rem) {
          bin = sg * L1_SEG + k;
          break;
        }
        acc += c;
      }
      s_bin[wv] = (unsigned)bin;
      s_rem[wv] = rem - acc;   // the rank within its bin
    }
  }
  __syncthreads();
  if (t == 0) {   // pool slices of the distinct bins
    unsigned off = 0;
    int fall = 0;
    for (int r = 0; r < 4; ++r) {
      int src = r;
      for (int q = r - 1; q >= 0; --q)
        if (s_bin[q] == s_bin[r]) src = q;
      s_list[r] = src;
      if (src == r) {
        s_off[r] = off;
        s_cnt[r] = 0u;
        if (s_bin[r] != 0u) off += hist[s_bin[r]];   // (the zero bin is not pooled: its key is 0)
      }
    }
    fall = off > (unsigned)L1_POOL;
    s_fall = fall;
    s_total = off;
  }
  __syncthreads();
  LSQ_STAMP(2);
  const bool fall = s_fall != 0;
  unsigned lb[4];
  int lsrc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    lb[r] = s_bin[r];
    lsrc[r] = s_list[r];
  }
  double s11 = 0, s12 = 0, s22 = 0, t1 = 0, t2 = 0;
  auto add_terms = [&](float d, float mv, float cv) __attribute__((always_inline)) {
    const float m = fabsf(mv);
    const float cc = fabsf(cv) * 0.9f + 0.1f;
    const float w = sqrtf(cc);
    const float a1 = m * w, y = fabsf(d) * w;
    s11 += (double)a1 * a1;
    s12 += (double)a1 * w;
    s22 += (double)w * w;
    t1 += (double)a1 * y;
    t2 += (double)w * y;
  };
  // the zero keys' terms (d = 0: no t1 / t2 part), kept apart until the band is known: they are
  // inside it iff the lower quantile is 0, possible only when the floor rank's bin is the zero bin
  double z11 = 0, z12 = 0, z22 = 0;
  const bool zero_lo = lb[0] == 0u;
  auto add_zero = [&](float mv, float cv) __attribute__((always_inline)) {
    const float m = fabsf(mv);
    const float w = sqrtf(fabsf(cv) * 0.9f + 0.1f);
    const float a1 = m * w;
    z11 += (double)a1 * a1;
    z12 += (double)a1 * w;
    z22 += (double)w * w;
  };
  if (!fall) {
    // B: copy the selected bins' keys (and indices) into their pool slices (wave-aggregated
    // appends); the normal equations of the keys strictly between the quantiles' bins
    const unsigned in_lo = lb[1], in_hi = lb[2];   // (b0 <= b1 <= b2 <= b3)
    auto append = [&](unsigned k, int j, bool valid) __attribute__((always_inline)) {
      const unsigned bin = bin_of(k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (lsrc[r] != r || lb[r] == 0u) continue;   // (uniform; the zero bin is not pooled)
        const bool hit = valid && bin == lb[r];
        const unsigned long long m = __ballot(hit);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        unsigned base = 0;
        if (lane == leader) base = atomicAdd(&s_cnt[r], (unsigned)__popcll(m));
        base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
        if (hit) {
          const unsigned at = s_off[r] + base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
          pool[at] = k;
          hist[at] = (unsigned)j;
        }
      }
    };
    for (int base = 0; base < n; base += 8 * LSQ_THREADS) {
      unsigned kv[8];
      float mv[8], cv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {   // (clamped loads, all in flight together)
        const int jc = min(base + c * LSQ_THREADS + t, n - 1);
        kv[c] = key_of(dd[jc]);
        mv[c] = md[jc];
        cv[c] = cd[jc];
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int j = base + c * LSQ_THREADS + t;
        const unsigned bin = bin_of(kv[c]);
        append(kv[c], j, j < n);
        if (j < n && bin > in_lo && bin < in_hi) add_terms(__uint_as_float(kv[c]), mv[c], cv[c]);
        if (zero_lo && j < n && bin == 0u) add_zero(mv[c], cv[c]);
      }
    }
    __syncthreads();
  LSQ_STAMP(3);
    // C: the low 17 bits of each rank's key as a 9-bit and an 8-bit digit (seg reused as [4][512])
    if (t < 4) s_pre[t] = lb[t] ? (lb[t] - 1u) << L1_SHIFT : 0u;   // (a zero-bin rank: key 0, done)
    for (int pass = 0; pass < 2; ++pass) {
      const int sh = pass == 0 ? 8 : 0, bits = pass == 0 ? 9 : 8;   // bits 16..8, then 7..0
      for (int i = t; i < 4 * 512; i += LSQ_THREADS) seg[i] = 0u;
      __syncthreads();
      unsigned pre[4];
      int src[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pre[r] = s_pre[r];
        src[r] = r;
        for (int q = r - 1; q >= 0; --q)   // (same bin too: a bin-1 rank's prefix is 0 like the zero bin's)
          if (pre[q] == pre[r] && lb[q] == lb[r]) src[r] = q;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (src[r] != r || lb[r] == 0u) continue;   // (uniform)
        const int L = lsrc[r];
        const unsigned cnt = s_cnt[L], off = s_off[L];
        for (unsigned e0 = 0; e0 < cnt; e0 += LSQ_THREADS) {
          const unsigned e = e0 + t;
          const unsigned k = e < cnt ? pool[off + e] : 0u;
          const bool match = e < cnt && (pass == 0 || ((k ^ pre[r]) >> (sh + bits)) == 0u);
          hist_add(seg + 512 * r, (k >> sh) & ((1u << bits) - 1u), match);
        }
      }
      __syncthreads();
      if (wv < 4 && pick4(lb, wv) != 0u) {
        int d;
        unsigned below;
        wave_find<8>(seg + 512 * pick4(src, wv), s_rem[wv], d, below);
        if (lane == 0) {
          s_rem[wv] -= below;
          s_pre[wv] = pick4(pre, wv) | ((unsigned)d << sh);
        }
      }
      __syncthreads();
    }
  } else {
    if (t < 4) {
      const float r = (t < 2) ? r_lo : r_hi;
      s_rem[t] = (unsigned)((t & 1) ? ceilf(r) : truncf(r));
    }
    __syncthreads();
    lsq_select_radix(dd, n, hist, s_pre, s_rem);
  }
  LSQ_STAMP(4);
  if (t < 2) {
    const float r = t == 0 ? r_lo : r_hi;
    const float lo = __uint_as_float(s_pre[2 * t]), hi = __uint_as_float(s_pre[2 * t + 1]);
    qv[t] = lerp_ref(lo, hi, r - truncf(r));
  }
  __syncthreads();
  LSQ_STAMP(5);
  const float qlo = qv[0], qhi = qv[1];
  if (!fall && zero_lo && qlo <= 0.0f) {   // the zeros are inside the band (d = 0 >= lo = 0)
    s11 += z11;
    s12 += z12;
    s22 += z22;
  }
  if (!fall) {   // the pooled keys inside the band
    const unsigned total = s_total;
    for (unsigned e = t; e < total; e += LSQ_THREADS) {
      const float d = __uint_as_float(pool[e]);
      if (qlo <= d && d <= qhi) {
        const unsigned j = hist[e];
        add_terms(d, md[j], cd[j]);
      }
    }
  } else {   // (the fallback: every key against the band)
    for (int base = 0; base < n; base += 8 * LSQ_THREADS) {
      float dv[8], mv[8], cv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int j = base + c * LSQ_THREADS + t, jc = min(j, n - 1);
        dv[c] = __uint_as_float(key_of(dd[jc]));
        if (j >= n) dv[c] = -1.0f;   // (outside every band)
        mv[c] = md[jc];
        cv[c] = cd[jc];
      }
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (qlo <= dv[c] && dv[c] <= qhi) add_terms(dv[c], mv[c], cv[c]);
    }
  }
  s11 = block_sum(s11, red);
  s12 = block_sum(s12, red);
  s22 = block_sum(s22, red);
  t1 = block_sum(t1, red);
  t2 = block_sum(t2, red);
  LSQ_STAMP(6);
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
    const unsigned *hr = gh + 256 * pick4(src, wv);
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
      st->prefix[wv] = pick4(pre, wv) | (sel << shift_);
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
  lsq1_kernel<<<B, LSQ_THREADS, 0, s>>>(mde, disp, conf, n_per_b, q_lo, q_hi, scale, shift);
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

#ifdef SA_LSQ_CLOCK
extern "C" int sa_lsq_clock_read(long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lsq_clock), sizeof(long long) * 8) == hipSuccess ? 0 : -1;
}
#endif
