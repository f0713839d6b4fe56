// Full-resolution tail of the mono hourglass as fused direct 3-D convolutions.
//
// Reference: Hourglass.forward tail (hourglass.py:325-329) = trilinear upsample +
// cat + final_agg (three BasicConv3d: conv -> InstanceNorm3d -> LeakyReLU,
// submodule.py:25-53) + final_feature_atts_up (DoubleFeatureAtt, submodule.py:113-140),
// then classifier_mono / classifier_monoconf (stereoanywhere.py:73-74, 165-166).
//
// At 544x960 these run on [B, 8, 240, 136, 240] volumes (7.8 M voxels per channel per
// pair): with 8 channels the convolutions are tiny GEMMs, and the library path spent
// ~14 ms per conv plus separate statistic / normalise / activation / gate passes.
// Here every layer is one pass over HBM:
//   * the conv applies the PREVIOUS layer's InstanceNorm + LeakyReLU (+ gate) to its
//     input while staging it in LDS (zero padding applies to the activated input);
//   * the epilogue writes the raw conv output and per-block (sum, sum of squares) of
//     each (b, co) channel for the NEXT layer's InstanceNorm (float64 partials, reduced
//     in fixed order by sa_instnorm_finalize: deterministic);
//   * the first layer (1x1x1 over cat(orig, up(x))) evaluates the trilinear upsample of
//     the half-resolution branch on the fly, so the 16-channel full-res upsampled
//     tensor and the concatenation are never materialised;
//   * both classifiers share one conv launch (Cout = 2).
// Layout everywhere: [B, C, D, H, W] with D = W2 (right pixel), W = W1 (left pixel).
#include <cmath>
#include <type_traits>

#include "sa_common.h"

// Convolution sums have no reference summation order to reproduce (MIOpen picks its own
// algorithm), so let a*b+c contract to (packed) FMA here; the library builds with
// -ffp-contract=off for the element-wise kernels that mirror torch expressions.
#pragma clang fp contract(fast)

namespace {

// Output tiles: 256 threads = TWx (along W) x THx (along H), each thread owning TDx
// planes along D.  A 64-lane wave stages one input row of the tile's halo per load, so
// the halo row must fit 64 floats: stride-1 tiles use 62 of their 64 columns, stride-2
// tiles 31 of 32 (same tile counts as 64 / 32 for the volume widths the model has).
constexpr int TW = 64;  // pointwise tiles along W
constexpr int TH = 4;   // along H
constexpr int TD = 4;   // output planes per thread along D
constexpr int ROW = 64; // LDS row pitch (floats)

struct InXform {
  const float *mean, *rstd;   // per (b, ci), or null
  const float *gl, *gr;       // gate maps [B, C, H, W] and [B, C, H, D] (sigmoid'ed), or null
  float slope;                // LeakyReLU slope
  int act;                    // apply LeakyReLU
};

__device__ __forceinline__ float xform(float v, const InXform &t, long bc, int d, int h, int w, int H, int W, int D) {
  if (t.mean) v = (v - t.mean[bc]) * t.rstd[bc];
  if (t.act) v = v > 0.0f ? v : v * t.slope;
  if (t.gl) {
    const float g = t.gl[(bc * H + h) * W + w] * t.gr[(bc * H + h) * D + d];
    v = g * v;
  }
  return v;
}

#ifndef SA_STATS_DPP
#define SA_STATS_DPP 1   // the wave sums of block_stats on DPP (0: __shfl_xor butterfly)
#endif
// block partial sums of (x, x^2) over the tile for each of NC channels -> partial[bc][blk].
// A thread's own values (at most TD of them) are summed in fp32, everything above in fp64.
template <int NC>
__device__ __forceinline__ void block_stats(const float (&s)[NC], const float (&q)[NC], double *red,
                                            double *partial, long b, int nparts, int blk, int Cout, int c0 = 0) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#if SA_STATS_DPP
    // (DPP: the ds_bpermute butterfly is 12 dependent LDS round trips per channel)
    const double a = sa::wave_sum_dpp_lane63((double)s[c]), e = sa::wave_sum_dpp_lane63((double)q[c]);
    if (lane == 63) {
#else
    double a = (double)s[c], e = (double)q[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      e += __shfl_xor(e, o);
    }
    if (lane == 0) {
#endif
      red[(c * 4 + wv) * 2] = a;
      red[(c * 4 + wv) * 2 + 1] = e;
    }
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    const int c = threadIdx.x;
    double a = 0.0, e = 0.0;
    for (int w = 0; w < 4; ++w) {
      a += red[(c * 4 + w) * 2];
      e += red[(c * 4 + w) * 2 + 1];
    }
    double *p = partial + ((b * Cout + c0 + c) * (long)nparts + blk) * 2;
    p[0] = a;
    p[1] = e;
  }
}

// The masked mono volume (stereoanywhere.py:161, mono_volume.hip) is one-hot over its
// nbins channels: cell (n, d, h, w) = 1.73 * (nL[h,w] . nR[h,d]) / sqrt(3) if the left pixel
// (h, w) and the right pixel (h, d) are both in depth bin n, else 0.  Its two consumers
// evaluate the cells from per-pixel records (n0, n1, n2, bin) (sa_mono_bin_records) instead of
// reading 8 channels of which 7 are zero: a tap costs one weight-row gather W[bin][tap][:].
struct OneHotVol {
  const float4 *recL;   // [B, H, W]: left pixels (the volume's W axis = W1)
  const float4 *recR;   // [B, H, D]: right pixels (its D axis = W2)
  float gain;
};

// the masked_volume_kernel's value, same operation order, no contraction; bin -1 (none) or a
// padding sentinel never matches
__device__ __forceinline__ float onehot_cell(const float4 l, const float4 r, float gain, int &bin) {
#pragma clang fp contract(off)
  const float v = gain * ((l.x * r.x + l.y * r.y + l.z * r.z) / sqrtf(3.0f));
  const bool m = l.w == r.w && l.w >= 0.0f;
  bin = m ? (int)l.w : 0;
  return m ? v : 0.0f;
}

// Stride-2 3x3x3 conv (pad 1, no bias) of the one-hot volume (down_layers[0][0],
// hourglass.py:27-33 / submodule.py:25-53): out[co] = sum over taps of W[bin][tap][co] * cell.
// Thread = one (w, h) output column x TDx output planes along D; block 64 (w) x 4 (h).  The
// taps' records come from L1/L2 (the left record of (h, w) serves every d, the right records
// of (h, d) every w); weight rows in LDS at a pitch that puts the 8 bins' 16-byte reads on
// disjoint banks.
template <int COUT, int TDx>
__global__ __launch_bounds__(256) void conv3d_onehot_s2_kernel(OneHotVol v, int nbins, int D, int H, int W, int Do,
                                                               int Ho, int Wo, const float *__restrict__ wt,
                                                               float *__restrict__ out, double *__restrict__ partial,
                                                               int tilesD) {
  constexpr int WP = 27 * COUT + 4;   // weight row pitch: (WP / 4) odd -> 8 rows on disjoint 16-byte banks
  static_assert(COUT % 4 == 0 && (WP / 4) % 2 == 1, "weight pitch");
  __shared__ __attribute__((aligned(16))) float ws[8 * WP];
  __shared__ double red[COUT * 4 * 2];
  for (int i = threadIdx.x; i < nbins * 27 * COUT; i += 256) {
    const int n = i / (27 * COUT), r = i - n * 27 * COUT;
    ws[n * WP + r] = wt[i];
  }
  __syncthreads();
  const int tx_ = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int wo = blockIdx.x * 64 + tx_, ho = blockIdx.y * 4 + ty;
  const int b = blockIdx.z / tilesD, d0 = (blockIdx.z % tilesD) * TDx;
  const bool ok = wo < Wo && ho < Ho;
  const int woc = min(wo, Wo - 1), hoc = min(ho, Ho - 1);
  const float4 *rl = v.recL + (long)b * H * W, *rr = v.recR + (long)b * H * D;
  const float4 pad_l = make_float4(0.f, 0.f, 0.f, -3.f), pad_r = make_float4(0.f, 0.f, 0.f, -2.f);
  float acc[TDx][COUT];
#pragma unroll
  for (int i = 0; i < TDx; ++i)
#pragma unroll
    for (int c = 0; c < COUT; ++c) acc[i][c] = 0.f;
  constexpr int ND = 2 * TDx + 1;   // input planes of the thread's outputs
#pragma unroll 1
  for (int kh = 0; kh < 3; ++kh) {
    const int h = 2 * hoc - 1 + kh;
    const bool hok = h >= 0 && h < H;
    float4 r[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int d = 2 * d0 - 1 + i;
      r[i] = (hok && d >= 0 && d < D) ? rr[(long)h * D + d] : pad_r;
    }
#pragma unroll 1
    for (int kw = 0; kw < 3; ++kw) {
      const int w = 2 * woc - 1 + kw;
      const float4 l = (hok && w >= 0 && w < W) ? rl[(long)h * W + w] : pad_l;
      float cv[ND];
      int cb[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) cv[i] = onehot_cell(l, r[i], v.gain, cb[i]);
#pragma unroll
      for (int od = 0; od < TDx; ++od)
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          const int i = 2 * od + kd;
          const float4 *wp = reinterpret_cast<const float4 *>(ws + cb[i] * WP + ((kd * 3 + kh) * 3 + kw) * COUT);
#pragma unroll
          for (int g = 0; g < COUT / 4; ++g) {
            const float4 w4 = wp[g];
            acc[od][4 * g + 0] += w4.x * cv[i];
            acc[od][4 * g + 1] += w4.y * cv[i];
            acc[od][4 * g + 2] += w4.z * cv[i];
            acc[od][4 * g + 3] += w4.w * cv[i];
          }
        }
    }
  }
  float s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0f;
  if (ok) {
#pragma unroll
    for (int od = 0; od < TDx; ++od) {
      const int d = d0 + od;
      if (d < Do) {
#pragma unroll
        for (int co = 0; co < COUT; ++co) {
          out[(((long)b * COUT + co) * Do + d) * (long)Ho * Wo + (long)ho * Wo + wo] = acc[od][co];
          s[co] += acc[od][co];
          q[co] += acc[od][co] * acc[od][co];
        }
      }
    }
  }
  if (partial) {
    const int nparts = gridDim.x * gridDim.y * tilesD;
    const int blk = (blockIdx.z % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
    block_stats<COUT>(s, q, red, partial, b, nparts, blk, COUT);
  }
}

// F(4,3) transforms (points 0, +-1, +-2, inf; the same B^T / A^T as conv2d_wino4.hip), for
// correlation along one axis: out[i] = sum_k g[k] x[i + k] = A^T ((G g) . (B^T x))
__device__ __forceinline__ void bt6(const float x0, const float x1, const float x2, const float x3, const float x4,
                                    const float x5, float *o) {
  const float a = x4 - 4.0f * x2, b = x3 - 4.0f * x1, c = x4 - x2, e = x3 - x1;
  o[0] = 4.0f * x0 - 5.0f * x2 + x4;
  o[1] = a + b;
  o[2] = a - b;
  o[3] = 2.0f * e + c;
  o[4] = c - 2.0f * e;
  o[5] = 4.0f * x1 - 5.0f * x3 + x5;
}
__device__ __forceinline__ void at6(const float *m, float *o) {
  const float a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], e = m[3] - m[4];
  o[0] = m[0] + a + c;
  o[1] = b + 2.0f * e;
  o[2] = a + 4.0f * c;
  o[3] = b + 8.0f * e + m[5];
}

template <int S, int TWx>
struct ConvTile {
  static constexpr int valid_w = TWx - (S == 1 ? 2 : 1);  // output columns per tile
};

// 3x3x3, stride S, padding 1, no bias; CIN input channels, COUT outputs.
//   staging: the halo of input channel ci+1 is fetched into registers (one 64-lane row load
//   per row, row coordinates wave-uniform) while channel ci is convolved out of LDS, then
//   transformed (InstanceNorm / LeakyReLU / gate of the producer) and written to the other
//   LDS buffer; one barrier per input channel.
//   compute: for each (kh, kw) the thread reads the LD input planes its TDx outputs touch
//   once and reuses them across the 3 kd taps; weights [ci][tap][co] come in as scalars.
template <int CIN, int COUT, int S, int TDx, int TWx, int THx>
__global__ __launch_bounds__(256) void conv3d_kernel(const float *__restrict__ in, int Di, int Hi, int Wi, int Do,
                                                     int Ho, int Wo, const float *__restrict__ wt, InXform tx,
                                                     float *__restrict__ out, double *__restrict__ partial,
                                                     int tilesD) {
  static_assert(TWx * THx == 256, "256 threads per block");
  constexpr int TWV = ConvTile<S, TWx>::valid_w;
  constexpr int LW = (TWV - 1) * S + 3, LH = (THx - 1) * S + 3, LD = (TDx - 1) * S + 3;
  static_assert(LW <= ROW, "halo row must fit one wave");
  constexpr int ROWS = LD * LH, RPW = (ROWS + 3) / 4;  // rows per wave
  static_assert(RPW <= 32, "row mask is 32 bits");
  constexpr int LBUF = ROWS * ROW + 2 * ROW;            // + slack for the idle columns' reads
  __shared__ float tile[2][LBUF];
  __shared__ double red[COUT * 4 * 2];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tx_ = threadIdx.x % TWx, ty = threadIdx.x / TWx;
  const int w0 = blockIdx.x * TWV, h0 = blockIdx.y * THx;
  const int b = blockIdx.z / tilesD, d0 = (blockIdx.z % tilesD) * TDx;
  const long vol = (long)Di * Hi * Wi;
  const int iw0 = w0 * S - 1, ih0 = h0 * S - 1, id0 = d0 * S - 1;
  const int wl = iw0 + lane;                              // this lane's input column
  const bool lane_ok = lane < LW && wl >= 0 && wl < Wi;
  float acc[TDx][COUT];
#pragma unroll
  for (int i = 0; i < TDx; ++i)
#pragma unroll
    for (int c = 0; c < COUT; ++c) acc[i][c] = 0.f;

  // branch-free staging: clamped addresses, padding selected to zero at commit (divergent
  // branches per row would keep one saved exec mask per row live in SGPRs)
  float pv[RPW], pg[RPW];
  unsigned okm = 0;
  const int wcl = min(max(wl, 0), Wi - 1);
  auto fetch_rows = [&](auto gated, int ci) __attribute__((always_inline)) {
    constexpr bool G = decltype(gated)::value;
    const long bc = (long)b * CIN + ci;
    const float *src = in + bc * vol;  // plane bases in 64 bits once; offsets in a plane fit 32
    const float *glb = G ? tx.gl + bc * Hi * Wi : nullptr;
    const float *grb = G ? tx.gr + bc * Hi * Di : nullptr;
    okm = 0;
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      int r = wv + 4 * k;
      asm volatile("" : "+s"(r));  // recompute the row math per fetch (SALU) instead of hoisting it into SGPRs
      const int dd = r / LH, hh = r - dd * LH;
      const int d = id0 + dd, h = ih0 + hh;
      const bool rok = r < ROWS && d >= 0 && d < Di && h >= 0 && h < Hi;
      const int dc = min(max(d, 0), Di - 1), hc = min(max(h, 0), Hi - 1);
      const float *rowp = src + (unsigned)((dc * Hi + hc) * Wi);  // scalar row base, lane offset
      pv[k] = rowp[(unsigned)wcl];
      if (G) pg[k] = glb[(unsigned)(hc * Wi) + (unsigned)wcl] * grb[hc * Di + dc];
      okm |= (rok && lane_ok) ? (1u << k) : 0u;
    }
  };
  auto fetch = [&](int ci) __attribute__((always_inline)) {
    if (tx.gl) fetch_rows(std::true_type{}, ci);
    else fetch_rows(std::false_type{}, ci);
  };
  auto commit = [&](int ci, int buf) __attribute__((always_inline)) {
    const long bc = (long)b * CIN + ci;
    float mean = 0.0f, rstd = 1.0f;
    if (tx.mean) {
      mean = tx.mean[bc];
      rstd = tx.rstd[bc];
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int r = wv + 4 * k;
      if (r < ROWS) {
        float v = pv[k];
        if (tx.mean) v = (v - mean) * rstd;
        if (tx.act) v = v > 0.0f ? v : v * tx.slope;
        if (tx.gl) v = pg[k] * v;
        tile[buf][r * ROW + lane] = ((okm >> k) & 1u) ? v : 0.0f;
      }
    }
  };

  fetch(0);
  commit(0, 0);
  __syncthreads();
  constexpr int KWU = COUT <= 8 ? 3 : 1;
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    const int buf = ci & 1;
    if (ci + 1 < CIN) fetch(ci + 1);
    const float *tb = tile[buf] + (ty * S) * ROW + tx_ * S;
    const float *wc = wt + (long)ci * 27 * COUT;  // weights pre-arranged [ci][tap][co]
#pragma unroll 1
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll KWU
      for (int kw = 0; kw < 3; ++kw) {
        float v[LD];
#pragma unroll
        for (int p = 0; p < LD; ++p) v[p] = tb[(p * LH + kh) * ROW + kw];
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          const float *wp = wc + ((kd * 3 + kh) * 3 + kw) * COUT;
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float wv_ = wp[co];
#pragma unroll
            for (int od = 0; od < TDx; ++od) acc[od][co] += wv_ * v[od * S + kd];
          }
        }
      }
    }
    if (ci + 1 < CIN) commit(ci + 1, buf ^ 1);
    __syncthreads();
  }

  const int w = w0 + tx_, h = h0 + ty;
  float s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0f;
  if (tx_ < TWV && w < Wo && h < Ho) {
#pragma unroll
    for (int od = 0; od < TDx; ++od) {
      const int d = d0 + od;
      if (d < Do) {
#pragma unroll
        for (int co = 0; co < COUT; ++co) {
          out[(((long)b * COUT + co) * Do + d) * (long)Ho * Wo + (long)h * Wo + w] = acc[od][co];
          s[co] += acc[od][co];
          q[co] += acc[od][co] * acc[od][co];
        }
      }
    }
  }
  if (partial) {
    const int nparts = gridDim.x * gridDim.y * tilesD;
    const int blk = (blockIdx.z % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
    block_stats<COUT>(s, q, red, partial, b, nparts, blk, COUT);
  }
}

// Stride-1 3x3x3 conv of 8 input channels (final_agg[1], final_agg[2] and the classifier pair:
// hourglass.py:329, submodule.py:25-53, stereoanywhere.py:165-166) as Winograd F(4,3) along D:
// for each (ci, kh, kw) the 3 D-taps of the kernel act on a column of the input along D, so the
// column is transformed once when it is staged (6 points per 4 outputs, points 0, +-1, +-2, inf:
// B^T / A^T of conv2d_wino4.hip) and every tap pair (kh, kw) multiplies it by the transformed
// kernel G g: 6 products per 4 outputs instead of 12 (12 + 12 FMA per column and output channel
// instead of 24 for the two D-tiles of a thread).  The products accumulate in the transform
// domain over (ci, kh, kw); one A^T per output column at the end.
//   block  = 64 (w) x 4 (h) threads, each 2 D-tiles (8 planes) x COUT channels; the staged slab
//            of one input channel is [6 h rows][64 w columns][12 points] (16-byte reads of a
//            column's points: a wave's 16-lane groups hit disjoint banks at the 48-byte stride)
//   staging = the producer's InstanceNorm + LeakyReLU (+ gate), zero padding, then B^T along D,
//            fetched one input channel ahead; one barrier per input channel
//   weights = (G g)[ci][kh][kw][p][co] (sa_conv3d_wd weight layout), wave-uniform (SGPR) operands
//   WL     = the weights staged in LDS a channel ahead with the input (per channel 54 x COUT
//            floats, double-buffered), read as wave-uniform LDS vectors instead of SGPR loads
//            (the scalar-load variant spends 42% of its wave cycles at waitcnt / barrier);
//            measured slower, so off by default (sa_conv3d_wd_set_variant)
//   PK     = (NT = 2) the two D-tiles' points interleaved in the slab, (t0 p, t1 p) pairs, so a
//            16-byte read is two aligned register pairs and each (p, co) product pair is one
//            v_pk_fma_f32 with the weight broadcast from its SGPR.  Without it the compiler packs
//            over output-channel pairs and copies the X values that sit in odd registers into
//            pairs whose other half can be a pending global load of the next channel's prefetch:
//            the copy then waits for that load (s_waitcnt vmcnt) inside the first tap pair of
//            every channel, and the prefetch stops overlapping the FMAs.
//   DMA    = the next channel's raw columns fetched by LDS-DMA (buffer_load_dword ... lds) into
//            a [6 rows][LD planes][64 lanes] staging area instead of 2 x LD VGPRs per thread; each
//            wave reads back only its own lanes' words, after its own vmcnt(0) in commit
#ifndef SA_WD_BUF
#define SA_WD_BUF 0   // 1: the staging loads as buffer loads (diagnostic: 8 -> 8 then needs 175 VGPRs)
#endif
//   COTT   = the conv's total output channels when a block computes COUT of them (COUT = 16 of
//            32: the 32-channel stride-1 conv as two channel halves, blockIdx.z = (b, D tile, half))
template <int CIN, int COUT, int NT, bool GATED, bool WL = false, bool PK = false, bool DMA = false, int COTT = 0>
__global__ __launch_bounds__(256) void conv3d_wd_kernel(const float *__restrict__ in, int D, int H, int W,
                                                        const float *__restrict__ wt, InXform tx,
                                                        float *__restrict__ out, double *__restrict__ partial,
                                                        int tilesD) {
  constexpr int TD = 4 * NT, LD = TD + 2, NP = 6 * NT, LH = 6, TWV = 62;
  constexpr int ROWP = 64 * NP + 4;   // row pitch (floats); 16-byte aligned
  // a column's points: 16-byte accesses at a 48-byte lane stride (NT = 2) or 8-byte ones at 24
  // (NT = 1); either way a wave's lane groups hit disjoint banks
  using VT = typename std::conditional<NP % 4 == 0, float4, float2>::type;
  constexpr int VW = sizeof(VT) / 4;
  static_assert(ROWP % 4 == 0, "row alignment");
  constexpr int CC = COUT < 8 ? COUT : 8;   // output channels per weight group (48 SGPRs)
  constexpr int COT = COTT ? COTT : COUT, NS = COT / COUT;
  static_assert(COT % COUT == 0 && (NS == 1 || !WL), "channel split");
  __shared__ __attribute__((aligned(16))) float slab[2][LH * ROWP];
  __shared__ double red[COUT * 4 * 2];
  __shared__ float raw[DMA ? LH : 1][DMA ? LD : 1][64];
  constexpr int WPC = 54 * COUT, NWL = (WPC + 255) / 256;   // weights per input channel, per thread
  __shared__ __attribute__((aligned(16))) float wsl[WL ? 2 : 1][WL ? WPC : 4];
  float pw[NWL];
  auto wfetch = [&](int ci) __attribute__((always_inline)) {
    if constexpr (WL) {
#pragma unroll
      for (int q = 0; q < NWL; ++q) {
        const int idx = (int)threadIdx.x + 256 * q;
        pw[q] = idx < WPC ? wt[(long)ci * WPC + idx] : 0.0f;
      }
    }
  };
  auto wcommit = [&](int buf) __attribute__((always_inline)) {
    if constexpr (WL) {
#pragma unroll
      for (int q = 0; q < NWL; ++q) {
        const int idx = (int)threadIdx.x + 256 * q;
        if (idx < WPC) wsl[buf][idx] = pw[q];
      }
    }
  };
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w0 = blockIdx.x * TWV, h0 = blockIdx.y * 4;
  // (NS == 1: the unsigned blockIdx.z arithmetic of the unsplit kernel, whose tap-loop schedule
  // the 16-channel conv is sensitive to: 575 against 640 us with the signed form)
  const unsigned zc = blockIdx.z / NS;
  const int co0 = NS == 1 ? 0 : (int)(blockIdx.z % NS) * COUT;
  const int b = zc / tilesD, d0 = (zc % tilesD) * TD;
  const int hw = H * W;
  const int wl = w0 - 1 + lane;
  const bool wok = wl >= 0 && wl < W;
  const int wcl = min(max(wl, 0), W - 1);
  // D-validity of the LD staged planes (block-uniform)
  unsigned dmask = 0;
#pragma unroll
  for (int j = 0; j < LD; ++j) dmask |= (d0 - 1 + j >= 0 && d0 - 1 + j < D) ? (1u << j) : 0u;
  // this lane's plane offset for the gate_r vector load (lane j < LD holds plane d0 - 1 + j)
  const int dlane = min(max(d0 - 1 + min(lane, LD - 1), 0), D - 1);

  // staging columns of this thread: (row wv, lane) and, for waves 0-1, (row wv + 4, lane)
  constexpr int NCOL = 2;
  float pv[NCOL][DMA ? 1 : LD];
  float pgl[NCOL], pgr[NCOL];
  float pmean, prstd;   // the channel's InstanceNorm, fetched with its columns
  auto fetch = [&](int ci) __attribute__((always_inline)) {
    const long bc = (long)b * CIN + ci;
    const float *src = in + bc * (long)D * hw;
    if constexpr (NT == 2) {   // (the 16-channel convs measured ~8% slower with this)
      pmean = tx.mean[bc];
      prstd = tx.rstd[bc];
    }
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int hh = wv + 4 * k;
      if ((NT == 2 && k == 0) || hh < LH) {   // (row wv < 4 always exists)
        const int hc = min(max(h0 - 1 + hh, 0), H - 1);
        const float *colp = src + hc * W + wcl;
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          int off = min(max(d0 - 1 + j, 0), D - 1) * hw;
          if constexpr (DMA) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src), (short)0, D * hw * 4, 0x00020000);
            // the LDS address laundered through an SGPR: the DMA then carries no alias scope, and
            // the compiler does not make the slab reads of the tap loop wait for it (vmcnt(0));
            // commit waits for this wave's DMAs itself
            unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void *)&raw[hh][j][0];
            asm volatile("" : "+s"(la));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(uintptr_t)la, 4,
                                                     (off + hc * W + wcl) * 4, 0, 0, 0);
          } else if constexpr (SA_WD_BUF) {
            // a buffer load at a 32-bit lane offset from the channel's base (no 64-bit address
            // per load); the plane offset in a VGPR (SGPRs hold the weights)
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src), (short)0, D * hw * 4, 0x00020000);
            int vo = (off + hc * W + wcl) * 4;
            asm volatile("" : "+v"(vo));
            pv[k][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
          } else {
            asm volatile("" : "+v"(off));   // plane offsets in VGPRs: SGPRs hold the weights
            pv[k][j] = colp[off];
          }
        }
        if (GATED) {
          pgl[k] = tx.gl[(bc * H + hc) * W + wcl];
          pgr[k] = tx.gr[(bc * H + hc) * D + dlane];   // one plane per lane, read back by readlane
        }
      }
    }
  };
  auto commit = [&](int ci, int buf) __attribute__((always_inline)) {
    // NT = 2: mean / rstd were fetched with the columns.  Loading them here, the loads' target
    // registers were reused by the tap loop, and at its head the compiler waited for every
    // outstanding load (s_waitcnt vmcnt(0)), i.e. for the next channel's prefetch: 8 -> 8
    // 1100 -> 970 us without that wait
    const long bc = (long)b * CIN + ci;
    const float mean = NT == 2 ? pmean : tx.mean[bc], rstd = NT == 2 ? prstd : tx.rstd[bc];
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs landed
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int hh = wv + 4 * k;
      if ((NT == 2 && k == 0) || hh < LH) {
        const int h = h0 - 1 + hh;
        const bool cok = wok && h >= 0 && h < H;
        float x[LD];
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          float v = ((DMA ? raw[hh][j][lane] : pv[k][j]) - mean) * rstd;
          v = v > 0.0f ? v : v * tx.slope;
          if (GATED) {   // gate_l[h, w] * gate_r[h, d] (xform's order)
            const float gr = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pgr[k]), j));
            v = (pgl[k] * gr) * v;
          }
          x[j] = (cok && ((dmask >> j) & 1u)) ? v : 0.0f;
        }
        float o[NP];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          bt6(x[4 * t], x[4 * t + 1], x[4 * t + 2], x[4 * t + 3], x[4 * t + 4], x[4 * t + 5], o + 6 * t);
        VT *dst = reinterpret_cast<VT *>(slab[buf] + hh * ROWP + lane * NP);
#pragma unroll
        for (int q = 0; q < NP / VW; ++q) {
          VT v;
#pragma unroll
          for (int e = 0; e < VW; ++e) {
            const int i = VW * q + e;   // slab position; PK: (t0 p, t1 p) pairs
            reinterpret_cast<float *>(&v)[e] = PK ? o[6 * (i & 1) + (i >> 1)] : o[i];
          }
          dst[q] = v;
        }
      }
    }
  };

  static_assert(!PK || NT == 2, "PK pairs the two D-tiles");
  using f2 = __attribute__((ext_vector_type(2))) float;
  float M[PK ? 1 : NT][6][COUT];
  f2 M2[PK ? 6 : 1][PK ? COUT : 1];
#pragma unroll
  for (int t = 0; t < (PK ? 1 : NT); ++t)
#pragma unroll
    for (int p = 0; p < 6; ++p)
#pragma unroll
      for (int c = 0; c < COUT; ++c) M[t][p][c] = 0.0f;
  if constexpr (PK) {
#pragma unroll
    for (int p = 0; p < 6; ++p)
#pragma unroll
      for (int c = 0; c < COUT; ++c) M2[p][c] = f2{0.0f, 0.0f};
  }

  fetch(0);
  wfetch(0);
  commit(0, 0);
  wcommit(0);
  __syncthreads();
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    const int buf = ci & 1;
    if (ci + 1 < CIN) {
      fetch(ci + 1);
      wfetch(ci + 1);
    }
    // lanes 62-63 (no output column) read lane 61's columns: lane + kw stays inside the 64
    // staged columns of the row
    const float *lb = slab[buf] + wv * ROWP + min(lane, TWV - 1) * NP;
    const float *wc = WL ? wsl[buf] : wt + (long)ci * 9 * 6 * COT + (NS == 1 ? 0 : co0);
    // the kw loop unrolled for the 16-channel convs and the classifier pair (the scalar weight
    // loads of the next kw then overlap this one's FMAs: 711 -> 567 and 568 -> 506 us), rolled
    // for 8 -> 8 (unrolled it measured 1057 -> 1310 us: SGPR pressure of 48 weights per kw;
    // with 4- or 2-channel weight groups 1460 / 1900 us, rolled with 4-channel groups 1130)
    constexpr int KW_UNR = (NT == 1 || COUT <= 2) ? 3 : 1;
#pragma unroll 1
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll KW_UNR
      for (int kw = 0; kw < 3; ++kw) {
        const VT *xp = reinterpret_cast<const VT *>(lb + kh * ROWP + kw * NP);
        float X[NP];
#pragma unroll
        for (int q = 0; q < NP / VW; ++q) {
          const VT v = xp[q];
#pragma unroll
          for (int e = 0; e < VW; ++e) X[VW * q + e] = reinterpret_cast<const float *>(&v)[e];
        }
        const float *wp = wc + (kh * 3 + kw) * 6 * COT;
#pragma unroll
        for (int cg = 0; cg < COUT / CC; ++cg) {
          if (cg) __builtin_amdgcn_sched_barrier(0);   // one channel group's weights live at a time
#pragma unroll
          for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int c = cg * CC; c < cg * CC + CC; ++c) {
              const float wv_ = wp[p * COT + c];
              if constexpr (PK) {
                const f2 xp2 = f2{X[2 * p], X[2 * p + 1]};
                M2[p][c] = __builtin_elementwise_fma(xp2, f2{wv_, wv_}, M2[p][c]);
              } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) M[t][p][c] += X[6 * t + p] * wv_;
              }
            }
        }
      }
    }
    if (ci + 1 < CIN) {
      commit(ci + 1, buf ^ 1);
      wcommit(buf ^ 1);
    }
    __syncthreads();
  }

  // A^T along D, stores, InstanceNorm partials
  const int w = w0 + lane, h = h0 + wv;
  const bool ok = lane < TWV && w < W && h < H;
  float s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int c = 0; c < COUT; ++c) {
      float m[6], o[4];
#pragma unroll
      for (int p = 0; p < 6; ++p) m[p] = PK ? M2[p][c][t] : M[t][p][c];
      at6(m, o);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = d0 + 4 * t + i;
        if (ok && d < D) {
          out[(((long)b * COT + co0 + c) * D + d) * (long)hw + (long)h * W + w] = o[i];
          s[c] += o[i];
          q[c] += o[i] * o[i];
        }
      }
    }
  if (partial) {
    const int nparts = gridDim.x * gridDim.y * tilesD;
    const int blk = (zc % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
    block_stats<COUT>(s, q, red, partial, b, nparts, blk, COT, co0);
  }
}

// 1x1x1 conv with the producer's transform on load: out = W . T(in), no statistics.
// Projects the low-resolution branch of an up-cat conv onto the output channels before it
// is upsampled (W_u . up(T(u)) = up(W_u . T(u)): trilinear interpolation is linear).
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void pointwise_kernel(const float *__restrict__ in, InXform tx, int D, int H, int W,
                                                        long n, const float *__restrict__ wt,
                                                        float *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long dhw = (long)D * H * W;
  const long b = i / dhw, pos = i - b * dhw;
  const int w = (int)(pos % W), h = (int)((pos / W) % H), d = (int)(pos / ((long)W * H));
  float r[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) r[co] = 0.0f;
#pragma unroll 4
  for (int c = 0; c < CIN; ++c) {
    const long bc = b * CIN + c;
    const float v = xform(in[bc * dhw + pos], tx, bc, d, h, w, H, W, D);
#pragma unroll
    for (int co = 0; co < COUT; ++co) r[co] += wt[c * COUT + co] * v;
  }
#pragma unroll
  for (int co = 0; co < COUT; ++co) out[(b * COUT + co) * dhw + pos] = r[co];
}

// 1x1x1 conv over cat(Ta(a), trilinear_up(u)) -> COUT channels, + IN partial statistics,
// evaluated as Wa . Ta(a) + up(p) with p = Wu . T(u) already at the low resolution
// (pointwise_kernel).  The block's low-resolution footprint of p (at most 4 x 4 x 34
// voxels for an upsampling factor >= 2) is staged in LDS as [d][h][w][co], so each
// voxel's 8 trilinear corners are COUT/4 float4 reads apiece.
// OH: a is the one-hot mono volume given by its records (OneHotVol): Wa . a = Wa[bin] * cell,
// one weight-row gather per voxel instead of CA products.
template <int CA, int COUT, bool AX, bool OH = false>
__global__ __launch_bounds__(256) void pointwise_upcat_kernel(const float *__restrict__ a, InXform ta, OneHotVol oh,
                                                              const float *__restrict__ pu, int D, int H, int W,
                                                              int Du, int Hu, int Wu, float sd, float sh, float sw,
                                                              const float *__restrict__ wt, float *__restrict__ out,
                                                              double *__restrict__ partial, int tilesD) {
  constexpr int TWV = TW;  // no halo: full, aligned 64-wide tiles
  constexpr int ED = 4, EH = 4, EW = 34;
  static_assert(COUT % 4 == 0, "float4 corners");
  __shared__ float4 pt[ED * EH * EW * (COUT / 4)];
  __shared__ double red[COUT * 4 * 2];
  __shared__ float4 wa[OH ? CA * COUT / 4 : 1];
  if (OH)
    for (int i = threadIdx.x; i < CA * COUT; i += 256) reinterpret_cast<float *>(wa)[i] = wt[i];
  const int tx_ = threadIdx.x & 63;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // one H row per wave
  const int w0 = blockIdx.x * TWV, h0 = blockIdx.y * TH;
  const int w = w0 + tx_, h = h0 + ty;
  const int b = blockIdx.z / tilesD, d0 = (blockIdx.z % tilesD) * TD;
  const long vol = (long)D * H * W;
  // upsample_trilinear3d(align_corners=True): source index floor(s * dst), monotone in dst
  const int dlo = (int)(sd * (float)d0), hlo = (int)(sh * (float)h0), wlo = (int)(sw * (float)w0);
  {
    float *ptf = reinterpret_cast<float *>(pt);
    for (int i = threadIdx.x; i < ED * EH * EW * COUT; i += 256) {
      const int ww = i % EW, r = i / EW, hh = r % EH, r2 = r / EH, dd = r2 % ED, co = r2 / ED;
      const int dz = dlo + dd, hy = hlo + hh, wx = wlo + ww;
      float v = 0.0f;
      if (dz < Du && hy < Hu && wx < Wu) v = pu[(((long)b * COUT + co) * Du + dz) * (long)Hu * Wu + (long)hy * Wu + wx];
      ptf[((dd * EH + hh) * EW + ww) * COUT + co] = v;
    }
  }
  __syncthreads();
  float s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0f;
  const bool col_ok = tx_ < TWV && w < W && h < H;
  const int wc = min(w, W - 1), hc = min(h, H - 1);
  // Wa . Ta(a): all TD planes of this (h, w) column per input channel
  float r[TD][COUT];
#pragma unroll
  for (int od = 0; od < TD; ++od)
#pragma unroll
    for (int co = 0; co < COUT; ++co) r[od][co] = 0.0f;
  const long pos0 = ((long)min(d0, D - 1) * H + hc) * W + wc;
  if constexpr (OH) {
    // the sum over the CA channels has one non-zero term: r = Wa[bin] * cell (as the dense sum
    // gives it: zero products add nothing)
    const float4 l = oh.recL[((long)b * H + hc) * W + wc];
    const float4 *rr = oh.recR + ((long)b * H + hc) * D;
#pragma unroll
    for (int od = 0; od < TD; ++od) {
      int bin;
      const float cv = onehot_cell(l, rr[min(d0 + od, D - 1)], oh.gain, bin);
#pragma unroll
      for (int g = 0; g < COUT / 4; ++g) {
        const float4 w4 = wa[bin * (COUT / 4) + g];
        r[od][4 * g + 0] += w4.x * cv;
        r[od][4 * g + 1] += w4.y * cv;
        r[od][4 * g + 2] += w4.z * cv;
        r[od][4 * g + 3] += w4.w * cv;
      }
    }
  }
#pragma unroll 2
  for (int c = 0; c < (OH ? 0 : CA); ++c) {
    const long bc = (long)b * CA + c;
    const float *ap = a + bc * vol + pos0;
    float av[TD];
#pragma unroll
    for (int od = 0; od < TD; ++od) av[od] = d0 + od < D ? ap[(long)od * H * W] : 0.0f;
    if (AX) {
      float mean = 0.0f, rstd = 1.0f, gl = 1.0f;
      if (ta.mean) {
        mean = ta.mean[bc];
        rstd = ta.rstd[bc];
      }
      if (ta.gl) gl = ta.gl[(bc * H + hc) * W + wc];
#pragma unroll
      for (int od = 0; od < TD; ++od) {
        float v = av[od];
        if (ta.mean) v = (v - mean) * rstd;
        if (ta.act) v = v > 0.0f ? v : v * ta.slope;
        if (ta.gl) v = (gl * ta.gr[(bc * H + hc) * D + min(d0 + od, D - 1)]) * v;
        av[od] = v;
      }
    }
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      const float wv_ = wt[c * COUT + co];
#pragma unroll
      for (int od = 0; od < TD; ++od) r[od][co] += wv_ * av[od];
    }
  }
  // + up(p) from the LDS footprint
  const float rh = sh * (float)hc, rw = sw * (float)wc;
  const int h1 = (int)rh, w1 = (int)rw;
  const int h1p = h1 < Hu - 1 ? 1 : 0, w1p = w1 < Wu - 1 ? 1 : 0;
  const float hl1 = rh - (float)h1, hl0 = 1.0f - hl1, wl1 = rw - (float)w1, wl0 = 1.0f - wl1;
  const int lh = h1 - hlo, lw = w1 - wlo;
#pragma unroll
  for (int od = 0; od < TD; ++od) {
    const int d = d0 + od;
    const float rd = sd * (float)min(d, D - 1);
    const int d1 = (int)rd;
    const int d1p = d1 < Du - 1 ? 1 : 0;
    const float dl1 = rd - (float)d1, dl0 = 1.0f - dl1;
    const float4 *c000 = pt + (((d1 - dlo) * EH + lh) * EW + lw) * (COUT / 4);
    const int od_ = d1p * EH * EW * (COUT / 4), oh_ = h1p * EW * (COUT / 4), ow_ = w1p * (COUT / 4);
#pragma unroll
    for (int g = 0; g < COUT / 4; ++g) {
      const float4 p000 = c000[g], p001 = c000[ow_ + g], p010 = c000[oh_ + g], p011 = c000[oh_ + ow_ + g];
      const float4 p100 = c000[od_ + g], p101 = c000[od_ + ow_ + g], p110 = c000[od_ + oh_ + g],
                   p111 = c000[od_ + oh_ + ow_ + g];
#define SA_TRI(F)                                                                                 \
  (dl0 * (hl0 * (wl0 * p000.F + wl1 * p001.F) + hl1 * (wl0 * p010.F + wl1 * p011.F)) +            \
   dl1 * (hl0 * (wl0 * p100.F + wl1 * p101.F) + hl1 * (wl0 * p110.F + wl1 * p111.F)))
      r[od][4 * g + 0] += SA_TRI(x);
      r[od][4 * g + 1] += SA_TRI(y);
      r[od][4 * g + 2] += SA_TRI(z);
      r[od][4 * g + 3] += SA_TRI(w);
#undef SA_TRI
    }
    if (col_ok && d < D) {
      const long pos = ((long)d * H + h) * W + w;
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        out[((long)b * COUT + co) * vol + pos] = r[od][co];
        s[co] += r[od][co];
        q[co] += r[od][co] * r[od][co];
      }
    }
  }
  const int nparts = gridDim.x * gridDim.y * tilesD;
  const int blk = (blockIdx.z % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
  block_stats<COUT>(s, q, red, partial, b, nparts, blk, COUT);
}

// T(x) materialised (for the low-resolution branch an up-cat conv reads at 8 corners)
__global__ __launch_bounds__(256) void vol_apply_kernel(const float *__restrict__ in, InXform tx, int C, int D, int H,
                                                        int W, long n, float *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int w = (int)(i % W);
  const long r = i / W;
  const int h = (int)(r % H);
  const long r2 = r / H;
  const int d = (int)(r2 % D);
  const long bc = r2 / D;
  out[i] = xform(in[i], tx, bc, d, h, w, H, W, D);
}

// one block per (b, c): fixed-shape tree reduction of the float64 partials (deterministic)
__global__ __launch_bounds__(256) void instnorm_finalize_kernel(const double *__restrict__ partial, int nparts,
                                                                double count, float eps, float *__restrict__ mean,
                                                                float *__restrict__ rstd) {
  __shared__ double rs[256], rq[256];
  const int bc = blockIdx.x, t = threadIdx.x;
  const double *p = partial + (long)bc * nparts * 2;
  double s = 0.0, q = 0.0;
  for (int i = t; i < nparts; i += 256) {
    s += p[2 * i];
    q += p[2 * i + 1];
  }
  rs[t] = s;
  rq[t] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      rs[t] += rs[t + o];
      rq[t] += rq[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double m = rs[0] / count;
    double var = rq[0] / count - m * m;
    if (var < 0.0) var = 0.0;
    mean[bc] = (float)m;
    rstd[bc] = (float)(1.0 / std::sqrt(var + (double)eps));
  }
}

struct ConvGeo {
  int td, tw, th;  // tw: threads along W (valid output columns: tw - 2 at stride 1, tw - 1 at 2)
  int stride;
  int valid_w() const { return tw - (stride == 1 ? 2 : 1); }
};

inline ConvGeo conv_geo(int cout, int stride) {
  if (stride == 2) return {2, 32, 8, 2};
  if (cout <= 8) return {8, 64, 4, 1};  // few outputs: longer D columns reuse each LDS read more
  return {cout >= 32 ? 2 : 4, 64, 4, 1};
}

inline dim3 conv_grid(int B, int Do, int Ho, int Wo, ConvGeo g, int &tilesD) {
  tilesD = (Do + g.td - 1) / g.td;
  return dim3((Wo + g.valid_w() - 1) / g.valid_w(), (Ho + g.th - 1) / g.th, tilesD * B);
}

// up-cat pointwise tiles: TD x TH x TW, aligned, no halo
inline dim3 upcat_grid(int B, int D, int H, int W, int &tilesD) {
  tilesD = (D + TD - 1) / TD;
  return dim3((W + TW - 1) / TW, (H + TH - 1) / TH, tilesD * B);
}

inline int out_size(int n, int stride) { return (n - 1) / stride + 1; }  // k3, pad 1

}  // namespace

extern "C" long sa_conv3d_stat_parts(int Cout, int stride, int Do, int Ho, int Wo) {
  int tilesD;
  dim3 g = conv_grid(1, Do, Ho, Wo, conv_geo(Cout, stride), tilesD);
  return (long)g.x * g.y * g.z;
}

extern "C" long sa_conv3d_wd_stat_parts(int Cout, int D, int H, int W) {
  return sa_conv3d_stat_parts(Cout < 16 ? Cout : 16, 1, D, H, W);
}

extern "C" long sa_conv3d_upcat_stat_parts(int D, int H, int W) {
  int tilesD;
  dim3 g = upcat_grid(1, D, H, W, tilesD);
  return (long)g.x * g.y * g.z;
}

extern "C" int sa_conv3d(const float *in, int B, int Cin, int Di, int Hi, int Wi, int stride, const float *weight,
                         int Cout, const float *in_mean, const float *in_rstd, int act, float slope,
                         const float *gate_l, const float *gate_r, float *out, double *stats_partial, void *stream) {
  SA_REQUIRE(in && weight && out, "sa_conv3d: null pointer");
  SA_REQUIRE(B > 0 && Di > 0 && Hi > 0 && Wi > 0, "sa_conv3d: empty shape");
  SA_REQUIRE((in_mean == nullptr) == (in_rstd == nullptr), "sa_conv3d: mean and rstd go together");
  SA_REQUIRE((gate_l == nullptr) == (gate_r == nullptr), "sa_conv3d: both gate maps or none");
  SA_REQUIRE((long)Di * Hi * Wi < (1L << 31), "sa_conv3d: a channel plane must hold < 2^31 voxels");
  const int Do = out_size(Di, stride), Ho = out_size(Hi, stride), Wo = out_size(Wi, stride);
  const ConvGeo geo = conv_geo(Cout, stride);
  int tilesD;
  dim3 grid = conv_grid(B, Do, Ho, Wo, geo, tilesD);
  InXform tx{in_mean, in_rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
#define SA_CONV(CI, CO, S, TDV, TWV, THV)                                                                   \
  if (Cin == CI && Cout == CO && stride == S) {                                                              \
    conv3d_kernel<CI, CO, S, TDV, TWV, THV><<<grid, 256, 0, s>>>(in, Di, Hi, Wi, Do, Ho, Wo, weight, tx, out, \
                                                                stats_partial, tilesD);                      \
    return sa::check_launch("sa_conv3d");                                                                    \
  }
  SA_CONV(8, 8, 1, 8, 64, 4)
  SA_CONV(8, 2, 1, 8, 64, 4)
  SA_CONV(16, 16, 1, 4, 64, 4)
  SA_CONV(32, 32, 1, 2, 64, 4)
  SA_CONV(8, 16, 2, 2, 32, 8)
  SA_CONV(16, 32, 2, 2, 32, 8)
#undef SA_CONV
  sa::set_error("sa_conv3d: no kernel built for Cin %d -> Cout %d, stride %d", Cin, Cout, stride);
  return SA_E_ARG;
}

// 0: wave-uniform scalar weight loads (default); 1: the weights staged in LDS (conv3d_wd_kernel
// WL), measured slower: bench_hourglass whole hourglass 8.62 against 7.73 ms, the 8 -> 8 convs
// 1.29-1.36 against 1.08-1.11 ms (LDS reads in the FMA loop cost more than the SGPR waits)
// 0 (default): scalar weights; points in D-tile order, or paired for the 8 -> 2 classifier pair
// (507 vs 547 us; 8 -> 8 is faster unpaired, 970 vs 1050 us); 1: LDS-staged weights (slower);
// 2: paired points for every 8-input-channel conv (the 16-channel ones have one D-tile);
// 3: variant 2 with the channel prefetch by LDS-DMA (slower: the compiler makes the tap loop's
// slab reads wait for the DMA)
static int sa_conv3d_wd_variant = 0;
extern "C" void sa_conv3d_wd_set_variant(int variant) { sa_conv3d_wd_variant = variant; }
extern "C" int sa_conv3d_wd_get_variant() { return sa_conv3d_wd_variant; }

extern "C" int sa_conv3d_wd(const float *in, int B, int Cin, int D, int H, int W, const float *weight_wd, int Cout,
                            const float *in_mean, const float *in_rstd, int act, float slope, const float *gate_l,
                            const float *gate_r, float *out, double *stats_partial, void *stream) {
  SA_REQUIRE(in && weight_wd && out, "sa_conv3d_wd: null pointer");
  SA_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, "sa_conv3d_wd: empty shape");
  SA_REQUIRE((in_mean == nullptr) == (in_rstd == nullptr), "sa_conv3d_wd: mean and rstd go together");
  SA_REQUIRE((gate_l == nullptr) == (gate_r == nullptr), "sa_conv3d_wd: both gate maps or none");
  SA_REQUIRE((long)D * H * W * 4 < (1L << 31), "sa_conv3d_wd: a channel volume must hold < 2^31 bytes");
  SA_REQUIRE((Cin == 8 && (Cout == 8 || Cout == 2)) || (Cin == 16 && Cout == 16) || (Cin == 32 && Cout == 32),
             "sa_conv3d_wd: built for 8 -> 8, 8 -> 2, 16 -> 16 and 32 -> 32 (got %d -> %d)", Cin, Cout);
  // the tiling of sa_conv3d's for 8 and 16 outputs (8 or 4 planes x 4 rows x 62 columns): the
  // statistic parts of sa_conv3d_wd_stat_parts (= sa_conv3d_stat_parts for those shapes)
  const ConvGeo geo = conv_geo(Cout < 16 ? Cout : 16, 1);
  SA_REQUIRE(geo.td == (Cin == 8 ? 8 : 4) && geo.tw == 64 && geo.th == 4, "sa_conv3d_wd: tiling");
  int tilesD;
  dim3 grid = conv_grid(B, D, H, W, geo, tilesD);
  InXform tx{in_mean, in_rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  SA_REQUIRE(in_mean && act, "sa_conv3d_wd: built for an InstanceNorm + LeakyReLU producer");
#define SA_WD(CI, CO, NTV, G)                                                                                   \
  if (Cin == CI && Cout == CO && (gate_l != nullptr) == G) {                                                    \
    if (sa_conv3d_wd_variant == 1)                                                                              \
      conv3d_wd_kernel<CI, CO, NTV, G, true><<<grid, 256, 0, s>>>(in, D, H, W, weight_wd, tx, out, stats_partial, \
                                                                  tilesD);                                      \
    else if ((sa_conv3d_wd_variant == 2 || (sa_conv3d_wd_variant == 0 && CO == 2)) && NTV == 2)                 \
      conv3d_wd_kernel<CI, CO, NTV, G, false, NTV == 2><<<grid, 256, 0, s>>>(in, D, H, W, weight_wd, tx, out,    \
                                                                             stats_partial, tilesD);            \
    else if (sa_conv3d_wd_variant == 3)                                                                         \
      conv3d_wd_kernel<CI, CO, NTV, G, false, NTV == 2, true><<<grid, 256, 0, s>>>(in, D, H, W, weight_wd, tx,   \
                                                                                   out, stats_partial, tilesD); \
    else                                                                                                        \
      conv3d_wd_kernel<CI, CO, NTV, G><<<grid, 256, 0, s>>>(in, D, H, W, weight_wd, tx, out, stats_partial, tilesD); \
    return sa::check_launch("sa_conv3d_wd");                                                                     \
  }
  SA_WD(8, 8, 2, false)
  SA_WD(8, 2, 2, true)
  SA_WD(8, 8, 2, true)
  SA_WD(8, 2, 2, false)
  SA_WD(16, 16, 1, false)
  SA_WD(16, 16, 1, true)
#undef SA_WD
  if (Cin == 32 && Cout == 32 && gate_l == nullptr) {   // two 16-channel halves per tile
    grid.z *= 2;
    conv3d_wd_kernel<32, 16, 1, false, false, false, false, 32><<<grid, 256, 0, s>>>(in, D, H, W, weight_wd, tx, out,
                                                                                  stats_partial, tilesD);
    return sa::check_launch("sa_conv3d_wd");
  }
  sa::set_error("sa_conv3d_wd: no kernel for %d -> %d", Cin, Cout);
  return SA_E_ARG;
}

extern "C" int sa_conv3d_pointwise(const float *in, int B, int Cin, int D, int H, int W, const float *mean,
                                   const float *rstd, int act, float slope, const float *gate_l, const float *gate_r,
                                   const float *weight, int Cout, float *out, void *stream) {
  SA_REQUIRE(in && weight && out && B > 0 && D > 0 && H > 0 && W > 0, "sa_conv3d_pointwise: bad arguments");
  SA_REQUIRE((mean == nullptr) == (rstd == nullptr), "sa_conv3d_pointwise: mean and rstd go together");
  SA_REQUIRE((gate_l == nullptr) == (gate_r == nullptr), "sa_conv3d_pointwise: both gate maps or none");
  const long n = (long)B * D * H * W;
  InXform tx{mean, rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
#define SA_PJ(CI, CO)                                                                                        \
  if (Cin == CI && Cout == CO) {                                                                             \
    pointwise_kernel<CI, CO><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in, tx, D, H, W, n, weight, out);   \
    return sa::check_launch("sa_conv3d_pointwise");                                                         \
  }
  SA_PJ(16, 8)
  SA_PJ(32, 16)
#undef SA_PJ
  sa::set_error("sa_conv3d_pointwise: no kernel built for %d -> %d", Cin, Cout);
  return SA_E_ARG;
}

extern "C" int sa_conv3d_pointwise_upcat(const float *a, int Ca, const float *a_mean, const float *a_rstd, int a_act,
                                         const float *a_gl, const float *a_gr, const float *p, int Dp, int Hp, int Wp,
                                         int B, int D, int H, int W, float slope, const float *weight, int Cout,
                                         float *out, double *stats_partial, void *stream) {
  SA_REQUIRE(a && p && weight && out && stats_partial, "sa_conv3d_pointwise_upcat: null pointer");
  SA_REQUIRE(B > 0 && D > 1 && H > 1 && W > 1 && Dp > 0 && Hp > 0 && Wp > 0,
             "sa_conv3d_pointwise_upcat: bad shape");
  // the LDS footprint assumes upsampling by at least 2 along every axis
  SA_REQUIRE(2 * (Dp - 1) <= D - 1 && 2 * (Hp - 1) <= H - 1 && 2 * (Wp - 1) <= W - 1,
             "sa_conv3d_pointwise_upcat: the low-resolution branch must be at most half size");
  int tilesD;
  dim3 grid = upcat_grid(B, D, H, W, tilesD);
  // area_pixel_compute_scale(align_corners=True) = (in - 1) / (out - 1)
  const float sd = (float)(Dp - 1) / (float)(D - 1), sh = (float)(Hp - 1) / (float)(H - 1),
              sw = (float)(Wp - 1) / (float)(W - 1);
  InXform ta{a_mean, a_rstd, a_gl, a_gr, slope, a_act};
  const bool ax = a_mean || a_act || a_gl;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
#define SA_PW(CA, CO, AXV)                                                                                    \
  if (Ca == CA && Cout == CO && ax == AXV) {                                                                 \
    pointwise_upcat_kernel<CA, CO, AXV><<<grid, 256, 0, s>>>(a, ta, OneHotVol{}, p, D, H, W, Dp, Hp, Wp, sd, sh, \
                                                             sw, weight, out, stats_partial, tilesD);        \
    return sa::check_launch("sa_conv3d_pointwise_upcat");                                                    \
  }
  SA_PW(8, 8, false)
  SA_PW(16, 16, true)
#undef SA_PW
  sa::set_error("sa_conv3d_pointwise_upcat: no kernel built for %d -> %d (a transform %d)", Ca, Cout, ax);
  return SA_E_ARG;
}

extern "C" long sa_conv3d_onehot_stat_parts(int Do, int Ho, int Wo) {
  return (long)((Wo + 63) / 64) * ((Ho + 3) / 4) * ((Do + 1) / 2);
}

extern "C" int sa_conv3d_onehot(const float *rec_l, const float *rec_r, int B, int nbins, int D, int H, int W,
                                int stride, float gain, const float *weight, int Cout, float *out,
                                double *stats_partial, void *stream) {
  SA_REQUIRE(rec_l && rec_r && weight && out, "sa_conv3d_onehot: null pointer");
  SA_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, "sa_conv3d_onehot: empty shape");
  SA_REQUIRE(((uintptr_t)rec_l & 15) == 0 && ((uintptr_t)rec_r & 15) == 0, "sa_conv3d_onehot: records need 16-byte alignment");
  SA_REQUIRE(nbins == 8 && stride == 2 && Cout == 16,
             "sa_conv3d_onehot: built for 8 bins, stride 2, 16 outputs (got %d, %d, %d)", nbins, stride, Cout);
  SA_REQUIRE((long)D * H * W < (1L << 31), "sa_conv3d_onehot: a channel plane must hold < 2^31 voxels");
  const int Do = out_size(D, 2), Ho = out_size(H, 2), Wo = out_size(W, 2);
  const int tilesD = (Do + 1) / 2;
  const dim3 grid((Wo + 63) / 64, (Ho + 3) / 4, tilesD * B);
  SA_REQUIRE((long)grid.x * grid.y * tilesD == sa_conv3d_onehot_stat_parts(Do, Ho, Wo), "sa_conv3d_onehot: parts");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  OneHotVol v{reinterpret_cast<const float4 *>(rec_l), reinterpret_cast<const float4 *>(rec_r), gain};
  conv3d_onehot_s2_kernel<16, 2><<<grid, 256, 0, s>>>(v, nbins, D, H, W, Do, Ho, Wo, weight, out, stats_partial,
                                                      tilesD);
  return sa::check_launch("sa_conv3d_onehot");
}

extern "C" int sa_conv3d_pointwise_upcat_onehot(const float *rec_l, const float *rec_r, int nbins, float gain,
                                                const float *p, int Dp, int Hp, int Wp, int B, int D, int H, int W,
                                                const float *weight, int Cout, float *out, double *stats_partial,
                                                void *stream) {
  SA_REQUIRE(rec_l && rec_r && p && weight && out && stats_partial, "sa_conv3d_pointwise_upcat_onehot: null pointer");
  SA_REQUIRE(((uintptr_t)rec_l & 15) == 0 && ((uintptr_t)rec_r & 15) == 0,
             "sa_conv3d_pointwise_upcat_onehot: records need 16-byte alignment");
  SA_REQUIRE(B > 0 && D > 1 && H > 1 && W > 1 && Dp > 0 && Hp > 0 && Wp > 0,
             "sa_conv3d_pointwise_upcat_onehot: bad shape");
  SA_REQUIRE(2 * (Dp - 1) <= D - 1 && 2 * (Hp - 1) <= H - 1 && 2 * (Wp - 1) <= W - 1,
             "sa_conv3d_pointwise_upcat_onehot: the low-resolution branch must be at most half size");
  SA_REQUIRE(nbins == 8 && Cout == 8, "sa_conv3d_pointwise_upcat_onehot: built for 8 bins -> 8 outputs");
  int tilesD;
  dim3 grid = upcat_grid(B, D, H, W, tilesD);
  const float sd = (float)(Dp - 1) / (float)(D - 1), sh = (float)(Hp - 1) / (float)(H - 1),
              sw = (float)(Wp - 1) / (float)(W - 1);
  OneHotVol v{reinterpret_cast<const float4 *>(rec_l), reinterpret_cast<const float4 *>(rec_r), gain};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  pointwise_upcat_kernel<8, 8, false, true><<<grid, 256, 0, s>>>(nullptr, InXform{}, v, p, D, H, W, Dp, Hp, Wp, sd,
                                                                  sh, sw, weight, out, stats_partial, tilesD);
  return sa::check_launch("sa_conv3d_pointwise_upcat_onehot");
}

extern "C" int sa_vol_apply(const float *in, int B, int C, int D, int H, int W, const float *mean, const float *rstd,
                            int act, float slope, const float *gate_l, const float *gate_r, float *out, void *stream) {
  SA_REQUIRE(in && out && B > 0 && C > 0 && D > 0 && H > 0 && W > 0, "sa_vol_apply: bad arguments");
  const long n = (long)B * C * D * H * W;
  InXform tx{mean, rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  vol_apply_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in, tx, C, D, H, W, n, out);
  return sa::check_launch("sa_vol_apply");
}

extern "C" int sa_instnorm_finalize(const double *partial, int bc_count, long nparts, long count, float eps,
                                    float *mean, float *rstd, void *stream) {
  SA_REQUIRE(partial && mean && rstd && bc_count > 0 && nparts > 0 && count > 0,
             "sa_instnorm_finalize: bad arguments");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  instnorm_finalize_kernel<<<bc_count, 256, 0, s>>>(partial, (int)nparts, (double)count, eps, mean, rstd);
  return sa::check_launch("sa_instnorm_finalize");
}
