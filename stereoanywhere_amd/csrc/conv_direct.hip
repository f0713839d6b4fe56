// Direct convolution on fp32 MFMA (implicit GEMM) for the encoder convs that the Winograd
// kernel does not cover (extractor.py:62-300):
//   * the 7x7 stems, 3 -> 64 channels at full resolution (fnet / cnet conv1), and
//   * the stride-2 3x3 conv of each stage's first residual block together with that block's
//     1x1 stride-2 downsample (extractor.py:22-40): both read the same input pixels (the 1x1
//     conv's input is the 3x3 conv's centre tap), so one launch computes both.
// MIOpen runs these as NHWC implicit GEMMs plus layout transposes, 5-7x slower than this.
//
//   block  = 8 waves; output tile 8 rows (one per wave) x 32 columns x NC = 16*NTL channels
//   chunk  = KC input channels: the stride-aware input patch ((8-1)*S+K rows x (32-1)*S+K
//            columns, zero padded) and the chunk's weights [tap][ci][NC] are staged in LDS;
//            the next chunk's global loads are in flight while this one multiplies
//   MFMA   = v_mfma_f32_16x16x4_f32 (exact fp32 products): K runs tap-major over the chunk,
//            so every LDS offset of a K-step is a compile-time immediate; each wave owns 2
//            row segments of 16 pixels x all NC channels (+ NC downsample channels)
//   output = raw conv (no bias: the encoders fold it into the following norm) and optional
//            float64 InstanceNorm partials per (image, channel, block), as the Winograd conv
//            writes them (sa_instnorm_finalize)
//   close  = (CL, sa_conv_direct_close) the input is a residual block's output not yet written:
//            relu(relu((c2 - mean) * rstd) + skip) per (image, channel) plane, formed while the
//            patch is staged (c2 and skip loaded at the same offsets; zero padding outside the
//            image), the arithmetic of sa_norm_act's pass exactly (no contraction)
#include "sa_common.h"

#pragma clang fp contract(fast)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
using f16x4 = __attribute__((ext_vector_type(4))) _Float16;

// Split products (SP, sa_conv_direct_split): the weights are f16 (hi, lo) pairs of w * 2^12 in
// one dword each (sa_conv_direct_weights_split), the patch values are split in registers, and
// each v_mfma_f32_16x16x4_f32 becomes one v_mfma_f32_16x16x16_f16 over the four products
// hi*bhi + hi*blo + lo*bhi + lo*blo (A = (hi, hi, lo, lo), B = (bhi, blo, bhi, blo)): exact
// products, fp32 accumulation, half the MFMA cycles (as conv2d_wino4.hip's W4Split).
constexpr float DSP_SCALE = 4096.0f;
__device__ __forceinline__ f16x4 dsplit(const float x) {
  const f16x2 hh = __builtin_convertvector(f32x2{x, x}, f16x2);
  float l;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(__builtin_bit_cast(unsigned, hh)), "v"(x));
  const f16x2 ll = __builtin_convertvector(f32x2{l, l}, f16x2);
  return __builtin_shufflevector(hh, ll, 0, 1, 2, 3);
}

// the fp32 value w * 2^12 of a split weight dword (hi, lo): exact in fp32
__device__ __forceinline__ float dunsplit(const float packed) {
  const f16x2 p = __builtin_bit_cast(f16x2, packed);
  return (float)p[0] + (float)p[1];
}

// blocks the split kernel's range guard recomputed on fp32 MFMA (sa_split_redo_blocks)
__device__ unsigned g_direct_redo_blocks;

constexpr int DOTH = 8, DOTW = 32, MT = 2;   // output tile; row segments of 16 pixels per wave

template <int K, int S, int KC, int NTL, bool DS>
struct DCfg {
  static constexpr int PH = (DOTH - 1) * S + K, PW = (DOTW - 1) * S + K;
  static constexpr int PWP = PW;
  // plane pitch: the A read's two 16-lane k-rows of a half-wave fall in disjoint banks
  // (stride 1: 16 consecutive columns -> offset 16 mod 32; stride 2: even columns -> odd offset)
  static constexpr int PL0 = PH * PWP, PR = S == 1 ? 16 : 17;
  static constexpr int PLANE = PL0 + ((PR - PL0 % 32) + 32) % 32;
  static constexpr int XN = KC * PLANE;                    // patch floats per chunk
  static constexpr int NC = 16 * NTL;                      // conv output channels per block
  static constexpr int KK = K * K;
  static constexpr int WN = KC * KK * NC;                  // conv weights per chunk, [tap*KC + ci][NC]
  static constexpr int DN = DS ? KC * NC : 0;              // downsample weights per chunk, [ci][NC]
  static constexpr int NCP = NC + 16;                      // LDS row pitch of the weights (bank halves)
  static constexpr int WROWS = KC * KK + (DS ? KC : 0);    // conv rows then downsample rows
  static constexpr int XPT = (XN + 511) / 512, WPT = (WN + DN) / 4 / 512 + (((WN + DN) / 4) % 512 ? 1 : 0);
  static constexpr int KSTEPS = KC * KK / 4;
  static constexpr int NACC = NTL * (DS ? 2 : 1);
  static constexpr int SMEM = XN + WROWS * NCP + 4;   // + a spare float4 for slot-less commits
  static_assert(KC % 4 == 0, "a K-step of 4 must stay inside one tap");
  static_assert((WN + DN) % 4 == 0, "weights are staged as float4");
  static_assert(SMEM * 4 <= 160 * 1024, "LDS budget");
  static_assert(8 * 2 * NACC * 16 * 2 <= SMEM, "the stats reduction reuses the staging LDS");
};

struct DirArgs {
  const float *in;
  long in_bs;
  const float *skip, *cm, *cs;   // CL: the close's skip planes and per-(image, channel) mean / rstd
  long skip_bs;
  int Cin, H, W, Ho, Wo;
  const float *wg, *wd;   // arranged weights (sa_conv_direct_weights layout)
  int Cout, co_blocks, tiles_w, tiles, nchunks;
  float *out, *out_ds;
  long out_bs, out_ds_bs;
  double *part, *part_ds;
};

// relu(relu((v - m) * s) + k) as sa_norm_act computes it (separate rounding of each operation)
__device__ __forceinline__ float close_value(float v, float m, float s, float k) {
#pragma clang fp contract(off)
  const float y = fmaxf((v - m) * s + 0.0f, 0.0f);
  return fmaxf(y + k, 0.0f);
}

template <int K, int S, int KC, int NTL, bool DS, bool SP = false, bool CL = false>
__global__ __launch_bounds__(512, DS ? 2 : 4) void conv_direct_kernel(const DirArgs a) {
  using C = DCfg<K, S, KC, NTL, DS>;
  constexpr int NC = C::NC, NCP = C::NCP, PLANE = C::PLANE, PWP = C::PWP;
  __shared__ __attribute__((aligned(16))) float sm[C::SMEM];
  // CL: the (mean, rstd) of the staged chunk's channels, double-buffered by chunk parity
  __shared__ float ctab[CL ? 2 : 1][CL ? 2 * KC : 1];
  float *sx = sm, *sw = sm + C::XN, *sd = sw + KC * C::KK * NCP;
  constexpr int SPARE = C::SMEM - 4;   // slot-less threads commit here (never read)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned wid = sa::xcd_remap(blockIdx.x, gridDim.x);   // co blocks of a tile together
  const int cb = wid % a.co_blocks;
  const int st = (wid / a.co_blocks) % a.tiles;
  const int n = wid / (a.co_blocks * a.tiles);
  const int oy0 = (st / a.tiles_w) * DOTH, ox0 = (st % a.tiles_w) * DOTW;
  const int iy0 = oy0 * S - K / 2, ix0 = ox0 * S - K / 2;
  const long hw = (long)a.H * a.W;
  const float *src = a.in + (long)n * a.in_bs;

  // staging slots, fixed for all chunks: patch element -> image offset.  Channels past Cin
  // (only a single-chunk stem pads Cin = 3 to KC = 4) read a real channel: their weights are
  // zero, so any finite value gives the exact result.
  // Branch-free staging: buffer loads whose out-of-range VGPR offset returns 0 give the zero
  // padding, and threads without a slot commit to a spare LDS float4.
  constexpr int OOB = 0x7ffffff0;
  const __amdgpu_buffer_rsrc_t xin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(src), (short)0, (int)((long)a.Cin * hw * 4), 0x00020000);
  int xoff[C::XPT], xl[C::XPT];
#pragma unroll
  for (int j = 0; j < C::XPT; ++j) {
    const int i = tid + 512 * j;
    const int ci = i / PLANE, rem = i % PLANE, r = rem / PWP, c = rem % PWP;
    const int y = iy0 + r, x = ix0 + c;
    const bool ok = i < C::XN && rem < C::PH * PWP && c < C::PW && y >= 0 && y < a.H && x >= 0 && x < a.W;
    xoff[j] = ok ? (int)((min(ci, a.Cin - 1) * hw + (long)y * a.W + x) * 4) : OOB;
    xl[j] = i < C::XN ? i : SPARE;
  }
  // weights: conv rows then downsample rows, float4 units; LDS slot with the padded pitch
  constexpr int WQ = (C::WN + C::DN) / 4;
  const __amdgpu_buffer_rsrc_t win = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(a.wg) + (long)cb * a.nchunks * C::WN, (short)0, (int)((long)a.nchunks * C::WN * 4),
      0x00020000);
  const __amdgpu_buffer_rsrc_t din = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(DS ? a.wd + (long)cb * a.nchunks * C::DN : a.wg), (short)0,
      (int)((long)a.nchunks * (DS ? C::DN : 0) * 4), 0x00020000);
  int woff[C::WPT], wl[C::WPT];
  bool wds[C::WPT];
#pragma unroll
  for (int j = 0; j < C::WPT; ++j) {
    const int i = tid + 512 * j;
    wds[j] = i >= C::WN / 4;
    woff[j] = i < WQ ? (wds[j] ? (i - C::WN / 4) * 16 : i * 16) : OOB;
    const int row = (4 * i) / NC, col = (4 * i) % NC;
    wl[j] = i < WQ ? row * NCP + col : SPARE;
  }
  const __amdgpu_buffer_rsrc_t kin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(CL ? a.skip + (long)n * a.skip_bs : src), (short)0, (int)((long)a.Cin * hw * 4), 0x00020000);
  float xr[C::XPT], kr[CL ? C::XPT : 1];
  float tv = 0.0f;   // CL: this thread's entry of the next chunk's (mean, rstd) table (tid < 2 KC)
  f32x4 wr[C::WPT];
  auto fetch = [&](int chunk) __attribute__((always_inline)) {
    const int xs = chunk * KC * (int)hw * 4;
#pragma unroll
    for (int j = 0; j < C::XPT; ++j) xr[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xin, xoff[j], xs, 0));
    if constexpr (CL) {
#pragma unroll
      for (int j = 0; j < C::XPT; ++j) kr[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(kin, xoff[j], xs, 0));
      if (tid < 2 * KC) {
        const int c = min(chunk * KC + tid % KC, a.Cin - 1);
        tv = (tid < KC ? a.cm : a.cs)[(long)n * a.Cin + c];
      }
    }
#pragma unroll
    for (int j = 0; j < C::WPT; ++j) {
      const auto v = wds[j] ? __builtin_amdgcn_raw_buffer_load_b128(din, woff[j], chunk * C::DN * 4, 0)
                            : __builtin_amdgcn_raw_buffer_load_b128(win, woff[j], chunk * C::WN * 4, 0);
      wr[j] = f32x4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])};
    }
  };
  auto put_tab = [&](int chunk) __attribute__((always_inline)) {
    if (CL && tid < 2 * KC) ctab[CL ? chunk & 1 : 0][tid] = tv;
  };
  auto commit = [&](int chunk) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < C::XPT; ++j) {
      float v = xr[j];
      if constexpr (CL) {
        const int cl = min((tid + 512 * j) / PLANE, KC - 1);
        const float *tb = ctab[chunk & 1];
        v = xoff[j] == OOB ? 0.0f : close_value(v, tb[cl], tb[KC + cl], kr[j]);
      }
      sx[xl[j]] = v;
    }
#pragma unroll
    for (int j = 0; j < C::WPT; ++j) *reinterpret_cast<f32x4 *>(sw + wl[j]) = wr[j];
  };

  f32x4 acc[MT][C::NACC];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < C::NACC; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // operand lanes (16x16x4): A[m = lane & 15][k = lane >> 4], B[k = lane >> 4][n = lane & 15]
  const int kq = lane >> 4, ml = lane & 15;
  int abase[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) abase[m] = kq * PLANE + (wv * S) * PWP + (m * 16 + ml) * S;
  const int bbase = kq * NCP + ml;

  fetch(0);
  if constexpr (CL) {
    put_tab(0);
    __syncthreads();
  }
  commit(0);
  __syncthreads();
#pragma unroll 1
  for (int chunk = 0; chunk < a.nchunks; ++chunk) {
    if (chunk + 1 < a.nchunks) fetch(chunk + 1);
#pragma unroll
    for (int s = 0; s < C::KSTEPS; ++s) {
      const int tap = (4 * s) / KC, ci0 = (4 * s) % KC;
      const int koff = ci0 * PLANE + (tap / K) * PWP + (tap % K);
      float av[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = sx[abase[m] + koff];
      auto prod = [&](const float bv, f32x4 *ac) __attribute__((always_inline)) {
        if constexpr (SP) {
          const f16x4 b = __builtin_bit_cast(f16x4, f32x2{bv, bv});
#pragma unroll
          for (int m = 0; m < MT; ++m) ac[m * C::NACC] = __builtin_amdgcn_mfma_f32_16x16x16f16(dsplit(av[m]), b, ac[m * C::NACC], 0, 0, 0);
        } else {
#pragma unroll
          for (int m = 0; m < MT; ++m) ac[m * C::NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv, ac[m * C::NACC], 0, 0, 0);
        }
      };
#pragma unroll
      for (int t = 0; t < NTL; ++t) prod(sw[bbase + 4 * s * NCP + t * 16], &acc[0][t]);
      if (DS && tap == (K / 2) * K + K / 2) {
#pragma unroll
        for (int t = 0; t < NTL; ++t) prod(sd[bbase + ci0 * NCP + t * 16], &acc[0][NTL + t]);
      }
    }
    if (CL && chunk + 1 < a.nchunks) put_tab(chunk + 1);   // (its buffer was last read two chunks ago)
    __syncthreads();
    if (chunk + 1 < a.nchunks) {
      commit(chunk + 1);
      __syncthreads();
    }
  }
  if constexpr (SP) {
    // Range guard (as conv2d_wino4.hip's split kernel): a patch value >= 65520 in magnitude
    // overflows its f16 hi half and leaves NaN in the accumulators it fed; the block then
    // recomputes on fp32 MFMA products
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < C::NACC; ++t) sum += acc[m][t];
    const float tot = (sum.x + sum.y) + (sum.z + sum.w);
    if (__syncthreads_or(!__builtin_isfinite(tot))) {
      if (tid == 0) atomicAdd(&g_direct_redo_blocks, 1u);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < C::NACC; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      // a plain (unpipelined, rolled) loop: this path is rare, and a second copy of the
      // pipelined one would raise the main loop's register pressure
#pragma unroll 1
      for (int chunk = 0; chunk < a.nchunks; ++chunk) {
        fetch(chunk);
        if constexpr (CL) {
          put_tab(chunk);
          __syncthreads();
        }
        commit(chunk);
        __syncthreads();
#pragma unroll 1
        for (int s = 0; s < C::KSTEPS; ++s) {
          const int tap = (4 * s) / KC, ci0 = (4 * s) % KC;
          const int koff = ci0 * PLANE + (tap / K) * PWP + (tap % K);
#pragma unroll
          for (int t = 0; t < NTL; ++t) {
            const float w = dunsplit(sw[bbase + 4 * s * NCP + t * 16]);
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sx[abase[m] + koff], w, acc[m][t], 0, 0, 0);
          }
          if (DS && tap == (K / 2) * K + K / 2) {
#pragma unroll
            for (int t = 0; t < NTL; ++t) {
              const float w = dunsplit(sd[bbase + ci0 * NCP + t * 16]);
#pragma unroll
              for (int m = 0; m < MT; ++m)
                acc[m][NTL + t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sx[abase[m] + koff], w, acc[m][NTL + t], 0, 0, 0);
            }
          }
        }
        __syncthreads();
      }
    }
  }

  if constexpr (SP) {   // the weights' 2^12 (exact)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < C::NACC; ++t) acc[m][t] *= 1.0f / DSP_SCALE;
  }
  // ---- epilogue: lane holds channel t*16 + (lane & 15), pixels 4*(lane>>4) + r of segment m.
  // The stats reduction reuses the staging LDS (free after the loop's last barrier).
  double *red = reinterpret_cast<double *>(sm);   // [8 waves][2][NACC * 16]
  constexpr int RC = C::NACC * 16;
  const int oy = oy0 + wv;
  const bool stats = a.part != nullptr;
  const bool interior = oy0 + DOTH <= a.Ho && ox0 + DOTW <= a.Wo && (a.Wo & 3) == 0;
#pragma unroll
  for (int t = 0; t < C::NACC; ++t) {
    const bool ds = DS && t >= NTL;
    const int co = cb * NC + (ds ? t - NTL : t) * 16 + ml;
    float *dst = (ds ? a.out_ds + (long)n * a.out_ds_bs : a.out + (long)n * a.out_bs) + (long)co * a.Ho * a.Wo;
    double s1 = 0.0, s2 = 0.0;
    if (interior) {   // block-uniform: every output in range, rows float4-aligned
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int ox = ox0 + m * 16 + 4 * kq;   // 4 consecutive pixels of one row
        *reinterpret_cast<float4 *>(dst + (long)oy * a.Wo + ox) =
            make_float4(acc[m][t][0], acc[m][t][1], acc[m][t][2], acc[m][t][3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = acc[m][t][r];
          s1 += v;
          s2 += v * v;
        }
      }
    } else {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int ox = ox0 + m * 16 + 4 * kq;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (oy < a.Ho && ox + r < a.Wo) {
            const float v = acc[m][t][r];
            dst[(long)oy * a.Wo + ox + r] = v;
            s1 += (double)v;
            s2 += (double)v * v;
          }
        }
      }
    }
    if (stats) {
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      if (kq == 0) {
        red[(wv * 2 + 0) * RC + t * 16 + ml] = s1;
        red[(wv * 2 + 1) * RC + t * 16 + ml] = s2;
      }
    }
  }
  if (stats) {
    __syncthreads();
    for (int c = tid; c < RC; c += 512) {
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s1 += red[(w * 2 + 0) * RC + c];
        s2 += red[(w * 2 + 1) * RC + c];
      }
      const bool ds = DS && c >= NC;
      double *pp = ds ? a.part_ds : a.part;
      if (pp) {
        const int co = cb * NC + (ds ? c - NC : c);
        pp += (((long)n * a.Cout + co) * a.tiles + st) * 2;
        pp[0] = s1;
        pp[1] = s2;
      }
    }
  }
}

// weight arrangement: w [Cout][Cin][K][K] -> [co block][chunk][tap][ci in chunk][NC], Cin padded
// with zeros to a multiple of KC; downsample wd [Cout][Cin] -> [co block][chunk][ci][NC]
__global__ void direct_weights_kernel(const float *__restrict__ w, int Cout, int Cin, int K, int KC, int NC,
                                      int nchunks, int ds, float *__restrict__ out) {
  const long total = (long)Cout * nchunks * KC * K * K;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  // output index decomposition
  const int n = (int)(i % NC);
  long r = i / NC;
  const int ci = (int)(r % KC);
  r /= KC;
  const int tap = (int)(r % (K * K));
  r /= K * K;
  const int chunk = (int)(r % nchunks);
  const int cblk = (int)(r / nchunks);
  const int co = cblk * NC + n, cin = chunk * KC + ci;
  (void)ds;
  out[i] = cin < Cin ? w[((long)co * Cin + cin) * K * K + tap] : 0.0f;
}

// the built configurations: (K, S, Cout) -> channel chunk KC and output tile NTL * 16; the
// stride-2 3x3 launches always carry the 1x1 downsample (K = 1 arranges its weights)
bool pick(int K, int S, int Cout, int &KC, int &NTL) {
  KC = K == 7 ? 4 : 8;
  if (K == 7 && S == 1 && Cout % 64 == 0) { NTL = 4; return true; }
  if ((K == 3 || K == 1) && S == 2 && Cout == 96) { NTL = 6; return true; }
  if ((K == 3 || K == 1) && S == 2 && Cout % 128 == 0) { NTL = 8; return true; }
  return false;
}

}  // namespace

extern "C" int sa_conv_direct_weights(const float *weight, int Cout, int Cin, int K, int S, int with_ds,
                                      float *out, void *stream) {
  int KC = 0, NTL = 0;
  SA_REQUIRE(weight && out && Cout > 0 && Cin > 0, "sa_conv_direct_weights: bad arguments");
  SA_REQUIRE(pick(K, S, Cout, KC, NTL) && (K != 1 || with_ds), "sa_conv_direct_weights: no kernel for K=%d S=%d Cout=%d",
             K, S, Cout);
  const int NC = 16 * NTL, nchunks = (Cin + KC - 1) / KC;
  const long total = (long)Cout * nchunks * KC * K * K;
  hipStream_t s = sa::as_stream(stream);
  direct_weights_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, K, KC, NC, nchunks, 0,
                                                                       out);
  return sa::check_launch("sa_conv_direct_weights");
}

namespace {
// arranged fp32 weights (sa_conv_direct_weights) -> the split kernel's f16 (hi, lo) pairs of
// w * 2^12, one dword per weight in the same layout
__global__ void direct_split_kernel(const float *__restrict__ w, long n, unsigned *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double u = (double)w[i] * DSP_SCALE;
  const _Float16 hi = (_Float16)(float)u;
  const _Float16 lo = (_Float16)(float)(u - (double)hi);
  out[i] = (unsigned)__builtin_bit_cast(unsigned short, hi) | ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
}

}  // namespace

extern "C" int sa_conv_direct_weights_split(const float *arranged, long n, void *out, void *stream) {
  SA_REQUIRE(arranged && out && n > 0, "sa_conv_direct_weights_split: bad arguments");
  hipStream_t s = sa::as_stream(stream);
  direct_split_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(arranged, n, static_cast<unsigned *>(out));
  return sa::check_launch("sa_conv_direct_weights_split");
}

long sa_direct_redo_blocks_internal(int reset) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_direct_redo_blocks), sizeof v) != hipSuccess) return -1;
  if (reset) {
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_direct_redo_blocks), &z, sizeof z) != hipSuccess) return -1;
  }
  return v;
}

extern "C" long sa_conv_direct_weights_size(int Cout, int Cin, int K, int S, int with_ds) {
  int KC = 0, NTL = 0;
  if (!pick(K, S, Cout, KC, NTL) || (K == 1 && !with_ds)) return -1;
  return (long)Cout * ((Cin + KC - 1) / KC) * KC * K * K;
}

extern "C" long sa_conv_direct_stat_parts(int Ho, int Wo) {
  return (long)((Wo + DOTW - 1) / DOTW) * ((Ho + DOTH - 1) / DOTH);
}

template <bool SP>
static int conv_direct_launch(const float *in, long in_bs, int N, int Cin, int H, int W, int K, int S,
                              const float *wg, const float *wd, int Cout, float *out, long out_bs, float *out_ds,
                              long out_ds_bs, double *part, double *part_ds, void *stream,
                              const float *skip = nullptr, long skip_bs = 0, const float *cm = nullptr,
                              const float *cs = nullptr) {
  int KC = 0, NTL = 0;
  const bool ds = wd != nullptr, cl = skip != nullptr;
  SA_REQUIRE(in && wg && out && N > 0 && Cin > 0 && H > 0 && W > 0, "sa_conv_direct: bad arguments");
  SA_REQUIRE(!ds || out_ds, "sa_conv_direct: downsample weights without an output");
  SA_REQUIRE(K != 1 && pick(K, S, Cout, KC, NTL) && ds == (S == 2),
             "sa_conv_direct: no kernel for K=%d S=%d Cout=%d ds=%d", K, S, Cout, (int)ds);
  SA_REQUIRE((long)Cin * H * W < (1L << 31), "sa_conv_direct: image too large");
  SA_REQUIRE(Cin % KC == 0 || Cin <= KC, "sa_conv_direct: Cin must be a multiple of %d (or at most %d)", KC, KC);
  SA_REQUIRE(!cl || (cm && cs && K == 3 && Cin % KC == 0),
             "sa_conv_direct_close: needs mean / rstd, a 3x3 stride-2 conv and Cin %% %d == 0", KC);
  const int p = K / 2;
  const int Ho = (H + 2 * p - K) / S + 1, Wo = (W + 2 * p - K) / S + 1;
  const int tiles_w = (Wo + DOTW - 1) / DOTW, tiles = tiles_w * ((Ho + DOTH - 1) / DOTH);
  const int co_blocks = Cout / (16 * NTL);
  const DirArgs a{in, in_bs, skip, cm, cs, skip_bs, Cin, H, W, Ho, Wo, wg, wd, Cout, co_blocks, tiles_w, tiles,
                  (Cin + KC - 1) / KC, out, out_ds, out_bs, out_ds_bs, part, part_ds};
  const long nblk = (long)N * tiles * co_blocks;
  SA_REQUIRE(nblk < (1L << 31), "sa_conv_direct: grid too large");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV_DIRECT, s);
  if (K == 7) {
    conv_direct_kernel<7, 1, 4, 4, false, SP><<<(unsigned)nblk, 512, 0, s>>>(a);
  } else if (NTL == 6) {
    if (cl) conv_direct_kernel<3, 2, 8, 6, true, SP, true><<<(unsigned)nblk, 512, 0, s>>>(a);
    else conv_direct_kernel<3, 2, 8, 6, true, SP><<<(unsigned)nblk, 512, 0, s>>>(a);
  } else {
    // (no close form here: staging the skip too would spill the 128-channel kernel's registers)
    SA_REQUIRE(!cl, "sa_conv_direct_close: no close form for Cout = %d", Cout);
    conv_direct_kernel<3, 2, 8, 8, true, SP><<<(unsigned)nblk, 512, 0, s>>>(a);
  }
  return sa::check_launch("sa_conv_direct");
}

extern "C" int sa_conv_direct(const float *in, long in_bs, int N, int Cin, int H, int W, int K, int S,
                              const float *wg, const float *wd, int Cout, float *out, long out_bs, float *out_ds,
                              long out_ds_bs, double *part, double *part_ds, void *stream) {
  return conv_direct_launch<false>(in, in_bs, N, Cin, H, W, K, S, wg, wd, Cout, out, out_bs, out_ds, out_ds_bs, part,
                                   part_ds, stream);
}

// the same with split weights (sa_conv_direct_weights_split for wg and wd)
extern "C" int sa_conv_direct_split(const float *in, long in_bs, int N, int Cin, int H, int W, int K, int S,
                                    const void *wg, const void *wd, int Cout, float *out, long out_bs, float *out_ds,
                                    long out_ds_bs, double *part, double *part_ds, void *stream) {
  return conv_direct_launch<true>(in, in_bs, N, Cin, H, W, K, S, static_cast<const float *>(wg),
                                  static_cast<const float *>(wd), Cout, out, out_bs, out_ds, out_ds_bs, part, part_ds,
                                  stream);
}

// 1 when sa_conv_direct_close has a kernel for this conv (the 96-channel stride-2 3x3 + downsample)
extern "C" int sa_conv_direct_close_supported(int K, int S, int Cout) {
  int KC = 0, NTL = 0;
  return K == 3 && S == 2 && pick(K, S, Cout, KC, NTL) && NTL == 6 ? 1 : 0;
}

// The stride-2 3x3 conv + 1x1 downsample (sa_conv_direct / _split, split != 0) of a residual
// block's output that was not written: the input is relu(relu((c2 - mean) * rstd) + skip), mean /
// rstd per (image, channel) ([N][Cin]), formed while the patch is staged (sa_norm_act's arithmetic)
extern "C" int sa_conv_direct_close(const float *c2, long c2_bs, const float *skip, long skip_bs, const float *mean,
                                    const float *rstd, int N, int Cin, int H, int W, int K, int S, const void *wg,
                                    const void *wd, int split, int Cout, float *out, long out_bs, float *out_ds,
                                    long out_ds_bs, double *part, double *part_ds, void *stream) {
  SA_REQUIRE(skip, "sa_conv_direct_close: null skip");
  if (split)
    return conv_direct_launch<true>(c2, c2_bs, N, Cin, H, W, K, S, static_cast<const float *>(wg),
                                    static_cast<const float *>(wd), Cout, out, out_bs, out_ds, out_ds_bs, part, part_ds,
                                    stream, skip, skip_bs, mean, rstd);
  return conv_direct_launch<false>(c2, c2_bs, N, Cin, H, W, K, S, static_cast<const float *>(wg),
                                   static_cast<const float *>(wd), Cout, out, out_bs, out_ds, out_ds_bs, part, part_ds,
                                   stream, skip, skip_bs, mean, rstd);
}
