// 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on v_mfma_f32_16x16x32_f16 with split
// operands (the encoder and update-block 3x3 convs, extractor.py:6-60, update.py:46-110).
//
// GEMM view: out[co][p] = sum over (tap, ci) of W[co][ci][tap] * X[ci][p + off(tap)], K = 9 Cin.
// Every operand is an f16 pair v = hi + lo (hi = f16(v), lo = f16(v - hi), 22 significant bits;
// the weights scaled by 2^12 first, the accumulators by 2^-12 after the main loop, both exact) and
// each product runs as the three f16 MFMAs hi*hi + hi*lo + lo*hi: f16 x f16 products are exact
// in fp32, so the result differs from an fp32 conv by the operands' rounding (<= 2^-22 relative
// for |v| >= 2^-3, the lo halves subnormal below: an absolute 2^-25) and the omitted lo*lo term
// (<= 2^-22 relative), and the accumulation order.  Three products per K = 32 slots run at 16/3
// times the fp32 MFMA rate (the F(4x4) split kernel's 16x16x16 form: 2 times, on 4 x 36/144 of
// the products).
//
//   block  = 8 waves (two per SIMD), 128 output channels x 256 output pixels (16 x 16, 8 x 32 or
//            4 x 64, whichever pads the image least); wave = 32 channels x 128 pixels (2 x 8
//            MFMA tiles, 64 accumulators)
//   chunk  = 32 input channels (the MFMA's K).  The input patch (TH + 2) x (TW + 2) of the chunk
//            is loaded to registers, split, and written to LDS as [hl][8-channel group][pixel]
//            16-byte entries (8 channels of one pixel: one ds_read_b128 per lane and operand;
//            planes of a multiple of 256 bytes make the B-operand reads conflict-free at any
//            tap offset), double-buffered: the next chunk's patch is staged during the current
//            chunk's 9 taps, one barrier per chunk
//   weights = pre-split, pre-arranged so that every MFMA A operand of a wave is one coalesced
//            1 KiB global load (16 bytes per lane) from L2, two taps ahead in registers: no LDS
//            and no barrier for them
//   epilogue = the accumulators staged in LDS per channel plane, then bias + ReLU, InstanceNorm
//            partials or the ConvGRU gates (as conv2d_wino4.hip's w4_emit) with float4 stores
#include "sa_common.h"

#include <type_traits>

#pragma clang fp contract(fast)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr int IG_LOG2 = 12;        // weight scale 2^12 (the split weights' lo halves stay normal)
constexpr int KCH = 32;            // input channels per chunk
constexpr int MAX_PROB = 8;
constexpr unsigned IG_OOB = 0x80000000u;   // out-of-range buffer offset: the load returns 0
#ifndef IG_DIAG
#define IG_DIAG 0   // timing diagnostics only (wrong results): 1 no weight loads in the loop, 2 no patch
                    // staging in the loop, 3 no chunk barrier, 4 = 1 + 2 + 3, 5 no MFMAs
#endif
#ifndef IG_STAGGER
#define IG_STAGGER 4   // tap rotation of the pixel-half-1 waves (0: all waves in tap order)
#endif

template <int LTW_>
struct IgCfg {
  static constexpr int NW = 8, NTHR = 512;
  static constexpr int CO_T = 128, WCO = 32, NCF = WCO / 16;   // 4 (channels) x 2 (pixels) waves
  static constexpr int PX_T = 256, NPF = 8;                    // pixel fragments (16 px) per wave
  static constexpr int LTW = LTW_, TW = 1 << LTW, TH = PX_T / TW, FPR = TW / 16, RPW = NPF / FPR;
  static constexpr int PR = TH + 2, PC = TW + 2, NPIX = PR * PC;
  static constexpr int PLANE = (NPIX + 15) / 16 * 16;          // 16-byte entries per (hl, group) plane
  static constexpr int XBUF = 2 * 4 * PLANE * 16;              // bytes per chunk buffer
  static constexpr int XJOBS = (4 * NPIX + NTHR - 1) / NTHR;   // (group, pixel) jobs per thread
  static constexpr int OPP = PX_T + 4;                         // output staging pitch (floats, 4 mod 32)
  static constexpr int STAGE = CO_T * OPP * 4;
  static constexpr int SMEM = 2 * XBUF > STAGE ? 2 * XBUF : STAGE;
  static constexpr int WSTEP = 2 * (CO_T / 16) * 1024;         // weight bytes per (chunk, tap): [hl][co/16][1 KiB]
  static_assert(XJOBS <= 4, "the patch jobs fit taps 0-7");
  static_assert(SMEM + 512 * 8 <= 160 * 1024, "LDS budget");
};

struct IgProb {
  const float *in;
  long in_bs;
  int Cin, H, W;
  const unsigned char *wt;   // split weights (sa_conv2d_igemm_weights)
  int Cout;
  const float *bias;
  int relu;
  float *out;
  long out_bs;
  int ltw, tiles_w, tiles_hw, co_blocks;
  double *partial;
  const float *in_m, *in_s, *in_t;
  int in_pstride, in_act;
  int pitch;
};
struct IgGate {
  int mode;
  const float *ctx;
  long ctx_bs;
  const float *h;
  long h_bs;
  const float *z;
  long z_bs;
  const float *add;
  long add_bs;
  float *out2;
  long out2_bs;
};
struct IgLaunch {
  IgProb p[MAX_PROB];
  IgGate gate[MAX_PROB];
  unsigned end[MAX_PROB];
  unsigned nblk[MAX_PROB];
  int nprob;
  int guard;   // range guard (a block with a finite input beyond the f16 range recomputes itself scaled)
};

__device__ unsigned g_ig_redo_blocks;

// The block's staged outputs (ot: [channel][pixel], pitch OPP; the accumulators times 2^-12):
// bias + ReLU, InstanceNorm partials (one part per block and channel: parts = tiles of the image),
// then float4 stores or the ConvGRU gate epilogue (update.py:16-27):
//   mode 1 (z | r over cat(h, x)): z = sigmoid(. + ctx) -> out, r * h -> out2 (block-uniform half)
//   mode 2 (q over r*h):           h' = (1 - z) h + z tanh((add + .) + ctx) -> out (in place on h)
template <class C, bool GATED>
__device__ __forceinline__ void ig_emit(const IgProb &P, const IgGate *gate, float *ot, const int n, const int co0,
                                        const int st, const int y0, const int x0, const int tid) {
  constexpr int NTHR = C::NTHR, OPP = C::OPP, CO_T = C::CO_T, TW = C::TW, PX_T = C::PX_T, LTW = C::LTW;
  const int H = P.H, W = P.W, pitch = P.pitch, hw = H * pitch;
  auto tail0 = [&](f32x4 v, const int x) __attribute__((always_inline)) {
    if (x + 4 > W) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (x + e >= W) v[e] = 0.0f;
    }
    return v;
  };
  // bias + ReLU in place (the statistics and the gates see the conv output with its bias)
  {
    constexpr int NJ = CO_T * PX_T / 4 / NTHR;
    const bool relu = P.relu != 0;
#pragma unroll 4
    for (int j = 0; j < NJ; ++j) {
      const int i4 = tid + NTHR * j, c = i4 / (PX_T / 4), p = (i4 % (PX_T / 4)) * 4;
      f32x4 *q = reinterpret_cast<f32x4 *>(ot + c * OPP + p);
      const float b = P.bias ? P.bias[co0 + c] : 0.0f;
      f32x4 v = *q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = v[e] + b;
        if (relu) v[e] = fmaxf(v[e], 0.0f);
      }
      *q = v;
    }
    __syncthreads();
  }
  if (P.partial) {
    constexpr int TPC = NTHR / CO_T, PPT = PX_T / TPC;   // threads per channel, pixels per thread
    const int c = tid / TPC, part = tid % TPC;
    double ssum = 0.0, ssq = 0.0;
#pragma unroll 4
    for (int p = part * PPT; p < (part + 1) * PPT; p += 4) {
      const int r = p >> LTW, cx = p & (TW - 1);
      if (y0 + r < H && x0 + cx < W) {
        const f32x4 v = tail0(*reinterpret_cast<const f32x4 *>(ot + c * OPP + p), x0 + cx);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double d = v[e];
          ssum += d;
          ssq += d * d;
        }
      }
    }
#pragma unroll
    for (int o = TPC / 2; o > 0; o >>= 1) {
      ssum += __shfl_xor(ssum, o);
      ssq += __shfl_xor(ssq, o);
    }
    if (part == 0) {
      double *pp = P.partial + (((long)n * P.Cout + co0 + c) * P.tiles_hw + st) * 2;
      pp[0] = ssum;
      pp[1] = ssq;
    }
  }
  float *dst = P.out + (long)n * P.out_bs;
  constexpr int NJ = CO_T * PX_T / (4 * NTHR);
  auto plain_stores = [&]() __attribute__((always_inline)) {
#pragma unroll 4
    for (int j = 0; j < NJ; ++j) {
      const int i4 = tid + NTHR * j;
      const int c = i4 / (PX_T / 4), p = (i4 % (PX_T / 4)) * 4, r = p >> LTW, cx = p & (TW - 1);
      const int y = y0 + r, x = x0 + cx;
      if (y < H && x < W)
        *reinterpret_cast<f32x4 *>(dst + (long)(co0 + c) * hw + (long)y * pitch + x) =
            tail0(*reinterpret_cast<const f32x4 *>(ot + c * OPP + p), x);
    }
  };
  if constexpr (!GATED) {
    plain_stores();
    return;
  } else {
    const IgGate &GT = *gate;
    if (GT.mode == 0) {
      plain_stores();
      return;
    }
    const int half = P.Cout / 2;
    const bool rhalf = co0 >= half;
    const float *ctxb = GT.ctx + (long)n * GT.ctx_bs;
    const float *hb = GT.h + (long)n * GT.h_bs;
    const float *ab = GT.add + (long)n * GT.add_bs;
    const float *zb = GT.z + (long)n * GT.z_bs;
    // the gate planes of a batch of store iterations are loaded together (out-of-image positions
    // read the block's first pixel and are not stored): all of a batch's loads in flight at once
    auto gate_stores = [&](auto gjb_c, auto mode_c) __attribute__((always_inline)) {
      constexpr int GJB = decltype(gjb_c)::value < NJ ? decltype(gjb_c)::value : NJ, MODE = decltype(mode_c)::value;
      static_assert(NJ % GJB == 0, "gate batches");
#pragma unroll 1
      for (int jb = 0; jb < NJ; jb += GJB) {
        int pos[GJB];
        bool ok[GJB];
        f32x4 cv[GJB], hv[GJB], av[GJB], zv[GJB];
#pragma unroll
        for (int u = 0; u < GJB; ++u) {
          const int i4 = tid + NTHR * (jb + u);
          const int c = i4 / (PX_T / 4), p = (i4 % (PX_T / 4)) * 4, r = p >> LTW, cx = p & (TW - 1);
          const int y = y0 + r, x = x0 + cx;
          ok[u] = y < H && x < W;
          pos[u] = (co0 + c) * hw + (ok[u] ? y * pitch + x : y0 * pitch + x0);
          cv[u] = *reinterpret_cast<const f32x4 *>(ctxb + pos[u]);
          if (MODE == 1) {
            if (rhalf) hv[u] = *reinterpret_cast<const f32x4 *>(hb + (pos[u] - half * hw));
          } else {
            av[u] = *reinterpret_cast<const f32x4 *>(ab + pos[u]);
            zv[u] = *reinterpret_cast<const f32x4 *>(zb + pos[u]);
            hv[u] = *reinterpret_cast<const f32x4 *>(hb + pos[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < GJB; ++u) {
          if (!ok[u]) continue;
          const int i4 = tid + NTHR * (jb + u);
          const int c = i4 / (PX_T / 4), p = (i4 % (PX_T / 4)) * 4;
          const int xg = x0 + (p & (TW - 1));
          const f32x4 v = *reinterpret_cast<const f32x4 *>(ot + c * OPP + p);
          f32x4 o;
          if (MODE == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = sa::sigmoidf_ref(v[e] + cv[u][e]);
            if (!rhalf) {
              *reinterpret_cast<f32x4 *>(dst + pos[u]) = tail0(o, xg);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] = o[e] * hv[u][e];
              *reinterpret_cast<f32x4 *>(GT.out2 + (long)n * GT.out2_bs + (pos[u] - half * hw)) = tail0(o, xg);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float q = tanhf((av[u][e] + v[e]) + cv[u][e]);
              o[e] = (1.0f - zv[u][e]) * hv[u][e] + zv[u][e] * q;
            }
            *reinterpret_cast<f32x4 *>(dst + pos[u]) = tail0(o, xg);
          }
        }
      }
    };
    if (GT.mode == 1) gate_stores(std::integral_constant<int, 16>{}, std::integral_constant<int, 1>{});
    else gate_stores(std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{});
  }
}

// One work item (128 output channels x one pixel tile of one image).
template <class C, bool GATED, bool AFF>
__device__ __forceinline__ void ig_body(const IgProb &P, const IgGate *gate, const unsigned wid, char *smem,
                                        float2 *atab, const bool guard) {
  constexpr int NTHR = C::NTHR, TW = C::TW, TH = C::TH, PC = C::PC, NPIX = C::NPIX, PLANE = C::PLANE,
                XBUF = C::XBUF, XJOBS = C::XJOBS, NCF = C::NCF, NPF = C::NPF, FPR = C::FPR, RPW = C::RPW,
                WSTEP = C::WSTEP, OPP = C::OPP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 3, pw = wv >> 2;   // the wave's 32-channel quarter and 128-pixel half
  const int co_blocks = P.co_blocks;
  const int cb = (int)(wid % (unsigned)co_blocks), tile = (int)(wid / (unsigned)co_blocks);
  const int st = tile % P.tiles_hw, n = tile / P.tiles_hw;
  const int y0 = (st / P.tiles_w) * TH, x0 = (st % P.tiles_w) * TW;
  const int H = P.H, W = P.W, pitch = P.pitch, hw = H * pitch;
  const int Cin = P.Cin, nchunks = Cin / KCH;
  const int co0 = cb * C::CO_T;

  // ---- input patch staging: job j = (8-channel group g, patch pixel q) ----
  // All global loads of the main loop are inline asm (asm volatile keeps their program order; the
  // compiler neither sinks the prefetches toward their uses nor counts them): the waits are placed by
  // hand, ig_wait<N> at the top of every tap, N = the loads issued since the data needed there.
  const __amdgpu_buffer_rsrc_t xin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(P.in + (long)n * P.in_bs), (short)0, Cin * hw * 4, 0x00020000);
  unsigned xoff[XJOBS];
  bool xin_img[XJOBS];
#pragma unroll
  for (int j = 0; j < XJOBS; ++j) {
    const int J = tid + NTHR * j;
    const int g = J / NPIX, q = J - g * NPIX, r = q / PC, c = q - r * PC;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    const bool ok = J < 4 * NPIX && y >= 0 && y < H && x >= 0 && x < W;
    xin_img[j] = ok;
    xoff[j] = ok ? (unsigned)((8 * g * hw + y * pitch + x) * 4) : IG_OOB;
  }
  // job j's LDS entry (group g, pixel q) = J + g (PLANE - NPIX), recomputed at its write (registers);
  // a slot-less lane writes the spare entry past the planes (branch-free, never read)
  auto xdst = [&](const int j) __attribute__((always_inline)) {
    const int J = tid + NTHR * j, g = J / NPIX;
    return J < 4 * NPIX ? (J + g * (PLANE - NPIX)) * 16 : 8 * PLANE * 16;
  };
  float xv[2][8];   // two jobs in flight (a job's loads go out three tap positions before its write)
  // range guard: a finite operand outside the f16 range; the largest finite magnitude staged
  bool bad = false;
  float xmax = 0.0f;
  float xscale = 1.0f;   // the recompute pass's power-of-two input scale
  auto xload = [&](const int j, const int chunk) __attribute__((always_inline)) {
    const int cs = chunk * KCH * hw * 4;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const unsigned o = xoff[j] + (unsigned)(e * hw * 4);
      asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(xv[j & 1][e]) : "v"(o), "s"(xin), "s"(cs));
    }
  };
  const float act_floor = P.in_act ? 0.0f : -INFINITY;
  auto xwrite = [&](const int j, const int chunk, char *buf) __attribute__((always_inline)) {
    f16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = xv[j & 1][e];
      if constexpr (AFF) {
        if (xin_img[j]) {
          const float2 ab = atab[chunk * KCH + 8 * ((tid + NTHR * j) / NPIX) + e];
          v = fmaxf(v * ab.x + ab.y, act_floor);
        }
      }
      const float a = __builtin_fabsf(v);
      const bool fin = a < INFINITY;   // (false for NaN too)
      bad |= fin && a >= 65504.0f;
      xmax = fmaxf(xmax, fin ? a : 0.0f);
      v *= xscale;
      const _Float16 h = (_Float16)v;
      hi[e] = h;
      lo[e] = (_Float16)(v - (float)h);
    }
    const int d = xdst(j);
    *reinterpret_cast<f16x8 *>(buf + d) = hi;
    *reinterpret_cast<f16x8 *>(buf + d + 4 * PLANE * 16) = lo;
  };

  // ---- weights: A operands straight from L2, two taps ahead ----
  // [co block][chunk][tap][hl][16-channel group][g][co % 16][8]: the wave's fragment (hl, cf) of a
  // step is 1 KiB at wbase + step * WSTEP + hl * WSTEP / 2 + cf * 1024
  const unsigned char *wbase = P.wt + (long)cb * nchunks * 9 * WSTEP + (wc * NCF) * 1024 + lane * 16;
  const int nsteps = nchunks * 9;
  static_assert(NCF == 2, "four weight fragments per step");
  f16x8 wr[3][2][NCF];
  auto wload = [&](f16x8 (&w)[2][NCF], int step) __attribute__((always_inline)) {
    step = step < nsteps ? step : nsteps - 1;   // (past the end: a harmless re-read, no branch)
    const unsigned char *q = wbase + (long)step * WSTEP;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(w[0][0]) : "v"(q));
    asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(w[0][1]) : "v"(q));
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(w[1][0]) : "v"(q + WSTEP / 2));
    asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(w[1][1]) : "v"(q + WSTEP / 2));
  };
  // s_waitcnt vmcnt(N) tied to the registers it guards (no use is scheduled above it)
  auto wait_w = [](auto n_c, f16x8 (&w)[2][NCF]) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1])
                 : "n"(decltype(n_c)::value));
  };
  auto wait_x = [](auto n_c, float (&x)[8]) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(%8)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]),
                 "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "n"(decltype(n_c)::value));
  };

  // input transform table (the producer's norm + activation, applied as the patch is split)
  if constexpr (AFF) {
    for (int c = tid; c < Cin; c += NTHR) {
      const int pi = n * P.in_pstride + c;
      const float m0 = P.in_m ? P.in_m[pi] : 0.0f, sc = P.in_s ? P.in_s[pi] : 1.0f, t0 = P.in_t ? P.in_t[pi] : 0.0f;
      atab[c] = make_float2(sc, t0 - m0 * sc);
    }
    __syncthreads();
  }

  // Pass 0 on the inputs as they are; pass 1 (block-uniform, only when pass 0 staged a finite value
  // beyond the f16 range) on the inputs times 2^-k, which brings the block's largest one below 2^15
  // (exact scaling; the accumulators are scaled back by 2^k).
  f32x4 acc[NCF][NPF];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
  // prologue: chunk 0's patch, then the first two taps' weights
#pragma unroll
  for (int j = 0; j < XJOBS; ++j) {
    xload(j, 0);
    wait_x(std::integral_constant<int, 0>{}, xv[j & 1]);
    xwrite(j, 0, smem);
  }
  const int toff = IG_STAGGER && pw ? IG_STAGGER : 0;   // (wave-uniform)
  wload(wr[0], toff);
  wload(wr[1], toff + 1 >= 9 ? toff - 8 : toff + 1);

#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int f = 0; f < NPF; ++f) acc[cf][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the lane's B-operand entry: group lane / 16, pixel (lane % 16) of fragment 0 of the wave
  const int xlane = ((lane >> 4) * PLANE + (lane & 15) + pw * RPW * PC) * 16;
  __syncthreads();

  // Per tap: (top) wait for this tap's weights (and the patch job loaded two taps ago), write that
  // job's split values into the next chunk's buffer, 16 B-operand reads + 48 MFMAs, then (end)
  // the next patch job's loads (even taps) and the weights of the tap after next.  Every chunk
  // issues its patch loads (the last one re-reads its own chunk into the idle buffer), so the
  // counts are static.
#pragma unroll 1
  for (int kc = 0; kc < nchunks; ++kc) {
    const char *xb = smem + (kc & 1) * XBUF + xlane;
    char *xn = smem + ((kc + 1) & 1) * XBUF;
    const bool more = kc + 1 < nchunks;
    const int kn = more ? kc + 1 : kc;
#pragma unroll
    for (int pos = 0; pos < 9; ++pos) {
      // the tap at this position: the pixel-half-1 waves (SIMD partners of the half-0 waves) run the
      // taps rotated by IG_STAGGER, so partners' LDS bursts and MFMA runs interleave
      int tap = pos + toff;
      tap = tap >= 9 ? tap - 9 : tap;
      f16x8(&w)[2][NCF] = wr[pos % 3];
      // Loads in issue order, at the end of each position p: the next chunk's patch job p / 2 (even
      // p <= 6), then the weights of position p + 2.  Job j is written three positions after its
      // loads (top of 2j + 3; job 3 at the end of position 8).  So the loads issued after this
      // position's weights are the next position's weights and, after an even position, a patch
      // job; on an odd position that waits for the job loaded at the end of p - 3 as well.
      if ((pos & 1) && (pos - 1) / 2 < XJOBS) {
        wait_w(std::integral_constant<int, 12>{}, w);
        if (pos >= 3 && (pos - 3) / 2 < XJOBS) {
          wait_x(std::integral_constant<int, 12>{}, xv[((pos - 3) / 2) & 1]);   // (ties the job's registers)
          if (IG_DIAG != 2 && IG_DIAG != 4) xwrite((pos - 3) / 2, kn, xn);
        }
      } else {
        wait_w(std::integral_constant<int, 4>{}, w);
        if ((pos & 1) && pos >= 3 && (pos - 3) / 2 < XJOBS) {
          wait_x(std::integral_constant<int, 4>{}, xv[((pos - 3) / 2) & 1]);
          if (IG_DIAG != 2 && IG_DIAG != 4) xwrite((pos - 3) / 2, kn, xn);
        }
      }
      const char *xt = xb + ((tap / 3) * PC + tap % 3) * 16;
      // the 8 pixel fragments in two halves of 4 (the B operands of a half: 32 VGPRs), each
      // half's products hi*hi, hi*lo, lo*hi over its 4 x 2 tiles (consecutive MFMAs on different
      // accumulators)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f16x8 bh[NPF / 2], bl[NPF / 2];
#pragma unroll
        for (int u = 0; u < NPF / 2; ++u) {
          const int f = hf * (NPF / 2) + u, qf = (f / FPR) * PC + (f % FPR) * 16;
          bh[u] = *reinterpret_cast<const f16x8 *>(xt + qf * 16);
          bl[u] = *reinterpret_cast<const f16x8 *>(xt + qf * 16 + 4 * PLANE * 16);
        }
        if constexpr (IG_DIAG == 5) {
#pragma unroll
          for (int u = 0; u < NPF / 2; ++u)
            acc[0][hf * 4 + u][0] += (float)(bh[u][0] + bl[u][1] + w[0][0][u] + w[1][1][u]);
        } else {
#pragma unroll
          for (int u = 0; u < NPF / 2; ++u)
#pragma unroll
            for (int cf = 0; cf < NCF; ++cf)
              acc[cf][hf * 4 + u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0][cf], bh[u], acc[cf][hf * 4 + u], 0, 0, 0);
#pragma unroll
          for (int u = 0; u < NPF / 2; ++u)
#pragma unroll
            for (int cf = 0; cf < NCF; ++cf)
              acc[cf][hf * 4 + u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0][cf], bl[u], acc[cf][hf * 4 + u], 0, 0, 0);
#pragma unroll
          for (int u = 0; u < NPF / 2; ++u)
#pragma unroll
            for (int cf = 0; cf < NCF; ++cf)
              acc[cf][hf * 4 + u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[1][cf], bh[u], acc[cf][hf * 4 + u], 0, 0, 0);
        }
      }
      if (!(pos & 1) && pos / 2 < XJOBS && IG_DIAG != 2 && IG_DIAG != 4) xload(pos / 2, kn);
      {
        int t2 = pos + 2 + toff, c2 = kc;
        if (pos + 2 >= 9) {
          t2 -= 9;
          c2 += 1;
        }
        t2 = t2 >= 9 ? t2 - 9 : t2;
        // (past the last chunk: clamped re-reads, so that every position's wait count is static;
        // no branch on `more` around a wait: the compiler once merged such paths with register
        // copies of loads still in flight, scripts/check_asm_loads.py)
        if (IG_DIAG != 1 && IG_DIAG != 4) wload(wr[(pos + 2) % 3], c2 * 9 + t2);
        else {   // (diagnostic: the same random operands, no loads)
#pragma unroll
          for (int hl = 0; hl < 2; ++hl)
#pragma unroll
            for (int cf = 0; cf < NCF; ++cf) wr[(pos + 2) % 3][hl][cf] = wr[pos % 3][hl][cf];
        }
      }
    }
    if constexpr (XJOBS == 4) {   // job 3 (loaded at the end of position 6; complete since position 8's wait)
      wait_x(std::integral_constant<int, 8>{}, xv[1]);
      if (IG_DIAG != 2 && IG_DIAG != 4) xwrite(3, kn, xn);
    }
    if (IG_DIAG != 3 && IG_DIAG != 4) __syncthreads();   // chunk kc + 1's patch is written; chunk kc's buffer is free
  }
  // nothing in flight past the loop; the wait names every register an asm load may still be
  // writing (so none of them is dead, copied or reused before it)
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(wr[0][0][0]), "+v"(wr[0][0][1]), "+v"(wr[0][1][0]), "+v"(wr[0][1][1]), "+v"(wr[1][0][0]),
                 "+v"(wr[1][0][1]), "+v"(wr[1][1][0]), "+v"(wr[1][1][1]), "+v"(wr[2][0][0]), "+v"(wr[2][0][1]),
                 "+v"(wr[2][1][0]), "+v"(wr[2][1][1])
               :
               : "memory");
  asm volatile("" : "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[0][4]), "+v"(xv[0][5]),
               "+v"(xv[0][6]), "+v"(xv[0][7]), "+v"(xv[1][0]), "+v"(xv[1][1]), "+v"(xv[1][2]), "+v"(xv[1][3]),
               "+v"(xv[1][4]), "+v"(xv[1][5]), "+v"(xv[1][6]), "+v"(xv[1][7]));
  if (pass == 1 || !guard || !__syncthreads_or(bad)) break;
  // the block's largest finite input: wave maxima through LDS (the patch buffers are free)
  {
    float *red = reinterpret_cast<float *>(smem);
    const float wmax = sa::wave_max_dpp(xmax);
    if (lane == 0) red[wv] = wmax;
    __syncthreads();
    float m = red[0];
#pragma unroll
    for (int w = 1; w < C::NW; ++w) m = fmaxf(m, red[w]);
    int e;
    (void)frexpf(m, &e);             // m < 2^e
    xscale = ldexpf(1.0f, 15 - e);   // m * xscale < 2^15
    __syncthreads();
    if (tid == 0) atomicAdd(&g_ig_redo_blocks, 1u);
  }
  }

  // accumulators -> LDS planes [channel][pixel] (times 2^-12)
  float *ot = reinterpret_cast<float *>(smem);
  const float inv = 1.0f / ((float)(1 << IG_LOG2) * xscale);
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int f = 0; f < NPF; ++f) {
      const int p = (pw * NPF + f) * 16 + (lane & 15);
      const int c = wc * C::WCO + cf * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) ot[(c + e) * OPP + p] = acc[cf][f][e] * inv;
    }
  __syncthreads();
  ig_emit<C, GATED>(P, gate, ot, n, co0, st, y0, x0, tid);
}

template <bool GATED, bool AFF>
__global__ __launch_bounds__(512, 1) void ig_kernel(const IgLaunch L) {
  const unsigned g = blockIdx.x;
  int pi = 0;
#pragma unroll
  for (int i = 1; i < MAX_PROB; ++i) pi += (i < L.nprob && g >= L.end[i - 1]) ? 1 : 0;
  const IgProb &P = L.p[pi];
  const unsigned base = pi ? L.end[pi - 1] : 0u, nb = L.nblk[pi];
  if (g - base >= nb) return;
  __shared__ __attribute__((aligned(16))) char smem[IgCfg<5>::SMEM > IgCfg<6>::SMEM ? IgCfg<5>::SMEM : IgCfg<6>::SMEM];
  __shared__ float2 atab[AFF ? 512 : 1];
  const unsigned wid = sa::xcd_remap(g - base, nb);
  const IgGate *gp = GATED ? &L.gate[pi] : nullptr;
  const bool guard = L.guard != 0;
  if (P.ltw == 4) ig_body<IgCfg<4>, GATED, AFF>(P, gp, wid, smem, atab, guard);
  else if (P.ltw == 5) ig_body<IgCfg<5>, GATED, AFF>(P, gp, wid, smem, atab, guard);
  else ig_body<IgCfg<6>, GATED, AFF>(P, gp, wid, smem, atab, guard);
}

// w[co][ci][3][3] -> [Cout/128][Cin/32][9][hl][co/16 % 8][g][co % 16][8] f16 of w * 2^12
// (hl 0: hi = f16(v), 1: lo = f16(v - hi))
__global__ __launch_bounds__(256) void ig_weights_kernel(const float *__restrict__ w, int Cout, int Cin,
                                                         _Float16 *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * 9) return;
  const int tap = (int)(i % 9), ci = (int)((i / 9) % Cin), co = (int)(i / (9L * Cin));
  const float v = w[i] * (float)(1 << IG_LOG2);
  const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
  const int nch = Cin / KCH, cb = co / 128, cg = (co % 128) / 16, c16 = co % 16, kc = ci / KCH, g = (ci % KCH) / 8,
            j = ci % 8;
  const long base = ((long)(cb * nch + kc) * 9 + tap) * 2;
  const long e = ((long)cg * 4 + g) * 16 * 8 + c16 * 8 + j;
  out[(base + 0) * 8 * 512 + e] = hi;
  out[(base + 1) * 8 * 512 + e] = lo;
}

// geometry with the fewest padded output pixels (ties: the smaller halo, 16 x 16 first)
int ig_ltw(int H, int W) {
  int best = 4;
  long barea = -1;
  for (int ltw = 4; ltw <= 6; ++ltw) {
    const int tw = 1 << ltw, th = 256 / tw;
    const long a = (long)((W + tw - 1) / tw) * tw * ((H + th - 1) / th) * th;
    if (barea < 0 || a < barea) {
      barea = a;
      best = ltw;
    }
  }
  return best;
}

}  // namespace

extern "C" long sa_conv2d_igemm_weights_size(int Cout, int Cin) {
  if (Cout <= 0 || Cin <= 0 || Cout % 128 || Cin % KCH) return -1;
  return (long)Cout * Cin * 9;   // dwords (an f16 hi / lo pair per weight)
}

extern "C" int sa_conv2d_igemm_weights(const float *weight, int Cout, int Cin, void *out, void *stream) {
  SA_REQUIRE(weight && out && sa_conv2d_igemm_weights_size(Cout, Cin) > 0,
             "sa_conv2d_igemm_weights: needs Cout %% 128 == 0 and Cin %% 32 == 0 (got %d, %d)", Cout, Cin);
  const long n = (long)Cout * Cin * 9;
  hipStream_t s = sa::as_stream(stream);
  ig_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, static_cast<_Float16 *>(out));
  return sa::check_launch("sa_conv2d_igemm_weights");
}

extern "C" long sa_conv2d_igemm_stat_parts(int H, int W) {
  if (H <= 0 || W <= 0) return -1;
  const int ltw = ig_ltw(H, W), tw = 1 << ltw, th = 256 / tw;
  return (long)((W + tw - 1) / tw) * ((H + th - 1) / th);
}

extern "C" long sa_conv2d_igemm_blocks(int N, int Cout, int H, int W) {
  const long parts = sa_conv2d_igemm_stat_parts(H, W);
  if (N <= 0 || Cout <= 0 || Cout % 128 || parts < 0) return -1;
  return (long)N * parts * (Cout / 128);
}

long sa_igemm_redo_blocks_internal(int reset) {   // (sa_split_redo_blocks adds it up; synchronised there)
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ig_redo_blocks), sizeof v) != hipSuccess) return -1;
  if (reset) {
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ig_redo_blocks), &z, sizeof z) != hipSuccess) return -1;
  }
  return (long)v;
}

extern "C" int sa_conv2d_k3_igemm(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates, int guard,
                                  void *stream) {
  SA_REQUIRE(nprob >= 1 && nprob <= MAX_PROB && probs, "sa_conv2d_k3_igemm: 1..%d problems", MAX_PROB);
  IgLaunch L{};
  long total = 0;
  bool gated = false, aff = false;
  for (int i = 0; i < nprob; ++i) {
    const SaWinoProblem &q = probs[i];
    SA_REQUIRE(q.in && q.U && q.out && q.N > 0 && q.H > 0 && q.W > 0, "sa_conv2d_k3_igemm: bad arguments");
    SA_REQUIRE(!q.skip, "sa_conv2d_k3_igemm: the residual epilogue is F(4x4) only");
    SA_REQUIRE(q.Cin % KCH == 0 && q.Cout % 128 == 0,
               "sa_conv2d_k3_igemm: needs Cin %% 32 == 0 and Cout %% 128 == 0 (got %d, %d)", q.Cin, q.Cout);
    const int pitch = q.pitch ? q.pitch : q.W;
    SA_REQUIRE(pitch >= q.W, "sa_conv2d_k3_igemm: pitch %d < W %d", pitch, q.W);
    SA_REQUIRE(pitch % 4 == 0 && (reinterpret_cast<uintptr_t>(q.out) & 15) == 0 && q.out_bs % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(q.U) & 15) == 0,
               "sa_conv2d_k3_igemm: needs the row pitch %% 4 == 0, 16-byte aligned output planes and weights");
    SA_REQUIRE((long)q.Cin * q.H * pitch * 4 < (1L << 30) && (long)q.H * pitch * 4 * 8 < (1L << 31),
               "sa_conv2d_k3_igemm: an image exceeds the buffer-descriptor range");
    const bool qaff = q.in_m || q.in_s || q.in_t || q.in_act;
    SA_REQUIRE(q.in_act == 0 || q.in_act == 1, "sa_conv2d_k3_igemm: input activation none or ReLU (got %d)", q.in_act);
    SA_REQUIRE(q.in_pstride == 0 || q.in_pstride == q.Cin, "sa_conv2d_k3_igemm: in_pstride must be 0 or Cin");
    SA_REQUIRE(!qaff || q.Cin <= 512, "sa_conv2d_k3_igemm: an input transform needs Cin <= 512");
    aff = aff || qaff;
    const int ltw = ig_ltw(q.H, q.W), tw = 1 << ltw, th = 256 / tw;
    const int tiles_w = (q.W + tw - 1) / tw, tiles_h = (q.H + th - 1) / th;
    L.p[i] = IgProb{q.in, q.in_bs, q.Cin, q.H, q.W, reinterpret_cast<const unsigned char *>(q.U), q.Cout, q.bias,
                    q.relu, q.out, q.out_bs, ltw, tiles_w, tiles_w * tiles_h, q.Cout / 128, q.stats_partial,
                    q.in_m, q.in_s, q.in_t, q.in_pstride, q.in_act, pitch};
    L.gate[i] = IgGate{};
    if (gates && gates[i].mode != 0) {
      const SaGateEpilogue &e = gates[i];
      auto a16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
      SA_REQUIRE(e.mode == 1 || e.mode == 2, "sa_conv2d_k3_igemm: gate mode %d (1 or 2)", e.mode);
      SA_REQUIRE(!q.relu && !q.stats_partial, "sa_conv2d_k3_igemm: a gate epilogue takes no ReLU / statistics");
      SA_REQUIRE(e.ctx && e.h && a16(e.ctx) && a16(e.h) && e.ctx_bs % 4 == 0 && e.h_bs % 4 == 0,
                 "sa_conv2d_k3_igemm: gate needs 16-byte aligned ctx and h planes");
      if (e.mode == 1)
        SA_REQUIRE(q.Cout % 256 == 0 && e.out2 && a16(e.out2) && e.out2_bs % 4 == 0,
                   "sa_conv2d_k3_igemm: z/r gate needs Cout %% 256 == 0 and an aligned r*h output");
      else
        SA_REQUIRE(e.z && e.add && a16(e.z) && a16(e.add) && e.z_bs % 4 == 0 && e.add_bs % 4 == 0,
                   "sa_conv2d_k3_igemm: state gate needs aligned z and addend planes");
      L.gate[i] = IgGate{e.mode, e.ctx, e.ctx_bs, e.h, e.h_bs, e.z, e.z_bs, e.add, e.add_bs, e.out2, e.out2_bs};
      gated = true;
    }
    const long nb = (long)q.N * L.p[i].tiles_hw * L.p[i].co_blocks;
    total = (i + 1 < nprob ? (total + nb + 7) / 8 * 8 : total + nb);
    SA_REQUIRE(total < (1L << 27), "sa_conv2d_k3_igemm: grid too large");
    L.end[i] = (unsigned)total;
    L.nblk[i] = (unsigned)nb;
  }
  for (int i = nprob; i < MAX_PROB; ++i) {
    L.end[i] = (unsigned)total;
    L.nblk[i] = 0;
  }
  L.nprob = nprob;
  SA_REQUIRE(!(aff && gated), "sa_conv2d_k3_igemm: an input transform and a gate epilogue in one launch");
  L.guard = guard ? 1 : 0;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV2D_IG, s);
  aff     ? ig_kernel<false, true><<<(unsigned)total, 512, 0, s>>>(L)
  : gated ? ig_kernel<true, false><<<(unsigned)total, 512, 0, s>>>(L)
          : ig_kernel<false, false><<<(unsigned)total, 512, 0, s>>>(L);
  return sa::check_launch("sa_conv2d_k3_igemm");
}
