// 3x3 / stride 1 / pad 1 convolution as fused Winograd F(4x4, 3x3) on fp32 MFMA.
//
// Same role as conv2d_wino.hip (the encoder and update-block 3x3 convs, extractor.py:6-300,
// update.py:46-110) with 36 products per 4x4 outputs instead of 16 per 2x2: 2.25 products
// per output against 4, so the fp32 MFMA peak is 629 TF/s direct-equivalent.  Transform
// points 0, +-1, +-2, inf (B^T, G, A^T below; filters transformed in fp64, rounded once).
//
//   block  = 8 waves, 64 Winograd tiles (16 x 64 or 8 x 128 output pixels, chosen per conv
//            to waste the fewest padded pixels) x 32 output channels
//   wave   = 16 tiles (one MFMA M-block) x 32 output channels x one half of the 36 transform
//            points (columns 0-2 or 3-5 of the 6 x 6 point grid): 144 fp32 accumulators, each
//            transformed input feeding two MFMAs.  The output transform runs in registers as
//            far as each half allows; the two halves' partial outputs meet in LDS.
//   chunk  = 8 input channels.  The input patch and the chunk's transformed filters are
//            copied global -> LDS by LDS-DMA (buffer_load ... lds, no staging registers),
//            one chunk ahead, one barrier per chunk.  Zero padding = out-of-range loads
//            (the patch is staged 16-byte aligned, so every 4-float group is wholly inside
//            or outside the image; needs W % 4 == 0).
//   input transform straight into MFMA operands: lane (k, m) of a v_mfma_f32_16x16x4_f32
//            holds A[tile m][channel k], which is exactly one (tile, channel) transform job,
//            so V = B^T d B never goes through LDS: the lane reads its 6 patch rows (all in
//            flight together), runs its half of the row pass (3 of 6 outputs per row), then
//            each of its 3 column passes yields the A operands of 6 x 2 MFMAs
//   filters B operands of the two output-channel halves as one float2 per lane (U[point][channel]
//            [co % 16][co / 16]: conflict-free ds_read_b64)
//
// No transform work is duplicated: each (tile, channel, point) value is computed once, by the
// lane that feeds it to its two MFMAs (about 2 VALU operations per MFMA).
#include "sa_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#pragma clang fp contract(fast)

// diagnostic switch (build-time)
#ifndef SA_W4_DIAG
#define SA_W4_DIAG 0   // timing diagnostics only (wrong results): 1 no DMA in the loop, 2 no
                       // transform / MFMA, 3 no DMA and no barrier in the loop, 4 as 3 and no
                       // DMA at all, 5 no column pass, 6 no row pass, 7 no filter reads in the loop,
                       // 8 neither row nor column pass (no input transform), 9 the loop waits for
                       // chunk kc - 1's DMAs only (the floor of a ring that issues two chunks ahead)
#endif
#ifndef SA_W4_PAIR
#define SA_W4_PAIR 1   // split kernel: a lane's two channels (jobs) in one MFMA pair (w4_pair_split, round 6)
#endif
#ifndef SA_W4_PAIR_AFF
// the affine-input split kernel on the paired loop too: it spills 28 B per lane (loop-invariant values
// around the main loop, one reload per chunk in the affine pass) and is still faster: forward
// 58.7 -> 58.1 ms/step, two interleaved passes (profiles/ab/r06_w4_pair_ab.txt)
#define SA_W4_PAIR_AFF 1
#endif
#ifndef SA_W4_GJB
#define SA_W4_GJB 4    // gate-epilogue store iterations whose plane loads go out together (mode 2)
#endif
#ifndef SA_W4_GJB1
#define SA_W4_GJB1 8   // the same for mode 1 (8 / 16 measured the same, 49.99 vs 50.01 ms/step, but
                       // with them the range guard's second body made the gated kernel spill 2 KiB)
#endif

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
using f16x4 = __attribute__((ext_vector_type(4))) _Float16;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr int NPT = 36;                   // transform points

// Two block shapes of the same algorithm.  Large (the default): 8 waves, 64 tiles, 8-channel
// chunks, one block per CU (158 KiB of LDS).  Small (block_shape 2): 4 waves, 32 tiles,
// 4-channel chunks, 66 KiB, two blocks per CU, so one block's first DMA wait and epilogue
// overlap the other's MFMAs (per block ~6-8k cycles until the first chunk lands and ~9k of
// epilogue around 6.8k per chunk, scripts/w4_clock.py); it is not faster in the forward.
// (Measured slower and removed, in git history: a wide 64-channel shape, a quadrant shape, a
// persistent kernel, the split products on the small shape, and the K = 32 / duplicated-read split
// forms)
template <int NW_, int KC_, bool SPLIT_ = false>
struct W4Cfg {
  // SPLIT: the products on f16 MFMA with hi/lo operand pairs (W4Split below)
  static constexpr bool SPLIT = SPLIT_;
  static constexpr int NW = NW_, NTHR = 64 * NW_, TG = NW_ / 2, NT = 16 * TG, KC = KC_, JPC = KC_ / 4;
  static constexpr int NR = 6;                              // point rows per wave
  static constexpr int CO = 32, CG = 2;                     // output channels per block, 16-channel groups
  static constexpr int SB = 4 * CO;                         // filters per (point, 4-channel job): [k][n][g]
  static constexpr int PS_MAX = NT == 64 ? 340 : 204;       // (BH + 2)(BW / 4 + 2), largest geometry
  static constexpr int PBUF = (KC * PS_MAX + 63) / 64 * 64 * 4;   // whole DMA pieces (the last one's idle lanes write zeros)
  static constexpr int UBUF = NPT * KC * CO;                // filters per chunk (dwords)
  static constexpr int BUF = PBUF + UBUF;                   // one buffer: patch, then filters
  static constexpr int OPP = NT * 16 + 4;                   // output staging plane pitch (4 mod 32)
  // (past the output staging: the flow head's taps and the range guard's per-wave flags)
  static constexpr int SMEM = 2 * BUF > CO * OPP + CO * 9 + 8 ? 2 * BUF : CO * OPP + CO * 9 + 8;
  static constexpr int PDMA = ((KC * PS_MAX + 63) / 64 + NW - 1) / NW;   // patch DMA pieces per wave
  static constexpr int UDMA = UBUF / 256;                   // filter DMA pieces (1 KiB) per chunk
  static constexpr int UPW = (UDMA + NW - 1) / NW;          // per wave
  static_assert(SMEM * 4 <= 160 * 1024, "LDS budget");
  static constexpr int PPART = (PDMA > UPW ? PDMA : UPW) > 6 ? 3 : 2;   // DMA pieces per part
  static_assert(PDMA <= 3 * PPART && UPW <= 3 * PPART, "three DMA parts");
  static_assert(OPP % 32 == 4, "conflict-free staging");
  // input (scale, shift) table of an input-transform launch in the LDS left over
  static constexpr int AFF_MAX = (160 * 1024 - SMEM * 4) / 8 > 512 ? 512 : (160 * 1024 - SMEM * 4) / 8;
};
using W4Big = W4Cfg<8, 8>;
using W4Small = W4Cfg<4, 4>;
// Split: the 8-wave shape whose Winograd-domain products run on v_mfma_f32_16x16x16_f16 instead of
// v_mfma_f32_16x16x4_f32.  Each operand is an f16 hi/lo pair (x = hi + lo, 22 significant bits;
// filters scaled by 2^W4S_LOG2 before the split and the accumulators by 2^-W4S_LOG2 after the main
// loop, both exact), and one MFMA's K = 16 slots hold a lane's channel as the four products
// hi*bhi + hi*blo + lo*bhi + lo*blo: the A operand (hi, hi, lo, lo) is the lane's transformed value
// (3 VALU to split), the B operand (bhi, blo, bhi, blo) is the filter's (bhi, blo) dword twice: the
// LDS image holds each pair once (sa_conv2d_wino4_weights_split; the same bytes per chunk as the
// fp32 filters, so the same L2 -> LDS intake per channel, which bounds this kernel family), one
// ds_read_b64 gives a lane both output-channel groups' pairs, and the copy is a register move.
// Products of f16 pairs are exact in fp32, so the result differs from the fp32 kernel only by the
// operands' rounding (<= 2^-22 relative; below 2^-14 the lo halves are subnormal, an absolute
// 2^-25) and the accumulation order.  |V| must stay below 65504 (the f16 range): V = B^T d B grows
// at most 100-fold over the input patch.
using W4Split = W4Cfg<8, 8, true>;
constexpr int W4S_LOG2 = 12;
static_assert(2 * W4Small::SMEM * 4 <= 160 * 1024, "two small blocks per CU");

struct W4Prob {
  const float *in;
  long in_bs;
  int Cin, H, W;
  const float *U;
  int Cout;
  const float *bias;
  int relu;
  float *out;
  long out_bs;
  int ltw;                 // log2 of Winograd tiles per block row: 4 (16 x 64 px) or 5 (8 x 128 px)
  int tiles_w, tiles_hw, co_blocks;
  double *partial;
  // input transform (the producer's norm + ReLU, SaWinoProblem in_m / in_s / in_t / in_act)
  const float *in_m, *in_s, *in_t;
  int in_pstride, in_act;
  int pitch;               // row pitch of the input / output / gate planes (>= W, % 4 == 0; SaWinoProblem)
  // residual epilogue (SaWinoProblem skip ...): out = oact(act(conv + bias) + skip_act(skip * s + t))
  const float *skip;
  long skip_bs;
  const float *skip_s, *skip_t;
  int skip_act, out_act;
};
constexpr int MAX_PROB = 8;

// work item -> (output-channel block, tile in the image, image): a tile's channel blocks adjacent
__device__ __forceinline__ void w4_item(const unsigned wid, const int co_blocks, const int tiles_hw, int &cb, int &st,
                                        int &n) {
  cb = wid % co_blocks;
  const int gt = wid / co_blocks;
  st = gt % tiles_hw;
  n = gt / tiles_hw;
}
// GRU gate epilogues (SaGateEpilogue in the header), read by the store loop only
struct W4Gate {
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
  const float *head_w;   // mode 3 (w4_flowhead)
  float *head_part;
  long head_part_bs;
};
struct W4Launch {
  W4Prob p[MAX_PROB];
  W4Gate gate[MAX_PROB];
  unsigned end[MAX_PROB];
  unsigned nblk[MAX_PROB];
  int nprob;
  int guard;   // the split kernel's range guard (an overflowed block runs again on scaled inputs)
};

// x as the f16 A operand (hi, hi, lo, lo): hi = f16(x), lo = f16(x - hi) (x - hi is exact in
// fp32; one v_fma_mix_f32 reads hi as f16), both round-to-nearest-even
__device__ __forceinline__ f16x4 w4_split(const float x) {
  const f16x2 hh = __builtin_convertvector(f32x2{x, x}, f16x2);
  float l;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(__builtin_bit_cast(unsigned, hh)), "v"(x));
  const f16x2 ll = __builtin_convertvector(f32x2{l, l}, f16x2);
  return __builtin_shufflevector(hh, ll, 0, 1, 2, 3);
}

// The two channels of a lane's jobs (c and c + 4) as the A operands of one MFMA pair (SA_W4_PAIR):
// ahi = (hi0, hi0, hi1, hi1), alo = (lo0, 0, lo1, 0) against B = (bhi0, blo0, bhi1, blo1), the two
// channels' filter (hi, lo) dwords of one output channel, adjacent in the job-innermost LDS image
// (one ds_read_b128 per point holds both groups' pairs): ahi . B = hi0 bhi0 + hi0 blo0 + hi1 bhi1 +
// hi1 blo1, alo . B = lo0 bhi0 + lo1 bhi1,
// i.e. per channel hi*bhi + hi*blo + lo*bhi (the dropped lo*lo term is below 2^-22 of the product).
// The B operand needs no register copy (the one-channel form duplicates the (bhi, blo) dword: one
// v_mov per MFMA, ~1 of the kernel's 5-7 VALU per MFMA) at the same MFMA and LDS instruction counts.
__device__ __forceinline__ void w4_pair_split(const float x0, const float x1, f16x4 &ahi, f16x4 &alo) {
  const f16x2 h0 = __builtin_convertvector(f32x2{x0, x0}, f16x2);
  const f16x2 h1 = __builtin_convertvector(f32x2{x1, x1}, f16x2);
  float l0, l1;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l0) : "v"(__builtin_bit_cast(unsigned, h0)), "v"(x0));
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l1) : "v"(__builtin_bit_cast(unsigned, h1)), "v"(x1));
  const f16x2 q0 = __builtin_convertvector(f32x2{l0, 0.0f}, f16x2);
  const f16x2 q1 = __builtin_convertvector(f32x2{l1, 0.0f}, f16x2);
  ahi = __builtin_shufflevector(h0, h1, 0, 1, 2, 3);
  alo = __builtin_shufflevector(q0, q1, 0, 1, 2, 3);
}

// Range guard of the split kernel: blocks whose f16 operands overflowed (|V| >= 65520 turns hi
// into inf, so every product of that value, and the outputs it feeds, are NaN) run their item
// again inside the launch on exactly scaled inputs (w4_body's xscale); this counts them
// (sa_split_redo_blocks)
__device__ unsigned g_w4_redo_blocks;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, float *lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds, 16, voff, soff, 0, 0);
}

// B^T x for x = 6 samples (rows of B^T: [4,0,-5,0,1,0] [0,-4,-4,1,1,0] [0,4,-4,-1,1,0]
// [0,-2,-1,2,1,0] [0,2,-1,-2,1,0] [0,4,0,-5,0,1])
__device__ __forceinline__ void bt6(const float x0, const float x1, const float x2, const float x3, const float x4,
                                    const float x5, float *o) {
  // 12 FMA-unit operations (explicit fmaf: no separate multiplies)
  const float a = fmaf(-4.0f, x2, x4), b = fmaf(-4.0f, x1, x3), c = x4 - x2, e = x3 - x1;
  o[0] = fmaf(4.0f, x0, fmaf(-5.0f, x2, x4));
  o[1] = a + b;
  o[2] = a - b;
  o[3] = fmaf(2.0f, e, c);
  o[4] = fmaf(-2.0f, e, c);
  o[5] = fmaf(4.0f, x1, fmaf(-5.0f, x3, x5));
}

// A^T m for m = 6 points (rows [1,1,1,1,1,0] [0,1,-1,2,-2,0] [0,1,1,4,4,0] [0,1,-1,8,-8,1])
__device__ __forceinline__ void at6(const float *m, float *o) {
  const float a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], e = m[3] - m[4];
  o[0] = m[0] + a + c;
  o[1] = b + 2.0f * e;
  o[2] = a + 4.0f * c;
  o[3] = b + 8.0f * e + m[5];
}

// A^T restricted to its columns 0-2 (H = 0: rows [1,1,1] [0,1,-1] [0,1,1] [0,1,-1]) or 3-5
// (H = 1: [1,1,0] [2,-2,0] [4,4,0] [8,-8,1]) applied to those 3 points: a partial of at6
template <int H>
__device__ __forceinline__ f32x4 at6h(const float u0, const float u1, const float u2) {
  if (H == 0) {
    const float p = u1 + u2, q = u1 - u2;
    return f32x4{u0 + p, q, p, q};
  } else {
    const float p = u0 + u1, q = u0 - u1;
    return f32x4{p, 2.0f * q, 4.0f * p, 8.0f * q + u2};
  }
}

// Tile (within a wave's 16) of MFMA row m.  The patch rows' ds_read_b128 serves four 16-lane
// groups, {0-3, 12-15, 20-27} and {4-11, 16-19, 28-31} (+ 32): channel k = lane / 16 of two
// adjacent channels in one group, their planes 16 (mod 64) dwords apart (PS * 4 for either
// geometry).  With tile = m the two channels' 4-bank slots overlap (2-way); mapping rows 4-11 to
// tiles {0,1,4,5,8,9,12,13} and the others to {2,3,6,7,10,11,14,15} (sets invariant under a
// shift of 4 slots) makes every group hit 16 distinct slots.
__device__ __forceinline__ int w4_tile_of_row(int m) {
  const bool mid = m >= 4 && m < 12;
  const int j = mid ? m - 4 : (m < 4 ? m : m - 8);
  return (mid ? 0 : 2) + 4 * (j >> 1) + (j & 1);
}

// half HF of B^T x: outputs 0-2 (HF = 0) or 3-5 (HF = 1)
template <int HF>
__device__ __forceinline__ void bt6h(const float x0, const float x1, const float x2, const float x3, const float x4,
                                     const float x5, float *o) {
  if (HF == 0) {
    const float a = fmaf(-4.0f, x2, x4), b = fmaf(-4.0f, x1, x3);
    o[0] = fmaf(4.0f, x0, fmaf(-5.0f, x2, x4));
    o[1] = a + b;
    o[2] = a - b;
  } else {
    const float c = x4 - x2, e = x3 - x1;
    o[0] = fmaf(2.0f, e, c);
    o[1] = fmaf(-2.0f, e, c);
    o[2] = fmaf(4.0f, x1, fmaf(-5.0f, x3, x5));
  }
}

// The block's staged outputs, channels [cbase, cbase + NCH) of its CO at ot (plane c - cbase,
// pitch OPP): InstanceNorm partials (if requested), then float4 stores or the GRU gate epilogue.
template <class C, bool GATED, int NCH>
__device__ __forceinline__ void w4_emit(const W4Prob &P, const W4Gate *gate, const float *ot, const int cbase,
                                        const int n, const int co0, const int st, const int tiles_w, const int y0,
                                        const int x0, const int BH, const int BW, const int lbw, const int tid) {
  constexpr int NT = C::NT, NTHR = C::NTHR, OPP = C::OPP;
  const int H = P.H, W = P.W, Cout = P.Cout, pitch = P.pitch, hw = H * pitch;
  const int cb0 = co0 + cbase;   // first output channel of this pass
  // a group of 4 that straddles the last column (pitch > W): its columns >= W stay zero
  auto tail0 = [&](f32x4 v, const int x) __attribute__((always_inline)) {
    if (x + 4 > W) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (x + e >= W) v[e] = 0.0f;
    }
    return v;
  };
  if (P.partial) {
    // InstanceNorm partials, indexed by the small blocks' tiling (BH rows of a large block = 2
    // small tiles), so both block shapes fill the same [N * Cout][parts][2] array: TPC threads
    // per (channel, small tile), each over consecutive pixels of it, fixed-order reduction
    constexpr int NSUB = NT / 32, TPC = NTHR / (NCH * NSUB), PPT = 32 * 16 / TPC;
    const int c = tid / (TPC * NSUB), sub = (tid / TPC) % NSUB, part = tid % TPC;
    const int sub_rows = BH / NSUB, fine_h = (H + sub_rows - 1) / sub_rows;
    const int frow = (st / tiles_w) * NSUB + sub;
    double ssum = 0.0, ssq = 0.0;
#pragma unroll 2
    for (int p = sub * 512 + part * PPT; p < sub * 512 + (part + 1) * PPT; p += 4) {
      const int r = p >> lbw, cx = p & (BW - 1);
      if (y0 + r < H && x0 + cx < W) {   // (the straddling group of a pitched plane: masked)
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
    if (part == 0 && frow < fine_h) {
      const long fst = (long)frow * tiles_w + st % tiles_w;
      double *pp = P.partial + (((long)n * Cout + cb0 + c) * ((long)fine_h * tiles_w) + fst) * 2;
      pp[0] = ssum;
      pp[1] = ssq;
    }
  }
  // float4 stores: NT * 4 per channel plane of the block
  float *dst = P.out + (long)n * P.out_bs;
  constexpr int NJ = (NCH * NT * 16) / (4 * NTHR);
  auto plain_stores = [&]() __attribute__((always_inline)) {
    if (P.skip) {   // residual epilogue: oact(act(conv + bias) + skip_act(skip * s + t))
      const float *sk = P.skip + (long)n * P.skip_bs;
#pragma unroll 4
      for (int j = 0; j < NJ; ++j) {
        const int i4 = tid + NTHR * j;
        const int c = i4 / (NT * 4), p = (i4 % (NT * 4)) * 4, r = p >> lbw, cx = p & (BW - 1);
        const int y = y0 + r, x = x0 + cx;
        if (y < H && x < W) {
          const long off = (long)(cb0 + c) * hw + (long)y * pitch + x;
          const f32x4 sv = *reinterpret_cast<const f32x4 *>(sk + off);
          const float ss = P.skip_s ? P.skip_s[cb0 + c] : 1.0f, st_ = P.skip_t ? P.skip_t[cb0 + c] : 0.0f;
          f32x4 v = *reinterpret_cast<const f32x4 *>(ot + c * OPP + p);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float a = sv[e] * ss + st_;
            if (P.skip_act) a = fmaxf(a, 0.0f);
            v[e] = v[e] + a;
            if (P.out_act) v[e] = fmaxf(v[e], 0.0f);
          }
          *reinterpret_cast<f32x4 *>(dst + off) = tail0(v, x);
        }
      }
      return;
    }
#pragma unroll 4
    for (int j = 0; j < NJ; ++j) {
      const int i4 = tid + NTHR * j;
      const int c = i4 / (NT * 4), p = (i4 % (NT * 4)) * 4, r = p >> lbw, cx = p & (BW - 1);
      const int y = y0 + r, x = x0 + cx;
      if (y < H && x < W)
        *reinterpret_cast<f32x4 *>(dst + (long)(cb0 + c) * hw + (long)y * pitch + x) =
            tail0(*reinterpret_cast<const f32x4 *>(ot + c * OPP + p), x);
    }
  };
  if constexpr (!GATED) {
    plain_stores();
    return;
  } else {
  // GRU gates (update.py:16-27): conv (+ bias, staged) + context, then
  //   mode 1 (z | r over cat(h, x)): z = sigmoid(.) -> out, r * h -> out2 (block-uniform half)
  //   mode 2 (q over r*h):           h' = (1 - z) h + z tanh(. + add) -> out (in place on h)
  // the gate parameters are read here, not at the kernel's start (they would lengthen the
  // prologue before chunk 0's DMA)
  const W4Gate &GT = *gate;
  if (GT.mode == 0) {
    plain_stores();
    return;
  }
  const int half = Cout / 2;
  const bool rhalf = co0 >= half;
  const float *ctxb = GT.ctx + (long)n * GT.ctx_bs;
  // The gate planes are loaded for a batch of store iterations at once (out-of-image
  // positions read the block's first pixel, whose load is always in range, and are not
  // stored), so all of a batch's loads are in flight together instead of a branchy loop
  // waiting for its own loads every iteration (the accumulators are dead here: registers are
  // free).  Batches: 16 iterations in mode 1 (ctx, and h for the r half), 8 in mode 2 (four
  // planes): 128 registers either way.
  const float *hb = GT.h + (long)n * GT.h_bs;
  const float *ab = GT.add + (long)n * GT.add_bs;
  const float *zb = GT.z + (long)n * GT.z_bs;
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
        const int c = i4 / (NT * 4), p = (i4 % (NT * 4)) * 4, r = p >> lbw, cx = p & (BW - 1);
        const int y = y0 + r, x = x0 + cx;
        ok[u] = y < H && x < W;
        pos[u] = (cb0 + c) * hw + (ok[u] ? y * pitch + x : y0 * pitch + x0);
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
        const int c = i4 / (NT * 4), p = (i4 % (NT * 4)) * 4;
        const int xg = x0 + (p & (BW - 1));
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
  if (GT.mode == 1) gate_stores(std::integral_constant<int, SA_W4_GJB1>{}, std::integral_constant<int, 1>{});
  else gate_stores(std::integral_constant<int, SA_W4_GJB>{}, std::integral_constant<int, 2>{});
  }
}


// Mode 3, the flow head (update.py:98-110): the block's staged outputs are relu(conv1(h08) + b1)
// of its 32 channels over its BH x BW pixels (ot, [channel][row][col], pitch OPP); conv2's
// output channel 0 (the only one the model reads, stereoanywhere.py:283) gets from them a partial
// 3x3 sum over the tile plus its one-pixel border, written to head_part as [N][channel block]
// [tile][BH + 2][BW + 2]; sa_flow_head_reduce adds the channel blocks and the overlapping borders.
// f1 (the 256-channel conv1 output) is never written.  Thread item: one interior border-region
// column c (1..BW) of one channel group (NQ groups: NQ * BW = 512 items), all BH + 2 region rows;
// the two outer columns (c = 0, BW + 1, one tap column each) are a second, short pass.
template <class C, int LTW>
__device__ __forceinline__ void w4_flowhead(const W4Prob &P, const W4Gate &GT, float *smem, const int n, const int co0,
                                            const int st, const int y0, const int x0, const int tid,
                                            const float wpre) {
  constexpr int BW = 4 << LTW, BH = 4 * (C::NT >> LTW), RH = BH + 2, RW = BW + 2, CO = C::CO, OPP = C::OPP;
  constexpr int NQ = C::NTHR / BW, CPQ = CO / NQ;
  static_assert(NQ * BW == C::NTHR && CPQ * NQ == CO, "flow head item mapping");
  static_assert(NQ * RH * RW <= CO * OPP, "partial staging in the output planes");
  static_assert(CO * OPP + CO * 9 <= C::SMEM, "head weights after the output planes");
  const float *ot = smem;
  float *wl = smem + CO * OPP;   // conv2's taps of this block's channels [ch][9]
  if (tid < CO * 9) wl[tid] = wpre;
  __syncthreads();
  const int H = P.H, W = P.W;
  auto item = [&](const int q, const int c, const int dx0, const int dx1, float *acc) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < RH; ++r) acc[r] = 0.0f;
    for (int ch = q * CPQ; ch < (q + 1) * CPQ; ++ch) {
      const float *plane = ot + ch * OPP;
#pragma unroll
      for (int dx = dx0; dx <= dx1; ++dx) {
        const int fc = c + dx - 2;   // f1 column of tap dx for region column c (tile-relative)
        if (fc < 0 || fc >= BW || x0 + fc >= W) continue;
        float col[BH];
#pragma unroll
        for (int r = 0; r < BH; ++r) col[r] = y0 + r < H ? plane[r * BW + fc] : 0.0f;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const float w = wl[ch * 9 + dy * 3 + dx];
#pragma unroll
          for (int r = 0; r < BH; ++r) acc[r - dy + 2] = fmaf(w, col[r], acc[r - dy + 2]);
        }
      }
    }
  };
  float acc[RH];
  const int q = tid / BW, c = 1 + tid % BW;
  item(q, c, 0, 2, acc);
  float acc2[RH];
  const bool edge = tid < 2 * NQ;   // outer columns: c = 0 (tap dx = 2) or BW + 1 (dx = 0)
  const int eq = tid >> 1, ec = (tid & 1) ? RW - 1 : 0;
  if (edge) item(eq, ec, (tid & 1) ? 0 : 2, (tid & 1) ? 0 : 2, acc2);
  __syncthreads();   // every item's reads of the output planes are done: reuse them
  float *red = smem;   // [NQ][RH][RW]
#pragma unroll
  for (int r = 0; r < RH; ++r) red[(q * RH + r) * RW + c] = acc[r];
  if (edge) {
#pragma unroll
    for (int r = 0; r < RH; ++r) red[(eq * RH + r) * RW + ec] = acc2[r];
  }
  __syncthreads();
  float *dst = GT.head_part + (long)n * GT.head_part_bs + ((long)(co0 / CO) * P.tiles_hw + st) * (RH * RW);
  for (int i = tid; i < RH * RW; i += C::NTHR) {
    float v = red[i];
#pragma unroll
    for (int g = 1; g < NQ; ++g) v += red[g * RH * RW + i];
    dst[i] = v;
  }
}

#ifdef SA_W4_CLOCK
// diagnostic build only: per block (s_memtime, s_memrealtime) at the start and the end of wave 0,
// then s_memtime after the first chunk's barrier and after the main loop
__device__ unsigned long long g_w4_clock[65536][12];   // + [8] chunk 0 issued, [9] last wave's start,
                                                      // [10] work item decoded, [11] chunk 0's filter DMA issued
#endif

// One work item: the block's 64 tiles x 32 output channels (HF: this wave's point-column half).
// Returns true (block-uniform) when the split kernel's range guard found an overflow: nothing was
// written, and the caller runs the item again with xscale = 0: the body then scans the block's input
// patch (every chunk, from global memory; after the producer's transform), takes the power of two
// xscale that brings 100 max|d| >= max|V| below 2^15, multiplies the staged patch by it (the same
// in-LDS pass as the input transform) and the accumulators by 1 / xscale: the same split products
// on exactly scaled operands.  (A second, fp32 instantiation of the body in the same kernel made the
// register allocator spill the gated split kernel: wino4 49.8 -> 79.0 ms/step.)
template <class C, int HF, int LTW, bool GATED, bool AFF>
__device__ __forceinline__ bool w4_body(const W4Prob &P, const W4Gate *gate, const unsigned wid, float *smem,
                                        float2 *atab, const bool guard = false, float xscale = 1.0f) {
  constexpr int NWAVE = C::NW, NTHR = C::NTHR, KC = C::KC, JPC = C::JPC, NT = C::NT, PDMA = C::PDMA,
                UDMA = C::UDMA, UPW = C::UPW, UBUF = C::UBUF, BUF = C::BUF, PBUF = C::PBUF, OPP = C::OPP,
                CO = C::CO, CG = C::CG, SB = C::SB, NR = C::NR;
  constexpr bool SPLIT = C::SPLIT;
  static_assert(!SPLIT || NWAVE == 8, "split: the 8-wave shape");
  // a lane's filter operands of a point: one float, or (split) one f16 (hi, lo) pair, per group
  using f32xg = float __attribute__((ext_vector_type(CG)));
  const int Cin = P.Cin, H = P.H;
  // block geometry as compile-time constants (the patch offsets divide by PS and PG)
  constexpr int ltw = LTW, tw = 1 << ltw, tr = NT >> ltw;
  constexpr int BH = 4 * tr, BW = 4 * tw, PG = tw + 2, PR = BH + 2, PS = PR * PG;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co_blocks = P.co_blocks, tiles_hw = P.tiles_hw, tiles_w = P.tiles_w;
  int cb, st, n;
  w4_item(wid, co_blocks, tiles_hw, cb, st, n);
  const int y0 = (st / tiles_w) * BH, x0 = (st % tiles_w) * BW;
  const int co0 = cb * CO;
  const int pitch = P.pitch, hw = H * pitch;
  const int nchunks = Cin / KC;

  const __amdgpu_buffer_rsrc_t xin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(P.in + (long)n * P.in_bs), (short)0, Cin * hw * 4, 0x00020000);
  // the filters' global layout has 8-channel chunks (sa_conv2d_wino4_weights); a 4-channel
  // chunk is every other SB-float piece of one (the DMA gathers it by its source addresses)
  const __amdgpu_buffer_rsrc_t uin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(P.U + (long)cb * Cin * NPT * CO), (short)0, Cin * NPT * CO * 4, 0x00020000);
  auto u_src = [&](int piece) {   // byte offset of this lane's 16 bytes of filter DMA piece `piece`
    const int f = piece * 256 + lane * 4;
    return (JPC == 2 ? f : f + (f / SB) * SB) * 4;
  };
  auto u_chunk = [&](int chunk) {   // byte offset of a chunk's filters
    return JPC == 2 ? chunk * UBUF * 4 : (chunk >> 1) * 2 * UBUF * 4 + (chunk & 1) * SB * 4;
  };

  // patch DMA: the chunk's image is [channel][PR rows][PG groups of 4 floats], dense, starting
  // at (y0 - 1, x0 - 4); wave-instruction gi fills groups 64 gi .. 64 gi + 63 (lane-linear)
  // chunk 0's filters first: their offsets need no patch geometry
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][10] = __builtin_amdgcn_s_memtime();
#endif
  if (SA_W4_DIAG != 4) {
#pragma unroll
    for (int j = 0; j < UPW; ++j)
      if (wv + NWAVE * j < UDMA)
        dma16(uin, smem + PBUF + (wv + NWAVE * j) * 256, u_src(wv + NWAVE * j), u_chunk(0));
  }
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][11] = __builtin_amdgcn_s_memtime();
#endif
  const int npi = (KC * PS + 63) >> 6;
  int po[PDMA];
  // input transform: per piece j, 4 bits at 4j = the group's channel in the chunk + 1 (0: padding
  // or an idle lane), one register for all pieces
  unsigned pcs = 0;
  static_assert(PDMA <= 8 && KC < 15, "4-bit channel fields");
#pragma unroll
  for (int j = 0; j < PDMA; ++j) {
    const int s = (wv + NWAVE * j) * 64 + lane;
    const int ci = s / PS, rem = s - ci * PS, r = rem / PG, g = rem - r * PG;
    const int y = y0 - 1 + r, x = x0 - 4 + 4 * g;
    // (a pitched plane's columns W .. pitch - 1 are zero: they load as the right padding)
    const bool ok = s < KC * PS && y >= 0 && y < H && x >= 0 && x < pitch;
    po[j] = ok ? (ci * hw + y * pitch + x) * 4 : 0x7ffffff0;   // out of range: the load returns 0
    pcs |= (ok && wv + NWAVE * j < (KC * PS + 63) / 64 ? (unsigned)ci + 1u : 0u) << (4 * j);
  }
  if constexpr (C::SPLIT) {
    if (xscale == 0.0f) {   // the range guard's second pass: the scale from the block's largest input
      float *red = smem;   // (patch buffer 0: only chunk 0's filters are in flight, into the filter area)
      const char *ib = reinterpret_cast<const char *>(P.in + (long)n * P.in_bs);
      float mx = 0.0f;
      // (8 chunks per iteration: their loads in flight together; one at a time the scan cost
      // a round trip per chunk, ~30% of the fp32 pass it precedes)
#pragma unroll 8
      for (int kc = 0; kc < nchunks; ++kc)
#pragma unroll
        for (int j = 0; j < PDMA; ++j) {
          const int pcj = (int)((pcs >> (4 * j)) & 15u) - 1;
          if (pcj < 0) continue;
          const f32x4 v = *reinterpret_cast<const f32x4 *>(ib + po[j] + (long)kc * KC * hw * 4);
          float a = 1.0f, b = 0.0f, fl = -INFINITY;
          if constexpr (AFF) {
            const int pi = n * P.in_pstride + kc * KC + pcj;
            const float m0 = P.in_m ? P.in_m[pi] : 0.0f, t0 = P.in_t ? P.in_t[pi] : 0.0f;
            a = P.in_s ? P.in_s[pi] : 1.0f;
            b = t0 - m0 * a;
            fl = P.in_act ? 0.0f : -INFINITY;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t = __builtin_fabsf(fmaxf(v[e] * a + b, fl));
            mx = fmaxf(mx, t < INFINITY ? t : 0.0f);
          }
        }
      mx = sa::wave_max_dpp(mx);
      if (lane == 0) red[wv] = mx;
      __syncthreads();
      mx = red[0];
#pragma unroll
      for (int w = 1; w < NWAVE; ++w) mx = fmaxf(mx, red[w]);
      __syncthreads();   // (before chunk 0's patch DMA lands there)
      int e2;
      (void)frexpf(100.0f * mx, &e2);   // 100 max|d| < 2^e2
      xscale = mx > 0.0f ? ldexpf(1.0f, 15 - e2) : 1.0f;
    }
  }
  const bool scaled = xscale != 1.0f;
  // the chunk's DMAs in three parts (part -1: all at once), spread over the first job's three
  // column phases (each piece costs tens of issue cycles; clustered after the barrier they
  // would delay the first reads)
  auto issue_part = [&](int chunk, int buf, int part) __attribute__((always_inline)) {
    float *pb = smem + buf * BUF;
    const int xs = chunk * KC * hw * 4;
    float *ub = pb + PBUF;
    const int us = u_chunk(chunk);
#pragma unroll
    for (int j = 0; j < PDMA; ++j)
      if ((part < 0 || j / C::PPART == part) && wv + NWAVE * j < npi) dma16(xin, pb + (wv + NWAVE * j) * 256, po[j], xs);
#pragma unroll
    for (int j = 0; j < UPW; ++j)
      if ((part < 0 || j / C::PPART == part) && wv + NWAVE * j < UDMA)
        dma16(uin, ub + (wv + NWAVE * j) * 256, u_src(wv + NWAVE * j), us);
  };
  auto issue = [&](int chunk, int buf) __attribute__((always_inline)) { issue_part(chunk, buf, -1); };
  auto issue_p0 = [&]() __attribute__((always_inline)) {   // chunk 0's patch (its filters went first)
#pragma unroll
    for (int j = 0; j < PDMA; ++j)
      if (wv + NWAVE * j < npi) dma16(xin, smem + (wv + NWAVE * j) * 256, po[j], 0);
  };

  // lane roles: MFMA A operand A[m][k] = (tile m, channel k); B operands B[k][n] = (channel k,
  // output channel n of each 16-channel half)
  const int tg = wv % C::TG;
  const int k = lane >> 4, m = lane & 15;
  const int tidx = tg * 16 + w4_tile_of_row(m), trow = tidx >> ltw, tcol = tidx & (tw - 1);
  // patch row 0 of the tile (input row y0 + 4 trow - 1), columns 4 tcol + 2 .. 4 tcol + 9
  // (input x0 + 4 tcol - 2 ...): the tile's 6 inputs are columns 3..8 of that span
  // the main loop addresses the patch with run-time PS / PG (as before the geometry became a
  // template argument: with immediate offsets its schedule measured ~1% slower)
  int PSv = PS, PGv = PG;
  asm volatile("" : "+s"(PSv), "+s"(PGv));
  const int pread = k * PSv * 4 + 4 * trow * PGv * 4 + 4 * tcol + 2;
  const int uread = (k * 16 + m) * CG * (SPLIT ? JPC : 1);   // (split: [k][n][g][job], wino4s_weights_kernel)

  // acc[i][jj][g]: point (row i, column 3 HF + jj) of output-channel group g
  f32x4 acc[NR][3][CG];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
#pragma unroll
      for (int g = 0; g < CG; ++g) acc[i][jj][g] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the bias of the channel groups this lane finishes in the epilogue, loaded now (a load
  // there would wait a global round trip between the two LDS phases)
  float bpre[CG / 2];
#pragma unroll
  for (int k = 0; k < CG / 2; ++k) bpre[k] = P.bias ? P.bias[co0 + (2 * k + HF) * 16 + (lane & 15)] : 0.0f;
  // static priority for waves 4-7 (split kernel forward: 66.8 -> 66.5 ms/step, two interleaved passes)
  if (HF == 1) __builtin_amdgcn_s_setprio(1);
  // (issuing each piece as soon as its offset is known, ~1.6k cycles earlier, did not land chunk 0
  // any sooner: 6.6k vs 6.2k cycles at xc08, forward 59.6 vs 59.8 ms/step, scripts/w4_clock.py)
  if (SA_W4_DIAG != 4) issue_p0();
  // Input transform: v -> act(v * scale + shift), scale = s, shift = t - m * s per channel
  // (in_pstride 0) or per (image, channel) (in_pstride = Cin).  Each lane transforms the
  // 4-float groups its own DMAs brought in (in the LDS, after its own vmcnt wait, before the
  // chunk's barrier); padding groups stay zero, as in the reference (padding of the activated
  // input).  One read-modify-write per staged float, against the standalone pass's HBM round
  // trip of the whole input.
  const float act_floor = P.in_act ? 0.0f : -INFINITY;
  if constexpr (AFF) {
    for (int c = tid; c < Cin; c += NTHR) {
      const int pi = n * P.in_pstride + c;
      const float m0 = P.in_m ? P.in_m[pi] : 0.0f, sc = P.in_s ? P.in_s[pi] : 1.0f, t0 = P.in_t ? P.in_t[pi] : 0.0f;
      atab[c] = make_float2(sc * xscale, (t0 - m0 * sc) * xscale);   // (ReLU commutes with a scale > 0)
    }
    __syncthreads();
  }
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][8] = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = kc & 1;
    if constexpr (AFF) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this lane's DMAs of chunk kc landed
      float *pbuf = smem + cur * BUF;
#pragma unroll
      for (int j = 0; j < PDMA; ++j) {
        const int pcj = (int)((pcs >> (4 * j)) & 15u) - 1;
        if (pcj >= 0) {
          f32x4 *q = reinterpret_cast<f32x4 *>(pbuf + ((wv + NWAVE * j) * 64 + lane) * 4);
          const float2 ab = atab[kc * KC + pcj];
          f32x4 v = *q;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * ab.x + ab.y, act_floor);
          *q = v;
        }
      }
    }
    if constexpr (SPLIT && !AFF) {
      if (scaled) {   // the range guard's second pass: this lane's staged groups times xscale
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float *pbuf = smem + cur * BUF + (wv * 64 + lane) * 4;
        // (one group at a time: the accumulators are live here)
#pragma unroll 1
        for (int j = 0; j < PDMA; ++j) {
          if (wv + NWAVE * j < npi) {
            f32x4 *q = reinterpret_cast<f32x4 *>(pbuf + NWAVE * j * 256);
            *q = *q * xscale;
          }
        }
      }
    }
    if (SA_W4_DIAG == 9 && !AFF && !scaled) {
      // timing only: wait for chunk kc - 1's DMAs, not chunk kc's (every wave issues >= 9 pieces
      // per chunk), i.e. the floor of a ring that issues each chunk two chunks ahead
      if (kc == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else if (SA_W4_DIAG < 3 || AFF || scaled) {
      __syncthreads();   // chunk kc landed (vmcnt(0) precedes the barrier); buffer cur ^ 1 is free
    }
#ifdef SA_W4_CLOCK
    if (kc == 0 && HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][4] = __builtin_amdgcn_s_memtime();
#endif
    if (SA_W4_DIAG == 2 && kc + 1 < nchunks) issue(kc + 1, cur ^ 1);
    if (SA_W4_DIAG == 2) continue;
    const float *pb = smem + cur * BUF + pread;
    const float *ub = smem + cur * BUF + PBUF + uread;
    // Per job s (channel k, then k + 4) the lane reads its tile's 6 patch rows (8 floats each;
    // the inputs are a.y, b.xyzw, c.x), runs its half of the row pass t[r][jj] =
    // (B^T d_r)[3 HF + jj], then 3 column passes V[i][3 HF + jj] = (B^T t)[i][jj] that feed
    // 6 x 2 MFMAs each.  Software pipeline (the scheduler is fenced per column to bound its
    // register use): the filter operands of the next column and rows 0-2 of the next job are
    // read under the current column's MFMAs.
    // (ds_read_b32 + b128 + b32 of just the 6 inputs measured 4-7% slower)
    f32x2 ra[6], rc[6];
    f32x4 rb[6];
    auto load_rows = [&](int s, int r0, int r1) __attribute__((always_inline)) {
      const float *p = pb + s * 4 * PSv * 4;
#pragma unroll
      for (int r = r0; r < r1; ++r) {
        ra[r] = *reinterpret_cast<const f32x2 *>(p + r * PGv * 4);
        rb[r] = *reinterpret_cast<const f32x4 *>(p + r * PGv * 4 + 2);
        rc[r] = *reinterpret_cast<const f32x2 *>(p + r * PGv * 4 + 6);
      }
    };
    f32xg bc[NR], bn[NR];
    auto load_b = [&](int s, int jj, f32xg *b) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        if constexpr (SPLIT) {   // (the job's dwords of both groups: one ds_read2_b32)
          const float *q = ub + (6 * i + 3 * HF + jj) * JPC * SB + s;
          b[i] = f32xg{q[0], q[JPC]};
        } else {
          b[i] = *reinterpret_cast<const f32xg *>(ub + ((6 * i + 3 * HF + jj) * JPC + s) * SB);
        }
      }
    };
    if constexpr (SPLIT && SA_W4_PAIR != 0 && JPC == 2 && (!AFF || SA_W4_PAIR_AFF)) {
      // both jobs' row passes first, then per column both jobs' column passes feed one MFMA pair per
      // (row, output-channel group) (w4_pair_split); a column's filter operands are read under its
      // two column passes
      float t0[6][3], t1[6][3];
      load_rows(0, 0, 6);
#pragma unroll
      for (int r = 0; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t0[r]);
      load_rows(1, 0, 6);
#pragma unroll
      for (int r = 0; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t1[r]);
      f32x4 pc_[NR];   // (group 0: job 0, job 1; group 1: job 0, job 1)
      auto load_bp = [&](int jj, int i0, int i1, f32x4 (&b)[NR]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = i0; i < i1; ++i) b[i] = *reinterpret_cast<const f32x4 *>(ub + (6 * i + 3 * HF + jj) * JPC * SB);
      };
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        if ((SA_W4_DIAG == 0 || SA_W4_DIAG == 9) && kc + 1 < nchunks) {
          issue_part(kc + 1, cur ^ 1, jj);
          __builtin_amdgcn_sched_barrier(0);
        }
        load_bp(jj, 0, NR / 2, pc_);   // (rows 0-2 under the column passes, 3-5 under rows 0-2's MFMAs:
                                       // a whole column at once, or the next column's, spills)
        float v0[6], v1[6];
        bt6(t0[0][jj], t0[1][jj], t0[2][jj], t0[3][jj], t0[4][jj], t0[5][jj], v0);
        bt6(t1[0][jj], t1[1][jj], t1[2][jj], t1[3][jj], t1[4][jj], t1[5][jj], v1);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          if (i == 1) load_bp(jj, NR / 2, NR, pc_);
          f16x4 ahi, alo;
          w4_pair_split(v0[i], v1[i], ahi, alo);
#pragma unroll
          for (int g = 0; g < CG; ++g) {
            const f16x4 bp = __builtin_bit_cast(f16x4, g == 0 ? pc_[i].xy : pc_[i].zw);
            acc[i][jj][g] = __builtin_amdgcn_mfma_f32_16x16x16f16(ahi, bp, acc[i][jj][g], 0, 0, 0);
            acc[i][jj][g] = __builtin_amdgcn_mfma_f32_16x16x16f16(alo, bp, acc[i][jj][g], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // bound the scheduler's hoisting (register pressure)
      }
      continue;
    }
    load_rows(0, 0, 6);
    load_b(0, 0, bc);
#pragma unroll
    for (int s = 0; s < JPC; ++s) {
      if (s == 1) load_rows(1, 3, 6);
      float t[6][3];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        if (SA_W4_DIAG == 6 || SA_W4_DIAG == 8) {   // timing only: no row pass
          t[r][0] = ra[r].y; t[r][1] = rb[r].x; t[r][2] = rc[r].x;
        } else {
          bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t[r]);
        }
      }
      if (s + 1 < JPC) load_rows(1, 0, 3);
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        // the next chunk's DMA part jj goes out before column jj's pass of the first job (the
        // chunk time is bound by the DMA's latency: one column earlier than after its MFMAs,
        // wino4 51.0 -> 50.1 ms/step; all parts at once delay the row reads)
        if ((SA_W4_DIAG == 0 || SA_W4_DIAG == 9) && s == 0 && kc + 1 < nchunks) {
          issue_part(kc + 1, cur ^ 1, jj);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (SA_W4_DIAG != 7 && (s + 1 < JPC || jj < 2)) load_b(jj < 2 ? s : s + 1, jj < 2 ? jj + 1 : 0, bn);
        float v[6];
        if (SA_W4_DIAG == 5 || SA_W4_DIAG == 8) {   // timing only: no column pass
#pragma unroll
          for (int i = 0; i < NR; ++i) v[i] = t[i][jj];
        } else {
          bt6(t[0][jj], t[1][jj], t[2][jj], t[3][jj], t[4][jj], t[5][jj], v);
        }
        if constexpr (SPLIT) {
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            const f16x4 a = w4_split(v[i]);
            const f16x4 b0 = __builtin_bit_cast(f16x4, f32x2{bc[i][0], bc[i][0]});
            const f16x4 b1 = __builtin_bit_cast(f16x4, f32x2{bc[i][1], bc[i][1]});
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b0, acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b1, acc[i][jj][1], 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NR; ++i)
#pragma unroll
            for (int g = 0; g < CG; ++g)
              acc[i][jj][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[i], bc[i][g],
                                                                    acc[i][jj][g], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // bound the scheduler's hoisting (register pressure)

#pragma unroll
        for (int i = 0; i < NR; ++i) bc[i] = bn[i];
      }
    }
  }
  __syncthreads();
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][5] = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (SPLIT) {   // the filters' 2^W4S_LOG2 and the inputs' xscale (exact)
    const float inv_scale = 1.0f / ((float)(1 << W4S_LOG2) * xscale);
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
#pragma unroll
        for (int g = 0; g < CG; ++g) acc[i][jj][g] *= inv_scale;
  }

  // ---- output transform.  Lane holds tiles tg * 16 + 4 (lane >> 4) + i of output channels
  // g * 16 + (lane & 15), points of columns 3 HF .. 3 HF + 2.  Y = A^T M A: the column-wise
  // A^T runs per column, the row-wise A^T only over this half's columns (a partial sum).  The
  // halves meet in LDS, O[co][row][x] (one float4 per output row of a tile), balanced: half HF
  // finishes the channel groups g with g % 2 == HF: in phase 0 each half stages its partials of
  // the OTHER half's groups; in phase 1 it adds its own partials, the bias and the ReLU.  Plane pitch OPP =
  // 4 (mod 32) floats: the 8 lanes of a ds_write_b128 group (8 output channels) hit disjoint
  // banks.
  float *ot = smem;
  const int relu = P.relu;
  f32x4 chk = f32x4{0.f, 0.f, 0.f, 0.f};   // the split kernel's range guard (below)
  // the flow head's conv2 taps (mode 3), loaded under the output transform
  float whead = 0.0f;
  if constexpr (GATED && C::NTHR == 512)
    if (gate->mode == 3 && tid < C::CO * 9) whead = gate->head_w[co0 * 9 + tid];
#pragma unroll
  for (int phase = 0; phase < 2; ++phase) {
#pragma unroll
  for (int gi = 0; gi < CG / 2; ++gi) {
    const int g = 2 * gi + (phase == 0 ? 1 - HF : HF);
    const int col = g * 16 + (lane & 15);
    const float bv = phase == 1 ? bpre[gi] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ti = tg * 16 + w4_tile_of_row(4 * (lane >> 4) + i), orow = (ti >> ltw) * 4, ocol = (ti & (tw - 1)) * 4;
      float u[4][3];
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        float mcol[6], o[4];
#pragma unroll
        for (int a = 0; a < 6; ++a) mcol[a] = acc[a][jj][g][i];
        at6(mcol, o);
#pragma unroll
        for (int a = 0; a < 4; ++a) u[a][jj] = o[a];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        // A^T rows restricted to columns 0-2: [1,1,1] [0,1,-1] [0,1,1] [0,1,-1];
        // columns 3-5: [1,1,0] [2,-2,0] [4,4,0] [8,-8,1]
        f32x4 y;
        if (HF == 0) {
          const float p = u[a][1] + u[a][2], q = u[a][1] - u[a][2];
          y = f32x4{u[a][0] + p, q, p, q};
        } else {
          const float p = u[a][0] + u[a][1], q = u[a][0] - u[a][1];
          y = f32x4{p, 2.0f * q, 4.0f * p, 8.0f * q + u[a][2]};
        }
        f32x4 *o = reinterpret_cast<f32x4 *>(ot + col * OPP + (orow + a) * BW + ocol);
        if (phase == 0) {
          *o = y;
        } else {
          // half 1's partial + half 0's: (p1 + p0) + bias for either finishing half
          f32x4 v = (HF == 0 ? (*o + y) : (y + *o)) + bv;
          if constexpr (SPLIT) chk += v;   // (the range guard, before the ReLU that would mask a NaN)
          if (relu) v = f32x4{fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f)};
          *o = v;
        }
      }
    }
  }
    if (phase == 0) __syncthreads();
  }
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][6] = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (SPLIT) {
    // Range guard: an f16 operand overflow (|V| >= 65520: hi = inf, lo = -inf) makes every product
    // of that value NaN, and so the staged outputs it feeds (checked before the ReLU).  Such a
    // block writes nothing (its epilogue may update h in place) and runs its item again right away
    // on exactly scaled inputs (wino_f4k3_kernel, w4_body's xscale): no list, no second launch,
    // every overflowed block in parallel.  Genuine NaN inputs take the same path and give NaN.
    // One int per wave past the output planes and the flow head's taps (nothing else uses that
    // LDS after the main loop).
    static_assert(C::CO * C::OPP + C::CO * 9 + NWAVE <= C::SMEM, "range guard flags");
    int *flags = reinterpret_cast<int *>(smem + C::CO * C::OPP + C::CO * 9);
    const float t = (chk.x + chk.y) + (chk.z + chk.w);
    const bool wbad = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(t)) != 0;
    if (lane == 0) flags[wv] = wbad ? 1 : 0;
    __syncthreads();
    int any = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) any |= flags[w];
    if (any && guard) return true;
  } else {
    __syncthreads();
  }
  if constexpr (GATED && C::NTHR == 512) {
    if (gate->mode == 3) {
      w4_flowhead<C, LTW>(P, *gate, smem, n, co0, st, y0, x0, tid, whead);
      return false;
    }
  }
  w4_emit<C, GATED, C::CO>(P, gate, ot, 0, n, co0, st, tiles_w, y0, x0, BH, BW, ltw + 2, tid);
  return false;
}

#ifndef SA_W4_REDO
#define SA_W4_REDO 1
#endif
template <class C, bool GATED, bool AFF = false>
__global__ __launch_bounds__(C::NTHR, C::NW == 8 ? 1 : 2) void wino_f4k3_kernel(const W4Launch L) {
  // problem of the block from its raw id (ranges padded to multiples of 8: every XCD gets an
  // equal share of each problem), then the L2-locality remap within it (conv2d_wino.hip)
  const unsigned g = blockIdx.x;
  // the problem index from the range ends alone, then only that problem's fields are loaded
  // (selecting among all eight by value loaded every one of them: ~70 scalar loads before the
  // first DMA)
  int pi = 0;
#pragma unroll
  for (int i = 1; i < MAX_PROB; ++i) pi += (i < L.nprob && g >= L.end[i - 1]) ? 1 : 0;
  const unsigned base = pi ? L.end[pi - 1] : 0u, nb = L.nblk[pi];
  if (g - base >= nb) return;
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  __shared__ float2 atab[AFF ? C::AFF_MAX : 1];
#ifdef SA_W4_CLOCK
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == C::NTHR - 64 && blockIdx.x < 65536) g_w4_clock[blockIdx.x][9] = t0;
#endif
  // the first half of the waves takes point columns 0-2, the second half 3-5 (wave-uniform)
  const unsigned wid = sa::xcd_remap(g - base, nb);
  const bool guard = C::SPLIT && L.guard;
  // the range guard: an overflowed block (block-uniform) runs its item again on scaled inputs
  const W4Prob &P = L.p[pi];
  const W4Gate *gp = GATED ? &L.gate[pi] : nullptr;
  bool over;
#define SA_W4_B(CC_, HF_, LTW_, G_, XS_) w4_body<CC_, HF_, LTW_, GATED, AFF>(P, gp, wid, smem, atab, G_, XS_)
  if (threadIdx.x < C::NTHR / 2) over = P.ltw == 4 ? SA_W4_B(C, 0, 4, guard, 1.0f) : SA_W4_B(C, 0, 5, guard, 1.0f);
  else over = P.ltw == 4 ? SA_W4_B(C, 1, 4, guard, 1.0f) : SA_W4_B(C, 1, 5, guard, 1.0f);
  if constexpr (C::SPLIT && SA_W4_REDO) {
    if (over) {
      __syncthreads();   // the first pass's LDS reads are over
      if (threadIdx.x == 0) atomicAdd(&g_w4_redo_blocks, 1u);
      // the second pass's arguments through opaque copies: nothing of it is hoisted (CSE'd) into
      // the first pass, whose registers stay its own
      int pil = __builtin_amdgcn_readfirstlane(pi);
      unsigned widl = __builtin_amdgcn_readfirstlane(wid);
      asm volatile("" : "+s"(pil), "+s"(widl));
      const W4Prob &P2 = L.p[pil];
      const W4Gate *gp2 = GATED ? &L.gate[pil] : nullptr;
#define SA_W4_B2(HF_, LTW_) w4_body<C, HF_, LTW_, GATED, AFF>(P2, gp2, widl, smem, atab, false, 0.0f)
      if (threadIdx.x < C::NTHR / 2) {
        if (P2.ltw == 4) SA_W4_B2(0, 4);
        else SA_W4_B2(0, 5);
      } else {
        if (P2.ltw == 4) SA_W4_B2(1, 4);
        else SA_W4_B2(1, 5);
      }
#undef SA_W4_B2
    }
  }
#undef SA_W4_B
#ifdef SA_W4_CLOCK
  if (threadIdx.x == 0 && g < 65536) {
    g_w4_clock[g][0] = t0;
    g_w4_clock[g][1] = r0;
    g_w4_clock[g][2] = __builtin_amdgcn_s_memtime();
    g_w4_clock[g][3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// U = G g G^T for g = w[co][ci] (3x3), fp64, rounded once.  Layout
// [Cout/32][Cin/8][36][2][4][16][2]: per (output block, chunk) one contiguous 36 KiB image of
// the LDS filter buffer; channel ci = 8 chunk + 4 s + k, output co = 32 cb + 16 h + n at
// [n][h].
__global__ __launch_bounds__(256) void wino4_weights_kernel(const float *__restrict__ w, int Cout, int Cin, int CB,
                                                            float *__restrict__ U) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin) return;
  const int co = (int)(i / Cin), ci = (int)(i % Cin);
  const float *g = w + i * 9;
  const double G[6][3] = {{0.25, 0.0, 0.0},
                          {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                          {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                          {1.0 / 24, 1.0 / 12, 1.0 / 6},
                          {1.0 / 24, -1.0 / 12, 1.0 / 6},
                          {0.0, 0.0, 1.0}};
  double t[6][3];
  for (int a = 0; a < 6; ++a)
    for (int c = 0; c < 3; ++c) t[a][c] = G[a][0] * g[c] + G[a][1] * g[3 + c] + G[a][2] * g[6 + c];
  const int chunk = ci / 8, s = (ci % 8) / 4, k = ci % 4, cb = co / CB, c = co % CB, ng = CB / 16;
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) {
      const double u = t[a][0] * G[b][0] + t[a][1] * G[b][1] + t[a][2] * G[b][2];
      const int pt = 6 * a + b;
      U[(((((long)cb * (Cin / 8) + chunk) * NPT + pt) * 2 + s) * 4 + k) * CB + (c & 15) * ng + (c >> 4)] = (float)u;
    }
}

// Filters of the split kernel (W4Split): U = G g G^T in fp64, times 2^W4S_LOG2, as the f16
// pair hi = f16(u), lo = f16(u - hi) in one dword (hi in the low half); per (32-channel block,
// 8-channel chunk, point) [k][n][g][job]: a lane's four operands of a point (both groups, both
// jobs' channels k and k + 4) are one 16-byte LDS read, the MFMA pairs' B operands as they stand.
__global__ __launch_bounds__(256) void wino4s_weights_kernel(const float *__restrict__ w, int Cout, int Cin,
                                                             unsigned *__restrict__ U) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin) return;
  const int co = (int)(i / Cin), ci = (int)(i % Cin);
  const float *g = w + i * 9;
  const double G[6][3] = {{0.25, 0.0, 0.0},
                          {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                          {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                          {1.0 / 24, 1.0 / 12, 1.0 / 6},
                          {1.0 / 24, -1.0 / 12, 1.0 / 6},
                          {0.0, 0.0, 1.0}};
  double t[6][3];
  for (int a = 0; a < 6; ++a)
    for (int c = 0; c < 3; ++c) t[a][c] = G[a][0] * g[c] + G[a][1] * g[3 + c] + G[a][2] * g[6 + c];
  const int chunk = ci / 8, s = (ci % 8) / 4, k = ci % 4, cb = co / 32, gg = (co % 32) / 16, n = co % 16;
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) {
      const double u = (t[a][0] * G[b][0] + t[a][1] * G[b][1] + t[a][2] * G[b][2]) * (double)(1 << W4S_LOG2);
      const _Float16 hi = (_Float16)(float)u;
      const _Float16 lo = (_Float16)(float)(u - (double)hi);
      const unsigned pr = (unsigned)__builtin_bit_cast(unsigned short, hi) |
                          ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
      const int pt = 6 * a + b;
      U[((((((long)cb * (Cin / 8) + chunk) * NPT + pt) * 4 + k) * 16 + n) * 2 + gg) * 2 + s] = pr;
    }
}

// geometry with the fewest padded output pixels (ties: 16 x 64, the smaller halo)

// sa_flow_head_reduce: per pixel, conv2's channel 0 = bias0 + the partial sums of every channel block
// from the (up to four) tiles whose bordered region holds the pixel, in a fixed order (channel
// block, then tile row, then tile column); then the coordinates / flow update of sa_flow_update.
__global__ __launch_bounds__(256) void flow_head_reduce_kernel(const float *__restrict__ part, long part_bs, int ncb,
                                                               int H, int W, int BH, int BW, int tiles_w,
                                                               int tiles_hw, const float *__restrict__ bias0,
                                                               float *__restrict__ cx, float *__restrict__ fa,
                                                               long fa_bs, float *__restrict__ fb, long fb_bs) {
  const unsigned r = blockIdx.x * 256u + threadIdx.x;
  const unsigned hw = (unsigned)(H * W);
  if (r >= hw) return;
  const long b = blockIdx.y;
  const int y = (int)(r / (unsigned)W), x = (int)(r % (unsigned)W);
  const int RH = BH + 2, RW = BW + 2, tiles_h = tiles_hw / tiles_w;
  const int ty0 = y / BH, tx0 = x / BW;
  // the tiles whose bordered region holds (y, x): its own, the one above / below when the pixel is
  // on its tile's first / last row, the one left / right on its first / last column, and the
  // diagonal one when both; summed in that fixed order per channel block
  const bool up = y % BH == 0 && ty0 > 0, dn = y % BH == BH - 1 && ty0 + 1 < tiles_h;
  const bool lf = x % BW == 0 && tx0 > 0, rt = x % BW == BW - 1 && tx0 + 1 < tiles_w;
  const int ty1 = up ? ty0 - 1 : ty0 + 1, tx1 = lf ? tx0 - 1 : tx0 + 1;
  auto off = [&](int ty, int tx) { return ((long)(ty * tiles_w + tx) * RH + (y - (ty * BH - 1))) * RW + (x - (tx * BW - 1)); };
  const bool hy = up || dn, hx = lf || rt;
  // (absent neighbours read the pixel's own partial and add nothing: no branches between the loads)
  const long o0 = off(ty0, tx0), o1 = hx ? off(ty0, tx1) : o0, o2 = hy ? off(ty1, tx0) : o0,
             o3 = hx && hy ? off(ty1, tx1) : o0;
  float d = bias0[0];
  const float *pc = part + b * part_bs;
  const long cbs = (long)tiles_hw * RH * RW;
  // 8 channel blocks' 32 loads go out together (clamped block index, summed only below ncb),
  // then the sums in the fixed order
  for (int cb0 = 0; cb0 < ncb; cb0 += 8) {
    float a[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float *q = pc + (long)min(cb0 + j, ncb - 1) * cbs;
      a[j][0] = q[o0];
      a[j][1] = q[o1];
      a[j][2] = q[o2];
      a[j][3] = q[o3];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in = cb0 + j < ncb;
      d = in ? d + a[j][0] : d;
      d = in && hx ? d + a[j][1] : d;
      d = in && hy ? d + a[j][2] : d;
      d = in && hx && hy ? d + a[j][3] : d;
    }
  }
  const long i = b * hw + r;
  const float c = cx[i] + d;
  cx[i] = c;
  const float fx = c - (float)x;
  if (fa) {
    fa[b * fa_bs + r] = fx;
    fa[b * fa_bs + hw + r] = 0.0f;
  }
  if (fb) {
    fb[b * fb_bs + r] = fx;
    fb[b * fb_bs + hw + r] = 0.0f;
  }
}

int w4_ltw(int H, int W) {
  const long a16 = (long)((W + 63) / 64) * 64 * ((H + 15) / 16) * 16;
  const long a32 = (long)((W + 127) / 128) * 128 * ((H + 7) / 8) * 8;
  return a32 < a16 ? 5 : 4;
}

}  // namespace

extern "C" int sa_conv2d_wino4_weights(const float *weight, int Cout, int Cin, float *U, void *stream) {
  SA_REQUIRE(weight && U && Cout > 0 && Cin > 0 && Cin % 8 == 0 && Cout % 32 == 0,
             "sa_conv2d_wino4_weights: bad arguments (Cin %% 8, Cout %% 32)");
  const long n = (long)Cout * Cin;
  hipStream_t s = sa::as_stream(stream);
  wino4_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, 32, U);
  return sa::check_launch("sa_conv2d_wino4_weights");
}

extern "C" int sa_conv2d_wino4_weights_split(const float *weight, int Cout, int Cin, void *U, void *stream) {
  SA_REQUIRE(weight && U && Cout > 0 && Cin > 0 && Cin % 8 == 0 && Cout % 32 == 0,
             "sa_conv2d_wino4_weights_split: bad arguments (Cin %% 8, Cout %% 32)");
  const long n = (long)Cout * Cin;
  hipStream_t s = sa::as_stream(stream);
  wino4s_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, static_cast<unsigned *>(U));
  return sa::check_launch("sa_conv2d_wino4_weights_split");
}

#ifdef SA_W4_CLOCK
extern "C" int sa_w4_clock_read(unsigned long long *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w4_clock), sizeof(unsigned long long) * 12 * n) == hipSuccess ? 0 : -1;
}
#endif

extern "C" long sa_flow_head_part_size(int N, int Cout, int H, int W) {
  if (N <= 0 || Cout <= 0 || Cout % 32 || H <= 0 || W <= 0) return -1;
  const int ltw = w4_ltw(H, W), bw = 4 << ltw, bh = 4 * (W4Big::NT >> ltw);
  const long tiles = (long)((W + bw - 1) / bw) * ((H + bh - 1) / bh);
  return (long)N * (Cout / 32) * tiles * (bh + 2) * (bw + 2);
}

extern "C" int sa_flow_head_reduce(const float *part, int N, int Cout, int H, int W, const float *bias0,
                                   float *coords_x, float *flow_a, long flow_a_bs, float *flow_b, long flow_b_bs,
                                   void *stream) {
  SA_REQUIRE(part && bias0 && coords_x, "sa_flow_head_reduce: null pointer");
  const long per = sa_flow_head_part_size(1, Cout, H, W);
  SA_REQUIRE(per > 0 && N > 0 && N <= 65535 && (long)H * W < (1L << 31), "sa_flow_head_reduce: bad shape");
  const int ltw = w4_ltw(H, W), bw = 4 << ltw, bh = 4 * (W4Big::NT >> ltw);
  const int tiles_w = (W + bw - 1) / bw, tiles_hw = tiles_w * ((H + bh - 1) / bh);
  const unsigned hw = (unsigned)((long)H * W);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  flow_head_reduce_kernel<<<dim3((hw + 255) / 256, N), 256, 0, s>>>(part, per, Cout / 32, H, W, bh, bw, tiles_w,
                                                                     tiles_hw, bias0, coords_x, flow_a, flow_a_bs,
                                                                     flow_b, flow_b_bs);
  return sa::check_launch("sa_flow_head_reduce");
}

long sa_direct_redo_blocks_internal(int reset);   // conv_direct.hip

// blocks of the split kernels (F(4x4) and direct) that the range guards recomputed
// since the last reset; synchronises the device (tests and bench.py, outside timed regions)
extern "C" long sa_split_redo_blocks(int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_w4_redo_blocks), sizeof v) != hipSuccess) return -1;
  if (reset) {
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_w4_redo_blocks), &z, sizeof z) != hipSuccess) return -1;
  }
  const long d = sa_direct_redo_blocks_internal(reset);
  return d < 0 ? -1 : (long)v + d;
}

// InstanceNorm partial count: the small blocks' tiling (a large block writes its two halves)
extern "C" long sa_conv2d_k3_wino4_stat_parts(int H, int W) {
  const int ltw = w4_ltw(H, W), bw = 4 << ltw, bh = 4 * (32 >> ltw);
  return (long)((W + bw - 1) / bw) * ((H + bh - 1) / bh);
}

extern "C" int sa_conv2d_k3_wino4_multi(int nprob, const SaWinoProblem *probs, void *stream) {
  return sa_conv2d_k3_wino4_multi_gate(nprob, probs, nullptr, 0, stream);
}

extern "C" int sa_conv2d_k3_wino4_multi_gate(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates,
                                             int block_shape, void *stream) {
  return sa_conv2d_k3_wino4_launch(nprob, probs, gates, block_shape, 0, stream);
}

extern "C" int sa_conv2d_k3_wino4_launch(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates,
                                         int block_shape, int guard, void *stream) {
  SA_REQUIRE(nprob >= 1 && nprob <= MAX_PROB && probs, "sa_conv2d_k3_wino4_multi: 1..%d problems", MAX_PROB);
  SA_REQUIRE(block_shape == 0 || block_shape == 1 || block_shape == 2 || block_shape == 6,
             "sa_conv2d_k3_wino4_multi: block_shape 0, 1, 2 or 6 (got %d)", block_shape);
  // Large blocks unless the caller asks for small ones (block_shape 2).  The small shape measured
  // 2-8% faster on standalone launches of Cin <= 128 with a few rounds of blocks (qh08, convc2) but
  // not faster in the forward as a blanket choice.  block_shape 6: the split kernel (W4Split;
  // filters from sa_conv2d_wino4_weights_split).
  const bool small = block_shape == 2, split = block_shape == 6;
  const int nt = small ? W4Small::NT : W4Big::NT;
  constexpr int CO = 32;
  const int aff_max = small ? W4Small::AFF_MAX : split ? W4Split::AFF_MAX : W4Big::AFF_MAX;
  W4Launch L{};
  long total = 0;
  bool gated = false, aff = false;
  for (int i = 0; i < nprob; ++i) {
    const SaWinoProblem &q = probs[i];
    SA_REQUIRE(q.in && q.U && q.out && q.N > 0 && q.H > 0 && q.W > 0, "sa_conv2d_k3_wino4: bad arguments");
    SA_REQUIRE(q.Cin % 8 == 0 && q.Cout % CO == 0,
               "sa_conv2d_k3_wino4: needs Cin %% 8 == 0 and Cout %% 32 == 0 (got %d, %d)", q.Cin, q.Cout);
    const int pitch = q.pitch ? q.pitch : q.W;
    SA_REQUIRE(pitch >= q.W, "sa_conv2d_k3_wino4: pitch %d < W %d", pitch, q.W);
    SA_REQUIRE(pitch % 4 == 0 && (reinterpret_cast<uintptr_t>(q.in) & 15) == 0 && q.in_bs % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(q.out) & 15) == 0 && q.out_bs % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(q.U) & 15) == 0,
               "sa_conv2d_k3_wino4: needs W (or the row pitch) %% 4 == 0 and 16-byte aligned input / output planes "
               "and filters");
    const bool qaff = q.in_m || q.in_s || q.in_t || q.in_act;
    SA_REQUIRE(q.in_act == 0 || q.in_act == 1, "sa_conv2d_k3_wino4: input activation none or ReLU (got %d)", q.in_act);
    SA_REQUIRE(q.in_pstride == 0 || q.in_pstride == q.Cin, "sa_conv2d_k3_wino4: in_pstride must be 0 or Cin");
    SA_REQUIRE(!qaff || q.Cin <= aff_max, "sa_conv2d_k3_wino4: an input transform needs Cin <= %d", aff_max);
    aff = aff || qaff;
    SA_REQUIRE((long)q.Cin * q.H * pitch * 4 < (1L << 31) - 64 && 36L * q.Cin * q.Cout * 4 < (1L << 31),
               "sa_conv2d_k3_wino4: an image or the filter bank exceeds the 2 GB buffer-descriptor range");
    const int ltw = w4_ltw(q.H, q.W), bw = 4 << ltw, bh = 4 * (nt >> ltw);
    const int tiles_w = (q.W + bw - 1) / bw, tiles_h = (q.H + bh - 1) / bh;
    if (q.skip) {
      SA_REQUIRE(!q.stats_partial && !(gates && gates[i].mode != 0) && (reinterpret_cast<uintptr_t>(q.skip) & 15) == 0 &&
                     q.skip_bs % 4 == 0 && (q.skip_act == 0 || q.skip_act == 1) && (q.out_act == 0 || q.out_act == 1),
                 "sa_conv2d_k3_wino4: a residual epilogue takes no statistics or gate and a 16-byte aligned skip "
                 "plane (skip_act none or ReLU)");
    }
    L.p[i] = W4Prob{q.in, q.in_bs, q.Cin, q.H, q.W, q.U, q.Cout, q.bias, q.relu, q.out, q.out_bs,
                    ltw, tiles_w, tiles_w * tiles_h, q.Cout / CO, q.stats_partial,
                    q.in_m, q.in_s, q.in_t, q.in_pstride, q.in_act, pitch,
                    q.skip, q.skip_bs, q.skip_s, q.skip_t, q.skip_act, q.out_act};
    L.gate[i] = W4Gate{};
    if (gates && gates[i].mode != 0) {
      const SaGateEpilogue &e = gates[i];
      auto a16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
      SA_REQUIRE(e.mode >= 1 && e.mode <= 3, "sa_conv2d_k3_wino4: gate mode %d", e.mode);
      if (e.mode == 3) {
        SA_REQUIRE(e.head_w && e.head_part && !q.stats_partial && !q.pitch && (block_shape == 0 || block_shape == 6),
                   "sa_conv2d_k3_wino4: the flow-head epilogue needs head_w / head_part, no statistics, dense "
                   "planes and the 8-wave 32-channel shape (block_shape 0 or 6)");
        SA_REQUIRE(e.head_part_bs >= sa_flow_head_part_size(1, q.Cout, q.H, q.W),
                   "sa_conv2d_k3_wino4: head_part_bs too small");
        L.gate[i] = W4Gate{};
        L.gate[i].mode = 3;
        L.gate[i].head_w = e.head_w;
        L.gate[i].head_part = e.head_part;
        L.gate[i].head_part_bs = e.head_part_bs;
        gated = true;
        const long nb3 = (long)q.N * L.p[i].tiles_hw * L.p[i].co_blocks;
        total = (i + 1 < nprob ? (total + nb3 + 7) / 8 * 8 : total + nb3);
        SA_REQUIRE(total < (1L << 31), "sa_conv2d_k3_wino4: grid too large");
        L.end[i] = (unsigned)total;
        L.nblk[i] = (unsigned)nb3;
        continue;
      }
      SA_REQUIRE(!q.relu && !q.stats_partial, "sa_conv2d_k3_wino4: a gate epilogue takes no ReLU / statistics");
      SA_REQUIRE(e.ctx && e.h && a16(e.ctx) && a16(e.h) && e.ctx_bs % 4 == 0 && e.h_bs % 4 == 0,
                 "sa_conv2d_k3_wino4: gate needs 16-byte aligned ctx and h planes");
      if (e.mode == 1)   // a block's channels lie wholly in the z half or the r half
        SA_REQUIRE(q.Cout % (2 * CO) == 0 && e.out2 && a16(e.out2) && e.out2_bs % 4 == 0,
                   "sa_conv2d_k3_wino4: z/r gate needs Cout %% %d == 0 and an aligned r*h output", 2 * CO);
      else
        SA_REQUIRE(e.z && e.add && a16(e.z) && a16(e.add) && e.z_bs % 4 == 0 && e.add_bs % 4 == 0,
                   "sa_conv2d_k3_wino4: state gate needs aligned z and addend planes");
      L.gate[i] = W4Gate{e.mode, e.ctx, e.ctx_bs, e.h, e.h_bs, e.z, e.z_bs, e.add, e.add_bs, e.out2, e.out2_bs,
                         nullptr, nullptr, 0};
      gated = true;
    }
    const long nb = (long)q.N * L.p[i].tiles_hw * L.p[i].co_blocks;
    total = (i + 1 < nprob ? (total + nb + 7) / 8 * 8 : total + nb);
    SA_REQUIRE(total < (1L << 31), "sa_conv2d_k3_wino4: grid too large");
    L.end[i] = (unsigned)total;
    L.nblk[i] = (unsigned)nb;
  }
  for (int i = nprob; i < MAX_PROB; ++i) {
    L.end[i] = (unsigned)total;
    L.nblk[i] = 0;
  }
  L.nprob = nprob;
  SA_REQUIRE(!(aff && gated), "sa_conv2d_k3_wino4: an input transform and a gate epilogue in one launch");
  // the split kernel's range guard: a block whose operands overflowed runs again on scaled inputs
  L.guard = split && guard ? 1 : 0;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV2D_W4, s);
  if (split) {
    aff     ? wino_f4k3_kernel<W4Split, false, true><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L)
    : gated ? wino_f4k3_kernel<W4Split, true><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L)
            : wino_f4k3_kernel<W4Split, false><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L);
  }
  else if (aff && small)
    wino_f4k3_kernel<W4Small, false, true><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L);
  else if (aff)
    wino_f4k3_kernel<W4Big, false, true><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L);
  else if (small)
    gated ? wino_f4k3_kernel<W4Small, true><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L)
          : wino_f4k3_kernel<W4Small, false><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L);
  else
    gated ? wino_f4k3_kernel<W4Big, true><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L)
          : wino_f4k3_kernel<W4Big, false><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L);
  return sa::check_launch("sa_conv2d_k3_wino4");
}
