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

// diagnostic / A-B switches (build-time)
#ifndef SA_W4_SPREAD
#define SA_W4_SPREAD 1
#endif
#ifndef SA_W4_FENCE
#define SA_W4_FENCE 1
#endif
#ifndef SA_W4_DIAG
#define SA_W4_DIAG 0   // timing diagnostics only (wrong results): 1 no DMA in the loop, 2 no
                       // transform / MFMA, 3 no DMA and no barrier in the loop, 4 as 3 and no
                       // DMA at all, 5 no column pass, 6 no row pass, 7 no filter reads in the loop,
                       // 8 neither row nor column pass (no input transform)
#endif
#ifndef SA_W4_PERM
#define SA_W4_PERM 1   // lane -> tile permutation that makes the patch rows' ds_read_b128 conflict-free
#endif
#ifndef SA_W4_GJB
#define SA_W4_GJB 8    // gate-epilogue store iterations whose plane loads go out together (mode 2)
#endif
#ifndef SA_W4_GJB1
#define SA_W4_GJB1 16  // the same for mode 1
#endif
#ifndef SA_W4_DUP
#define SA_W4_DUP 0    // split kernel: each B operand (bhi, blo, bhi, blo) read as its (hi, lo) dword twice by one
                       // ds_read2st64_b32 (filter image [g][k][n] per point and job) instead of register copies;
                       // a column's pairs of points 0-2 / 3-5 are reloaded for the next column as soon as their
                       // MFMAs are issued (the same 24 VGPRs as the copied form's bc / bn)
#endif
#ifndef SA_W4_DMA_AT
#define SA_W4_DMA_AT 1 // the next chunk's DMA part jj: 0 after column jj's MFMAs of the first job, 1 before its
                       // column pass (wino4 51.0 -> 50.1 ms/step, scripts/ab_w4_variants.sh), 2 all three parts
                       // before column 0 (after the first job's row pass), 3 part 0 before the first job's row
                       // pass, part jj + 1 before column jj
#endif
#ifndef SA_W4_TGRP
#define SA_W4_TGRP 1   // work-item order: groups of TGRP tiles, output-channel block outer within a group
                       // (1: a tile's channel blocks adjacent).  The 32 blocks an XCD runs at once then share
                       // ~TGRP tiles' patches and ~32 / TGRP channel blocks' filters in its L2
#endif
#ifndef SA_W4_PPART
#define SA_W4_PPART 0  // DMA pieces per part of the spread next-chunk DMA (0: 2, or 3 when a wave has more than 6)
#endif
#ifndef SA_W4_UFIRST
#define SA_W4_UFIRST 0 // 1: a DMA part's filter pieces go out before its patch pieces
#endif
#ifndef SA_W4_PRIO
#define SA_W4_PRIO 1   // s_setprio 1 for the point-half-1 waves (split kernel forward: 66.8 -> 66.5 ms/step, wino4 49.8 -> 49.0 ms, two interleaved passes)
#endif
#ifndef SA_W4_PF
#define SA_W4_PF 1     // persistent kernel: prefetch the next item's chunk 0 (0: each item issues its own)
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
template <int NW_, int KC_, int CO_ = 32, bool QUAD_ = false, bool SPLIT_ = false, bool UNSPLIT_ = false>
struct W4Cfg {
  // UNSPLIT: fp32 MFMA products with the split kernel's (hi, lo) filter dwords read as hi + lo (the
  // range guard's redo kernel, wino_f4k3_redo_kernel)
  static constexpr bool UNSPLIT = UNSPLIT_;
  // QUAD: the waves of a tile group split the 6 x 6 points in quadrants (rows 0-2 / 3-5 x
  // columns 0-2 / 3-5) instead of column halves
  static constexpr bool QUAD = QUAD_;
  // SPLIT: the products on f16 MFMA with hi/lo operand pairs (W4Split below)
  static constexpr bool SPLIT = SPLIT_;
  static constexpr int NW = NW_, NTHR = 64 * NW_, TG = QUAD_ ? NW_ / 4 : NW_ / 2, NT = 16 * TG, KC = KC_, JPC = KC_ / 4;
  static constexpr int NR = QUAD_ ? 3 : 6;                  // point rows per wave
  static constexpr int CO = CO_, CG = CO_ / 16;                // output channels per block, 16-channel groups
  static constexpr int SB = 4 * CO_;                        // filters per (point, 4-channel job): [k][n][g]
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
  static constexpr int PPART = SA_W4_PPART ? SA_W4_PPART : (PDMA > UPW ? PDMA : UPW) > 6 ? 3 : 2;   // DMA pieces per part
  static_assert(PDMA <= 3 * PPART && UPW <= 3 * PPART, "three DMA parts");
  static_assert(OPP % 32 == 4, "conflict-free staging");
  // input (scale, shift) table of an input-transform launch in the LDS left over
  static constexpr int AFF_MAX = (160 * 1024 - SMEM * 4) / 8 > 512 ? 512 : (160 * 1024 - SMEM * 4) / 8;
};
using W4Big = W4Cfg<8, 8>;
using W4Small = W4Cfg<4, 4>;
// Wide: one wave per SIMD, 32 tiles x 64 output channels, 4-channel chunks.  Each transformed
// input value feeds four MFMAs (one per 16-channel group) instead of two, and one ds_read_b128
// hands a lane its four filter operands: half the transform VALU and the filter-read
// instructions per MFMA of the 8-wave shape (whose main loop measured VALU- and LDS-issue
// bound: -DSA_W4_DIAG=5/7 builds ran 20% / 15% faster).  288 accumulators per lane.
using W4Wide = W4Cfg<4, 4, 64>;
// Quad: 8 waves (two per SIMD), 32 tiles x 64 output channels, 4-channel chunks; a wave owns
// 16 tiles x 64 channels x one quadrant of the points (9 points x 4 channel groups = 144
// accumulators, as the 8-wave shape).  Per (tile, channel) job the row pass is the 8-wave
// shape's (3 of 6 outputs per row) but the column pass yields 3 instead of 6 points, and each
// transformed value feeds four MFMAs: ~1.5 instead of ~2 transform operations per MFMA, and one
// ds_read_b128 instead of two ds_read_b64 per four MFMAs.  The price: a barrier per 4 input
// channels and four partial output transforms meeting in LDS.
using W4Quad = W4Cfg<8, 4, 64, true>;
#ifndef W4S_KC
#define W4S_KC 8   // the split kernel's input-channel chunk (4: twice the barriers, measured slower)
#endif
#ifndef W4S_K32
#define W4S_K32 0  // 2: the paired form (both of a lane's channels per MFMA pair, hi then lo halves: no operand copies; 268 instead of ~375 VALU per chunk and wave, 1.0-1.06x on plain convs, but the forward 66.7 -> 68.3 ms);  1: plain launches take the products of both of a lane's channels on one v_mfma_f32_16x16x32_f16 (1.02-1.03x on the plain convs, but the gated / input-transform kernels then spill or read the filters as 2 x b32: forward 66.2 -> 72.4 ms)
#endif
static_assert(!W4S_K32 || W4S_KC == 8, "the K = 32 split form takes a lane's two channels of an 8-channel chunk");
// Split: the 8-wave shape (8- or 4-channel chunks) whose Winograd-domain products run on
// v_mfma_f32_16x16x16_f16 instead of v_mfma_f32_16x16x4_f32.  Each operand is an f16 hi/lo
// pair (x = hi + lo, 22 significant bits; filters scaled by 2^W4S_LOG2 before the split and
// the accumulators by 2^-W4S_LOG2 after the main loop, both exact), and one MFMA's K = 16
// slots hold a lane's channel as the four products hi*bhi + hi*blo + lo*bhi + lo*blo: the A
// operand (hi, hi, lo, lo) is the lane's transformed value (3 VALU to split), the B operand
// (bhi, blo, bhi, blo) is the filter's (bhi, blo) dword twice: the LDS image holds each pair
// once (sa_conv2d_wino4_weights_split; the same bytes per chunk as the fp32 filters, so the
// same L2 -> LDS intake per channel, which bounds this kernel family), one ds_read_b64 gives a
// lane both output-channel groups' pairs, and the copy is a register move.  Products of f16 pairs are
// exact in fp32, so the result differs from the fp32 kernel only by the operands' rounding
// (<= 2^-22 relative; below 2^-14 the lo halves are subnormal, an absolute 2^-25) and the
// accumulation order.  |V| must stay below 65504 (the f16 range): V = B^T d B grows at most
// 100-fold over the input patch.
using W4Split = W4Cfg<8, W4S_KC, 32, false, true>;
using W4SplitRedo = W4Cfg<8, W4S_KC, 32, false, false, true>;
// the split products on the 4-wave shape (block_shape 7): 32 tiles, 4-channel chunks, two blocks
// per CU, so one block's first-chunk wait and epilogue overlap the other's main loop
using W4SplitSmall = W4Cfg<4, 4, 32, false, true>;
using W4SplitRedoSmall = W4Cfg<4, 4, 32, false, false, true>;
constexpr int W4S_LOG2 = 12;
static_assert(2 * W4Small::SMEM * 4 <= 160 * 1024, "two small blocks per CU");
static_assert(2 * (W4SplitSmall::SMEM * 4 + W4SplitSmall::AFF_MAX * 8) <= 160 * 1024, "two small split blocks per CU");
static_assert(W4Wide::SMEM * 4 <= 160 * 1024, "one wide block per CU");

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
  int ntiles;              // N * tiles_hw
};
constexpr int MAX_PROB = 8;

// work item -> (output-channel block, tile in the image, image)
__device__ __forceinline__ void w4_item(const unsigned wid, const int co_blocks, const int tiles_hw, const int ntiles,
                                        int &cb, int &st, int &n) {
  int gt;
  if constexpr (SA_W4_TGRP <= 1) {
    cb = wid % co_blocks;
    gt = wid / co_blocks;
  } else {
    const int per = SA_W4_TGRP * co_blocks, g = wid / per, rem = wid - g * per, full = ntiles / SA_W4_TGRP;
    const int sz = g < full ? SA_W4_TGRP : ntiles - full * SA_W4_TGRP;
    cb = rem / sz;
    gt = g * SA_W4_TGRP + (rem - cb * sz);
  }
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
  // the split kernel's range guard: [0] = count, [1 ..] = (problem << 27 | work item) of the blocks
  // that skipped their epilogue; redo_cap entries (wino_f4k3_redo_kernel)
  unsigned *redo;
  unsigned redo_cap;
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

// x0, x1 as the A operand (hi0, hi0, hi1, hi1, lo0, lo0, lo1, lo1) of v_mfma_f32_16x16x32_f16
// (the B operand (p0, p1, p0, p1) with p = (bhi, blo): the four products of each channel)
[[maybe_unused]] __device__ __forceinline__ f16x8 w4_split2(const float x0, const float x1) {
  const f16x2 h0 = __builtin_convertvector(f32x2{x0, x0}, f16x2);
  const f16x2 h1 = __builtin_convertvector(f32x2{x1, x1}, f16x2);
  float l0, l1;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l0) : "v"(__builtin_bit_cast(unsigned, h0)), "v"(x0));
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l1) : "v"(__builtin_bit_cast(unsigned, h1)), "v"(x1));
  const f16x2 g0 = __builtin_convertvector(f32x2{l0, l0}, f16x2);
  const f16x2 g1 = __builtin_convertvector(f32x2{l1, l1}, f16x2);
  return __builtin_shufflevector(__builtin_shufflevector(h0, h1, 0, 1, 2, 3), __builtin_shufflevector(g0, g1, 0, 1, 2, 3),
                                 0, 1, 2, 3, 4, 5, 6, 7);
}

// the fp32 value w * 2^12 of a split filter dword (hi, lo): hi + lo is exact in fp32 (22 bits)
__device__ __forceinline__ float w4_unsplit(const float packed) {
  const f16x2 p = __builtin_bit_cast(f16x2, packed);
  return (float)p[0] + (float)p[1];
}

// (SA_W4_DUP) the dword at LDS byte address addr + 256 OFF into both registers of a pair: one
// ds_read2st64_b32 with equal offsets.  Inline asm: the compiler does not count it in its LDS
// waits, so every use is preceded by w4_lds_wait3 on the loaded pairs.
template <int OFF>
__device__ __forceinline__ f32x2 w4_lds_dup(unsigned addr) {
  f32x2 r;
  asm volatile("ds_read2st64_b32 %0, %1 offset0:%2 offset1:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
// the same with the offset as a value the unrolled loops make constant (the chain folds away)
template <int N>
__device__ __forceinline__ f32x2 w4_lds_dup_rt(unsigned addr, int off) {
  if constexpr (N < 0) {
    __builtin_unreachable();
    return f32x2{0.f, 0.f};
  } else {
    if (off == N) return w4_lds_dup<N>(addr);
    return w4_lds_dup_rt<N - 1>(addr, off);
  }
}
// s_waitcnt lgkmcnt(CNT) tied to three points' pairs (both groups), so no use is scheduled above
// it; CNT <= the LDS operations issued after those pairs' loads (LDS returns in order)
template <int CNT>
__device__ __forceinline__ void w4_lds_wait3(f32x2 &a0, f32x2 &a1, f32x2 &b0, f32x2 &b1, f32x2 &c0, f32x2 &c1) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1), "+v"(c0), "+v"(c1) : "n"(CNT));
}

// Range guard of the split kernel: blocks whose f16 operands overflowed (|V| >= 65520 turns hi
// into inf, so every product of that value, and the outputs it feeds, are NaN) skip their epilogue
// and are recomputed on fp32 MFMA by wino_f4k3_redo_kernel; this counts them (sa_split_redo_blocks)
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
  if (!SA_W4_PERM) return m;
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

// Chunk 0 (filters + patch) of work item `wid` of problem P into LDS buffer pb, with the patch
// geometry at run time (P.ltw): the persistent kernel issues it for its NEXT work item during
// the current item's last chunk, so the next item's first chunk lands under this item's
// epilogue instead of after it.  Same DMA pieces and lanes as w4_body's own chunk-0 issue.
template <class C>
__device__ __forceinline__ void w4_issue_chunk0(const W4Prob &P, const unsigned wid, float *pb, const int wv,
                                                const int lane) {
  constexpr int NWAVE = C::NW, KC = C::KC, PDMA = C::PDMA, UDMA = C::UDMA, UPW = C::UPW, PBUF = C::PBUF,
                NT = C::NT, CO = C::CO, SB = C::SB, JPC = C::JPC;
  const int Cin = P.Cin, H = P.H;
  const int ltw = P.ltw, tw = 1 << ltw, tr = NT >> ltw;
  const int BH = 4 * tr, BW = 4 * tw, PG = tw + 2, PR = BH + 2, PS = PR * PG;
  const int co_blocks = P.co_blocks, tiles_hw = P.tiles_hw, tiles_w = P.tiles_w;
  int cb, st, n;
  w4_item(wid, co_blocks, tiles_hw, P.ntiles, cb, st, n);
  const int y0 = (st / tiles_w) * BH, x0 = (st % tiles_w) * BW;
  const int pitch = P.pitch, hw = H * pitch;
  const __amdgpu_buffer_rsrc_t xin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(P.in + (long)n * P.in_bs), (short)0, Cin * hw * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t uin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(P.U + (long)cb * Cin * NPT * CO), (short)0, Cin * NPT * CO * 4, 0x00020000);
#pragma unroll
  for (int j = 0; j < UPW; ++j)
    if (wv + NWAVE * j < UDMA) {
      const int f = (wv + NWAVE * j) * 256 + lane * 4;
      dma16(uin, pb + PBUF + (wv + NWAVE * j) * 256, (JPC == 2 ? f : f + (f / SB) * SB) * 4, 0);
    }
  const int npi = (KC * PS + 63) >> 6;
  // rolled: this runs with the accumulators live (an unrolled loop's address math spilled)
#pragma unroll 1
  for (int j = 0; j < PDMA; ++j) {
    if (wv + NWAVE * j < npi) {
      const int s = (wv + NWAVE * j) * 64 + lane;
      const int ci = s / PS, rem = s - ci * PS, r = rem / PG, g = rem - r * PG;
      const int y = y0 - 1 + r, x = x0 - 4 + 4 * g;
      const bool ok = s < KC * PS && y >= 0 && y < H && x >= 0 && x < pitch;
      dma16(xin, pb + (wv + NWAVE * j) * 256, ok ? (ci * hw + y * pitch + x) * 4 : 0x7ffffff0, 0);
    }
  }
}

// The block's staged outputs, channels [cbase, cbase + NCH) of its CO at ot (plane c - cbase,
// pitch OPP): InstanceNorm partials (if requested), then float4 stores or the GRU gate epilogue.
template <class C, bool GATED, int NCH>
__device__ __forceinline__ void w4_emit(const W4Prob &P, const W4Gate *gate, const float *ot, const int cbase,
                                        const int n, const int co0, const int st, const int tiles_w, const int y0,
                                        const int x0, const int BH, const int BW, const int lbw, const int tid) {
  constexpr int NT = C::NT, NTHR = C::NTHR, OPP = C::OPP, CO = C::CO;
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
  // (the 64-channel shapes spill with 16 in mode 1: 8 there; a 16-channel pass of the persistent
  // kernel runs with the other group's accumulators live: 4)
  if (GT.mode == 1)
    gate_stores(std::integral_constant<int, NCH == 16 ? 4 : CO == 64 ? SA_W4_GJB : SA_W4_GJB1>{},
                std::integral_constant<int, 1>{});
  else gate_stores(std::integral_constant<int, NCH == 16 ? 4 : SA_W4_GJB>{}, std::integral_constant<int, 2>{});
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
__device__ unsigned long long g_w4_clock[65536][10];   // + [8] chunk 0 issued, [9] last wave's start
#endif

// PERSIST: a work item of the persistent kernel.  Its chunk kc is staged in LDS buffer
// (kc + par) & 1; `pre`: chunk 0 was issued by the previous item (w4_issue_chunk0); NP / nwid:
// the next item (if has_next), whose chunk 0 this item issues as its main loop ends.  The epilogue then stages
// one 16-channel group at a time in the last chunk's buffer (the other one receives the
// prefetch).
template <class C, int HF, int LTW, bool GATED, bool AFF, int RH = 0, bool PERSIST = false>
__device__ __forceinline__ void w4_body(const W4Prob &P, const W4Gate *gate, const unsigned wid, float *smem,
                                        float2 *atab, const int par = 0, const bool pre = false,
                                        const bool has_next = false, const W4Prob &NP = W4Prob{},
                                        const unsigned nwid = 0, unsigned *redo = nullptr,
                                        const unsigned redo_cap = 0, const unsigned redo_tag = 0) {
  constexpr int NWAVE = C::NW, NTHR = C::NTHR, KC = C::KC, JPC = C::JPC, NT = C::NT, PDMA = C::PDMA,
                UDMA = C::UDMA, UPW = C::UPW, UBUF = C::UBUF, BUF = C::BUF, PBUF = C::PBUF, OPP = C::OPP,
                CO = C::CO, CG = C::CG, SB = C::SB, NR = C::NR;
  constexpr bool QUAD = C::QUAD, SPLIT = C::SPLIT;
  static_assert(!SPLIT || (!QUAD && !PERSIST && CG == 2), "split: the 8-wave 32-channel shape");
  // a lane's filter operands of a point: one float, or (split) one f16 (hi, lo) pair, per group
  using f32xg = float __attribute__((ext_vector_type(CG)));
  const int Cin = P.Cin, H = P.H;
  // block geometry as compile-time constants (the patch offsets divide by PS and PG)
  constexpr int ltw = LTW, tw = 1 << ltw, tr = NT >> ltw;
  constexpr int BH = 4 * tr, BW = 4 * tw, PG = tw + 2, PR = BH + 2, PS = PR * PG;
  int tid = threadIdx.x;
  // persistent items: an opaque thread id per item keeps the compiler from hoisting the
  // lane-dependent offsets out of the item loop (live across it they cost ~20 VGPRs and spilled)
#ifndef SA_W4_OPAQUE
#define SA_W4_OPAQUE 1
#endif
  if constexpr (PERSIST && SA_W4_OPAQUE) asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co_blocks = P.co_blocks, tiles_hw = P.tiles_hw, tiles_w = P.tiles_w;
  int cb, st, n;
  w4_item(wid, co_blocks, tiles_hw, P.ntiles, cb, st, n);
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
  if (SA_W4_DIAG != 4 && !pre) {
#pragma unroll
    for (int j = 0; j < UPW; ++j)
      if (wv + NWAVE * j < UDMA)
        dma16(uin, smem + par * BUF + PBUF + (wv + NWAVE * j) * 256, u_src(wv + NWAVE * j), u_chunk(0));
  }
  const int npi = (KC * PS + 63) >> 6;
  int po[PDMA];
  int pc[PDMA];   // input transform: the group's channel in the chunk (-1: padding or idle lane)
#pragma unroll
  for (int j = 0; j < PDMA; ++j) {
    const int s = (wv + NWAVE * j) * 64 + lane;
    const int ci = s / PS, rem = s - ci * PS, r = rem / PG, g = rem - r * PG;
    const int y = y0 - 1 + r, x = x0 - 4 + 4 * g;
    // (a pitched plane's columns W .. pitch - 1 are zero: they load as the right padding)
    const bool ok = s < KC * PS && y >= 0 && y < H && x >= 0 && x < pitch;
    po[j] = ok ? (ci * hw + y * pitch + x) * 4 : 0x7ffffff0;   // out of range: the load returns 0
    pc[j] = ok && wv + NWAVE * j < (KC * PS + 63) / 64 ? ci : -1;
  }
  // the chunk's DMAs in three parts (part -1: all at once), spread over the first job's three
  // column phases (each piece costs tens of issue cycles; clustered after the barrier they
  // would delay the first reads)
  auto issue_part = [&](int chunk, int buf, int part) __attribute__((always_inline)) {
    float *pb = smem + buf * BUF;
    const int xs = chunk * KC * hw * 4;
    float *ub = pb + PBUF;
    const int us = u_chunk(chunk);
    auto pieces_u = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < UPW; ++j)
        if ((part < 0 || j / C::PPART == part) && wv + NWAVE * j < UDMA)
          dma16(uin, ub + (wv + NWAVE * j) * 256, u_src(wv + NWAVE * j), us);
    };
    if (SA_W4_UFIRST) pieces_u();
#pragma unroll
    for (int j = 0; j < PDMA; ++j)
      if ((part < 0 || j / C::PPART == part) && wv + NWAVE * j < npi) dma16(xin, pb + (wv + NWAVE * j) * 256, po[j], xs);
    if (!SA_W4_UFIRST) pieces_u();
  };
  auto issue = [&](int chunk, int buf) __attribute__((always_inline)) { issue_part(chunk, buf, -1); };
  auto issue_p0 = [&]() __attribute__((always_inline)) {   // chunk 0's patch (its filters went first)
#pragma unroll
    for (int j = 0; j < PDMA; ++j)
      if (wv + NWAVE * j < npi) dma16(xin, smem + par * BUF + (wv + NWAVE * j) * 256, po[j], 0);
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
  // (SA_W4_DUP: the split filter image is [g][k][n] per point and job, one 64-dword row per group)
  constexpr bool DUP = SA_W4_DUP && (SPLIT || C::UNSPLIT) && !W4S_K32;
  const int uread = DUP ? k * 16 + m : (k * 16 + m) * CG;

  // acc[i][jj][g]: point (row i, or 3 RH + i in a quadrant; column 3 HF + jj) of output-channel
  // group g
  f32x4 acc[NR][3][CG];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
#pragma unroll
      for (int g = 0; g < CG; ++g) acc[i][jj][g] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the bias of the channel groups this lane finishes in the epilogue, loaded now (a load
  // there would wait a global round trip between the two LDS phases)
  float bpre[QUAD ? 1 : CG / 2];
#pragma unroll
  for (int k = 0; k < (QUAD ? 1 : CG / 2); ++k)
    bpre[k] = P.bias ? P.bias[co0 + (QUAD ? 2 * RH + HF : 2 * k + HF) * 16 + (lane & 15)] : 0.0f;
  if (SA_W4_PRIO && HF == 1) __builtin_amdgcn_s_setprio(1);   // static priority for waves 4-7
  if (SA_W4_DIAG != 4 && !pre) issue_p0();
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
      atab[c] = make_float2(sc, t0 - m0 * sc);
    }
    __syncthreads();
  }
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][8] = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = (kc + par) & 1;
    if constexpr (AFF) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this lane's DMAs of chunk kc landed
      float *pbuf = smem + cur * BUF;
#pragma unroll
      for (int j = 0; j < PDMA; ++j) {
        if (pc[j] >= 0) {
          f32x4 *q = reinterpret_cast<f32x4 *>(pbuf + ((wv + NWAVE * j) * 64 + lane) * 4);
          const float2 ab = atab[kc * KC + pc[j]];
          f32x4 v = *q;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * ab.x + ab.y, act_floor);
          *q = v;
        }
      }
    }
    if (SA_W4_DIAG < 3 || AFF) __syncthreads();   // chunk kc landed (vmcnt(0) precedes the barrier); buffer cur ^ 1 is free
#ifdef SA_W4_CLOCK
    if (kc == 0 && HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][4] = __builtin_amdgcn_s_memtime();
#endif
    if (SA_W4_DIAG == 2 || (SA_W4_DIAG == 0 && !SA_W4_SPREAD))
      if (kc + 1 < nchunks) issue(kc + 1, cur ^ 1);
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
      for (int i = 0; i < NR; ++i)
        if constexpr (SPLIT && W4S_K32) {   // the K = 32 filter image [point][k][n][g][s], per channel
          const float *q = smem + cur * BUF + PBUF + (k * 16 + m) * 4 + (6 * i + 3 * HF + jj) * 256 + s;
          b[i] = f32xg{q[0], q[2]};
        } else if constexpr (DUP) {   // (the redo kernel's fp32 products on the [g][k][n] image)
          const float *q = ub + ((6 * i + 3 * HF + jj) * JPC + s) * SB;
          b[i] = f32xg{q[0], q[64]};
        } else {
          b[i] = *reinterpret_cast<const f32xg *>(ub + ((6 * (QUAD ? 3 * RH + i : i) + 3 * HF + jj) * JPC + s) * SB);
        }
    };
    if constexpr (SPLIT && W4S_K32 && ((!GATED && !AFF) || W4S_K32 >= 2)) {   // (the gated and input-transform kernels keep the per-channel form: with it they do not spill)
      // Both jobs' row passes, then per point column one v_mfma_f32_16x16x32_f16 per output
      // group over the lane's two channels (k, k + 4): half the MFMAs of the per-channel form
      // and one 64-bit register copy per group for the B operand's repeat.  The filter image is
      // [point][k][n][g][s] (sa_conv2d_wino4_weights_split): a lane's (p_s0, p_s1) pair of a
      // group is one ds_read_b64.
      const float *us = smem + cur * BUF + PBUF + (k * 16 + m) * 4;
      float t0[6][3], t1[6][3];
      load_rows(0, 0, 6);
      if (W4S_K32 == 3) {
        // channel k + 4's rows go out into the slots channel k's row pass has consumed, in
        // two halves, so their reads overlap that row pass instead of following it
#pragma unroll
        for (int r = 0; r < 3; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t0[r]);
        load_rows(1, 0, 3);
#pragma unroll
        for (int r = 3; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t0[r]);
        load_rows(1, 3, 6);
      } else {
#pragma unroll
        for (int r = 0; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t0[r]);
        load_rows(1, 0, 6);
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t1[r]);
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        float v0[6], v1[6];
        bt6(t0[0][jj], t0[1][jj], t0[2][jj], t0[3][jj], t0[4][jj], t0[5][jj], v0);
        bt6(t1[0][jj], t1[1][jj], t1[2][jj], t1[3][jj], t1[4][jj], t1[5][jj], v1);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const float *pp = us + (6 * i + 3 * HF + jj) * 256;
          const f32x2 q0 = *reinterpret_cast<const f32x2 *>(pp), q1 = *reinterpret_cast<const f32x2 *>(pp + 2);
          const f16x8 a = w4_split2(v0[i], v1[i]);
          if (W4S_K32 >= 2) {
            // paired: the B operand (p_s0, p_s1) of a group as loaded (no copies), once with the
            // hi halves (hi0, hi0, hi1, hi1) and once with the lo halves of both channels
            const f16x4 ah = __builtin_shufflevector(a, a, 0, 1, 2, 3), al = __builtin_shufflevector(a, a, 4, 5, 6, 7);
            const f16x4 b0 = __builtin_bit_cast(f16x4, q0), b1 = __builtin_bit_cast(f16x4, q1);
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, b0, acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, b1, acc[i][jj][1], 0, 0, 0);
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x16f16(al, b0, acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x16f16(al, b1, acc[i][jj][1], 0, 0, 0);
          } else {
            const f16x8 b0 = __builtin_bit_cast(f16x8, f32x4{q0.x, q0.y, q0.x, q0.y});
            const f16x8 b1 = __builtin_bit_cast(f16x8, f32x4{q1.x, q1.y, q1.x, q1.y});
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b0, acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b1, acc[i][jj][1], 0, 0, 0);
          }
        }
#if SA_W4_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
        if (SA_W4_DIAG == 0 && SA_W4_SPREAD && kc + 1 < nchunks) {
          issue_part(kc + 1, cur ^ 1, jj);
#if SA_W4_FENCE
          __builtin_amdgcn_sched_barrier(0);
#endif
        }
      }
      continue;
    }
    if constexpr (DUP && SPLIT) {
      const unsigned ua = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float *)ub;
      f32x2 P[6][2];   // the current column's pairs; points 0-2 / 3-5 refilled for the next column
      auto ldp = [&](int s, int jj, int i0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = i0; i < i0 + 3; ++i)
#pragma unroll
          for (int g = 0; g < 2; ++g) P[i][g] = w4_lds_dup_rt<143>(ua, ((6 * i + 3 * HF + jj) * JPC + s) * 2 + g);
      };
      load_rows(0, 0, 6);
      ldp(0, 0, 0);
      ldp(0, 0, 3);
#pragma unroll
      for (int s = 0; s < JPC; ++s) {
        if (s == 1) load_rows(1, 3, 6);
        float t[6][3];
#pragma unroll
        for (int r = 0; r < 6; ++r) bt6h<HF>(ra[r].y, rb[r].x, rb[r].y, rb[r].z, rb[r].w, rc[r].x, t[r]);
        if (s + 1 < JPC) load_rows(1, 0, 3);
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          const bool more = s + 1 < JPC || jj < 2;
          const int ns = jj < 2 ? s : s + 1, njj = jj < 2 ? jj + 1 : 0;
          if (SA_W4_DMA_AT == 1 && SA_W4_DIAG == 0 && SA_W4_SPREAD && s == 0 && kc + 1 < nchunks) {
            issue_part(kc + 1, cur ^ 1, jj);
#if SA_W4_FENCE
            __builtin_amdgcn_sched_barrier(0);
#endif
          }
          float v[6];
          bt6(t[0][jj], t[1][jj], t[2][jj], t[3][jj], t[4][jj], t[5][jj], v);
          f16x4 a[6];
#pragma unroll
          for (int i = 0; i < 6; ++i) a[i] = w4_split(v[i]);
          w4_lds_wait3<6>(P[0][0], P[0][1], P[1][0], P[1][1], P[2][0], P[2][1]);   // points 3-5's pairs may stay out
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x16f16(a[i], __builtin_bit_cast(f16x4, P[i][0]), acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x16f16(a[i], __builtin_bit_cast(f16x4, P[i][1]), acc[i][jj][1], 0, 0, 0);
          }
#if SA_W4_FENCE
          __builtin_amdgcn_sched_barrier(0);
#endif
          if (more) ldp(ns, njj, 0);
          if (more)
            w4_lds_wait3<6>(P[3][0], P[3][1], P[4][0], P[4][1], P[5][0], P[5][1]);   // the refill of 0-2 may stay out
          else
            w4_lds_wait3<0>(P[3][0], P[3][1], P[4][0], P[4][1], P[5][0], P[5][1]);
#pragma unroll
          for (int i = 3; i < 6; ++i) {
            acc[i][jj][0] = __builtin_amdgcn_mfma_f32_16x16x16f16(a[i], __builtin_bit_cast(f16x4, P[i][0]), acc[i][jj][0], 0, 0, 0);
            acc[i][jj][1] = __builtin_amdgcn_mfma_f32_16x16x16f16(a[i], __builtin_bit_cast(f16x4, P[i][1]), acc[i][jj][1], 0, 0, 0);
          }
#if SA_W4_FENCE
          __builtin_amdgcn_sched_barrier(0);
#endif
          if (more) ldp(ns, njj, 3);
          if (SA_W4_DMA_AT == 0 && SA_W4_DIAG == 0 && SA_W4_SPREAD && s == 0 && kc + 1 < nchunks) {
            issue_part(kc + 1, cur ^ 1, jj);
#if SA_W4_FENCE
            __builtin_amdgcn_sched_barrier(0);
#endif
          }
        }
      }
      continue;
    }
    load_rows(0, 0, 6);
    load_b(0, 0, bc);
#pragma unroll
    for (int s = 0; s < JPC; ++s) {
      if (s == 1) load_rows(1, 3, 6);
      if (SA_W4_DMA_AT == 3 && SA_W4_DIAG == 0 && SA_W4_SPREAD && s == 0 && kc + 1 < nchunks) {
        issue_part(kc + 1, cur ^ 1, 0);
#if SA_W4_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
      }
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
        if (SA_W4_DMA_AT >= 1 && SA_W4_DIAG == 0 && SA_W4_SPREAD && s == 0 && kc + 1 < nchunks) {
          if (SA_W4_DMA_AT == 1) issue_part(kc + 1, cur ^ 1, jj);
          if (SA_W4_DMA_AT == 2 && jj == 0) issue(kc + 1, cur ^ 1);
          if (SA_W4_DMA_AT == 3 && jj < 2) issue_part(kc + 1, cur ^ 1, jj + 1);
#if SA_W4_FENCE
          __builtin_amdgcn_sched_barrier(0);
#endif
        }
        if (SA_W4_DIAG != 7 && (s + 1 < JPC || jj < 2)) load_b(jj < 2 ? s : s + 1, jj < 2 ? jj + 1 : 0, bn);
        float v[6];
        if (SA_W4_DIAG == 5 || SA_W4_DIAG == 8) {   // timing only: no column pass
#pragma unroll
          for (int i = 0; i < NR; ++i) v[i] = t[i][jj];
        } else if constexpr (QUAD) {
          bt6h<RH>(t[0][jj], t[1][jj], t[2][jj], t[3][jj], t[4][jj], t[5][jj], v);
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
              acc[i][jj][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[i], C::UNSPLIT ? w4_unsplit(bc[i][g]) : bc[i][g],
                                                                    acc[i][jj][g], 0, 0, 0);
        }
#if SA_W4_FENCE
        __builtin_amdgcn_sched_barrier(0);   // bound the scheduler's hoisting (register pressure)
#endif
        if (SA_W4_DMA_AT == 0 && SA_W4_DIAG == 0 && SA_W4_SPREAD && s == 0 && kc + 1 < nchunks) {
          issue_part(kc + 1, cur ^ 1, jj);
#if SA_W4_FENCE
          __builtin_amdgcn_sched_barrier(0);
#endif
        }

#pragma unroll
        for (int i = 0; i < NR; ++i) bc[i] = bn[i];
      }
    }
  }
  __syncthreads();
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][5] = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (SPLIT || C::UNSPLIT) {   // the filters' 2^W4S_LOG2 (exact)
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
#pragma unroll
        for (int g = 0; g < CG; ++g) acc[i][jj][g] *= 1.0f / (1 << W4S_LOG2);
  }

#ifndef SA_W4_P2PASS
#define SA_W4_P2PASS 1   // 0 (diagnostic, with SA_W4_PF=0 only): the one-shot epilogue in persistent items
#endif
  if constexpr (PERSIST && SA_W4_P2PASS) {
    // Persistent item: the next item's chunk 0 is landing in the other buffer, so the outputs
    // are staged one 16-channel group at a time in this item's last buffer (16 planes of OPP
    // fit in BUF).  Group g is finished by half HF == g: both halves form their partial of g
    // in registers, half 1 - g stages its own, half g adds it (same order as below: p1 + p0),
    // then the group is emitted.
    static_assert(!QUAD && CG == 2 && 16 * OPP <= BUF, "persistent shape: 8 waves x 32 channels");
    // the next item's chunk 0 into the buffer after this item's last one (free since the last
    // chunk's barrier); issued here, not inside the last chunk, where the MFMA loop's registers
    // are live (the address math there spilled)
    if (SA_W4_PF && has_next) w4_issue_chunk0<C>(NP, nwid, smem + ((nchunks + par) & 1) * BUF, wv, lane);
    float *ot = smem + ((nchunks - 1 + par) & 1) * BUF;
    const int relu = P.relu;
    const int col = lane & 15;
#pragma unroll
    for (int g = 0; g < CG; ++g) {
      // this half's partial of group g at tile i (of the lane's 4), output rows 0-3
      auto partial = [&](int i, f32x4 *y) __attribute__((always_inline)) {
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
          if (HF == 0) {
            const float p = u[a][1] + u[a][2], q = u[a][1] - u[a][2];
            y[a] = f32x4{u[a][0] + p, q, p, q};
          } else {
            const float p = u[a][0] + u[a][1], q = u[a][0] - u[a][1];
            y[a] = f32x4{p, 2.0f * q, 4.0f * p, 8.0f * q + u[a][2]};
          }
        }
      };
      auto slot = [&](int i, int a) __attribute__((always_inline)) {
        const int ti = tg * 16 + w4_tile_of_row(4 * (lane >> 4) + i), orow = (ti >> ltw) * 4, ocol = (ti & (tw - 1)) * 4;
        return reinterpret_cast<f32x4 *>(ot + col * OPP + (orow + a) * BW + ocol);
      };
      if (HF != g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 y[4];
          partial(i, y);
#pragma unroll
          for (int a = 0; a < 4; ++a) *slot(i, a) = y[a];
        }
      }
      __syncthreads();
      if (HF == g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 y[4];
          partial(i, y);
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            f32x4 *o = slot(i, a);
            f32x4 v = (HF == 0 ? (*o + y[a]) : (y[a] + *o)) + bpre[0];
            if (relu) v = f32x4{fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f)};
            *o = v;
          }
        }
      }
      __syncthreads();
      w4_emit<C, GATED, 16>(P, gate, ot, 16 * g, n, co0, st, tiles_w, y0, x0, BH, BW, ltw + 2, tid);
      if (g + 1 < CG) __syncthreads();
    }
    return;
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
  if constexpr (GATED && !QUAD && C::CO == 32 && C::NTHR == 512)
    if (gate->mode == 3 && tid < C::CO * 9) whead = gate->head_w[co0 * 9 + tid];
  if constexpr (QUAD) {
    // Quadrant (RH, HF) contributes A_RH^T M_q A_HF (at6h along each, over its 3 x 3 points).
    // The four partials of a channel group meet in LDS in a rotation: in phase p quadrant
    // q = 2 RH + HF handles group (q + 1 + p) % 4 (store, add, add, then its own group: add,
    // bias, ReLU), so each group plane has one writer per phase.
    constexpr int QD = 2 * RH + HF;
#pragma unroll
    for (int phase = 0; phase < 4; ++phase) {
      const int g = (QD + 1 + phase) & 3;
      const int col = g * 16 + (lane & 15);
      const float bv = phase == 3 ? bpre[0] : 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ti = tg * 16 + w4_tile_of_row(4 * (lane >> 4) + i), orow = (ti >> ltw) * 4, ocol = (ti & (tw - 1)) * 4;
        f32x4 u[3];
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) u[jj] = at6h<RH>(acc[0][jj][g][i], acc[1][jj][g][i], acc[2][jj][g][i]);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const f32x4 y = at6h<HF>(u[0][a], u[1][a], u[2][a]);
          f32x4 *o = reinterpret_cast<f32x4 *>(ot + col * OPP + (orow + a) * BW + ocol);
          if (phase == 0) {
            *o = y;
          } else if (phase < 3) {
            *o = *o + y;
          } else {
            f32x4 v = (*o + y) + bv;
            if (relu) v = f32x4{fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f)};
            *o = v;
          }
        }
      }
      if (phase < 3) __syncthreads();
    }
  } else {
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
  }
#ifdef SA_W4_CLOCK
  if (HF == 0 && tid == 0) g_w4_clock[blockIdx.x & 65535][6] = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (SPLIT) {
    // Range guard: an f16 operand overflow (|V| >= 65520: hi = inf, lo = -inf) makes every product
    // of that value NaN, and so the staged outputs it feeds (checked before the ReLU).  Such a
    // block writes nothing (its epilogue may update h in place) and queues itself for
    // wino_f4k3_redo_kernel, which recomputes it on fp32 MFMA products right after this launch.
    // Genuine NaN inputs take the same path and give the fp32 kernel's NaN.  One int per wave past
    // the output planes and the flow head's taps (nothing else uses that LDS after the main loop).
    static_assert(C::CO * C::OPP + C::CO * 9 + NWAVE <= C::SMEM, "range guard flags");
    int *flags = reinterpret_cast<int *>(smem + C::CO * C::OPP + C::CO * 9);
    const float t = (chk.x + chk.y) + (chk.z + chk.w);
    const bool wbad = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(t)) != 0;
    if (lane == 0) flags[wv] = wbad ? 1 : 0;
    __syncthreads();
    int any = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) any |= flags[w];
    if (any) {
      if (tid == 0 && redo) {
        const unsigned slot = atomicAdd(redo, 1u);
        if (slot < redo_cap) redo[1 + slot] = redo_tag;
      }
      return;
    }
  } else {
    __syncthreads();
  }
  if constexpr (GATED && !QUAD && C::CO == 32 && C::NTHR == 512) {
    if (gate->mode == 3) {
      w4_flowhead<C, LTW>(P, *gate, smem, n, co0, st, y0, x0, tid, whead);
      return;
    }
  }
  w4_emit<C, GATED, C::CO>(P, gate, ot, 0, n, co0, st, tiles_w, y0, x0, BH, BW, ltw + 2, tid);
}

template <class C, bool GATED, bool AFF = false>
__global__ __launch_bounds__(C::NTHR, C::NW == 8 || C::CO == 64 ? 1 : 2) void wino_f4k3_kernel(const W4Launch L) {
  // problem of the block from its raw id (ranges padded to multiples of 8: every XCD gets an
  // equal share of each problem), then the L2-locality remap within it (conv2d_wino.hip)
  const unsigned g = blockIdx.x;
  // the problem index from the range ends alone, then only that problem's fields are loaded
  // (selecting among all eight by value loaded every one of them: ~70 scalar loads before the
  // first DMA)
  int pi = 0;
#pragma unroll
  for (int i = 1; i < MAX_PROB; ++i) pi += (i < L.nprob && g >= L.end[i - 1]) ? 1 : 0;
  const W4Prob &P = L.p[pi];
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
  const W4Gate *gp = GATED ? &L.gate[pi] : nullptr;
  if constexpr (C::QUAD) {   // quadrant 2 RH + HF = wave / TG
    const int qd = threadIdx.x / (C::NTHR / 4);
#define SA_W4_Q(HF_, RH_)                                                   \
  (P.ltw == 4 ? w4_body<C, HF_, 4, GATED, AFF, RH_>(P, gp, wid, smem, atab) \
              : w4_body<C, HF_, 5, GATED, AFF, RH_>(P, gp, wid, smem, atab))
    if (qd == 0) SA_W4_Q(0, 0);
    else if (qd == 1) SA_W4_Q(1, 0);
    else if (qd == 2) SA_W4_Q(0, 1);
    else SA_W4_Q(1, 1);
#undef SA_W4_Q
  } else {
    const unsigned tag = ((unsigned)pi << 27) | wid;
#define SA_W4_B(HF_, LTW_) \
  w4_body<C, HF_, LTW_, GATED, AFF>(P, gp, wid, smem, atab, 0, false, false, W4Prob{}, 0, L.redo, L.redo_cap, tag)
    if (threadIdx.x < C::NTHR / 2) {
      if (P.ltw == 4) SA_W4_B(0, 4);
      else SA_W4_B(0, 5);
    } else {
      if (P.ltw == 4) SA_W4_B(1, 4);
      else SA_W4_B(1, 5);
    }
#undef SA_W4_B
  }
#ifdef SA_W4_CLOCK
  if (threadIdx.x == 0 && g < 65536) {
    g_w4_clock[g][0] = t0;
    g_w4_clock[g][1] = r0;
    g_w4_clock[g][2] = __builtin_amdgcn_s_memtime();
    g_w4_clock[g][3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// Persistent variant of the 8-wave shape: one block per CU walks the launch's work items
// g = blockIdx.x, blockIdx.x + gridDim.x, ... (gridDim.x a multiple of 8, so an item stays on the
// XCD the one-shot grid would put it on, and the L2-locality remap is unchanged).  Each item
// issues the next item's chunk 0 as its main loop ends (w4_issue_chunk0), so the first-chunk
// wait of every item but the block's first is hidden under the previous item's epilogue.
// The split kernel's range guard, finished: one workgroup recomputes, on fp32 MFMA products (the
// split filters read as hi + lo), every block the preceding split launch queued in L.redo (the list
// holds every block of the launch), then clears the count.  Launched after every guarded split
// launch on its stream; with nothing queued it reads one word and exits.
template <class C, bool GATED, bool AFF>
__global__ __launch_bounds__(C::NTHR, 1) void wino_f4k3_redo_kernel(const W4Launch L) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  __shared__ float2 atab[AFF ? C::AFF_MAX : 1];
  const unsigned n = __atomic_load_n(L.redo, __ATOMIC_RELAXED);
  if (n == 0) return;
  const unsigned total = n < L.redo_cap ? n : L.redo_cap;
  unsigned done = 0;
  for (unsigned i = 0; i < total; ++i) {
    const unsigned tag = L.redo[1 + i];
    const int pi = (int)(tag >> 27);
    const unsigned wid = tag & ((1u << 27) - 1u);
    const W4Prob &P = L.p[pi];
    const W4Gate *gp = GATED ? &L.gate[pi] : nullptr;
    __syncthreads();   // the previous block's LDS use is over
    if (threadIdx.x < C::NTHR / 2) {
      if (P.ltw == 4) w4_body<C, 0, 4, GATED, AFF>(P, gp, wid, smem, atab);
      else w4_body<C, 0, 5, GATED, AFF>(P, gp, wid, smem, atab);
    } else {
      if (P.ltw == 4) w4_body<C, 1, 4, GATED, AFF>(P, gp, wid, smem, atab);
      else w4_body<C, 1, 5, GATED, AFF>(P, gp, wid, smem, atab);
    }
    ++done;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&g_w4_redo_blocks, done);
    __atomic_store_n(L.redo, 0u, __ATOMIC_RELAXED);
  }
}

template <class C, bool GATED, bool AFF = false>
__global__ __launch_bounds__(C::NTHR, 1) void wino_f4k3_persist_kernel(const W4Launch L) {
  static_assert(C::NW == 8 && C::CO == 32 && !C::QUAD, "persistent: the 8-wave 32-channel shape");
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  __shared__ float2 atab[AFF ? C::AFF_MAX : 1];
  const unsigned total = L.end[MAX_PROB - 1], G = gridDim.x;
  auto locate = [&](const unsigned g, int &pi, unsigned &wid) __attribute__((always_inline)) {
    pi = 0;
#pragma unroll
    for (int i = 1; i < MAX_PROB; ++i) pi += (i < L.nprob && g >= L.end[i - 1]) ? 1 : 0;
    const unsigned base = pi ? L.end[pi - 1] : 0u, nb = L.nblk[pi];
    if (g - base >= nb) return false;   // padding of a problem's range to a multiple of 8
    wid = sa::xcd_remap(g - base, nb);
    return true;
  };
  auto next_valid = [&](unsigned g, int &pi, unsigned &wid) __attribute__((always_inline)) {
    while (g < total && !locate(g, pi, wid)) g += G;
    return g;
  };
  int pi = 0, pi2 = 0;
  unsigned wid = 0, wid2 = 0;
  unsigned g = next_valid(blockIdx.x, pi, wid);
  int par = 0;
  bool pre = false;
  while (g < total) {
    const unsigned g2 = next_valid(g + G, pi2, wid2);
    const W4Prob &P = L.p[pi];
    // (a reference, not a pointer that may be null: a null-or-kernarg pointer made the compiler
    // copy the whole launch struct to scratch)
    const bool has_next = g2 < total;
    const W4Prob &NP = L.p[pi2];
    const W4Gate *gp = GATED ? &L.gate[pi] : nullptr;
    // wave-uniform (readfirstlane): a branch on threadIdx.x would be divergent to the compiler,
    // and the item loop's carried state would then live in VGPRs
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < C::NW / 2) {
      if (P.ltw == 4) w4_body<C, 0, 4, GATED, AFF, 0, true>(P, gp, wid, smem, atab, par, pre, has_next, NP, wid2);
      else w4_body<C, 0, 5, GATED, AFF, 0, true>(P, gp, wid, smem, atab, par, pre, has_next, NP, wid2);
    } else {
      if (P.ltw == 4) w4_body<C, 1, 4, GATED, AFF, 0, true>(P, gp, wid, smem, atab, par, pre, has_next, NP, wid2);
      else w4_body<C, 1, 5, GATED, AFF, 0, true>(P, gp, wid, smem, atab, par, pre, has_next, NP, wid2);
    }
    par = (par + P.Cin / C::KC) & 1;
    pre = SA_W4_PF && has_next;
    g = g2;
    pi = pi2;
    wid = wid2;
  }
}

int w4_num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
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
// pair hi = f16(u), lo = f16(u - hi) in one dword (hi in the low half): for the K = 32 form
// [Cout/32][Cin/8][36][4][16][2][2] (channel 8 chunk + 4 s + k, output co = 32 cb + 16 g + n at
// [k][n][g][s]), otherwise in the fp32 filters' layout (wino4_weights_kernel).
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
      if (W4S_K32)   // [Cout/32][Cin/8][36][4][16][2][2]: channel 8 chunk + 4 s + k at [k][n][g][s]
        U[(((((long)cb * (Cin / 8) + chunk) * NPT + pt) * 4 + k) * 16 + n) * 4 + gg * 2 + s] = pr;
      else if (SA_W4_DUP)   // [Cout/32][Cin/8][36][2][2][4][16]: [g][k][n] per point and job
        U[(((((long)cb * (Cin / 8) + chunk) * NPT + pt) * 2 + s) * 2 + gg) * 64 + k * 16 + n] = pr;
      else
        U[(((((long)cb * (Cin / 8) + chunk) * NPT + pt) * 2 + s) * 4 + k) * 32 + n * 2 + gg] = pr;
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

extern "C" int sa_conv2d_wino4_weights_cb(const float *weight, int Cout, int Cin, int co_block, float *U,
                                          void *stream) {
  SA_REQUIRE(co_block == 32 || co_block == 64, "sa_conv2d_wino4_weights: co_block 32 or 64");
  SA_REQUIRE(weight && U && Cout > 0 && Cin > 0 && Cin % 8 == 0 && Cout % co_block == 0,
             "sa_conv2d_wino4_weights: bad arguments (Cin %% 8, Cout %% %d)", co_block);
  const long n = (long)Cout * Cin;
  hipStream_t s = sa::as_stream(stream);
  wino4_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, co_block, U);
  return sa::check_launch("sa_conv2d_wino4_weights");
}

extern "C" int sa_conv2d_wino4_weights(const float *weight, int Cout, int Cin, float *U, void *stream) {
  return sa_conv2d_wino4_weights_cb(weight, Cout, Cin, 32, U, stream);
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
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w4_clock), sizeof(unsigned long long) * 10 * n) == hipSuccess ? 0 : -1;
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

// blocks of the split kernels (F(4x4) and direct) that the range guard recomputed on fp32 MFMA
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
  return sa_conv2d_k3_wino4_launch(nprob, probs, gates, block_shape, nullptr, 0, stream);
}

extern "C" int sa_conv2d_k3_wino4_launch(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates,
                                         int block_shape, unsigned *redo_ws, long redo_cap, void *stream) {
  SA_REQUIRE(nprob >= 1 && nprob <= MAX_PROB && probs, "sa_conv2d_k3_wino4_multi: 1..%d problems", MAX_PROB);
  SA_REQUIRE(block_shape >= 0 && block_shape <= 7, "sa_conv2d_k3_wino4_multi: block_shape 0..7");
  // Large blocks unless the caller asks for small ones (block_shape 2) or wide ones (3: 64
  // output channels per block, filters from sa_conv2d_wino4_weights_cb(..., 64, ...)).  The
  // small shape measured 2-8% faster on standalone launches of Cin <= 128 with a few rounds of
  // blocks (qh08, convc2) but not faster in the forward as a blanket choice.
  // block_shape 4: the quadrant shape (W4Quad), also on the 64-channel filter layout
  // block_shape 6: the split kernel (W4Split; filters from sa_conv2d_wino4_weights_split)
  // block_shape 7: the split kernel on the 4-wave shape (W4SplitSmall, the same split filters)
  const bool small = block_shape == 2, wide = block_shape == 3, quad = block_shape == 4, persist = block_shape == 5,
             split = block_shape == 6, split_small = block_shape == 7;
  const int nt = small || wide || quad || split_small ? W4Small::NT : W4Big::NT;
  const int CO = wide || quad ? 64 : 32;
  const int aff_max = small ? W4Small::AFF_MAX : quad ? W4Quad::AFF_MAX : split ? W4Split::AFF_MAX
                    : split_small ? W4SplitSmall::AFF_MAX : W4Big::AFF_MAX;
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
    SA_REQUIRE(!qaff || (!wide && q.Cin <= aff_max),
               "sa_conv2d_k3_wino4: an input transform needs the 8-wave, quadrant or 4-wave shape and Cin <= %d",
               aff_max);
    aff = aff || qaff;
    SA_REQUIRE((long)q.Cin * q.H * pitch * 4 < (1L << 31) - 64 && 36L * q.Cin * q.Cout * 4 < (1L << 31),
               "sa_conv2d_k3_wino4: an image or the filter bank exceeds the 2 GB buffer-descriptor range");
    const int ltw = w4_ltw(q.H, q.W), bw = 4 << ltw, bh = 4 * (nt >> ltw);
    const int tiles_w = (q.W + bw - 1) / bw, tiles_h = (q.H + bh - 1) / bh;
    L.p[i] = W4Prob{q.in, q.in_bs, q.Cin, q.H, q.W, q.U, q.Cout, q.bias, q.relu, q.out, q.out_bs,
                    ltw, tiles_w, tiles_w * tiles_h, q.Cout / CO, q.stats_partial,
                    q.in_m, q.in_s, q.in_t, q.in_pstride, q.in_act, pitch, q.N * tiles_w * tiles_h};
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
  // the split kernel's range guard: blocks whose operands overflowed queue themselves in redo_ws and
  // the redo kernel recomputes them on fp32 products (the list holds every block of the launch)
  const bool guard = (split || split_small) && redo_ws;
  if (guard) {
    SA_REQUIRE(redo_cap >= total && (reinterpret_cast<uintptr_t>(redo_ws) & 3) == 0,
               "sa_conv2d_k3_wino4: the redo workspace holds %ld entries, the launch has %ld blocks", redo_cap, total);
    L.redo = redo_ws;
    L.redo_cap = (unsigned)redo_cap;
  }
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV2D_W4, s);
  if (persist) {
    // one block per CU (rounded down to a multiple of 8: every block keeps its items on one XCD)
#ifndef SA_W4_PGRID
#define SA_W4_PGRID 1   // 0: one block per work item (timing diagnostic of the persistent code path)
#endif
    const unsigned grid = SA_W4_PGRID ? (unsigned)std::min<long>(total, std::max(8, w4_num_cus() / 8 * 8))
                                      : (unsigned)total;
    aff     ? wino_f4k3_persist_kernel<W4Big, false, true><<<grid, W4Big::NTHR, 0, s>>>(L)
    : gated ? wino_f4k3_persist_kernel<W4Big, true><<<grid, W4Big::NTHR, 0, s>>>(L)
            : wino_f4k3_persist_kernel<W4Big, false><<<grid, W4Big::NTHR, 0, s>>>(L);
  } else if (split) {
    aff     ? wino_f4k3_kernel<W4Split, false, true><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L)
    : gated ? wino_f4k3_kernel<W4Split, true><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L)
            : wino_f4k3_kernel<W4Split, false><<<(unsigned)total, W4Split::NTHR, 0, s>>>(L);
    if (guard)
      aff     ? wino_f4k3_redo_kernel<W4SplitRedo, false, true><<<1, W4SplitRedo::NTHR, 0, s>>>(L)
      : gated ? wino_f4k3_redo_kernel<W4SplitRedo, true, false><<<1, W4SplitRedo::NTHR, 0, s>>>(L)
              : wino_f4k3_redo_kernel<W4SplitRedo, false, false><<<1, W4SplitRedo::NTHR, 0, s>>>(L);
  } else if (split_small) {
    aff     ? wino_f4k3_kernel<W4SplitSmall, false, true><<<(unsigned)total, W4SplitSmall::NTHR, 0, s>>>(L)
    : gated ? wino_f4k3_kernel<W4SplitSmall, true><<<(unsigned)total, W4SplitSmall::NTHR, 0, s>>>(L)
            : wino_f4k3_kernel<W4SplitSmall, false><<<(unsigned)total, W4SplitSmall::NTHR, 0, s>>>(L);
    if (guard)
      aff     ? wino_f4k3_redo_kernel<W4SplitRedoSmall, false, true><<<1, W4SplitRedoSmall::NTHR, 0, s>>>(L)
      : gated ? wino_f4k3_redo_kernel<W4SplitRedoSmall, true, false><<<1, W4SplitRedoSmall::NTHR, 0, s>>>(L)
              : wino_f4k3_redo_kernel<W4SplitRedoSmall, false, false><<<1, W4SplitRedoSmall::NTHR, 0, s>>>(L);
  }
  else if (quad)
    aff     ? wino_f4k3_kernel<W4Quad, false, true><<<(unsigned)total, W4Quad::NTHR, 0, s>>>(L)
    : gated ? wino_f4k3_kernel<W4Quad, true><<<(unsigned)total, W4Quad::NTHR, 0, s>>>(L)
            : wino_f4k3_kernel<W4Quad, false><<<(unsigned)total, W4Quad::NTHR, 0, s>>>(L);
  else if (aff && small)
    wino_f4k3_kernel<W4Small, false, true><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L);
  else if (aff)
    wino_f4k3_kernel<W4Big, false, true><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L);
  else if (small)
    gated ? wino_f4k3_kernel<W4Small, true><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L)
          : wino_f4k3_kernel<W4Small, false><<<(unsigned)total, W4Small::NTHR, 0, s>>>(L);
  else if (wide)
    gated ? wino_f4k3_kernel<W4Wide, true><<<(unsigned)total, W4Wide::NTHR, 0, s>>>(L)
          : wino_f4k3_kernel<W4Wide, false><<<(unsigned)total, W4Wide::NTHR, 0, s>>>(L);
  else
    gated ? wino_f4k3_kernel<W4Big, true><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L)
          : wino_f4k3_kernel<W4Big, false><<<(unsigned)total, W4Big::NTHR, 0, s>>>(L);
  return sa::check_launch("sa_conv2d_k3_wino4");
}
