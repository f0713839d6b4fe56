// 3x3 / stride 1 / pad 1 convolution as fused Winograd F(2x2, 3x3) on fp32 MFMA.
//
// The 2-D convolutions of the encoders and the update block (extractor.py:6-300,
// update.py:46-110) are ~3/4 of the forward's time; MIOpen runs them as its assembly
// Winograd f2x3 kernels or NHWC implicit GEMM (+ layout transposes) at ~110 TF/s
// direct-equivalent.  This kernel does the whole Winograd pipeline per block:
//
//   block  = 8 waves, output tile 8 x 32 pixels (64 Winograd tiles of 2x2) x 32 channels
//   chunk  = 8 input channels: the 10 x 34 input patch -> LDS, input transform
//            V = B^T d B (one (channel, tile) per thread) -> LDS as V[xi][ci][tile],
//            transformed filters U[xi][ci][co] (sa_conv2d_wino_weights) -> LDS;
//            the next chunk's global loads are in flight while this one multiplies
//   MFMA   = v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate): wave w owns
//            16 tiles (one tile row) x 16 output channels for all 16 transform points,
//            so the output transform Y = A^T M A runs in registers
//   store  = + bias, optional ReLU, through LDS as 32-float rows (coalesced)
//
// 16 multiplies per 2x2 outputs instead of 36: the MFMA peak (157 TF/s fp32) is 354 TF/s
// direct-equivalent.  Numerics: the same algorithm as MIOpen's f2x3 path (transform
// coefficients 0, +-1, +-1/2); filters are transformed in fp64 and rounded once.
// Block -> XCD: the 2-D grid is walked with a bijective XCD remap so that the output-channel
// blocks of one spatial tile (which read the same input patch) share an XCD's L2.
#include "sa_common.h"

#pragma clang fp contract(fast)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int OTH = 8, OTW = 32;             // output tile (pixels)
constexpr int TR = OTH / 2, TC = OTW / 2;    // Winograd tiles: 4 rows x 16 cols
constexpr int NT = TR * TC;                  // 64
constexpr int KC = 8;                        // input channels per chunk
constexpr int PH = OTH + 2, PW = OTW + 2;    // input patch 10 x 34
constexpr int XS = 36;                       // LDS row pitch of the patch
constexpr int XCP = 384;                     // LDS channel-plane pitch (>= PH * XS)
constexpr int NX = KC * PH * PW;             // 2720 patch values per chunk
constexpr int XPT = (NX + 511) / 512;        // per thread (6)

// V and U live in LDS as rows of float2 pairs (channel c and c + 4 of a chunk: the two
// k-steps of an MFMA pair, one ds_read_b64).  An operand read puts rows r and r + 1 in one
// half-wave, so odd rows are stored with column ^ 16: the two rows then fall in disjoint
// bank halves without padding (b64 bank = dword address mod 64).
__device__ __forceinline__ int swz(int row, int col, int ncol) { return row * ncol + (col ^ ((row & 1) << 4)); }

// CG output-channel groups of 16 per wave; a block has 4 tile rows x 2 channel halves of waves
// and 32 * CG output channels.  CG = 2 halves the transform work and V traffic per FMA and
// reuses each A fragment for two MFMAs.
template <int CG>
struct Wino {
  static constexpr int CO = 32 * CG;
  static constexpr int UPT = (16 * 4 * CO / 2) / 512;   // float4 of U per thread per chunk
  static constexpr int COP = CO + 2;                    // output staging O[row][x][co] pitch
  static constexpr int XSZ = KC * XCP, X_OFF = 0, V_OFF = 2 * XSZ, VSZ = 16 * 4 * NT * 2, U_OFF = V_OFF + 2 * VSZ,
                       USZ = 16 * 4 * CO * 2, SMEM = U_OFF + 2 * USZ;
  static_assert(OTH * OTW * COP <= 2 * VSZ + 2 * USZ, "output staging fits V + U");
  static_assert(SMEM * 4 <= 160 * 1024, "LDS budget");
};

#ifndef SA_WINO_SCHED
#define SA_WINO_SCHED 0
#endif

#ifndef SA_WINO_WAVES_PER_EU
#define SA_WINO_WAVES_PER_EU 2
#endif

constexpr int MAX_CIN_AFFINE = 512;

// Optional producer epilogue applied on load and statistics of the output:
//   input  v -> act(v * scale[c] + shift[c]), scale = s, shift = t - m * s, with (m, s, t)
//          per channel (pstride 0) or per (image, channel) (pstride Cin), any of them NULL =
//          0 / 1 / 0 — the previous layer's bias / BatchNorm / InstanceNorm + ReLU; zero
//          padding applies to the activated input
//   stats  per-block float64 (sum, sum^2) of every output channel for the next
//          InstanceNorm: partial[(n * Cout + co) * tiles_hw + spatial tile][2]
struct WinoIO {
  const float *m, *s, *t;
  int pstride, act;
  double *partial;
};

// one convolution of a launch; a launch carries up to MAX_PROB independent convolutions
// with the same template configuration (their blocks share the grid, so one conv's tail
// round fills with another's blocks)
struct WinoProb {
  const float *in;
  long in_bs;
  int Cin, H, W;
  const float *U;
  int Cout;
  const float *bias;
  int relu;
  float *out;
  long out_bs;
  int tiles_w, tiles_hw, co_blocks;
  WinoIO io;
};
constexpr int MAX_PROB = 8;
struct WinoLaunch {
  WinoProb p[MAX_PROB];
  unsigned end[MAX_PROB];   // end of each problem's block range, ranges padded to multiples of 8
  unsigned nblk[MAX_PROB];  // the problem's own block count
  int nprob;
};

template <int CG, bool AFF>
__device__ __forceinline__ void wino_body(const WinoProb &P, const unsigned wid) {
  const float *__restrict__ in = P.in;
  const long in_bs = P.in_bs;
  const int Cin = P.Cin, H = P.H, W = P.W, Cout = P.Cout, relu = P.relu;
  const float *__restrict__ U = P.U;
  const float *__restrict__ bias = P.bias;
  float *__restrict__ out = P.out;
  const long out_bs = P.out_bs;
  const int tiles_w = P.tiles_w, tiles_hw = P.tiles_hw, co_blocks = P.co_blocks;
  const WinoIO io = P.io;
  using Cfg = Wino<CG>;
  constexpr int CO = Cfg::CO, UPT = Cfg::UPT;
  __shared__ float smem[Cfg::SMEM];
  __shared__ float2 tab[MAX_CIN_AFFINE];   // input (scale, shift) of this image's channels
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware work order (the launch remaps block ids): consecutive work ids = the co
  // blocks of one spatial tile
  const int cb = wid % co_blocks;
  const int st = (wid / co_blocks) % tiles_hw;
  const int n = wid / (co_blocks * tiles_hw);
  const int y0 = (st / tiles_w) * OTH, x0 = (st % tiles_w) * OTW;
  const int co0 = cb * CO;
  const float *src = in + (long)n * in_bs;
  const long hw = (long)H * W;

  // ---- per-thread load slots, fixed for all chunks: 32-bit byte offsets from the chunk's
  // channel-0 plane (clamped inside the image; padding selected at commit), read with buffer
  // loads (scalar base + chunk offset, no per-load address arithmetic)
  const __amdgpu_buffer_rsrc_t xin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(src), (short)0, (int)((long)Cin * hw * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t uin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(U), (short)0, (int)(16L * Cin * Cout * 4), 0x00020000);
  constexpr bool in_aff = AFF;  // producer epilogue on load (a template flag: free when off)
  if (in_aff) {
    for (int c = tid; c < Cin; c += 512) {
      const int pi = n * io.pstride + c;
      const float m = io.m ? io.m[pi] : 0.0f, sc = io.s ? io.s[pi] : 1.0f, t = io.t ? io.t[pi] : 0.0f;
      tab[c] = make_float2(sc, t - m * sc);
    }
  }
  int xo[XPT], xl[XPT], xc[XPT];   // global byte offset, LDS slot (-1: no slot), channel in chunk
  unsigned xpad = 0;
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int i = min(tid + 512 * j, NX - 1);
    const int ci = i / (PH * PW), r = (i / PW) % PH, cc = i % PW;
    const int y = y0 - 1 + r, x = x0 - 1 + cc;
    xc[j] = ci;
    xo[j] = (ci * (int)hw + min(max(y, 0), H - 1) * W + min(max(x, 0), W - 1)) * 4;
    // without an input transform, padding taps read past the buffer's range: the load
    // returns 0 (raw buffer range check on the VGPR offset), so no select is needed
    if (!AFF && (y < 0 || y >= H || x < 0 || x >= W)) xo[j] = 0x7ffffff0;
    // threads without a slot store into the unused tail of channel 0's plane (branch-free)
    xl[j] = tid + 512 * j < NX ? ci * XCP + r * XS + cc : XCP - 1;
    if (y < 0 || y >= H || x < 0 || x >= W) xpad |= 1u << j;
  }
  // U chunk image: global [xi][Cin/8][4][Cout][2] -> LDS rows (xi, ci4) of CO swizzled pairs
  int uo[UPT], ul[UPT];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int i4 = tid + 512 * j;
    const int q = i4 % (CO / 2), row = i4 / (CO / 2);   // row = xi * 4 + ci4
    uo[j] = (((row >> 2) * (Cin / KC) * 4 + (row & 3)) * Cout * 2 + co0 * 2 + q * 4) * 4;
    ul[j] = swz(row, 2 * q, CO) * 2;
  }
  float xr[XPT];
  f32x4 ur[UPT];
  auto fetch_x = [&](int chunk) __attribute__((always_inline)) {
    const int xs = chunk * KC * (int)hw * 4;
#pragma unroll
    for (int j = 0; j < XPT; ++j) xr[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xin, xo[j], xs, 0));
  };
  auto fetch_u = [&](int chunk) __attribute__((always_inline)) {
    const int us = chunk * 4 * Cout * 2 * 4;
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const auto w = __builtin_amdgcn_raw_buffer_load_b128(uin, uo[j], us, 0);
      ur[j] = f32x4{__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]), __uint_as_float(w[3])};
    }
  };
  const float act_floor = io.act ? 0.0f : -INFINITY;   // ReLU or identity, branch-free
  auto commit_x = [&](int buf, int chunk) __attribute__((always_inline)) {
    float *sx = smem + Cfg::X_OFF + buf * Cfg::XSZ;
    const int cb = min(chunk, Cin / KC - 1) * KC;
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      float v = xr[j];
      if (in_aff) {
        const float2 p = tab[cb + xc[j]];
        v = fmaxf(v * p.x + p.y, act_floor);
      }
      if (in_aff) v = ((xpad >> j) & 1u) ? 0.0f : v;
      sx[xl[j]] = v;
    }
  };
  auto commit_u = [&](int buf) __attribute__((always_inline)) {
    float *su = smem + Cfg::U_OFF + buf * Cfg::USZ;
#pragma unroll
    for (int j = 0; j < UPT; ++j) *reinterpret_cast<f32x4 *>(su + ul[j]) = ur[j];
  };
  // input transform V = B^T d B of (channel tid >> 6, tile tid & 63) into its slot of the
  // (c, c + 4) pair image; every thread has one job per chunk.  Split in three parts so the
  // work spreads over a chunk's MFMAs: read + row pass, then the column pass and writes of
  // transform rows 0-1 and 2-3.
  float tw[4][4];
  auto transform_read = [&](int buf) __attribute__((always_inline)) {
    const int ci = tid >> 6, t = tid & 63;
    const int ty = t / TC, tx = t % TC;
    const float *p = smem + Cfg::X_OFF + buf * Cfg::XSZ + ci * XCP + 2 * ty * XS + 2 * tx;
    float d[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) d[r][c] = p[r * XS + c];
    // B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      tw[0][c] = d[0][c] - d[2][c];
      tw[1][c] = d[1][c] + d[2][c];
      tw[2][c] = d[2][c] - d[1][c];
      tw[3][c] = d[1][c] - d[3][c];
    }
  };
  auto transform_write = [&](int buf, int r0) __attribute__((always_inline)) {
    const int ci = tid >> 6, t = tid & 63;
    // rows xi * 4 + (ci & 3) all have the parity of ci & 3: one swizzled column for all xi
    float *o = smem + Cfg::V_OFF + buf * Cfg::VSZ + swz(ci & 3, t, NT) * 2 + (ci >> 2);
#pragma unroll
    for (int r = r0; r < r0 + 2; ++r) {
      o[((r * 4 + 0) * 4) * NT * 2] = tw[r][0] - tw[r][2];
      o[((r * 4 + 1) * 4) * NT * 2] = tw[r][1] + tw[r][2];
      o[((r * 4 + 2) * 4) * NT * 2] = tw[r][2] - tw[r][1];
      o[((r * 4 + 3) * 4) * NT * 2] = tw[r][1] - tw[r][3];
    }
  };
  auto transform = [&](int buf) __attribute__((always_inline)) {
    transform_read(buf);
    transform_write(buf, 0);
    transform_write(buf, 2);
  };

  f32x4 acc[16][CG];
#pragma unroll
  for (int k = 0; k < 16; ++k)
#pragma unroll
    for (int g = 0; g < CG; ++g) acc[k][g] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tg = wv & 3, ch = wv >> 2;                 // tile row, output-channel half
  const int ak = lane >> 4, am = lane & 15;            // operand lane map (16x16x4)
  // the epilogue's bias values, loaded now (there a load would wait a global round trip)
  float bpre[CG];
#pragma unroll
  for (int g = 0; g < CG; ++g) bpre[g] = bias ? bias[co0 + (ch * CG + g) * 16 + (lane & 15)] : 0.0f;
  // operand slots (float2 units) of row xi * 4 + ak: the swizzle depends on ak's parity only
  const int a_slot = swz(ak, tg * TC + am, NT);
  int b_slot[CG];
#pragma unroll
  for (int g = 0; g < CG; ++g) b_slot[g] = swz(ak, (ch * CG + g) * 16 + am, CO);

  // software pipeline, one barrier per chunk.  Chunk c lives in X[c & 1], V[c & 1], U[c & 1].
  // Iteration k: barrier | MFMA(k) || transform(k+1) | commit U(k+1), X(k+2) | loads U(k+2), X(k+3).
  // Every buffer written in iteration k was last read in iteration k-1 (before the barrier),
  // every buffer read in iteration k was written in iteration k-1.  Past the last chunk the
  // fetches re-read the last chunk (clamped: branch-free) into buffers nobody reads again.
  // The chunk's MFMAs run as 4 groups of 4 transform points (16 MFMAs); operands are read one
  // group ahead and the side work is spread over the groups, so the matrix pipe is fed while
  // both waves of a SIMD do their share of it.
  const int nchunks = Cin / KC;
  if (in_aff) __syncthreads();  // the (scale, shift) table
  // static priority for the second half of the waves (the arbitration losers of each SIMD pair)
  if (wv >= 4) __builtin_amdgcn_s_setprio(1);
  fetch_x(0);
  fetch_u(0);
  commit_x(0, 0);
  commit_u(0);
  fetch_x(min(1, nchunks - 1));
  fetch_u(min(1, nchunks - 1));
  commit_x(1, 1);
  fetch_x(min(2, nchunks - 1));
  __syncthreads();
  transform(0);
#ifndef SA_WINO_DIAG
#define SA_WINO_DIAG 0   // timing diagnostics only (wrong results): 1 no side work, 2 also no barrier
#endif
#pragma unroll 1
  for (int k = 0; k < nchunks; ++k) {
    const int cur = k & 1, nxt = cur ^ 1;
    if (SA_WINO_DIAG < 2) __syncthreads();
    const float2 *va = reinterpret_cast<const float2 *>(smem + Cfg::V_OFF + cur * Cfg::VSZ) + a_slot;
    const float2 *vb = reinterpret_cast<const float2 *>(smem + Cfg::U_OFF + cur * Cfg::USZ);
    float2 a[2][4], b[2][4][CG];
    auto load_ops = [&](int q, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[slot][i] = va[(4 * q + i) * 4 * NT];
#pragma unroll
        for (int g = 0; g < CG; ++g) b[slot][i][g] = vb[(4 * q + i) * 4 * CO + b_slot[g]];
      }
    };
    auto mfma_group = [&](int q, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < CG; ++g)
          acc[4 * q + i][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[slot][i].x, b[slot][i][g].x, acc[4 * q + i][g], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < CG; ++g)
          acc[4 * q + i][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[slot][i].y, b[slot][i][g].y, acc[4 * q + i][g], 0, 0, 0);
    };
    load_ops(0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < 3) load_ops(q + 1, (q + 1) & 1);
      if (SA_WINO_DIAG == 0) {
      if (q == 0) transform_read(nxt);
      if (q == 1) transform_write(nxt, 0);
      if (q == 2) transform_write(nxt, 2);
      if (q == 3) {
        commit_u(nxt);
        commit_x(cur, k + 2);
        fetch_u(min(k + 2, nchunks - 1));
        fetch_x(min(k + 3, nchunks - 1));
      }
      }
      mfma_group(q, q & 1);
    }
#if SA_WINO_SCHED
    // issue order of the iteration: the first group's operand reads, then every MFMA
    // followed by one LDS access and one VALU op; the global loads sit in the last quarter
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x300, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      if (i >= 48 && i < 58) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
#endif
  }
  __syncthreads();

  // ---- output transform in registers: lane holds tiles (tg, 4*(lane>>4) + r) of channel
  // (ch * CG + g) * 16 + (lane & 15); staged as O[row][x][co] for row-contiguous stores
  float *ot = smem + Cfg::V_OFF;
  constexpr int COP = Cfg::COP;
#pragma unroll
  for (int g = 0; g < CG; ++g) {
    const int col = (ch * CG + g) * 16 + (lane & 15);
    const float bv = bpre[g];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tx = 4 * (lane >> 4) + r;
      float m[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) m[a][b] = acc[a * 4 + b][g][r];
      // A^T = [[1,1,1,0],[0,1,-1,-1]]
      float t0[4], t1[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        t0[b] = m[0][b] + m[1][b] + m[2][b];
        t1[b] = m[1][b] - m[2][b] - m[3][b];
      }
      float y[2][2];
      y[0][0] = t0[0] + t0[1] + t0[2];
      y[0][1] = t0[1] - t0[2] - t0[3];
      y[1][0] = t1[0] + t1[1] + t1[2];
      y[1][1] = t1[1] - t1[2] - t1[3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v = y[i][j] + bv;
          if (relu) v = fmaxf(v, 0.0f);
          ot[((2 * tg + i) * OTW + 2 * tx + j) * COP + col] = v;
        }
    }
  }
  __syncthreads();
  if (io.partial) {
    // InstanceNorm partials of the block: TPC threads per channel, fixed-order reduction
    constexpr int TPC = 512 / CO, PPT = OTH * OTW / TPC;
    const int c = tid / TPC, part = tid % TPC;
    double ssum = 0.0, ssq = 0.0;
#pragma unroll 4
    for (int p = part * PPT; p < (part + 1) * PPT; ++p) {
      const int r = p / OTW, cx = p % OTW;
      if (y0 + r < H && x0 + cx < W) {
        const double v = ot[(r * OTW + cx) * COP + c];
        ssum += v;
        ssq += v * v;
      }
    }
#pragma unroll
    for (int o = TPC / 2; o > 0; o >>= 1) {
      ssum += __shfl_xor(ssum, o);
      ssq += __shfl_xor(ssq, o);
    }
    if (part == 0) {
      double *pp = io.partial + (((long)n * Cout + co0 + c) * tiles_hw + st) * 2;
      pp[0] = ssum;
      pp[1] = ssq;
    }
  }
  // CO channels x 8 rows x 32 columns, one row-segment of 32 floats per half-wave
  float *dst = out + (long)n * out_bs;
#pragma unroll
  for (int j = 0; j < (CO * OTH * OTW) / 512; ++j) {
    const int i = tid + 512 * j;
    const int cx = i % OTW, r = (i / OTW) % OTH, c = i / (OTW * OTH);
    const int y = y0 + r, x = x0 + cx;
    if (y < H && x < W) dst[(long)(co0 + c) * hw + (long)y * W + x] = ot[(r * OTW + cx) * COP + c];
  }
}

template <int CG, bool AFF>
__global__ __launch_bounds__(512, SA_WINO_WAVES_PER_EU) void wino_f2k3_kernel(const WinoLaunch L) {
  // The block's problem from its raw id: blocks are dealt to the 8 XCDs round-robin and every
  // problem's range starts at a multiple of 8, so each XCD gets an equal share of each
  // problem (problems differ in work per block); the L2-locality remap applies within it.
  // Uniform selects with constant indices (a dynamic index into the kernel-argument struct
  // would copy it to scratch).
  const unsigned g = blockIdx.x;
  WinoProb P = L.p[0];
  unsigned base = 0, n = L.nblk[0];
#pragma unroll
  for (int i = 1; i < MAX_PROB; ++i) {
    if (i < L.nprob && g >= L.end[i - 1]) {
      P = L.p[i];
      base = L.end[i - 1];
      n = L.nblk[i];
    }
  }
  if (g - base >= n) return;   // padding block (before any barrier)
  wino_body<CG, AFF>(P, sa::xcd_remap(g - base, n));
}

// U = (G g G^T) for g = w[co][ci] (3x3), in fp64, rounded once
__global__ __launch_bounds__(256) void wino_weights_kernel(const float *__restrict__ w, int Cout, int Cin,
                                                           float *__restrict__ U) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin) return;
  const int co = (int)(i / Cin), ci = (int)(i % Cin);
  const float *g = w + i * 9;
  // G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]]
  double t[4][3];
  for (int c = 0; c < 3; ++c) {
    const double g0 = g[c], g1 = g[3 + c], g2 = g[6 + c];
    t[0][c] = g0;
    t[1][c] = 0.5 * (g0 + g1 + g2);
    t[2][c] = 0.5 * (g0 - g1 + g2);
    t[3][c] = g2;
  }
  for (int r = 0; r < 4; ++r) {
    const double u0 = t[r][0], u1 = 0.5 * (t[r][0] + t[r][1] + t[r][2]), u2 = 0.5 * (t[r][0] - t[r][1] + t[r][2]),
                 u3 = t[r][2];
    const double u[4] = {u0, u1, u2, u3};
    // layout [xi][Cin/8][ci%4][Cout][(ci%8)/4]: the chunk image the conv kernel stages
    for (int c = 0; c < 4; ++c)
      U[((((long)(r * 4 + c) * (Cin / 8) + ci / 8) * 4 + (ci % 4)) * Cout + co) * 2 + (ci % 8) / 4] = (float)u[c];
  }
}

}  // namespace

extern "C" int sa_conv2d_wino_weights(const float *weight, int Cout, int Cin, float *U, void *stream) {
  SA_REQUIRE(weight && U && Cout > 0 && Cin > 0 && Cin % 8 == 0, "sa_conv2d_wino_weights: bad arguments (Cin %% 8)");
  const long n = (long)Cout * Cin;
  hipStream_t s = sa::as_stream(stream);
  wino_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(weight, Cout, Cin, U);
  return sa::check_launch("sa_conv2d_wino_weights");
}

extern "C" long sa_conv2d_k3_wino_stat_parts(int H, int W) {
  return (long)((W + OTW - 1) / OTW) * ((H + OTH - 1) / OTH);
}

namespace {

// validate one problem and fill its kernel descriptor; returns its CG (0 on error)
int wino_prob(const SaWinoProblem &q, WinoProb &P, bool &aff) {
  SA_REQUIRE(q.pitch == 0 || q.pitch == q.W, "sa_conv2d_k3_wino: pitched planes are F(4x4) only");
  SA_REQUIRE(!q.skip, "sa_conv2d_k3_wino: the residual epilogue is F(4x4) only");
  SA_REQUIRE(q.in && q.U && q.out && q.N > 0 && q.H > 0 && q.W > 0, "sa_conv2d_k3_wino: bad arguments");
  SA_REQUIRE(q.Cin % KC == 0 && q.Cout % 32 == 0,
             "sa_conv2d_k3_wino: needs Cin %% 8 == 0 and Cout %% 32 == 0 (got %d, %d)", q.Cin, q.Cout);
  SA_REQUIRE((reinterpret_cast<uintptr_t>(q.U) & 15) == 0, "sa_conv2d_k3_wino: U must be 16-byte aligned");
  SA_REQUIRE((long)q.Cin * q.H * q.W * 4 < (1L << 31) && 16L * q.Cin * q.Cout * 4 < (1L << 31),
             "sa_conv2d_k3_wino: an image or the filter bank exceeds the 2 GB buffer-descriptor range");
  aff = q.in_m || q.in_s || q.in_t || q.in_act;
  SA_REQUIRE(!aff || q.Cin <= MAX_CIN_AFFINE, "sa_conv2d_k3_wino: input transform needs Cin <= %d", MAX_CIN_AFFINE);
  SA_REQUIRE(q.in_pstride == 0 || q.in_pstride == q.Cin, "sa_conv2d_k3_wino: in_pstride must be 0 or Cin");
  SA_REQUIRE(q.in_act == 0 || q.in_act == 1, "sa_conv2d_k3_wino: input activation none or ReLU (got %d)", q.in_act);
  const int cg = q.Cout % 64 == 0 ? 2 : 1;
  const int tiles_w = (q.W + OTW - 1) / OTW, tiles_h = (q.H + OTH - 1) / OTH;
  P = WinoProb{q.in, q.in_bs, q.Cin, q.H, q.W, q.U, q.Cout, q.bias, q.relu, q.out, q.out_bs, tiles_w,
               tiles_w * tiles_h, q.Cout / (32 * cg),
               WinoIO{q.in_m, q.in_s, q.in_t, q.in_pstride, q.in_act, q.stats_partial}};
  return cg;
}

}  // namespace

extern "C" int sa_conv2d_k3_wino_multi(int nprob, const SaWinoProblem *probs, void *stream) {
  SA_REQUIRE(nprob >= 1 && nprob <= MAX_PROB && probs, "sa_conv2d_k3_wino_multi: 1..%d problems", MAX_PROB);
  WinoLaunch L{};
  int cg = 0;
  bool aff = false;
  long total = 0;
  for (int i = 0; i < nprob; ++i) {
    bool a = false;
    const int c = wino_prob(probs[i], L.p[i], a);
    if (c == 0) return SA_E_ARG;
    SA_REQUIRE(i == 0 || (c == cg && a == aff),
               "sa_conv2d_k3_wino_multi: problems must share the output-channel grouping (Cout %% 64) and "
               "the presence of an input transform");
    cg = c;
    aff = a;
    const long nb = (long)probs[i].N * L.p[i].tiles_hw * L.p[i].co_blocks;
    total = (i + 1 < nprob ? (total + nb + 7) / 8 * 8 : total + nb);
    SA_REQUIRE(total < (1L << 31), "sa_conv2d_k3_wino: grid too large");
    L.end[i] = (unsigned)total;
    L.nblk[i] = (unsigned)nb;
  }
  for (int i = nprob; i < MAX_PROB; ++i) {
    L.end[i] = (unsigned)total;
    L.nblk[i] = 0;
  }
  L.nprob = nprob;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV2D, s);
#define SA_WINO(CGV, AFFV) wino_f2k3_kernel<CGV, AFFV><<<(unsigned)total, 512, 0, s>>>(L)
  if (cg == 2) {
    if (aff) SA_WINO(2, true); else SA_WINO(2, false);
  } else {
    if (aff) SA_WINO(1, true); else SA_WINO(1, false);
  }
#undef SA_WINO
  return sa::check_launch("sa_conv2d_k3_wino");
}

extern "C" int sa_conv2d_k3_wino_ex(const float *in, long in_bs, int N, int Cin, int H, int W, const float *U,
                                    int Cout, const float *bias, int relu, const float *in_m, const float *in_s,
                                    const float *in_t, int in_pstride, int in_act, float *out, long out_bs,
                                    double *stats_partial, void *stream) {
  const SaWinoProblem q{in, in_bs, N, Cin, H, W, U, Cout, bias, relu, in_m, in_s, in_t, in_pstride, in_act,
                        out, out_bs, stats_partial};
  return sa_conv2d_k3_wino_multi(1, &q, stream);
}

extern "C" int sa_conv2d_k3_wino(const float *in, long in_bs, int N, int Cin, int H, int W, const float *U, int Cout,
                                 const float *bias, int relu, float *out, long out_bs, void *stream) {
  return sa_conv2d_k3_wino_ex(in, in_bs, N, Cin, H, W, U, Cout, bias, relu, nullptr, nullptr, nullptr, 0, 0, out,
                              out_bs, nullptr, stream);
}
