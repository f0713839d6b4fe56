// 1x1 convolutions as GEMMs on split-f16 MFMA: the feature encoder's output conv (extractor.py:149,
// 128 -> 256 at 1/4 resolution) and the update block's mask head 1x1 (update.py:159-162, 191:
// 256 -> 576, x 0.25), which rocBLAS ran until round 5.  Two forms: the round-6 all-channel form
// (conv1x1_v2_kernel, below; Cin 64 / 128 / 256, the model's shapes) and the round-5 form described
// here (every other Cin).
//
//   out[b][co][p] = scale * (bias[co] + sum_ci W[co][ci] x[b][ci][p])     (p over the flat H*W plane)
//
// Products: each fp32 product w * x as hi(w) hi(x) + hi(w) lo(x) + lo(w) hi(x) of f16 pairs (x = hi
// + lo exactly in fp32, 22 significant bits per operand; the dropped lo * lo term is below 2^-22 of
// the product) on v_mfma_f32_16x16x32_f16, fp32 accumulation.  Weights are scaled by 2^12 before the
// split (exact; the accumulators are scaled back) so their lo halves stay normal f16.
//
//   block = 4 waves, 64 output channels x 128 pixels; wave = 64 channels x 32 pixels: 4 x 2 MFMA
//           tiles (D[m = channel][n = pixel]), 32 fp32 accumulators
//   chunk = 32 input channels: the block's x[32][128] is loaded as float4 (the next chunk's loads
//           in flight during this chunk's MFMAs) and written to LDS as it is, [k][pixel] (row
//           pitch 132 floats: conflict-free float4 writes, 2-way operand reads); a lane
//           reads its B operand's 8 k of one pixel as 8 dwords and splits them in registers (each
//           x value is split once, by the one wave that reads it); the A operands (8 consecutive k
//           of one channel, 16 B) come straight from the pre-split weights in global memory (L2:
//           every block of a channel range reads the same ones)
//   blocks of one pixel tile (all channel blocks) are consecutive in the remapped order, so they
//           run on one XCD and share its L2 copy of the tile's x
//   range guard: an input of magnitude >= 65504 (f16 overflow) makes the block recompute its
//           outputs with fp32 FMAs (exact products, the reference's arithmetic up to summation order)
#include "sa_common.h"

#include <cstdint>

namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int C1_CO = 64, C1_PX = 128, C1_K = 32, C1_THR = 256;
constexpr int C1_PITCH = 132;   // floats per LDS row (128 pixels + 4: the operand reads' rows 8 apart start
                                // 32 banks apart, so a ds_read_b32 of 16 pixels x 4 k-groups is 2-way)
constexpr float C1_WSCALE = 4096.0f;
#ifndef SA_C1_V2
#define SA_C1_V2 1   // the round-6 form (conv1x1_v2_kernel) for Cin <= 256; 0: the round-5 form everywhere
#endif

__device__ unsigned g_c1_redo_blocks;

__global__ __launch_bounds__(C1_THR, 2) void conv1x1_kernel(const float *__restrict__ x, long x_bs, int Cin, long P,
                                                            const _Float16 *__restrict__ whi,
                                                            const _Float16 *__restrict__ wlo, int Cout,
                                                            const float *__restrict__ bias, float scale,
                                                            float *__restrict__ out, long out_bs, int co_blocks,
                                                            long px_blocks) {
  __shared__ __attribute__((aligned(16))) float xs[C1_K * C1_PITCH];   // [k][pixel]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // remap: consecutive logical blocks (the channel blocks of a pixel tile) on one XCD
  const unsigned nwg = gridDim.x;
  const unsigned lid = sa::xcd_remap(blockIdx.x, nwg);
  const int cb = (int)(lid % (unsigned)co_blocks);
  const long rest = lid / (unsigned)co_blocks;
  const long pb = rest % px_blocks;
  const int b = (int)(rest / px_blocks);
  const int co0 = cb * C1_CO;
  const long p0 = pb * C1_PX;
  const float *xb = x + (long)b * x_bs;

  // staging: thread tid loads 4 float4 per chunk: channel kk = tid / 32 + 8 i, pixels 4 (tid % 32) .. + 3
  const int sp = (tid & 31) * 4;
  // (pixels past the plane's end load the plane's last group instead: unpredicated loads all stay in
  // flight, a load under a branch would be waited for at once; those outputs are never stored)
  const long pc = min(p0 + sp, P - 4);
  auto load_chunk = [&](int k0, f32x4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = *reinterpret_cast<const f32x4 *>(xb + (long)(k0 + (tid >> 5) + 8 * i) * P + pc);
  };
  auto stage = [&](const f32x4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4 *>(&xs[((tid >> 5) + 8 * i) * C1_PITCH + sp]) = v[i];
  };
  // A operands: channel co0 + 16 c + lane % 16, k = k0 + 8 (lane / 16) .. + 7
  const int am = lane & 15, ak = (lane >> 4) * 8;
  auto load_w = [&](int k0, f16x8 (&wh)[4], f16x8 (&wl)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int co = min(co0 + 16 * c + am, Cout - 1);
      const long o = (long)co * Cin + k0 + ak;
      wh[c] = *reinterpret_cast<const f16x8 *>(whi + o);
      wl[c] = *reinterpret_cast<const f16x8 *>(wlo + o);
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[c][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = Cin / C1_K;
  // B operands: pixel (wave's 32) + 16 q + lane % 16, k = 8 (lane / 16) .. + 7
  const int bp = wv * 32 + (lane & 15), bk = (lane >> 4) * 8;
  bool bad = false;   // an input beyond the f16 range (|x| >= 65504: its hi half is inf)
  // two register sets, each chunk's loads issued two chunks ahead: chunk kc + 2's inputs as soon as
  // chunk kc is staged, its weights once chunk kc's MFMAs have read theirs
  f32x4 xa[4], xb2[4];
  f16x8 wha[4], wla[4], whb[4], wlb[4];
  load_chunk(0, xa);
  load_w(0, wha, wla);
  if (nchunks > 1) {
    load_chunk(C1_K, xb2);
    load_w(C1_K, whb, wlb);
  }
  auto step = [&](int kc, f32x4 (&xv)[4], f16x8 (&wh)[4], f16x8 (&wl)[4]) __attribute__((always_inline)) {
    __syncthreads();   // the previous chunk's B reads are done
    stage(xv);
    __syncthreads();
    if (kc + 2 < nchunks) load_chunk((kc + 2) * C1_K, xv);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = xs[(bk + j) * C1_PITCH + bp + 16 * q];
      f16x8 bh, bl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)v[j];
        bh[j] = h;
        bl[j] = (_Float16)(v[j] - (float)h);   // exact in fp32
        bad |= !(__builtin_fabsf(v[j]) < 65504.0f);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[c], bh, acc[c][q], 0, 0, 0);
        acc[c][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[c], bl, acc[c][q], 0, 0, 0);
        acc[c][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[c], bh, acc[c][q], 0, 0, 0);
      }
    }
    if (kc + 2 < nchunks) load_w((kc + 2) * C1_K, wh, wl);
  };
#pragma unroll 1
  for (int kc = 0; kc < nchunks; kc += 2) {
    step(kc, xa, wha, wla);
    if (kc + 1 < nchunks) step(kc + 1, xb2, whb, wlb);
  }
  float *ob = out + (long)b * out_bs;
  // D layout: lane holds rows 4 (lane / 16) .. + 3 (channels), column lane % 16 (pixel)
  const int dn = lane & 15, dm = (lane >> 4) * 4;
  if (!__syncthreads_or(bad)) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const long p = p0 + wv * 32 + 16 * q + dn;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = co0 + 16 * c + dm + i;
          if (co < Cout && p < P) {
            const float bv = bias ? bias[co] : 0.0f;
            ob[(long)co * P + p] = (acc[c][q][i] * (1.0f / C1_WSCALE) + bv) * scale;
          }
        }
      }
    return;
  }
  // range guard: fp32 FMAs on the inputs and the split weights (hi + lo: 22 significant bits)
  if (tid == 0) atomicAdd(&g_c1_redo_blocks, 1u);
  for (int e = tid; e < C1_CO * C1_PX; e += C1_THR) {
    const int co = co0 + e / C1_PX;
    const long p = p0 + e % C1_PX;
    if (co >= Cout || p >= P) continue;
    float s = 0.0f;
    for (int k = 0; k < Cin; ++k) {
      const float w = ((float)whi[(long)co * Cin + k] + (float)wlo[(long)co * Cin + k]) * (1.0f / C1_WSCALE);
      s = fmaf(w, xb[(long)k * P + p], s);
    }
    ob[(long)co * P + p] = (s + (bias ? bias[co] : 0.0f)) * scale;
  }
}

// Round 6 form (the default for Cin <= 256): a block owns 64 pixels of one image for EVERY output
// channel.  The pixels' Cin inputs are read from HBM once, split into f16 hi / lo as they are
// staged, and kept in LDS as [k / 8][pixel][8] halves (a lane's B operand, 8 consecutive k of one
// pixel, is one 16-byte read, no VALU, conflict-free).  The Cout / 16 channel tiles are shared out
// among the 4 waves; a wave walks its tiles MT at a time against all 64 pixels (MT x 4 MFMA
// tiles, 3 products each per 32 k), so every A operand (pre-split weights, from L2) feeds 4 pixel
// tiles and the block reads the weights once.  (The round-5 form above reads each pixel tile once
// per 64-channel block and its waves read the weights once per 32 pixels.)  A pass's 32-k steps are
// unrolled (NKS = Cin / 32) so the waits on the weight loads stay partial; the stores go through a
// buffer resource (no branches) with the bias from LDS.
// Measured (configs[1] shapes, profiles/ab/r06_conv1x1_forms.txt): 8x128->256 302 -> 195 us,
// 4x256->576 451 -> 235 us.  What bounds it now is the A operands' L2 -> CU traffic: 2 KB of hi / lo
// weights per channel tile per 32 k feed 12 MFMAs (4 pixel tiles x 3 products), ~170 B per MFMA,
// about the vector cache's rate at the MFMA pipe's pace; the HBM floor is ~50 us per call.
constexpr int C2_PX = 64, C2_THR = 256, C2_KMAX = 256, C2_COMAX = 1024;

template <int MT, int NKS>
__global__ __launch_bounds__(C2_THR, 2) void conv1x1_v2_kernel(const float *__restrict__ x, long x_bs, int Cin, long P,
                                                               const _Float16 *__restrict__ whi,
                                                               const _Float16 *__restrict__ wlo, int Cout,
                                                               const float *__restrict__ bias, float scale,
                                                               float *__restrict__ out, long out_bs, long px_blocks) {
  __shared__ __attribute__((aligned(16))) _Float16 xh[C2_KMAX / 8 * C2_PX * 8], xl[C2_KMAX / 8 * C2_PX * 8];
  __shared__ float bs[C2_COMAX];   // the bias (zeros when absent): read at the stores without a global load
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned lid = sa::xcd_remap(blockIdx.x, gridDim.x);
  for (int i = tid; i < Cout; i += C2_THR) bs[i] = bias ? bias[i] : 0.0f;
  const long pb = lid % px_blocks;
  const int b = (int)(lid / px_blocks);
  const long p0 = pb * C2_PX;
  const float *xb = x + (long)b * x_bs;
  float *ob = out + (long)b * out_bs;
  const int ngrp = Cin / 8;
  // staging: thread (pixel tid % 64, k-groups tid / 64 + 4 i), 8 loads per group (each coalesced
  // over the wave's 64 pixels; the last tile's pixels past P load pixel P - 1 and are never stored)
  bool bad = false;
  {
    const long pc = min(p0 + (tid & 63), P - 1);
    for (int g0 = tid >> 6; g0 < ngrp; g0 += 16) {   // 4 groups per pass: their 32 loads in flight
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kg = min(g0 + 4 * u, ngrp - 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = xb[(long)(kg * 8 + j) * P + pc];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kg = g0 + 4 * u;
        if (kg >= ngrp) break;
        f16x8 h, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const _Float16 hh = (_Float16)v[u][j];
          h[j] = hh;
          l[j] = (_Float16)(v[u][j] - (float)hh);   // exact in fp32
          bad |= !(__builtin_fabsf(v[u][j]) < 65504.0f);
        }
        *reinterpret_cast<f16x8 *>(&xh[(kg * C2_PX + (tid & 63)) * 8]) = h;
        *reinterpret_cast<f16x8 *>(&xl[(kg * C2_PX + (tid & 63)) * 8]) = l;
      }
    }
  }
  if (__syncthreads_or(bad)) {   // range guard: the whole tile with fp32 FMAs (exact products)
    if (tid == 0) atomicAdd(&g_c1_redo_blocks, 1u);
    for (long e = tid; e < (long)Cout * C2_PX; e += C2_THR) {
      const int co = (int)(e / C2_PX);
      const long p = p0 + e % C2_PX;
      if (p >= P) continue;
      float s = 0.0f;
      for (int k = 0; k < Cin; ++k) {
        const float w = ((float)whi[(long)co * Cin + k] + (float)wlo[(long)co * Cin + k]) * (1.0f / C1_WSCALE);
        s = fmaf(w, xb[(long)k * P + p], s);
      }
      ob[(long)co * P + p] = (s + (bias ? bias[co] : 0.0f)) * scale;
    }
    return;
  }
  const int am = lane & 15, aq = lane >> 4;   // A: channel row am of a tile, k = 8 aq .. + 7; B: pixel am of a tile
  const int ntiles = (Cout + 15) / 16, tpw = (ntiles + 3) / 4;
  const int t0 = __builtin_amdgcn_readfirstlane(wv) * tpw, t1 = min(t0 + tpw, ntiles);
  const int npass = t1 > t0 ? (t1 - t0 + MT - 1) / MT : 0;
  constexpr int nks = NKS;   // (= Cin / 32)
  const int total = npass * nks;   // steps: (pass, 32 k)
  // A operands of step it (clamped: the loads past the last step are unconditional, never used)
  auto load_w = [&](int it, f16x8 (&wh)[MT], f16x8 (&wl)[MT]) __attribute__((always_inline)) {
    it = __builtin_amdgcn_readfirstlane(min(it, max(total - 1, 0)));
    const int ps = it / nks, ks = it - ps * nks;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const long o = (long)min(16 * (t0 + ps * MT + t) + am, Cout - 1) * Cin + ks * 32 + aq * 8;
      wh[t] = *reinterpret_cast<const f16x8 *>(whi + o);
      wl[t] = *reinterpret_cast<const f16x8 *>(wlo + o);
    }
  };
  f32x4 acc[MT][4];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  // D: lane holds channels 16 tile + 4 aq + i (rows), pixel 16 n + am (column).  Stores through a
  // buffer resource over the image's output: an element outside (channel tile past the wave's, channel
  // >= Cout, pixel >= P) gets an offset past the range and the hardware drops it (no branches, so
  // no waits on the loads in flight)
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(ob, 0, (int)((long)Cout * P * 4), 0x00020000);
  auto store = [&](int ps) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int tile = t0 + ps * MT + t;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = 16 * tile + 4 * aq + i;
        const float bv = bs[min(co, Cout - 1)];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const long p = p0 + 16 * n + am;
          const bool ok = tile < t1 && co < Cout && p < P;
          const int off = ok ? (int)(((long)co * P + p) * 4) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, (acc[t][n][i] * (1.0f / C1_WSCALE) + bv) * scale),
                                                orsrc, off, 0, 0);
        }
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto step = [&](int it, f16x8 (&wh)[MT], f16x8 (&wl)[MT]) __attribute__((always_inline)) {
    const int kg = (it % nks) * 4 + aq;
    f16x8 bh[4], bl[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      bh[n] = *reinterpret_cast<const f16x8 *>(&xh[(kg * C2_PX + 16 * n + am) * 8]);
      bl[n] = *reinterpret_cast<const f16x8 *>(&xl[(kg * C2_PX + 16 * n + am) * 8]);
    }
    // product-major: an accumulator's three products are MT x 4 MFMAs apart (the same order of
    // accumulation as the round-5 form: hi hi, hi lo, lo hi per 32 k)
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[t], bh[n], acc[t][n], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[t], bl[n], acc[t][n], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[t], bh[n], acc[t][n], 0, 0, 0);
    load_w(it + 2, wh, wl);   // two steps ahead (the next set is already in flight)
    __builtin_amdgcn_sched_barrier(0);   // (left to itself the scheduler sinks the first step's loads
                                         // past the second step's MFMAs: both sets then wait together)
  };
  // two register sets, each step's weights issued two steps ahead (a pass's steps unrolled: the
  // waits stay exact; nks even: the host sends Cin other than 64, 128, 256 to the round-5 form)
  f16x8 wha[MT], wla[MT], whb[MT], wlb[MT];
  load_w(0, wha, wla);
  load_w(1, whb, wlb);
#pragma unroll 1
  for (int ps = 0; ps < npass; ++ps) {
#pragma unroll
    for (int ks = 0; ks < nks; ks += 2) {
      step(ps * nks + ks, wha, wla);
      step(ps * nks + ks + 1, whb, wlb);
    }
    store(ps);
  }
}

// [Cout][Cin] fp32 -> hi, lo f16 planes of w * 2^12 (round to nearest even; w * 2^12 - hi is exact)
__global__ __launch_bounds__(256) void conv1x1_weights_kernel(const float *__restrict__ w, long n,
                                                              _Float16 *__restrict__ hi, _Float16 *__restrict__ lo) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = w[i] * C1_WSCALE;
  const _Float16 h = (_Float16)v;
  hi[i] = h;
  lo[i] = (_Float16)(v - (float)h);
}

}  // namespace

extern "C" long sa_conv1x1_weights_size(int Cout, int Cin) {
  if (Cout <= 0 || Cin <= 0) return -1;
  return 2L * Cout * Cin * (long)sizeof(_Float16);
}

extern "C" int sa_conv1x1_weights(const float *weight, int Cout, int Cin, void *out, void *stream) {
  SA_REQUIRE(weight && out, "sa_conv1x1_weights: null pointer");
  SA_REQUIRE(Cout > 0 && Cin > 0, "sa_conv1x1_weights: empty shape");
  SA_REQUIRE((reinterpret_cast<uintptr_t>(out) & 15) == 0, "sa_conv1x1_weights: out not 16-byte aligned");
  const long n = (long)Cout * Cin;
  _Float16 *hi = static_cast<_Float16 *>(out);
  conv1x1_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, sa::as_stream(stream)>>>(weight, n, hi, hi + n);
  return sa::check_launch("sa_conv1x1_weights");
}

extern "C" int sa_conv1x1(const float *x, long x_bs, int B, int Cin, int H, int W, const void *wsplit, int Cout,
                          const float *bias, float scale, float *out, long out_bs, void *stream) {
  SA_REQUIRE(x && wsplit && out, "sa_conv1x1: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0 && Cout > 0, "sa_conv1x1: empty shape");
  SA_REQUIRE(Cin > 0 && Cin % C1_K == 0, "sa_conv1x1: Cin must be a positive multiple of 32");
  const long P = (long)H * W;
  SA_REQUIRE(P % 4 == 0 && x_bs % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
             "sa_conv1x1: H*W, the batch stride and x must be 16-byte granular");
  SA_REQUIRE(x_bs >= (long)Cin * P && out_bs >= (long)Cout * P, "sa_conv1x1: batch stride below the planes");
  SA_REQUIRE((reinterpret_cast<uintptr_t>(wsplit) & 15) == 0, "sa_conv1x1: weights not 16-byte aligned");
  const int co_blocks = (Cout + C1_CO - 1) / C1_CO;
  const long px_blocks = (P + C1_PX - 1) / C1_PX;
  const long nblk = (long)co_blocks * px_blocks * B;
  SA_REQUIRE(nblk < (1L << 31), "sa_conv1x1: too many blocks");
  const _Float16 *hi = static_cast<const _Float16 *>(wsplit);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV1X1, s);
  if (SA_C1_V2 && (Cin == 64 || Cin == 128 || Cin == 256) && Cout <= C2_COMAX && (long)Cout * P * 4 < 0x7ffffff0L) {   // (32-bit store offsets)
    const long pb2 = (P + C2_PX - 1) / C2_PX;
    SA_REQUIRE(pb2 * B < (1L << 31), "sa_conv1x1: too many blocks");
    // channel tiles per wave: passes of 3 or 4 tiles, whichever wastes fewer MFMA rows (576: 9 = 3 x 3)
    const int tpw = ((Cout + 15) / 16 + 3) / 4;
    const bool mt3 = (tpw + 2) / 3 * 3 < (tpw + 3) / 4 * 4;
    const unsigned g = (unsigned)(pb2 * B);
    const _Float16 *lo = hi + (long)Cout * Cin;
#define SA_C1_V2_LAUNCH(MT, NKS) \
  conv1x1_v2_kernel<MT, NKS><<<g, C2_THR, 0, s>>>(x, x_bs, Cin, P, hi, lo, Cout, bias, scale, out, out_bs, pb2)
    if (Cin == 64) {
      if (mt3) SA_C1_V2_LAUNCH(3, 2); else SA_C1_V2_LAUNCH(4, 2);
    } else if (Cin == 128) {
      if (mt3) SA_C1_V2_LAUNCH(3, 4); else SA_C1_V2_LAUNCH(4, 4);
    } else {
      if (mt3) SA_C1_V2_LAUNCH(3, 8); else SA_C1_V2_LAUNCH(4, 8);
    }
#undef SA_C1_V2_LAUNCH
  } else {
    conv1x1_kernel<<<(unsigned)nblk, C1_THR, 0, s>>>(x, x_bs, Cin, P, hi, hi + (long)Cout * Cin, Cout, bias, scale,
                                                     out, out_bs, co_blocks, px_blocks);
  }
  return sa::check_launch("sa_conv1x1");
}

extern "C" long sa_conv1x1_redo_blocks(int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_c1_redo_blocks), sizeof v) != hipSuccess) return -1;
  if (reset) {
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_c1_redo_blocks), &z, sizeof z) != hipSuccess) return -1;
  }
  return v;
}
