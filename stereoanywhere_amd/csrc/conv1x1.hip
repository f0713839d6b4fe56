// 1x1 convolutions as GEMMs on split-f16 MFMA: the feature encoder's output conv (extractor.py:149,
// 128 -> 256 at 1/4 resolution) and the update block's mask head 1x1 (update.py:159-162, 191:
// 256 -> 576, x 0.25), which rocBLAS ran until round 5.
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
  conv1x1_kernel<<<(unsigned)nblk, C1_THR, 0, s>>>(x, x_bs, Cin, P, hi, hi + (long)Cout * Cin, Cout, bias, scale,
                                                   out, out_bs, co_blocks, px_blocks);
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
