// The motion encoder's convc1 (update.py:75, 84: 1x1 conv of the L*(2r+1) lookup taps to 64
// channels, + bias, ReLU) on fp32 MFMA, for the lookup kernels (corr_lookup.hip,
// corr_shear.hip) whose lanes each hold one pixel's taps.
//
// Per wave: 64 pixels x NT taps x 64 channels = a [64 x NT] x [NT x 64] GEMM, as 4 pixel blocks
// x 4 channel groups x NT/4 k-steps of v_mfma_f32_16x16x4_f32 (144 MFMAs for NT = 36) instead
// of NT * 64 VALU FMAs per lane.  The taps go through LDS once ([NT][80]: lane pixel p writes
// row k at column p; the A operand of lane (k, m) is row 4s + k, column 16q + m; pitch 80 =
// 16 (mod 64) keeps the four k rows of a read in distinct banks); the B operands (weights, [NT]
// [64] row-major) and the bias are per-lane registers.  Each output is the k-ordered fmaf
// chain bias + sum_k w[k] * tap[k] (MFMA numerics), the VALU path's order.
#pragma once

#include "sa_common.h"

namespace sa {

constexpr int C1_PITCH = 80;

template <int NT>
struct C1Weights {
  float b[NT / 4][4];   // B operand of (k-step s, channel group g)
  float bias[4];        // channel 16 g + (lane & 15)
};

template <int NT>
__device__ __forceinline__ void c1_load_weights(const float *__restrict__ wt, const float *__restrict__ bias,
                                                int lane, C1Weights<NT> &w) {
  static_assert(NT % 4 == 0, "k-steps of 4 taps");
  const int kk = lane >> 4, n = lane & 15;
#pragma unroll
  for (int s = 0; s < NT / 4; ++s)
#pragma unroll
    for (int g = 0; g < 4; ++g) w.b[s][g] = wt[(4 * s + kk) * 64 + 16 * g + n];
#pragma unroll
  for (int g = 0; g < 4; ++g) w.bias[g] = bias[16 * g + n];
}

// f: this lane's NT taps (its pixel = wave pixel `lane`); lds: the wave's [NT][C1_PITCH] floats.
// store(q, g, acc): the caller writes the 4 outputs acc[i] = channel 16 g + (lane & 15) of wave
// pixels 16 q + 4 (lane >> 4) + i (ReLU applied).
template <int NT, class Store>
__device__ __forceinline__ void c1_mfma(const float (&f)[NT], const C1Weights<NT> &w, float *lds, int lane,
                                        Store &&store) {
  using f32x4 = __attribute__((ext_vector_type(4))) float;
#pragma unroll
  for (int k = 0; k < NT; ++k) lds[k * C1_PITCH + lane] = f[k];
  // (the wave's own LDS writes precede its reads: DS operations of a wave complete in order)
  const int kk = lane >> 4, m = lane & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f32x4{w.bias[g], w.bias[g], w.bias[g], w.bias[g]};
#pragma unroll
    for (int s = 0; s < NT / 4; ++s) {
      const float a = lds[(4 * s + kk) * C1_PITCH + 16 * q + m];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w.b[s][g], acc[g], 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = fmaxf(acc[g][i], 0.0f);
      store(q, g, r);
    }
  }
}

// the 4 outputs of c1_mfma's store for wave pixels px .. px + 3 (global pixel index, px % 4 ==
// 0), channel ch, of out [B * nvol, 64, H, W] (sample b * nvol + v), pixels past npix skipped
template <class V4>
__device__ __forceinline__ void c1_store4(float *__restrict__ out, int px, int ch, int hw, int nvol, int v, int npix,
                                          const V4 &r) {
  if (px + 3 < npix && hw % 4 == 0) {   // one image, 16-byte aligned
    const int b = px / hw, rem = px - b * hw;
    *reinterpret_cast<V4 *>(out + (((long)b * nvol + v) * 64 + ch) * hw + rem) = r;
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = px + i;
    if (q < npix) {
      const int b = q / hw, rem = q - b * hw;
      out[(((long)b * nvol + v) * 64 + ch) * hw + rem] = r[i];
    }
  }
}

}  // namespace sa
