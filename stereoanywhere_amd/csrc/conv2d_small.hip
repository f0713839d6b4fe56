// Direct 2-D convolution for the motion encoder's flow stem (convf1 = Conv2d(2, 64, 7,
// padding=3) followed by ReLU, update.py:76, 85).
//
// With two input channels this conv is 1.6 GFLOP per 544x960 batch of four, but the
// library path lowered it to an NHWC implicit GEMM plus layout transposes (~1.7 ms per
// GRU iteration).  Here a 16x16-pixel block stages the (16+K-1)^2 halo of every input
// channel in LDS and each thread accumulates all COUT outputs of its pixel with
// wave-uniform (scalar) weights; bias and ReLU are applied in the epilogue.
#include "sa_common.h"

namespace {

constexpr int T = 16;

template <int K, int COUT>
__global__ __launch_bounds__(256) void conv2d_small_kernel(const float *__restrict__ in, long in_bs, int Cin, int H,
                                                           int W, const float *__restrict__ wt,
                                                           const float *__restrict__ bias, int relu,
                                                           float *__restrict__ out, long out_bs) {
  constexpr int L = T + K - 1, P = K / 2;
  __shared__ float tile[L * L];
  const int tx = threadIdx.x & (T - 1), ty = threadIdx.x / T;
  const int x0 = blockIdx.x * T, y0 = blockIdx.y * T, b = blockIdx.z;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
  for (int ci = 0; ci < Cin; ++ci) {
    const float *src = in + (long)b * in_bs + (long)ci * H * W;
    __syncthreads();
    for (int i = threadIdx.x; i < L * L; i += 256) {
      const int yy = y0 - P + i / L, xx = x0 - P + i % L;
      tile[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? src[(long)yy * W + xx] : 0.0f;
    }
    __syncthreads();
    const float *wc = wt + (long)ci * K * K * COUT;  // weights pre-arranged [ci][ky][kx][co]
#pragma unroll 1
    for (int ky = 0; ky < K; ++ky)
#pragma unroll 1
      for (int kx = 0; kx < K; ++kx) {
        const float v = tile[(ty + ky) * L + tx + kx];
        const float *wp = wc + (ky * K + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] += wp[co] * v;
      }
  }
  const int x = x0 + tx, y = y0 + ty;
  if (x < W && y < H) {
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float r = acc[co] + (bias ? bias[co] : 0.0f);
      if (relu) r = fmaxf(r, 0.0f);
      out[(long)b * out_bs + (long)co * H * W + (long)y * W + x] = r;
    }
  }
}

}  // namespace

extern "C" int sa_conv2d_small(const float *in, long in_bs, int B, int Cin, int H, int W, const float *weight,
                               const float *bias, int Cout, int ksize, int relu, float *out, long out_bs,
                               void *stream) {
  SA_REQUIRE(in && weight && out, "sa_conv2d_small: null pointer");
  SA_REQUIRE(B > 0 && Cin > 0 && Cin <= 8 && H > 0 && W > 0, "sa_conv2d_small: bad shape");
  SA_REQUIRE(ksize == 7 && Cout == 64, "sa_conv2d_small: built for 7x7 -> 64 channels (got %dx%d -> %d)", ksize,
             ksize, Cout);
  dim3 grid((W + T - 1) / T, (H + T - 1) / T, B);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  conv2d_small_kernel<7, 64><<<grid, 256, 0, s>>>(in, in_bs, Cin, H, W, weight, bias, relu, out, out_bs);
  return sa::check_launch("sa_conv2d_small");
}
