// K8 — convex upsampling of the final low-res flow (convex_upflow, utils.py:97-110).
//
// For each low-res pixel and each of the f x f sub-pixels (a, b): softmax over the 9
// mask logits mask[k*f*f + a*f + b] (k = 3x3 neighbour, row-major like F.unfold), then
// the weighted sum of the zero-padded 3x3 neighbourhood of f*flow.  One thread per
// output pixel; the f*f threads of one low-res pixel share its 9 flow values in L1.
#include "sa_common.h"

namespace {

__global__ __launch_bounds__(256) void convex_up_kernel(const float *__restrict__ flow,
                                                        const float *__restrict__ mask, long mask_bs,
                                                        int H, int W, int f, long n,
                                                        float *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int Wo = W * f, Ho = H * f;
  const int X = (int)(i % Wo);
  const int Y = (int)((i / Wo) % Ho);
  const long b = i / ((long)Wo * Ho);
  const int h = Y / f, a = Y % f, w = X / f, c = X % f;
  const long hw = (long)H * W;
  const float *m = mask + b * mask_bs + (long)(a * f + c) * hw + (long)h * W + w;
  const long kstride = (long)f * f * hw;
  float lg[9];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = m[k * kstride];
    mx = fmaxf(mx, lg[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = expf(lg[k] - mx);
    s += lg[k];
  }
  const float inv = 1.0f / s;
  const float *fl = flow + b * hw;
  const float ff = (float)f;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
    const float v = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? ff * fl[(long)yy * W + xx] : 0.0f;
    acc += (lg[k] * inv) * v;
  }
  out[i] = acc;
}

}  // namespace

extern "C" int sa_convex_upsample(const float *flow, const float *mask, long mask_bs, int B, int H, int W,
                                  int factor, float *out, void *stream) {
  SA_REQUIRE(flow && mask && out, "sa_convex_upsample: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0 && factor >= 1 && factor <= 8, "sa_convex_upsample: bad shape");
  const long n = (long)B * H * W * factor * factor;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_UPSAMPLE, s);
  convex_up_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(flow, mask, mask_bs, H, W, factor, n, out);
  return sa::check_launch("sa_convex_upsample");
}
