// K8 — convex upsampling of the final low-res flow (convex_upflow, utils.py:97-110).
//
// For each low-res pixel and each of the f x f sub-pixels (a, b): softmax over the 9
// mask logits mask[k*f*f + a*f + b] (k = 3x3 neighbour, row-major like F.unfold), then
// the weighted sum of the zero-padded 3x3 neighbourhood of f*flow.
//
// convex_up_px_kernel (round 6, f = 4, the model's factor): one thread per low-res pixel and
// sub-pixel row a (its 4 sub-pixels): each of the 144 mask planes is read by a wave as 64
// consecutive floats (whole 256-B runs; one thread per output pixel read each plane in 64-B pieces,
// 4 planes interleaved, and fetched ~1.3x the mask's bytes), its 36 logits all in flight together,
// and the 4 outputs are one float4 store.  The same operations per output, in the same order:
// bit-identical to convex_up_kernel (the other factors' path).
#include "sa_common.h"

#include <cstdint>

namespace {

__device__ __forceinline__ float convex_px(const float (&lg_in)[9], const float (&v)[9]) {
  float lg[9];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = lg_in[k];
    mx = fmaxf(mx, lg[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = expf(lg[k] - mx);
    s += lg[k];
  }
  const float inv = 1.0f / s;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) acc += (lg[k] * inv) * v[k];
  return acc;
}

__global__ __launch_bounds__(256) void convex_up_px_kernel(const float *__restrict__ flow,
                                                           const float *__restrict__ mask, long mask_bs, int H,
                                                           int W, long n, float *__restrict__ out) {
  constexpr int f = 4;
  // thread = (b, a, h, w), w fastest: a wave's lanes read 64 consecutive pixels of each mask plane
  // and write 64 consecutive float4 of output row 4 h + a
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long hw = (long)H * W;
  const int w = (int)(i % W);
  const long q = i / W;
  const int h = (int)(q % H);
  const int a = (int)((q / H) % f);
  const long b = q / ((long)H * f);
  const int r = h * W + w;
  const float *fl = flow + b * hw;
  float v[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {   // (clamped loads, then the zero padding as a select: no load under a branch)
    const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
    const float t = fl[(long)min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1)];
    v[k] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? (float)f * t : 0.0f;
  }
  const float *m = mask + b * mask_bs + (long)(a * f) * hw + r;
  const long kstride = (long)f * f * hw;
  float lg[f][9];
#pragma unroll
  for (int c = 0; c < f; ++c)
#pragma unroll
    for (int k = 0; k < 9; ++k) lg[c][k] = m[k * kstride + (long)c * hw];
  float4 o;
  o.x = convex_px(lg[0], v);
  o.y = convex_px(lg[1], v);
  o.z = convex_px(lg[2], v);
  o.w = convex_px(lg[3], v);
  const int Wo = W * f;
  *reinterpret_cast<float4 *>(out + b * hw * f * f + (long)(h * f + a) * Wo + w * f) = o;
}

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
  if (factor == 4 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const long np = (long)B * H * W * 4;
    convex_up_px_kernel<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(flow, mask, mask_bs, H, W, np, out);
    return sa::check_launch("sa_convex_upsample");
  }
  convex_up_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(flow, mask, mask_bs, H, W, factor, n, out);
  return sa::check_launch("sa_convex_upsample");
}
