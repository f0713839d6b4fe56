// The tiled harness's data movement around the model (mapreduce_v2/tile_wrapper.py:226-236, 169-185,
// 188-189), which ran as ATen launches per tile until round 5 (cfg5: 57 elementwise launches, 4
// concatenations and 4 replicate pads per image, ~2.5 ms):
//   sa_tile_gather_pad — the batch of tile rectangles cut from a full image and padded to the model's
//     multiple of 32 by edge replication (torch.cat of the views, then F.pad(mode="replicate")): one
//     launch per image tensor, a thread per 4 output pixels of a row;
//   sa_tile_stitch — the blend: for every pixel, the tiles covering it in the reference's order (a
//     duplicate rectangle counted each time it is listed) add d * w to the numerator and w to the
//     weight, then out = weight > 0 ? num / max(weight, 1e-4) : num.  The same fp32 operations in the
//     same order per pixel as the reference's sequence of slice updates, so the same bits.
#include "sa_common.h"

namespace {

// out[t][c][y][x] = src[c][ys(t) + clamp(y - pt, 0, th - 1)][xs(t) + clamp(x - pl, 0, tw - 1)]
__global__ __launch_bounds__(256) void tile_gather_pad_kernel(const float *__restrict__ src, long src_cs, int W,
                                                              const int *__restrict__ origin, int C, int th, int tw,
                                                              int pt, int pl, int Ho, int Wo,
                                                              float *__restrict__ out, long nrows) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;   // (row, 4-pixel group)
  const int groups = (Wo + 3) / 4;
  const long row = q / groups;
  if (row >= nrows) return;
  const int x0 = (int)(q - row * groups) * 4;
  const int y = (int)(row % Ho);
  const long tc = row / Ho;   // tile * C + c
  const int c = (int)(tc % C), t = (int)(tc / C);
  const int ys = origin[2 * t], xs = origin[2 * t + 1];
  const int yy = ys + min(max(y - pt, 0), th - 1);
  const float *s = src + (long)c * src_cs + (long)yy * W + xs;
  float *o = out + row * Wo + x0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int x = x0 + e;
    if (x < Wo) o[e] = s[min(max(x - pl, 0), tw - 1)];
  }
}

__global__ __launch_bounds__(256) void tile_stitch_kernel(const float *__restrict__ disp, long disp_ts, int dpitch,
                                                          const int *__restrict__ tiles, int ntiles, int th, int tw,
                                                          const float *__restrict__ wgt, int H, int W, int finalize,
                                                          float *__restrict__ num, float *__restrict__ den) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)H * W) return;
  const int y = (int)(p / W), x = (int)(p - (long)y * W);
  float s = num[p], w = den[p];
  for (int i = 0; i < ntiles; ++i) {   // tiles[i] = (y0, x0, slot of its disparity map)
    const int ty = y - tiles[3 * i], tx = x - tiles[3 * i + 1];
    if (ty < 0 || ty >= th || tx < 0 || tx >= tw) continue;
    const float wv = wgt[ty * tw + tx];
    const float d = disp[tiles[3 * i + 2] * disp_ts + (long)ty * dpitch + tx];
    s = s + d * wv;
    w = w + wv;
  }
  if (finalize) {
    num[p] = w > 0.0f ? s / fmaxf(w, 1e-4f) : s;
  } else {
    num[p] = s;
    den[p] = w;
  }
}

}  // namespace

extern "C" int sa_tile_gather_pad(const float *src, int C, int H, int W, const int *origin, int ntiles, int th,
                                  int tw, int pt, int pb, int pl, int pr, float *out, void *stream) {
  SA_REQUIRE(src && origin && out, "sa_tile_gather_pad: null pointer");
  SA_REQUIRE(C > 0 && H > 0 && W > 0 && ntiles > 0 && th > 0 && tw > 0 && th <= H && tw <= W,
             "sa_tile_gather_pad: bad shape");
  SA_REQUIRE(pt >= 0 && pb >= 0 && pl >= 0 && pr >= 0, "sa_tile_gather_pad: negative padding");
  const int Ho = th + pt + pb, Wo = tw + pl + pr;
  const long nrows = (long)ntiles * C * Ho;
  const long nthr = nrows * ((Wo + 3) / 4);
  SA_REQUIRE(nthr < (1L << 40), "sa_tile_gather_pad: too large");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  tile_gather_pad_kernel<<<(unsigned)((nthr + 255) / 256), 256, 0, s>>>(src, (long)H * W, W, origin, C, th, tw, pt,
                                                                         pl, Ho, Wo, out, nrows);
  return sa::check_launch("sa_tile_gather_pad");
}

extern "C" int sa_tile_stitch(const float *disp, long disp_ts, int dpitch, const int *tiles, int ntiles, int th,
                              int tw, const float *wgt, int H, int W, int finalize, float *num, float *den,
                              void *stream) {
  SA_REQUIRE(disp && tiles && wgt && num && den, "sa_tile_stitch: null pointer");
  SA_REQUIRE(ntiles > 0 && th > 0 && tw > 0 && H > 0 && W > 0 && dpitch >= tw && disp_ts >= (long)th * dpitch,
             "sa_tile_stitch: bad shape");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  const long n = (long)H * W;
  tile_stitch_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(disp, disp_ts, dpitch, tiles, ntiles, th, tw, wgt, H,
                                                                  W, finalize, num, den);
  return sa::check_launch("sa_tile_stitch");
}
