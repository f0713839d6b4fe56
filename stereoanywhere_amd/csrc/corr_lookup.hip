// K4 — correlation-pyramid lookup (CorrBlock1D.__call__, corr.py:93-115, through
// bilinear_sampler, utils.py:19-35).
//
// One thread per (volume, pixel): for each level l it reads the (2r+2) pyramid cells
// around x = coords_x / 2^l out of its own pixel row and writes the (2r+1) linearly
// interpolated taps; consecutive threads are consecutive pixels j, so every output
// plane store is coalesced.  Stereo and mono pyramids share one launch (blockIdx.y).
//
// Arithmetic mirrors the reference's grid_sample round trip in fp32:
//   xg = 2 (t + x/2^l) / (W_l - 1) - 1       (utils.py:25, corr.py:104)
//   ix = (xg + 1) * ((W_l - 1) / 2)          (ATen CPU grid_sample, align_corners=True)
//   out = v[floor] * (1 - w) + v[floor + 1] * w, zero outside [0, W_l - 1].
#include "sa_common.h"
#include "convc1_mfma.h"

namespace {

struct LGeo {
  int H, W1, L, r;
  long rs, cbs, obs;
  int off[4], wid[4];
};

__global__ __launch_bounds__(256) void lookup_kernel(const float *__restrict__ pa,
                                                     const float *__restrict__ pb,
                                                     const float *__restrict__ cx, LGeo g,
                                                     long npix, float *__restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int v = blockIdx.y;
  const float *__restrict__ pyr = v ? pb : pa;
  const long hw = (long)g.H * g.W1;
  const long b = p / hw, rem = p % hw;
  const float x = cx[b * g.cbs + rem];
  const float *__restrict__ row = pyr + p * g.rs;
  const int K = 2 * g.r + 1;
  float *__restrict__ o = out + b * g.obs + (long)v * g.L * K * hw + rem;
  for (int l = 0; l < g.L; ++l) {
    const int Wl = g.wid[l];
    const float *__restrict__ lv = row + g.off[l];
    const float xl = x / (float)(1 << l);
    const float denom = (float)(Wl - 1);
    const float sf = (float)(Wl - 1) / 2.0f;
    for (int t = -g.r; t <= g.r; ++t) {
      const float x0 = (float)t + xl;
      const float xg = 2.0f * x0 / denom - 1.0f;
      const float ix = (xg + 1.0f) * sf;
      float xw = floorf(ix);
      const float w = ix - xw;
      const float e = 1.0f - w;
      xw = fminf(fmaxf(xw, -2.0f), (float)Wl + 1.0f);  // keep the int conversion defined
      const int xi = (int)xw;
      const float v0 = (xi >= 0 && xi <= Wl - 1) ? lv[xi] : 0.0f;
      const float v1 = (xi + 1 >= 0 && xi + 1 <= Wl - 1) ? lv[xi + 1] : 0.0f;
      o[(long)(l * K + t + g.r) * hw] = v0 * e + v1 * w;
    }
  }
}

// Lookup fused with the motion encoder's first layer (update.py:75, 84): convc1 is a 1x1
// conv of the L*(2r+1) taps to COUT channels + bias + ReLU, applied by the thread that
// sampled them, so the taps never leave registers.  Weights [K][COUT] are wave-uniform
// (scalar loads); consecutive output channels pair up for packed FMAs.
// out: [B * nvol, COUT, H, W1], sample b * nvol + v (the reference's stereo / mono batch).
template <int L, int R, int COUT>
__global__ __launch_bounds__(256) void lookup_c1_kernel(const float *__restrict__ pa, const float *__restrict__ pb,
                                                        const float *__restrict__ cx, LGeo g, long npix,
                                                        const float *__restrict__ wt,
                                                        const float *__restrict__ bias, int nvol,
                                                        float *__restrict__ out) {
  constexpr int K = 2 * R + 1, NT = L * K;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int v = blockIdx.y;
  const float *__restrict__ pyr = v ? pb : pa;
  const long hw = (long)g.H * g.W1;
  const long b = p / hw, rem = p % hw;
  const float x = cx[b * g.cbs + rem];
  const float *__restrict__ row = pyr + p * g.rs;
  float f[NT];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int Wl = g.wid[l];
    const float *__restrict__ lv = row + g.off[l];
    const float xl = x / (float)(1 << l);
    const float denom = (float)(Wl - 1);
    const float sf = (float)(Wl - 1) / 2.0f;
#pragma unroll
    for (int t = -R; t <= R; ++t) {
      const float x0 = (float)t + xl;
      const float xg = 2.0f * x0 / denom - 1.0f;
      const float ix = (xg + 1.0f) * sf;
      float xw = floorf(ix);
      const float w = ix - xw;
      const float e = 1.0f - w;
      xw = fminf(fmaxf(xw, -2.0f), (float)Wl + 1.0f);
      const int xi = (int)xw;
      const float v0 = (xi >= 0 && xi <= Wl - 1) ? lv[xi] : 0.0f;
      const float v1 = (xi + 1 >= 0 && xi + 1 <= Wl - 1) ? lv[xi + 1] : 0.0f;
      f[l * K + t + R] = v0 * e + v1 * w;
    }
  }
  float *__restrict__ o = out + (b * nvol + v) * COUT * hw + rem;
#pragma unroll 4
  for (int c0 = 0; c0 < COUT; c0 += 8) {
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = bias[c0 + c];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = fmaf(wt[k * COUT + c0 + c], f[k], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) o[(long)(c0 + c) * hw] = fmaxf(acc[c], 0.0f);
  }
}

// The same, with each level's taps gathered from four aligned float4 buffer loads instead
// of 2 * (2R+1) scalar loads: one thread per pixel used to touch ~2 cache lines per tap load
// across 64 rows, which thrashes L1 and re-fetches every line from L2 for every tap.  The
// float4s cover [x_-R - 1, x_-R + 2R + 3] of the level (the floor of every tap's own grid
// position lies within 1 of x_-R + t; its fp32 rounding is reproduced exactly per tap), the
// alignment shift is undone with selects, and every tap picks its two cells with 3-way
// selects.  Loads past the buffer return 0 (cells outside [0, W_l - 1] are zeroed anyway).
// MF: convc1 on fp32 MFMA (convc1_mfma.h; the same k-ordered fmaf chain as the VALU loop)
template <int L, int R, int COUT, bool MF = false>
__global__ __launch_bounds__(256) void lookup_c1_vec_kernel(const float *__restrict__ pa, const float *__restrict__ pb,
                                                            const float *__restrict__ cx, LGeo g, int npix,
                                                            int pyr_bytes, const float *__restrict__ wt,
                                                            const float *__restrict__ bias, int nvol,
                                                            float *__restrict__ out) {
  constexpr int K = 2 * R + 1, NT = L * K, WIN = 2 * R + 4;   // cells x_-R - 1 .. x_-R + 2R + 2
  static_assert(WIN + 3 <= 16, "four float4s cover the window at any alignment");
  static_assert(!MF || COUT == 64, "MFMA convc1: 64 outputs");
  __shared__ float c1lds[MF ? 4 : 1][MF ? NT * sa::C1_PITCH : 1];
  const int p0 = blockIdx.x * 256 + threadIdx.x;
  if (!MF && p0 >= npix) return;
  // (MFMA: every lane of the wave takes part; lanes past the end sample the last pixel and
  // store nothing)
  const int p = p0 < npix ? p0 : npix - 1;
  const int v = blockIdx.y;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(v ? pb : pa), (short)0, pyr_bytes, 0x00020000);
  const int hw = g.H * g.W1;
  const int b = p / hw, rem = p - b * hw;
  const float x = cx[(long)b * g.cbs + rem];
  float f[NT];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int Wl = g.wid[l];
    const float xl = x / (float)(1 << l);
    const float denom = (float)(Wl - 1);
    const float sf = (float)(Wl - 1) / 2.0f;
    int xi[K];
    float wgt[K];
#pragma unroll
    for (int t = -R; t <= R; ++t) {
      const float x0 = (float)t + xl;
      const float xg = 2.0f * x0 / denom - 1.0f;
      const float ix = (xg + 1.0f) * sf;
      float xw = floorf(ix);
      wgt[t + R] = ix - xw;
      // a wide clamp only keeps the int conversion defined: consecutive taps then stay
      // within 1 of x_-R + t (a tight clamp to [-2, W_l + 1] would break that), and a
      // cell's in/out-of-range status is the same as the reference's
      xw = fminf(fmaxf(xw, -16777216.0f), 16777216.0f);
      xi[t + R] = (int)xw;
    }
    // window start (float index in the buffer) and its float4-aligned base
    const long start = (long)p * g.rs + g.off[l] + xi[0] - 1;
    float cell[WIN];   // cell[k] = level value at x_-R - 1 + k
    if (start >= 0) {
      const long abase = start & ~3L;
      const int sh = (int)(start - abase);
      float wv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (unsigned)(abase * 4) + 16 * q, 0, 0);
        wv[4 * q + 0] = __uint_as_float(u[0]);
        wv[4 * q + 1] = __uint_as_float(u[1]);
        wv[4 * q + 2] = __uint_as_float(u[2]);
        wv[4 * q + 3] = __uint_as_float(u[3]);
      }
#pragma unroll
      for (int k = 0; k < WIN; ++k)
        cell[k] = sh == 0 ? wv[k] : sh == 1 ? wv[k + 1] : sh == 2 ? wv[k + 2] : wv[k + 3];
    } else {   // only the buffer's first row, level 0, with x_-R <= 0: cells before it are unused
      const float *q = v ? pb : pa;
#pragma unroll
      for (int k = 0; k < WIN; ++k) cell[k] = start + k >= 0 ? q[start + k] : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int d = xi[t] - xi[0] - t;   // -1, 0 or +1 (fp32 rounding of the grid position)
      const float c0 = d == 0 ? cell[t + 1] : d < 0 ? cell[t] : cell[t + 2];
      const float c1 = d == 0 ? cell[t + 2] : d < 0 ? cell[t + 1] : cell[t + 3 < WIN ? t + 3 : WIN - 1];
      const float v0 = (xi[t] >= 0 && xi[t] <= Wl - 1) ? c0 : 0.0f;
      const float v1 = (xi[t] + 1 >= 0 && xi[t] + 1 <= Wl - 1) ? c1 : 0.0f;
      const float w = wgt[t];
      f[l * K + t] = v0 * (1.0f - w) + v1 * w;
    }
  }
  if constexpr (MF) {
    const int lane = threadIdx.x & 63;
    sa::C1Weights<NT> w;
    sa::c1_load_weights<NT>(wt, bias, lane, w);
    const int wp0 = p0 - lane;   // the wave's first pixel
    sa::c1_mfma<NT>(f, w, c1lds[threadIdx.x >> 6], lane, [&](int q, int gq, const auto &r) {
      sa::c1_store4(out, wp0 + 16 * q + 4 * (lane >> 4), 16 * gq + (lane & 15), hw, nvol, v, npix, r);
    });
    return;
  }
  float *__restrict__ o = out + ((long)b * nvol + v) * COUT * hw + rem;
#pragma unroll 4
  for (int c0 = 0; c0 < COUT; c0 += 8) {
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = bias[c0 + c];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = fmaf(wt[k * COUT + c0 + c], f[k], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) o[(long)(c0 + c) * hw] = fmaxf(acc[c], 0.0f);
  }
}

}  // namespace

// convc1 of the fused lookups on the VALU (0, default) or on fp32 MFMA (1): the MFMA form measured
// slower (scripts/bench_lookup.py: 64.9 vs 55.6 us at B = 4 x 136 x 240, 816 vs 707 us on the
// sheared booster batch): the lookup is bound by its gathers, and the taps' LDS round trip and
// the lower occupancy (3 instead of 4 waves per SIMD) cost more than the FMAs it removes
static int sa_lookup_mfma = 0;
extern "C" void sa_lookup_set_mfma(int on) { sa_lookup_mfma = on ? 1 : 0; }
extern "C" int sa_lookup_get_mfma() { return sa_lookup_mfma; }

extern "C" int sa_corr_lookup_conv1x1(const float *pyramid_a, const float *pyramid_b, int W2, long row_stride,
                                      int num_levels, int radius, const float *coords_x, long coords_bstride,
                                      int B, int H, int W1, const float *weight_kc, const float *bias, int Cout,
                                      float *out, void *stream) {
  SA_REQUIRE(pyramid_a && coords_x && out && weight_kc && bias, "sa_corr_lookup_conv1x1: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 0 && W2 > 0, "sa_corr_lookup_conv1x1: empty shape");
  SA_REQUIRE(num_levels == 4 && radius == 4 && Cout == 64,
             "sa_corr_lookup_conv1x1: built for 4 levels, radius 4, 64 outputs (got %d, %d, %d)", num_levels, radius,
             Cout);
  SA_REQUIRE(sa_pyramid_level_width(W2, num_levels - 1) >= 2,
             "sa_corr_lookup_conv1x1: level %d of width %d is too narrow to sample", num_levels - 1,
             sa_pyramid_level_width(W2, num_levels - 1));
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels), "sa_corr_lookup_conv1x1: row_stride too small");
  const int nvol = pyramid_b ? 2 : 1;
  LGeo g{};
  g.H = H;
  g.W1 = W1;
  g.L = num_levels;
  g.r = radius;
  g.rs = row_stride;
  g.cbs = coords_bstride;
  for (int i = 0; i < 4; ++i) {
    g.off[i] = sa_pyramid_level_offset(W2, i);
    g.wid[i] = sa_pyramid_level_width(W2, i);
  }
  const long npix = (long)B * H * W1;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LOOKUP, s);
  dim3 grid((unsigned)((npix + 255) / 256), nvol);
  const long pyr_bytes = npix * row_stride * 4;
  if (pyr_bytes < (1L << 31) - 64 && row_stride % 4 == 0 && (long)H * W1 < (1L << 30)) {
    if (sa_lookup_mfma)
      lookup_c1_vec_kernel<4, 4, 64, true><<<grid, 256, 0, s>>>(pyramid_a, pyramid_b ? pyramid_b : pyramid_a, coords_x,
                                                                g, (int)npix, (int)pyr_bytes, weight_kc, bias, nvol, out);
    else
      lookup_c1_vec_kernel<4, 4, 64><<<grid, 256, 0, s>>>(pyramid_a, pyramid_b ? pyramid_b : pyramid_a, coords_x, g,
                                                          (int)npix, (int)pyr_bytes, weight_kc, bias, nvol, out);
    return sa::check_launch("sa_corr_lookup_conv1x1");
  }
  lookup_c1_kernel<4, 4, 64><<<grid, 256, 0, s>>>(pyramid_a, pyramid_b ? pyramid_b : pyramid_a, coords_x, g, npix,
                                                  weight_kc, bias, nvol, out);
  return sa::check_launch("sa_corr_lookup_conv1x1");
}

extern "C" int sa_corr_lookup(const float *pyramid_a, const float *pyramid_b, int W2, long row_stride,
                              int num_levels, int radius, const float *coords_x, long coords_bstride,
                              int B, int H, int W1, float *out, long out_bstride, void *stream) {
  SA_REQUIRE(pyramid_a && coords_x && out, "sa_corr_lookup: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 0 && W2 > 0, "sa_corr_lookup: empty shape");
  SA_REQUIRE(num_levels >= 1 && num_levels <= 4, "sa_corr_lookup: num_levels must be 1..4");
  SA_REQUIRE(radius >= 0 && radius <= 16, "sa_corr_lookup: radius must be 0..16");
  SA_REQUIRE(sa_pyramid_level_width(W2, num_levels - 1) >= 2,
             "sa_corr_lookup: level %d of width %d is too narrow to sample", num_levels - 1,
             sa_pyramid_level_width(W2, num_levels - 1));
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels), "sa_corr_lookup: row_stride too small");
  const int nvol = pyramid_b ? 2 : 1;
  SA_REQUIRE(out_bstride >= (long)nvol * num_levels * (2 * radius + 1) * H * W1,
             "sa_corr_lookup: out batch stride too small");
  LGeo g{};
  g.H = H;
  g.W1 = W1;
  g.L = num_levels;
  g.r = radius;
  g.rs = row_stride;
  g.cbs = coords_bstride;
  g.obs = out_bstride;
  for (int i = 0; i < 4; ++i) {
    g.off[i] = sa_pyramid_level_offset(W2, i);
    g.wid[i] = sa_pyramid_level_width(W2, i);
  }
  const long npix = (long)B * H * W1;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LOOKUP, s);
  dim3 grid((unsigned)((npix + 255) / 256), nvol);
  lookup_kernel<<<grid, 256, 0, s>>>(pyramid_a, pyramid_b ? pyramid_b : pyramid_a, coords_x, g, npix, out);
  return sa::check_launch("sa_corr_lookup");
}
