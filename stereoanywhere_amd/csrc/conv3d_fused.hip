// Full-resolution tail of the mono hourglass as fused direct 3-D convolutions.
//
// Reference: Hourglass.forward tail (hourglass.py:325-329) = trilinear upsample +
// cat + final_agg (three BasicConv3d: conv -> InstanceNorm3d -> LeakyReLU,
// submodule.py:25-53) + final_feature_atts_up (DoubleFeatureAtt, submodule.py:113-140),
// then classifier_mono / classifier_monoconf (stereoanywhere.py:73-74, 165-166).
//
// At 544x960 these run on [B, 8, 240, 136, 240] volumes (7.8 M voxels per channel per
// pair): with 8 channels the convolutions are tiny GEMMs, and the library path spent
// ~14 ms per conv plus separate statistic / normalise / activation / gate passes.
// Here every layer is one pass over HBM:
//   * the conv applies the PREVIOUS layer's InstanceNorm + LeakyReLU (+ gate) to its
//     input while staging it in LDS (zero padding applies to the activated input);
//   * the epilogue writes the raw conv output and per-block (sum, sum of squares) of
//     each (b, co) channel for the NEXT layer's InstanceNorm (float64 partials, reduced
//     in fixed order by sa_instnorm_finalize: deterministic);
//   * the first layer (1x1x1 over cat(orig, up(x))) evaluates the trilinear upsample of
//     the half-resolution branch on the fly, so the 16-channel full-res upsampled
//     tensor and the concatenation are never materialised;
//   * both classifiers share one conv launch (Cout = 2).
// Layout everywhere: [B, C, D, H, W] with D = W2 (right pixel), W = W1 (left pixel).
#include <cmath>

#include "sa_common.h"

namespace {

// Output tiles: 256 threads = TW (along W) x TH (along H); each thread owns TD planes
// along D.  Stride-1 tiles are one wave wide (TW 64); stride-2 tiles are 32 x 8 so the
// (2*T+1)-wide input halo stays small.
constexpr int TW = 64;  // default tile (stride 1) along W
constexpr int TH = 4;   // along H
constexpr int TD = 4;   // output planes per thread along D

struct InXform {
  const float *mean, *rstd;   // per (b, ci), or null
  const float *gl, *gr;       // gate maps [B, C, H, W] and [B, C, H, D] (sigmoid'ed), or null
  float slope;                // LeakyReLU slope
  int act;                    // apply LeakyReLU
};

__device__ __forceinline__ float xform(float v, const InXform &t, long bc, int d, int h, int w, int H, int W, int D) {
  if (t.mean) v = (v - t.mean[bc]) * t.rstd[bc];
  if (t.act) v = v > 0.0f ? v : v * t.slope;
  if (t.gl) {
    const float g = t.gl[(bc * H + h) * W + w] * t.gr[(bc * H + h) * D + d];
    v = g * v;
  }
  return v;
}

// block partial sums of (x, x^2) over the tile for each of NC channels -> partial[bc][blk]
template <int NC>
__device__ __forceinline__ void block_stats(const double (&s)[NC], const double (&q)[NC], double *red,
                                            double *partial, long b, int nparts, int blk, int Cout) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double a = s[c], e = q[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      e += __shfl_xor(e, o);
    }
    if (lane == 0) {
      red[(c * 4 + wv) * 2] = a;
      red[(c * 4 + wv) * 2 + 1] = e;
    }
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    const int c = threadIdx.x;
    double a = 0.0, e = 0.0;
    for (int w = 0; w < 4; ++w) {
      a += red[(c * 4 + w) * 2];
      e += red[(c * 4 + w) * 2 + 1];
    }
    double *p = partial + ((b * Cout + c) * (long)nparts + blk) * 2;
    p[0] = a;
    p[1] = e;
  }
}

// 3x3x3, stride S, padding 1, no bias; CIN input channels, COUT outputs.
template <int CIN, int COUT, int S, int TDx, int TWx, int THx>
__global__ __launch_bounds__(256) void conv3d_kernel(const float *__restrict__ in, int Di, int Hi, int Wi, int Do,
                                                     int Ho, int Wo, const float *__restrict__ wt, InXform tx,
                                                     float *__restrict__ out, double *__restrict__ partial,
                                                     int tilesD) {
  static_assert(TWx * THx == 256, "256 threads per block");
  constexpr int LW = (TWx - 1) * S + 3, LH = (THx - 1) * S + 3, LD = (TDx - 1) * S + 3;
  constexpr int LPLANE = LD * LH * LW;
  __shared__ float tile[2][LPLANE];
  __shared__ double red[COUT * 4 * 2];
  const int tx_ = threadIdx.x % TWx, ty = threadIdx.x / TWx;
  const int w0 = blockIdx.x * TWx, h0 = blockIdx.y * THx;
  const int b = blockIdx.z / tilesD, d0 = (blockIdx.z % tilesD) * TDx;
  const long vol = (long)Di * Hi * Wi;
  const int iw0 = w0 * S - 1, ih0 = h0 * S - 1, id0 = d0 * S - 1;
  float acc[TDx][COUT];
#pragma unroll
  for (int i = 0; i < TDx; ++i)
#pragma unroll
    for (int c = 0; c < COUT; ++c) acc[i][c] = 0.f;

  auto stage = [&](int ci, int buf) {
    const long bc = (long)b * CIN + ci;
    const float *src = in + bc * vol;
    for (int i = threadIdx.x; i < LPLANE; i += 256) {
      const int ww = i % LW, r = i / LW, hh = r % LH, dd = r / LH;
      const int w = iw0 + ww, h = ih0 + hh, d = id0 + dd;
      float v = 0.0f;
      if (w >= 0 && w < Wi && h >= 0 && h < Hi && d >= 0 && d < Di)
        v = xform(src[((long)d * Hi + h) * Wi + w], tx, bc, d, h, w, Hi, Wi, Di);
      tile[buf][i] = v;
    }
  };

  stage(0, 0);
  __syncthreads();
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    const int buf = ci & 1;
    if (ci + 1 < CIN) stage(ci + 1, buf ^ 1);
    const float *tb = tile[buf] + (ty * S) * LW + tx_ * S;
    const float *wc = wt + (long)ci * 27 * COUT;  // weights pre-arranged [ci][tap][co]
#pragma unroll 1
    for (int kd = 0; kd < 3; ++kd) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float *tp = tb + (kd * LH + kh) * LW + kw;
          float v[TDx];
#pragma unroll
          for (int od = 0; od < TDx; ++od) v[od] = tp[od * S * LH * LW];
          const float *wp = wc + ((kd * 3 + kh) * 3 + kw) * COUT;
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float wv = wp[co];
#pragma unroll
            for (int od = 0; od < TDx; ++od) acc[od][co] += wv * v[od];
          }
        }
    }
    __syncthreads();
  }

  const int w = w0 + tx_, h = h0 + ty;
  double s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0;
  if (w < Wo && h < Ho) {
#pragma unroll
    for (int od = 0; od < TDx; ++od) {
      const int d = d0 + od;
      if (d < Do) {
#pragma unroll
        for (int co = 0; co < COUT; ++co) {
          out[(((long)b * COUT + co) * Do + d) * (long)Ho * Wo + (long)h * Wo + w] = acc[od][co];
          s[co] += (double)acc[od][co];
          q[co] += (double)acc[od][co] * acc[od][co];
        }
      }
    }
  }
  if (partial) {
    const int nparts = gridDim.x * gridDim.y * tilesD;
    const int blk = (blockIdx.z % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
    block_stats<COUT>(s, q, red, partial, b, nparts, blk, COUT);
  }
}

// 1x1x1 conv over cat(Ta(a), trilinear_up(u)) -> COUT channels, + IN partial statistics.
// The low-resolution branch u arrives already transformed (sa_vol_apply): evaluating its
// gate at all 8 corners of every voxel made this kernel load-issue bound.
template <int CA, int CU, int COUT, bool AX>
__global__ __launch_bounds__(256) void pointwise_upcat_kernel(const float *__restrict__ a, InXform ta,
                                                              const float *__restrict__ u, int D, int H,
                                                              int W, int Du, int Hu, int Wu, float sd, float sh,
                                                              float sw, const float *__restrict__ wt,
                                                              float *__restrict__ out, double *__restrict__ partial,
                                                              int tilesD) {
  __shared__ double red[COUT * 4 * 2];
  const int tx_ = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int w = blockIdx.x * TW + tx_, h = blockIdx.y * TH + ty;
  const int b = blockIdx.z / tilesD, d0 = (blockIdx.z % tilesD) * TD;
  const long vol = (long)D * H * W, volu = (long)Du * Hu * Wu;
  double s[COUT], q[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) s[c] = q[c] = 0.0;
  if (w < W && h < H) {
    // upsample_trilinear3d(align_corners=True) source coordinates (h, w fixed per thread)
    const float rh = sh * (float)h, rw = sw * (float)w;
    const int h1 = (int)rh, w1 = (int)rw;
    const int h1p = h1 < Hu - 1 ? 1 : 0, w1p = w1 < Wu - 1 ? 1 : 0;
    const float hl1 = rh - (float)h1, hl0 = 1.0f - hl1, wl1 = rw - (float)w1, wl0 = 1.0f - wl1;
    for (int od = 0; od < TD; ++od) {
      const int d = d0 + od;
      if (d >= D) break;
      const float rd = sd * (float)d;
      const int d1 = (int)rd;
      const int d1p = d1 < Du - 1 ? 1 : 0;
      const float dl1 = rd - (float)d1, dl0 = 1.0f - dl1;
      const long pos = ((long)d * H + h) * W + w;
      float r[COUT];
#pragma unroll
      for (int co = 0; co < COUT; ++co) r[co] = 0.0f;
      // weights pre-arranged [cin][co] with the a-rows first
#pragma unroll 1
      for (int c = 0; c < CA; ++c) {
        const long bc = (long)b * CA + c;
        const float av = a[bc * vol + pos];
        const float xv = AX ? xform(av, ta, bc, d, h, w, H, W, D) : av;
#pragma unroll
        for (int co = 0; co < COUT; ++co) r[co] += wt[c * COUT + co] * xv;
      }
      const long o000 = ((long)d1 * Hu + h1) * Wu + w1;
      const long od_ = (long)d1p * Hu * Wu, oh_ = (long)h1p * Wu, ow_ = w1p;
#pragma unroll 1
      for (int c = 0; c < CU; ++c) {
        const float *p = u + ((long)b * CU + c) * volu + o000;
        const float xv = dl0 * (hl0 * (wl0 * p[0] + wl1 * p[ow_]) + hl1 * (wl0 * p[oh_] + wl1 * p[oh_ + ow_])) +
                         dl1 * (hl0 * (wl0 * p[od_] + wl1 * p[od_ + ow_]) +
                                hl1 * (wl0 * p[od_ + oh_] + wl1 * p[od_ + oh_ + ow_]));
#pragma unroll
        for (int co = 0; co < COUT; ++co) r[co] += wt[(CA + c) * COUT + co] * xv;
      }
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        out[((long)b * COUT + co) * vol + pos] = r[co];
        s[co] += (double)r[co];
        q[co] += (double)r[co] * r[co];
      }
    }
  }
  const int nparts = gridDim.x * gridDim.y * tilesD;
  const int blk = (blockIdx.z % tilesD) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
  block_stats<COUT>(s, q, red, partial, b, nparts, blk, COUT);
}

// T(x) materialised (for the low-resolution branch an up-cat conv reads at 8 corners)
__global__ __launch_bounds__(256) void vol_apply_kernel(const float *__restrict__ in, InXform tx, int C, int D, int H,
                                                        int W, long n, float *__restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int w = (int)(i % W);
  const long r = i / W;
  const int h = (int)(r % H);
  const long r2 = r / H;
  const int d = (int)(r2 % D);
  const long bc = r2 / D;
  out[i] = xform(in[i], tx, bc, d, h, w, H, W, D);
}

// one block per (b, c): fixed-shape tree reduction of the float64 partials (deterministic)
__global__ __launch_bounds__(256) void instnorm_finalize_kernel(const double *__restrict__ partial, int nparts,
                                                                double count, float eps, float *__restrict__ mean,
                                                                float *__restrict__ rstd) {
  __shared__ double rs[256], rq[256];
  const int bc = blockIdx.x, t = threadIdx.x;
  const double *p = partial + (long)bc * nparts * 2;
  double s = 0.0, q = 0.0;
  for (int i = t; i < nparts; i += 256) {
    s += p[2 * i];
    q += p[2 * i + 1];
  }
  rs[t] = s;
  rq[t] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      rs[t] += rs[t + o];
      rq[t] += rq[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double m = rs[0] / count;
    double var = rq[0] / count - m * m;
    if (var < 0.0) var = 0.0;
    mean[bc] = (float)m;
    rstd[bc] = (float)(1.0 / std::sqrt(var + (double)eps));
  }
}

struct ConvGeo {
  int td, tw, th;
};

inline ConvGeo conv_geo(int cout, int stride) {
  if (stride == 2) return {2, 32, 8};
  return {cout >= 32 ? 2 : 4, 64, 4};
}

inline dim3 conv_grid(int B, int Do, int Ho, int Wo, ConvGeo g, int &tilesD) {
  tilesD = (Do + g.td - 1) / g.td;
  return dim3((Wo + g.tw - 1) / g.tw, (Ho + g.th - 1) / g.th, tilesD * B);
}

inline int out_size(int n, int stride) { return (n - 1) / stride + 1; }  // k3, pad 1

}  // namespace

extern "C" long sa_conv3d_stat_parts(int Cout, int stride, int Do, int Ho, int Wo) {
  int tilesD;
  dim3 g = conv_grid(1, Do, Ho, Wo, conv_geo(Cout, stride), tilesD);
  return (long)g.x * g.y * g.z;
}

extern "C" int sa_conv3d(const float *in, int B, int Cin, int Di, int Hi, int Wi, int stride, const float *weight,
                         int Cout, const float *in_mean, const float *in_rstd, int act, float slope,
                         const float *gate_l, const float *gate_r, float *out, double *stats_partial, void *stream) {
  SA_REQUIRE(in && weight && out, "sa_conv3d: null pointer");
  SA_REQUIRE(B > 0 && Di > 0 && Hi > 0 && Wi > 0, "sa_conv3d: empty shape");
  SA_REQUIRE((in_mean == nullptr) == (in_rstd == nullptr), "sa_conv3d: mean and rstd go together");
  SA_REQUIRE((gate_l == nullptr) == (gate_r == nullptr), "sa_conv3d: both gate maps or none");
  const int Do = out_size(Di, stride), Ho = out_size(Hi, stride), Wo = out_size(Wi, stride);
  const ConvGeo geo = conv_geo(Cout, stride);
  int tilesD;
  dim3 grid = conv_grid(B, Do, Ho, Wo, geo, tilesD);
  InXform tx{in_mean, in_rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
#define SA_CONV(CI, CO, S, TDV, TWV, THV)                                                                   \
  if (Cin == CI && Cout == CO && stride == S) {                                                              \
    conv3d_kernel<CI, CO, S, TDV, TWV, THV><<<grid, 256, 0, s>>>(in, Di, Hi, Wi, Do, Ho, Wo, weight, tx, out, \
                                                                stats_partial, tilesD);                      \
    return sa::check_launch("sa_conv3d");                                                                    \
  }
  SA_CONV(8, 8, 1, 4, 64, 4)
  SA_CONV(8, 2, 1, 4, 64, 4)
  SA_CONV(16, 16, 1, 4, 64, 4)
  SA_CONV(32, 32, 1, 2, 64, 4)
  SA_CONV(8, 16, 2, 2, 32, 8)
  SA_CONV(16, 32, 2, 2, 32, 8)
#undef SA_CONV
  sa::set_error("sa_conv3d: no kernel built for Cin %d -> Cout %d, stride %d", Cin, Cout, stride);
  return SA_E_ARG;
}

extern "C" int sa_conv3d_pointwise_upcat(const float *a, int Ca, const float *a_mean, const float *a_rstd, int a_act,
                                         const float *a_gl, const float *a_gr, const float *u, int Cu, int Du, int Hu,
                                         int Wu, int B, int D, int H, int W, float slope, const float *weight, int Cout,
                                         float *out, double *stats_partial, void *stream) {
  SA_REQUIRE(a && u && weight && out && stats_partial, "sa_conv3d_pointwise_upcat: null pointer");
  SA_REQUIRE(B > 0 && D > 1 && H > 1 && W > 1 && Du > 0 && Hu > 0 && Wu > 0,
             "sa_conv3d_pointwise_upcat: bad shape");
  const ConvGeo geo = conv_geo(8, 1);
  int tilesD;
  dim3 grid = conv_grid(B, D, H, W, geo, tilesD);
  // area_pixel_compute_scale(align_corners=True) = (in - 1) / (out - 1)
  const float sd = (float)(Du - 1) / (float)(D - 1), sh = (float)(Hu - 1) / (float)(H - 1),
              sw = (float)(Wu - 1) / (float)(W - 1);
  InXform ta{a_mean, a_rstd, a_gl, a_gr, slope, a_act};
  const bool ax = a_mean || a_act || a_gl;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
#define SA_PW(CA, CU, CO, AXV)                                                                                     \
  if (Ca == CA && Cu == CU && Cout == CO && ax == AXV) {                                                          \
    pointwise_upcat_kernel<CA, CU, CO, AXV><<<grid, 256, 0, s>>>(a, ta, u, D, H, W, Du, Hu, Wu, sd, sh, sw,       \
                                                                  weight, out, stats_partial, tilesD);             \
    return sa::check_launch("sa_conv3d_pointwise_upcat");                                                         \
  }
  SA_PW(8, 16, 8, false)
  SA_PW(16, 32, 16, true)
#undef SA_PW
  sa::set_error("sa_conv3d_pointwise_upcat: no kernel built for %d + %d -> %d (a transform %d)", Ca, Cu, Cout, ax);
  return SA_E_ARG;
}

extern "C" int sa_vol_apply(const float *in, int B, int C, int D, int H, int W, const float *mean, const float *rstd,
                            int act, float slope, const float *gate_l, const float *gate_r, float *out, void *stream) {
  SA_REQUIRE(in && out && B > 0 && C > 0 && D > 0 && H > 0 && W > 0, "sa_vol_apply: bad arguments");
  const long n = (long)B * C * D * H * W;
  InXform tx{mean, rstd, gate_l, gate_r, slope, act};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  vol_apply_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in, tx, C, D, H, W, n, out);
  return sa::check_launch("sa_vol_apply");
}

extern "C" int sa_instnorm_finalize(const double *partial, int bc_count, long nparts, long count, float eps,
                                    float *mean, float *rstd, void *stream) {
  SA_REQUIRE(partial && mean && rstd && bc_count > 0 && nparts > 0 && count > 0,
             "sa_instnorm_finalize: bad arguments");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  instnorm_finalize_kernel<<<bc_count, 256, 0, s>>>(partial, (int)nparts, (double)count, eps, mean, rstd);
  return sa::check_launch("sa_instnorm_finalize");
}
