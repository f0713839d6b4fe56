// Normalisation / activation / residual epilogues of the 2-D convolutions that stay on
// MIOpen: the feature and context encoders (extractor.py:6-300) and the update block's
// bias + ReLU pairs (update.py:64-90, 98-110).
//
// PyTorch runs each conv as conv + bias-add, then a norm (statistics + apply), then a ReLU,
// and a residual add + ReLU: four to six full passes over a tensor that is 1 GB at full
// resolution for the 8-image feature batch.  Here a conv output is written once by MIOpen
// (bias dropped) and then read by
//   sa_plane_stats  InstanceNorm2d statistics (biased variance, fp64 sums) per (b, c)
//                   plane — only for instance-norm layers;
//   sa_norm_act     out = act_out( act_in((x - m) * s + t) + skip_term ),
//                   skip_term = act_skip((skip - m') * s' + t')  or  act_skip(skip),
//                   so bias (m = -b), eval BatchNorm (m = mean - b, s = gamma / sqrt(var +
//                   eps), t = beta), InstanceNorm (m = mean, s = rstd), ReLU / tanh and the
//                   residual block's projection norm + add + ReLU are one pass.
// Parameters are per channel (pstride 0) or per (b, c) plane (pstride C).
#include <cmath>

#include "sa_common.h"

namespace {

constexpr int kAct_relu = 1, kAct_tanh = 2;  // 0: none

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == kAct_relu) return fmaxf(v, 0.0f);
  if (act == kAct_tanh) return tanhf(v);
  return v;
}

__global__ __launch_bounds__(256) void plane_stats_kernel(const float *__restrict__ x, long x_bs, int C, long hw,
                                                          float eps, float *__restrict__ mean,
                                                          float *__restrict__ rstd) {
  const int plane = blockIdx.x;
  const int b = plane / C, c = plane % C;
  const float *p = x + b * x_bs + (long)c * hw;
  double s = 0.0, q = 0.0;
  if ((hw & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    for (long i = threadIdx.x; i < hw / 4; i += 256) {
      const float4 v = p4[i];
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
      q += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
  } else {
    for (long i = threadIdx.x; i < hw; i += 256) {
      const double v = p[i];
      s += v;
      q += v * v;
    }
  }
  __shared__ double rs[4], rq[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double S = (rs[0] + rs[1]) + (rs[2] + rs[3]), Q = (rq[0] + rq[1]) + (rq[2] + rq[3]);
    const double m = S / (double)hw;
    double var = Q / (double)hw - m * m;
    if (var < 0.0) var = 0.0;
    mean[plane] = (float)m;
    rstd[plane] = (float)(1.0 / std::sqrt(var + (double)eps));
  }
}

struct Affine {
  const float *m, *s, *t;  // each nullable: 0 / 1 / 0
  int pstride;             // 0: per channel, C: per (b, c) plane
  __device__ __forceinline__ void load(int b, int c, float &mm, float &ss, float &tt) const {
    const int i = b * pstride + c;
    mm = m ? m[i] : 0.0f;
    ss = s ? s[i] : 1.0f;
    tt = t ? t[i] : 0.0f;
  }
};

// grid: x over the plane in chunks of 256 * VEC elements, y = b * C + c
template <int VEC>
__global__ __launch_bounds__(256) void norm_act_kernel(const float *__restrict__ x, long x_bs, int C, long hw,
                                                       Affine ax, int act_in, const float *__restrict__ skip,
                                                       long skip_bs, Affine as, int act_skip, int act_out,
                                                       float *__restrict__ out, long out_bs) {
  const int plane = blockIdx.y, b = plane / C, c = plane % C;
  float m, s, t, sm = 0.0f, ss = 1.0f, st = 0.0f;
  ax.load(b, c, m, s, t);
  if (skip) as.load(b, c, sm, ss, st);
  const bool skip_aff = as.m || as.s || as.t;
  const long base = (long)c * hw;
  const long i0 = ((long)blockIdx.x * 256 + threadIdx.x) * VEC;
  if (i0 >= hw) return;
  float v[VEC], k[VEC];
  if (VEC == 4) {
    const float4 a = *reinterpret_cast<const float4 *>(x + b * x_bs + base + i0);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    if (skip) {
      const float4 e = *reinterpret_cast<const float4 *>(skip + b * skip_bs + base + i0);
      k[0] = e.x; k[1] = e.y; k[2] = e.z; k[3] = e.w;
    }
  } else {
    v[0] = x[b * x_bs + base + i0];
    if (skip) k[0] = skip[b * skip_bs + base + i0];
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    float y = act_fn((v[j] - m) * s + t, act_in);
    if (skip) y = y + act_fn(skip_aff ? (k[j] - sm) * ss + st : k[j], act_skip);
    v[j] = act_fn(y, act_out);
  }
  if (VEC == 4) {
    *reinterpret_cast<float4 *>(out + b * out_bs + base + i0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    out[b * out_bs + base + i0] = v[0];
  }
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int sa_plane_stats(const float *x, long x_bs, int B, int C, long hw, float eps, float *mean, float *rstd,
                              void *stream) {
  SA_REQUIRE(x && mean && rstd && B > 0 && C > 0 && hw > 0, "sa_plane_stats: bad arguments");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_NORM, s);
  plane_stats_kernel<<<B * C, 256, 0, s>>>(x, x_bs, C, hw, eps, mean, rstd);
  return sa::check_launch("sa_plane_stats");
}

extern "C" int sa_norm_act(const float *x, long x_bs, int B, int C, long hw, const float *m, const float *sc,
                           const float *t, int pstride, int act_in, const float *skip, long skip_bs,
                           const float *skip_m, const float *skip_s, const float *skip_t, int skip_pstride,
                           int act_skip, int act_out, float *out, long out_bs, void *stream) {
  SA_REQUIRE(x && out && B > 0 && C > 0 && hw > 0, "sa_norm_act: bad arguments");
  SA_REQUIRE(act_in >= 0 && act_in <= 2 && act_out >= 0 && act_out <= 2 && act_skip >= 0 && act_skip <= 2,
             "sa_norm_act: unknown activation");
  SA_REQUIRE(pstride == 0 || pstride == C, "sa_norm_act: pstride must be 0 or C");
  SA_REQUIRE(skip_pstride == 0 || skip_pstride == C, "sa_norm_act: skip_pstride must be 0 or C");
  SA_REQUIRE((long)B * C <= 65535, "sa_norm_act: too many planes");
  Affine ax{m, sc, t, pstride}, as{skip_m, skip_s, skip_t, skip_pstride};
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_NORM, s);
  const bool vec = (hw % 4 == 0) && x_bs % 4 == 0 && out_bs % 4 == 0 && (!skip || skip_bs % 4 == 0) &&
                   aligned16(x) && aligned16(out) && (!skip || aligned16(skip));
  if (vec) {
    dim3 grid((unsigned)((hw / 4 + 255) / 256), (unsigned)(B * C));
    norm_act_kernel<4><<<grid, 256, 0, s>>>(x, x_bs, C, hw, ax, act_in, skip, skip_bs, as, act_skip, act_out, out,
                                            out_bs);
  } else {
    dim3 grid((unsigned)((hw + 255) / 256), (unsigned)(B * C));
    norm_act_kernel<1><<<grid, 256, 0, s>>>(x, x_bs, C, hw, ax, act_in, skip, skip_bs, as, act_skip, act_out, out,
                                            out_bs);
  }
  return sa::check_launch("sa_norm_act");
}
