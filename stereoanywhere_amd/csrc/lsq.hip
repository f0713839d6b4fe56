// Mono-scale alignment: softLRC, weighted LSQ with exact quantile band, mirror
// detector and initial coordinates.
//
// Reference: softlrc + disp_warping (utils.py:172-198), fuzzy_and (240-241),
// weighted_lsq (345-384), scaled mono maps (stereoanywhere.py:191-199),
// handcrafted_mirror_detector (utils.py:255-269), coords init (stereoanywhere.py:261-262).
//
// The reference's weighted_lsq runs torch.quantile + boolean indexing +
// torch.linalg.lstsq per sample: host syncs and a CPU-side LAPACK call on GPU.  Here
// one workgroup per sample finds the four order statistics the two linear quantiles
// need by an 8-bit-per-pass radix select on the float bits (relu'd values are
// non-negative, so their bit patterns order like the values), then accumulates the
// 2x2 weighted normal equations in float64 and solves them — no host round trip.
#include <cmath>

#include "sa_common.h"

namespace {

// ------------------------------------------------------------------ softLRC
__device__ __forceinline__ float softplus_ref(float x) {
  // torch softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}

// grid_sample(bilinear, zeros, align_corners=True) of one [H,W] plane at the grid
// point (gx, gy) already normalised to [-1, 1] (ATen CPU ApplyGridSample order).
__device__ __forceinline__ float sample_zero_ac(const float *__restrict__ img, int H, int W, float gx,
                                                float gy) {
  const float ix = (gx + 1.0f) * ((float)(W - 1) / 2.0f);
  const float iy = (gy + 1.0f) * ((float)(H - 1) / 2.0f);
  float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, e = 1.0f - w;
  const float n = iy - yn, s = 1.0f - n;
  const float nw = s * e, ne = s * w, sw = n * e, se = n * w;
  xw = fminf(fmaxf(xw, -2.0f), (float)W + 1.0f);
  yn = fminf(fmaxf(yn, -2.0f), (float)H + 1.0f);
  const int xi = (int)xw, yi = (int)yn;
  auto at = [&](int y, int x) {
    return (x >= 0 && x <= W - 1 && y >= 0 && y <= H - 1) ? img[(long)y * W + x] : 0.0f;
  };
  return at(yi, xi) * nw + at(yi, xi + 1) * ne + at(yi + 1, xi) * sw + at(yi + 1, xi + 1) * se;
}

// softlrc of pixel (y, x): compare d_self with d_other warped by relu(d_src)
// sign = -1: left map (sample at x - relu(d2)), +1: right map (x + relu(d3)).
__device__ __forceinline__ float softlrc_px(const float *__restrict__ dself, const float *__restrict__ dother,
                                            int H, int W, int y, int x, float sign, float th,
                                            float div) {
  const float dsrc = fmaxf(dself[(long)y * W + x], 0.0f);
  const float xn = sign < 0 ? ((float)x - dsrc) : ((float)x + dsrc);
  const float gx = 2.0f * (xn / (float)W) - 1.0f;
  const float gy = 2.0f * ((float)y / (float)H) - 1.0f;
  const float warped = sample_zero_ac(dother, H, W, gx, gy);
  const float d = dself[(long)y * W + x];
  return softplus_ref(-fabsf(d - warped) + th) / div;
}

__global__ __launch_bounds__(256) void softlrc_kernel(const float *__restrict__ d2, const float *__restrict__ d3,
                                                      const float *__restrict__ c2, const float *__restrict__ c3,
                                                      int H, int W, long bs, float th, float div, long npix,
                                                      float *__restrict__ s2, float *__restrict__ s3) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long b = p / hw, r = p % hw;
  const int y = (int)(r / W), x = (int)(r % W);
  const float *a = d2 + b * bs, *c = d3 + b * bs;
  // softlrc_disp2 uses warped_disp3 = disp_warping(relu(disp2), disp3, right_disp=False)
  float v2 = softlrc_px(a, c, H, W, y, x, -1.0f, th, div);
  float v3 = softlrc_px(c, a, H, W, y, x, +1.0f, th, div);
  if (c2) v2 = c2[b * bs + r] * v2;
  if (c3) v3 = c3[b * bs + r] * v3;
  s2[b * bs + r] = v2;
  s3[b * bs + r] = v3;
}

// ------------------------------------------------------------------ weighted LSQ
constexpr int LSQ_THREADS = 1024;

__device__ __forceinline__ unsigned key_of(float d) {
  d = fmaxf(d, 0.0f);  // F.relu (utils.py:352)
  if (d == 0.0f) d = 0.0f;  // -0 -> +0 so bit order == value order
  return __float_as_uint(d);
}

__device__ __forceinline__ float lerp_ref(float a, float b, float w) {
  // at::lerp CPU: |w| < 0.5 ? a + w (b - a) : b - (b - a)(1 - w)
  return fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < LSQ_THREADS / 64; ++i) t += red[i];  // fixed order: deterministic
  return t;
}

__global__ __launch_bounds__(LSQ_THREADS) void lsq_kernel(const float *__restrict__ mde, const float *__restrict__ disp,
                                                          const float *__restrict__ conf, int n, float q_lo,
                                                          float q_hi, float *__restrict__ scale,
                                                          float *__restrict__ shift) {
  __shared__ unsigned hist[4][256];
  __shared__ unsigned prefix[4];
  __shared__ unsigned remain[4];
  __shared__ double red[LSQ_THREADS / 64];
  __shared__ float qv[2];
  const int b = blockIdx.x;
  const float *md = mde + (long)b * n, *dd = disp + (long)b * n, *cd = conf + (long)b * n;
  const int t = threadIdx.x;

  // ranks of torch.quantile(linear): rank = q * (n - 1) in fp32
  const float r_lo = q_lo * (float)(n - 1), r_hi = q_hi * (float)(n - 1);
  if (t < 4) {
    const float r = (t < 2) ? r_lo : r_hi;
    const float idx = (t & 1) ? ceilf(r) : truncf(r);
    remain[t] = (unsigned)idx;
    prefix[t] = 0u;
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift_ = 24 - 8 * pass;
    for (int i = t; i < 4 * 256; i += LSQ_THREADS) (&hist[0][0])[i] = 0u;
    __syncthreads();
    unsigned pre[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pre[r] = prefix[r];
    for (int i = t; i < n; i += LSQ_THREADS) {
      const unsigned k = key_of(dd[i]);
      const unsigned bin = (k >> shift_) & 255u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool match = pass == 0 || ((k ^ pre[r]) >> (shift_ + 8)) == 0u;
        if (match) atomicAdd(&hist[r][bin], 1u);
      }
    }
    __syncthreads();
    if (t < 4) {
      unsigned rem = remain[t], acc = 0u, sel = 255u;
      for (unsigned bin = 0; bin < 256u; ++bin) {
        const unsigned c = hist[t][bin];
        if (acc + c > rem) {
          sel = bin;
          break;
        }
        acc += c;
      }
      remain[t] = rem - acc;
      prefix[t] |= sel << shift_;
    }
    __syncthreads();
  }
  if (t < 2) {
    const float r = t == 0 ? r_lo : r_hi;
    const float lo = __uint_as_float(prefix[2 * t]), hi = __uint_as_float(prefix[2 * t + 1]);
    qv[t] = lerp_ref(lo, hi, r - truncf(r));
  }
  __syncthreads();
  const float qlo = qv[0], qhi = qv[1];
  double s11 = 0, s12 = 0, s22 = 0, t1 = 0, t2 = 0;
  for (int i = t; i < n; i += LSQ_THREADS) {
    const float d = __uint_as_float(key_of(dd[i]));
    if (qlo <= d && d <= qhi) {
      const float m = fabsf(md[i]);
      const float c = fabsf(cd[i]) * 0.9f + 0.1f;
      const float w = sqrtf(c);
      const float a1 = m * w, y = fabsf(d) * w;
      s11 += (double)a1 * a1;
      s12 += (double)a1 * w;
      s22 += (double)w * w;
      t1 += (double)a1 * y;
      t2 += (double)w * y;
    }
  }
  s11 = block_sum(s11, red);
  s12 = block_sum(s12, red);
  s22 = block_sum(s22, red);
  t1 = block_sum(t1, red);
  t2 = block_sum(t2, red);
  if (t == 0) {
    const double det = s11 * s22 - s12 * s12;
    double sc, sh;
    if (s22 > 0 && fabs(det) > 1e-12 * s11 * s22) {
      sc = (s22 * t1 - s12 * t2) / det;
      sh = (s11 * t2 - s12 * t1) / det;
    } else if (s22 > 0) {
      // rank-deficient (all kept mono values equal): minimum-norm solution like gelsy
      const double m0 = s12 / s22, c0 = t2 / s22;
      sc = c0 * m0 / (m0 * m0 + 1.0);
      sh = c0 / (m0 * m0 + 1.0);
    } else {
      sc = 0.0;
      sh = 0.0;
    }
    scale[b] = (float)sc;
    shift[b] = (float)sh;
  }
}

// ------------------------------------------------------------------ scaled mono + mirror
__global__ __launch_bounds__(256) void scale_maps_kernel(const float *__restrict__ m2, const float *__restrict__ m3,
                                                         const float *__restrict__ scale,
                                                         const float *__restrict__ shift, long hw, long in_bs,
                                                         long npix, float *__restrict__ sm2,
                                                         float *__restrict__ sm3) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long b = p / hw, r = p % hw;
  const float s = scale[b], t = shift[b];
  sm2[p] = s * m2[b * in_bs + r] + t;
  sm3[p] = s * m3[b * in_bs + r] + t;
}

__global__ __launch_bounds__(256) void mirror_kernel(const float *__restrict__ sm2, const float *__restrict__ sm3,
                                                     const float *__restrict__ dL, const float *__restrict__ confl,
                                                     int H, int W, long in_bs, float th, float div,
                                                     float conf_th, long npix, float *__restrict__ mirror,
                                                     float *__restrict__ coords_x) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long b = p / hw, r = p % hw;
  const int y = (int)(r / W), x = (int)(r % W);
  const float lrc = softlrc_px(sm2 + b * hw, sm3 + b * hw, H, W, y, x, -1.0f, th, div);
  const float sc = confl[b * in_bs + r], md = sm2[p], sd = dL[b * in_bs + r];
  const float both = sc * lrc;
  const float near_ = sa::sigmoidf_ref(20.0f * (md - sd));
  const float a = both * near_;
  const float bb = (1.0f - sc) * lrc;
  const float better = a + bb - a * bb;
  mirror[p] = sa::sigmoidf_ref(20.0f * (better - conf_th));
  coords_x[p] = (float)x - md;
}

}  // namespace

extern "C" int sa_softlrc(const float *d2, const float *d3, const float *conf2, const float *conf3, int B,
                          int H, int W, long map_bs, float lrc_th, float *s2, float *s3, void *stream) {
  SA_REQUIRE(d2 && d3 && s2 && s3, "sa_softlrc: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_softlrc: empty shape");
  SA_REQUIRE(map_bs >= (long)H * W, "sa_softlrc: map_bs too small");
  const long npix = (long)B * H * W;
  const float div = (float)std::log(1.0 + std::exp((double)lrc_th));
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  softlrc_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(d2, d3, conf2, conf3, H, W, map_bs, lrc_th,
                                                                div, npix, s2, s3);
  return sa::check_launch("sa_softlrc");
}

extern "C" int sa_weighted_lsq(const float *mde, const float *disp, const float *conf, int B, int n_per_b,
                               float q_lo, float q_hi, float *scale, float *shift, void *stream) {
  SA_REQUIRE(mde && disp && conf && scale && shift, "sa_weighted_lsq: null pointer");
  SA_REQUIRE(B > 0 && n_per_b > 0, "sa_weighted_lsq: empty input");
  SA_REQUIRE(q_lo >= 0.f && q_lo <= q_hi && q_hi <= 1.f, "sa_weighted_lsq: quantiles out of order");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LSQ, s);
  lsq_kernel<<<B, LSQ_THREADS, 0, s>>>(mde, disp, conf, n_per_b, q_lo, q_hi, scale, shift);
  return sa::check_launch("sa_weighted_lsq");
}

extern "C" int sa_mono_scale_mirror(const float *m2, const float *m3, const float *scale, const float *shift,
                                    const float *dL, const float *conf_l, int B, int H, int W, long in_bs,
                                    float lrc_th, float conf_th, float *sm2, float *sm3, float *mirror,
                                    float *coords_x, void *stream) {
  SA_REQUIRE(m2 && m3 && scale && shift && dL && conf_l && sm2 && sm3 && mirror && coords_x,
             "sa_mono_scale_mirror: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_mono_scale_mirror: empty shape");
  SA_REQUIRE(in_bs >= (long)H * W, "sa_mono_scale_mirror: in_bs too small");
  const long npix = (long)B * H * W;
  const float div = (float)std::log(1.0 + std::exp((double)lrc_th));
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  const unsigned nb = (unsigned)((npix + 255) / 256);
  scale_maps_kernel<<<nb, 256, 0, s>>>(m2, m3, scale, shift, (long)H * W, in_bs, npix, sm2, sm3);
  int rc = sa::check_launch("sa_mono_scale_mirror/scale");
  if (rc) return rc;
  mirror_kernel<<<nb, 256, 0, s>>>(sm2, sm3, dL, conf_l, H, W, in_bs, lrc_th, div, conf_th, npix, mirror, coords_x);
  return sa::check_launch("sa_mono_scale_mirror/mirror");
}
