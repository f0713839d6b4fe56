// K7 — ConvGRU gate fusion and the update-block plumbing that feeds the GRU convs
// (SURVEY.md §8(a) rows a12, a13).
//
// Reference ConvGRU.forward (update.py:53-62):
//   hx = cat(h, x); z = sigmoid(convz(hx) + cz); r = sigmoid(convr(hx) + cr)
//   q = tanh(convq(cat(r*h, x)) + cq); h = (1 - z) h + z q
// The build splits every gate convolution by input, conv(cat(h, x)) = conv_h(h) +
// conv_x(x) (bias carried by conv_x), so the x part of all three gates is ONE conv with
// 3C outputs and neither concatenation is materialised.  These kernels are the
// elementwise halves: gru_zr fuses the z/r sigmoids, the context biases and r*h;
// gru_out fuses the q tanh and the state update, in place on h.
// The plumbing kernels write pool2x / interp / relu outputs straight into channel
// slices of the next conv's input buffer (update.py:124-132, 88-90).
#include "sa_common.h"

namespace {

__global__ __launch_bounds__(256) void gru_zr_kernel(const float *__restrict__ xc, long xc_bs,
                                                     const float *__restrict__ bx,
                                                     const float *__restrict__ hzr, long hzr_bs,
                                                     const float *__restrict__ cz, const float *__restrict__ cr,
                                                     long c_bs, const float *__restrict__ h, long h_bs,
                                                     int C, long HW, long n, float *__restrict__ z,
                                                     float *__restrict__ rh) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long per = (long)C * HW;
  const long b = i / per, r = i % per;
  float zx = xc[b * xc_bs + r], rx = xc[b * xc_bs + per + r];
  if (bx) {  // conv_x bias, added as MIOpen's conv + bias would (one rounding)
    const int c = (int)((unsigned)r / (unsigned)HW);
    zx = zx + bx[c];
    rx = rx + bx[C + c];
  }
  const float zh = hzr[b * hzr_bs + r], rhh = hzr[b * hzr_bs + per + r];
  const float zz = sa::sigmoidf_ref((zx + zh) + cz[b * c_bs + r]);
  const float rr = sa::sigmoidf_ref((rx + rhh) + cr[b * c_bs + r]);
  z[i] = zz;
  rh[i] = rr * h[b * h_bs + r];
}

__global__ __launch_bounds__(256) void gru_out_kernel(const float *__restrict__ xc, long xc_bs,
                                                      const float *__restrict__ bx,
                                                      const float *__restrict__ qh, long qh_bs,
                                                      const float *__restrict__ cq, long c_bs,
                                                      const float *__restrict__ z, int C, long HW, long n,
                                                      float *__restrict__ h, long h_bs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long per = (long)C * HW;
  const long b = i / per, r = i % per;
  float qx = xc[b * xc_bs + 2 * per + r];
  if (bx) qx = qx + bx[2 * C + (int)((unsigned)r / (unsigned)HW)];
  const float q = tanhf((qx + qh[b * qh_bs + r]) + cq[b * c_bs + r]);
  const float zz = z[i];
  const float hv = h[b * h_bs + r];
  h[b * h_bs + r] = (1.0f - zz) * hv + zz * q;
}

// F.avg_pool2d(x, 3, stride=2, padding=1), count_include_pad=True -> always / 9
__global__ __launch_bounds__(256) void pool2x_kernel(const float *__restrict__ in, long in_bs, int C, int H,
                                                     int W, int Ho, int Wo, long n, float *__restrict__ out,
                                                     long out_bs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int x = (int)(i % Wo);
  const int y = (int)((i / Wo) % Ho);
  const long bc = i / ((long)Wo * Ho);
  const long b = bc / C, c = bc % C;
  const float *p = in + b * in_bs + c * (long)H * W;
  float s = 0.f;
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = 2 * y + dy;
    if (yy < 0 || yy >= H) continue;
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = 2 * x + dx;
      if (xx < 0 || xx >= W) continue;
      s += p[(long)yy * W + xx];
    }
  }
  out[b * out_bs + c * (long)Ho * Wo + (long)y * Wo + x] = s / 9.0f;
}

// F.interpolate(bilinear, align_corners=True) (upsample_bilinear2d arithmetic)
__global__ __launch_bounds__(256) void interp_kernel(const float *__restrict__ in, long in_bs, int C, int H,
                                                     int W, int Ho, int Wo, float sh, float sw, long n,
                                                     float *__restrict__ out, long out_bs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int x = (int)(i % Wo);
  const int y = (int)((i / Wo) % Ho);
  const long bc = i / ((long)Wo * Ho);
  const long b = bc / C, c = bc % C;
  const float *p = in + b * in_bs + c * (long)H * W;
  const float ry = sh * (float)y, rx = sw * (float)x;
  const int y0 = (int)ry, x0 = (int)rx;
  const int yp = y0 < H - 1 ? 1 : 0, xp = x0 < W - 1 ? 1 : 0;
  const float ly1 = ry - (float)y0, ly0 = 1.0f - ly1;
  const float lx1 = rx - (float)x0, lx0 = 1.0f - lx1;
  const float *r0 = p + (long)y0 * W, *r1 = p + (long)(y0 + yp) * W;
  const float v = ly0 * (lx0 * r0[x0] + lx1 * r0[x0 + xp]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x0 + xp]);
  out[b * out_bs + c * (long)Ho * Wo + (long)y * Wo + x] = v;
}

__global__ __launch_bounds__(256) void relu_copy_kernel(const float *__restrict__ in, long in_bs, long per, long n,
                                                        float *__restrict__ out, long out_bs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long b = i / per, r = i % per;
  out[b * out_bs + r] = fmaxf(in[b * in_bs + r], 0.0f);
}

__global__ __launch_bounds__(256) void flow_update_kernel(float *__restrict__ cx, const float *__restrict__ delta,
                                                          long delta_bs, int W, long hw, long n,
                                                          float *__restrict__ fa, long fa_bs,
                                                          float *__restrict__ fb, long fb_bs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long b = i / hw, r = i % hw;
  float c = cx[i];
  if (delta) {
    c = c + delta[b * delta_bs + r];
    cx[i] = c;
  }
  const float fx = c - (float)(r % W);
  if (fa) {
    fa[b * fa_bs + r] = fx;
    fa[b * fa_bs + hw + r] = 0.0f;
  }
  if (fb) {
    fb[b * fb_bs + r] = fx;
    fb[b * fb_bs + hw + r] = 0.0f;
  }
}

inline unsigned nblocks(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int sa_gru_zr(const float *xc, long xc_bs, const float *bx, const float *hzr, long hzr_bs, const float *cz,
                         const float *cr, long c_bs, const float *h, long h_bs, int B, int C, int HW,
                         float *z, float *rh, void *stream) {
  SA_REQUIRE(xc && hzr && cz && cr && h && z && rh, "sa_gru_zr: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && HW > 0, "sa_gru_zr: empty shape");
  SA_REQUIRE((long)C * HW < (1L << 31), "sa_gru_zr: plane too large");
  const long n = (long)B * C * HW;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_GRU_ZR, s);
  gru_zr_kernel<<<nblocks(n), 256, 0, s>>>(xc, xc_bs, bx, hzr, hzr_bs, cz, cr, c_bs, h, h_bs, C, HW, n, z, rh);
  return sa::check_launch("sa_gru_zr");
}

extern "C" int sa_gru_out(const float *xc, long xc_bs, const float *bx, const float *qh, long qh_bs, const float *cq, long c_bs,
                          const float *z, int B, int C, int HW, float *h, long h_bs, void *stream) {
  SA_REQUIRE(xc && qh && cq && z && h, "sa_gru_out: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && HW > 0, "sa_gru_out: empty shape");
  const long n = (long)B * C * HW;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_GRU_OUT, s);
  gru_out_kernel<<<nblocks(n), 256, 0, s>>>(xc, xc_bs, bx, qh, qh_bs, cq, c_bs, z, C, HW, n, h, h_bs);
  return sa::check_launch("sa_gru_out");
}

extern "C" int sa_pool2x(const float *in, long in_bs, int B, int C, int H, int W, float *out, long out_bs,
                         void *stream) {
  SA_REQUIRE(in && out, "sa_pool2x: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0, "sa_pool2x: empty shape");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const long n = (long)B * C * Ho * Wo;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  pool2x_kernel<<<nblocks(n), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, n, out, out_bs);
  return sa::check_launch("sa_pool2x");
}

extern "C" int sa_interp_bilinear_ac(const float *in, long in_bs, int B, int C, int H, int W, int Ho, int Wo,
                                     float *out, long out_bs, void *stream) {
  SA_REQUIRE(in && out, "sa_interp_bilinear_ac: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, "sa_interp_bilinear_ac: empty shape");
  // area_pixel_compute_scale(align_corners=True): (in - 1) / (out - 1), 0 for out == 1
  const float sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.0f;
  const float sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.0f;
  const long n = (long)B * C * Ho * Wo;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  interp_kernel<<<nblocks(n), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, sh, sw, n, out, out_bs);
  return sa::check_launch("sa_interp_bilinear_ac");
}

extern "C" int sa_relu_copy(const float *in, long in_bs, int B, int C, int HW, float *out, long out_bs,
                            void *stream) {
  SA_REQUIRE(in && out, "sa_relu_copy: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && HW > 0, "sa_relu_copy: empty shape");
  const long per = (long)C * HW, n = (long)B * per;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  relu_copy_kernel<<<nblocks(n), 256, 0, s>>>(in, in_bs, per, n, out, out_bs);
  return sa::check_launch("sa_relu_copy");
}

extern "C" int sa_flow_update(float *coords_x, const float *delta, long delta_bs, int B, int H, int W,
                              float *flow_a, long flow_a_bs, float *flow_b, long flow_b_bs, void *stream) {
  SA_REQUIRE(coords_x, "sa_flow_update: null coords");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_flow_update: empty shape");
  const long hw = (long)H * W, n = (long)B * hw;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  flow_update_kernel<<<nblocks(n), 256, 0, s>>>(coords_x, delta, delta_bs, W, hw, n, flow_a, flow_a_bs, flow_b,
                                                 flow_b_bs);
  return sa::check_launch("sa_flow_update");
}
