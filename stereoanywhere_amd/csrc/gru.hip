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

// Every kernel here walks one image (blockIdx.y) or one (image, channel) plane (blockIdx.z)
// per grid row with 32-bit in-plane offsets: no 64-bit division per element (emulated,
// ~100 instructions each).  VEC = 4: float4 accesses (HW % 4 == 0, 16-byte aligned bases
// and batch strides), so a thread's 4 elements share one channel.
template <int VEC>
__device__ __forceinline__ void ldv(const float *p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4 *>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = *p;
  }
}
template <int VEC>
__device__ __forceinline__ void stv(float *p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    *p = v[0];
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void gru_zr_kernel(const float *__restrict__ xc, long xc_bs,
                                                     const float *__restrict__ bx,
                                                     const float *__restrict__ hzr, long hzr_bs,
                                                     const float *__restrict__ cz, const float *__restrict__ cr,
                                                     long c_bs, const float *__restrict__ h, long h_bs,
                                                     int C, unsigned HW, unsigned per, float *__restrict__ z,
                                                     float *__restrict__ rh) {
  const unsigned r = (blockIdx.x * 256u + threadIdx.x) * VEC;
  if (r >= per) return;
  const long b = blockIdx.y;
  float zx[VEC], rx[VEC], zh[VEC], rhh[VEC], czv[VEC], crv[VEC], hv[VEC], zo[VEC], ro[VEC];
  ldv<VEC>(xc + b * xc_bs + r, zx);
  ldv<VEC>(xc + b * xc_bs + per + r, rx);
  ldv<VEC>(hzr + b * hzr_bs + r, zh);
  ldv<VEC>(hzr + b * hzr_bs + per + r, rhh);
  ldv<VEC>(cz + b * c_bs + r, czv);
  ldv<VEC>(cr + b * c_bs + r, crv);
  ldv<VEC>(h + b * h_bs + r, hv);
  const int c = (int)(r / HW);
  const float bz = bx ? bx[c] : 0.0f, br = bx ? bx[C + c] : 0.0f;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    // conv_x bias added as MIOpen's conv + bias would (one rounding)
    const float a = bx ? zx[j] + bz : zx[j], e = bx ? rx[j] + br : rx[j];
    zo[j] = sa::sigmoidf_ref((a + zh[j]) + czv[j]);
    ro[j] = sa::sigmoidf_ref((e + rhh[j]) + crv[j]) * hv[j];
  }
  stv<VEC>(z + b * per + r, zo);
  stv<VEC>(rh + b * per + r, ro);
}

// qh2 (may be NULL): the second half of the r*h conv split over its input channels (the two
// partial sums are added here, qh + qh2)
template <int VEC>
__global__ __launch_bounds__(256) void gru_out_kernel(const float *__restrict__ xc, long xc_bs,
                                                      const float *__restrict__ bx,
                                                      const float *__restrict__ qh, const float *__restrict__ qh2,
                                                      long qh_bs,
                                                      const float *__restrict__ cq, long c_bs,
                                                      const float *__restrict__ z, int C, unsigned HW, unsigned per,
                                                      float *__restrict__ h, long h_bs) {
  const unsigned r = (blockIdx.x * 256u + threadIdx.x) * VEC;
  if (r >= per) return;
  const long b = blockIdx.y;
  float qx[VEC], qv[VEC], cv[VEC], zv[VEC], hv[VEC];
  ldv<VEC>(xc + b * xc_bs + 2 * (long)per + r, qx);
  ldv<VEC>(qh + b * qh_bs + r, qv);
  if (qh2) {
    float q2[VEC];
    ldv<VEC>(qh2 + b * qh_bs + r, q2);
#pragma unroll
    for (int j = 0; j < VEC; ++j) qv[j] += q2[j];
  }
  ldv<VEC>(cq + b * c_bs + r, cv);
  ldv<VEC>(z + b * per + r, zv);
  ldv<VEC>(h + b * h_bs + r, hv);
  const float bq = bx ? bx[2 * C + (int)(r / HW)] : 0.0f;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const float a = bx ? qx[j] + bq : qx[j];
    const float q = tanhf((a + qv[j]) + cv[j]);
    hv[j] = (1.0f - zv[j]) * hv[j] + zv[j] * q;
  }
  stv<VEC>(h + b * h_bs + r, hv);
}

// F.avg_pool2d(x, 3, stride=2, padding=1), count_include_pad=True -> always / 9.
// grid: x over output columns (64 per block), y over output rows (4 per block), z = (b, c)
// (in_p / out_p: row pitches of the planes, >= W / Wo: columns beyond the width are not read
// or written)
__global__ __launch_bounds__(256) void pool2x_kernel(const float *__restrict__ in, long in_bs, int C, int H,
                                                     int W, int Ho, int Wo, float *__restrict__ out, long out_bs,
                                                     int in_p, int out_p) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= Wo || y >= Ho) return;
  const int b = blockIdx.z / C, c = blockIdx.z % C;
  const float *p = in + b * in_bs + (long)c * H * in_p;
  float s = 0.f;
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = 2 * y + dy;
    if (yy < 0 || yy >= H) continue;
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = 2 * x + dx;
      if (xx < 0 || xx >= W) continue;
      s += p[yy * in_p + xx];
    }
  }
  out[b * out_bs + (long)c * Ho * out_p + y * out_p + x] = s / 9.0f;
}

// F.interpolate(bilinear, align_corners=True) (upsample_bilinear2d arithmetic); grid as pool2x
__global__ __launch_bounds__(256) void interp_kernel(const float *__restrict__ in, long in_bs, int C, int H,
                                                     int W, int Ho, int Wo, float sh, float sw,
                                                     float *__restrict__ out, long out_bs, int in_p, int out_p) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= Wo || y >= Ho) return;
  const int b = blockIdx.z / C, c = blockIdx.z % C;
  const float *p = in + b * in_bs + (long)c * H * in_p;
  const float ry = sh * (float)y, rx = sw * (float)x;
  const int y0 = (int)ry, x0 = (int)rx;
  const int yp = y0 < H - 1 ? 1 : 0, xp = x0 < W - 1 ? 1 : 0;
  const float ly1 = ry - (float)y0, ly0 = 1.0f - ly1;
  const float lx1 = rx - (float)x0, lx0 = 1.0f - lx1;
  const float *r0 = p + y0 * in_p, *r1 = p + (y0 + yp) * in_p;
  const float v = ly0 * (lx0 * r0[x0] + lx1 * r0[x0 + xp]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x0 + xp]);
  out[b * out_bs + (long)c * Ho * out_p + y * out_p + x] = v;
}

// interp_kernel with 4 consecutive outputs per thread and one float4 store (Wo % 4 == 0,
// 16-byte aligned output planes: the update block's maps); per-output arithmetic identical
// to interp_kernel. grid: x over quads of output columns (64 per block), y over rows (4)
__global__ __launch_bounds__(256) void interp_v4_kernel(const float *__restrict__ in, long in_bs, int C, int H,
                                                        int W, int Ho, int Wo, float sh, float sw,
                                                        float *__restrict__ out, long out_bs, int in_p) {
  const int xq = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (4 * xq >= Wo || y >= Ho) return;
  const int b = blockIdx.z / C, c = blockIdx.z % C;
  const float *p = in + b * in_bs + (long)c * H * in_p;
  const float ry = sh * (float)y;
  const int y0 = (int)ry;
  const int yp = y0 < H - 1 ? 1 : 0;
  const float ly1 = ry - (float)y0, ly0 = 1.0f - ly1;
  const float *r0 = p + y0 * in_p, *r1 = p + (y0 + yp) * in_p;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float rx = sw * (float)(4 * xq + j);
    const int x0 = (int)rx;
    const int xp = x0 < W - 1 ? 1 : 0;
    const float lx1 = rx - (float)x0, lx0 = 1.0f - lx1;
    v[j] = ly0 * (lx0 * r0[x0] + lx1 * r0[x0 + xp]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x0 + xp]);
  }
  *reinterpret_cast<float4 *>(out + b * out_bs + (long)c * Ho * Wo + y * Wo + 4 * xq) =
      make_float4(v[0], v[1], v[2], v[3]);
}

// pool2x with 4 consecutive outputs per thread and one float4 store (W % 8 == 0, 16-byte
// aligned planes: the update block's maps): the window columns of outputs 4q .. 4q + 3 are
// 8q - 1 .. 8q + 7, one scalar and two float4 loads per input row instead of 12 scalar loads.
__global__ __launch_bounds__(256) void pool2x_v4_kernel(const float *__restrict__ in, long in_bs, int C, int H, int W,
                                                        int Ho, int Wo, float *__restrict__ out, long out_bs) {
  const int xq = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (4 * xq >= Wo || y >= Ho) return;
  const int b = blockIdx.z / C, c = blockIdx.z % C;
  const float *p = in + b * in_bs + (long)c * H * W;
  const int x0 = 8 * xq;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = 2 * y + dy;
    if (yy < 0 || yy >= H) continue;
    const float *r = p + yy * W;
    const float4 a = *reinterpret_cast<const float4 *>(r + x0);   // x0 + 3 < W: Wo = W / 2
    const float4 e = x0 + 4 < W ? *reinterpret_cast<const float4 *>(r + x0 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float m = x0 > 0 ? r[x0 - 1] : 0.0f;
    s0 += (m + a.x) + a.y;
    s1 += (a.y + a.z) + a.w;
    s2 += (a.w + e.x) + e.y;
    s3 += (e.y + e.z) + e.w;
  }
  *reinterpret_cast<float4 *>(out + b * out_bs + (long)c * Ho * Wo + y * Wo + 4 * xq) =
      make_float4(s0 / 9.0f, s1 / 9.0f, s2 / 9.0f, s3 / 9.0f);
}

__global__ __launch_bounds__(256) void relu_copy_kernel(const float *__restrict__ in, long in_bs, unsigned per,
                                                        float *__restrict__ out, long out_bs) {
  const unsigned r = blockIdx.x * 256u + threadIdx.x;
  if (r >= per) return;
  const long b = blockIdx.y;
  out[b * out_bs + r] = fmaxf(in[b * in_bs + r], 0.0f);
}

__global__ __launch_bounds__(256) void flow_update_kernel(float *__restrict__ cx, const float *__restrict__ delta,
                                                          long delta_bs, int W, unsigned hw,
                                                          float *__restrict__ fa, long fa_bs,
                                                          float *__restrict__ fb, long fb_bs) {
  const unsigned r = blockIdx.x * 256u + threadIdx.x;
  if (r >= hw) return;
  const long b = blockIdx.y;
  const long i = b * hw + r;
  float c = cx[i];
  if (delta) {
    c = c + delta[b * delta_bs + r];
    cx[i] = c;
  }
  const float fx = c - (float)(r % (unsigned)W);
  if (fa) {
    fa[b * fa_bs + r] = fx;
    fa[b * fa_bs + hw + r] = 0.0f;
  }
  if (fb) {
    fb[b * fb_bs + r] = fx;
    fb[b * fb_bs + hw + r] = 0.0f;
  }
}

bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }


}  // namespace

extern "C" int sa_gru_zr(const float *xc, long xc_bs, const float *bx, const float *hzr, long hzr_bs, const float *cz,
                         const float *cr, long c_bs, const float *h, long h_bs, int B, int C, int HW,
                         float *z, float *rh, void *stream) {
  SA_REQUIRE(xc && hzr && cz && cr && h && z && rh, "sa_gru_zr: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && C > 0 && HW > 0, "sa_gru_zr: empty shape");
  SA_REQUIRE((long)C * HW < (1L << 31), "sa_gru_zr: plane too large");
  const unsigned per = (unsigned)((long)C * HW);
  const bool v4 = HW % 4 == 0 && al16(xc) && al16(hzr) && al16(cz) && al16(cr) && al16(h) && al16(z) && al16(rh) &&
                  xc_bs % 4 == 0 && hzr_bs % 4 == 0 && c_bs % 4 == 0 && h_bs % 4 == 0;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_GRU_ZR, s);
  if (v4) {
    gru_zr_kernel<4><<<dim3((per / 4 + 255) / 256, B), 256, 0, s>>>(xc, xc_bs, bx, hzr, hzr_bs, cz, cr, c_bs, h, h_bs,
                                                                     C, HW, per, z, rh);
  } else {
    gru_zr_kernel<1><<<dim3((per + 255) / 256, B), 256, 0, s>>>(xc, xc_bs, bx, hzr, hzr_bs, cz, cr, c_bs, h, h_bs, C,
                                                                 HW, per, z, rh);
  }
  return sa::check_launch("sa_gru_zr");
}

extern "C" int sa_gru_out_split(const float *xc, long xc_bs, const float *bx, const float *qh, const float *qh2,
                                long qh_bs, const float *cq, long c_bs, const float *z, int B, int C, int HW, float *h,
                                long h_bs, void *stream) {
  SA_REQUIRE(xc && qh && cq && z && h, "sa_gru_out: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && C > 0 && HW > 0, "sa_gru_out: empty shape");
  SA_REQUIRE((long)C * HW < (1L << 31), "sa_gru_out: plane too large");
  const unsigned per = (unsigned)((long)C * HW);
  const bool v4 = HW % 4 == 0 && al16(xc) && al16(qh) && (!qh2 || al16(qh2)) && al16(cq) && al16(z) && al16(h) &&
                  xc_bs % 4 == 0 && qh_bs % 4 == 0 && c_bs % 4 == 0 && h_bs % 4 == 0;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_GRU_OUT, s);
  if (v4) {
    gru_out_kernel<4><<<dim3((per / 4 + 255) / 256, B), 256, 0, s>>>(xc, xc_bs, bx, qh, qh2, qh_bs, cq, c_bs, z, C, HW,
                                                                      per, h, h_bs);
  } else {
    gru_out_kernel<1><<<dim3((per + 255) / 256, B), 256, 0, s>>>(xc, xc_bs, bx, qh, qh2, qh_bs, cq, c_bs, z, C, HW, per,
                                                                  h, h_bs);
  }
  return sa::check_launch("sa_gru_out");
}

extern "C" int sa_gru_out(const float *xc, long xc_bs, const float *bx, const float *qh, long qh_bs, const float *cq, long c_bs,
                          const float *z, int B, int C, int HW, float *h, long h_bs, void *stream) {
  return sa_gru_out_split(xc, xc_bs, bx, qh, nullptr, qh_bs, cq, c_bs, z, B, C, HW, h, h_bs, stream);
}

extern "C" int sa_pool2x_p(const float *in, long in_bs, int in_pitch, int B, int C, int H, int W, float *out,
                           long out_bs, int out_pitch, void *stream) {
  SA_REQUIRE(in && out, "sa_pool2x: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && (long)B * C <= 65535, "sa_pool2x: bad shape");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  SA_REQUIRE(in_pitch >= W && out_pitch >= Wo, "sa_pool2x: row pitch below the width");
  SA_REQUIRE((long)H * in_pitch < (1L << 31), "sa_pool2x: plane too large");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  if (in_pitch == W && out_pitch == Wo && W % 8 == 0 && Wo % 4 == 0 && al16(in) && al16(out) && in_bs % 4 == 0 &&
      out_bs % 4 == 0)
    pool2x_v4_kernel<<<dim3((Wo / 4 + 63) / 64, (Ho + 3) / 4, B * C), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, out,
                                                                                   out_bs);
  else
    pool2x_kernel<<<dim3((Wo + 63) / 64, (Ho + 3) / 4, B * C), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, out, out_bs,
                                                                            in_pitch, out_pitch);
  return sa::check_launch("sa_pool2x");
}

extern "C" int sa_pool2x(const float *in, long in_bs, int B, int C, int H, int W, float *out, long out_bs,
                         void *stream) {
  return sa_pool2x_p(in, in_bs, W, B, C, H, W, out, out_bs, (W + 2 - 3) / 2 + 1, stream);
}

extern "C" int sa_interp_bilinear_ac_p(const float *in, long in_bs, int in_pitch, int B, int C, int H, int W, int Ho,
                                       int Wo, float *out, long out_bs, int out_pitch, void *stream) {
  SA_REQUIRE(in && out, "sa_interp_bilinear_ac: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && (long)B * C <= 65535,
             "sa_interp_bilinear_ac: bad shape");
  SA_REQUIRE(in_pitch >= W && out_pitch >= Wo, "sa_interp_bilinear_ac: row pitch below the width");
  SA_REQUIRE((long)H * in_pitch < (1L << 31) && (long)Ho * out_pitch < (1L << 31),
             "sa_interp_bilinear_ac: plane too large");
  // area_pixel_compute_scale(align_corners=True): (in - 1) / (out - 1), 0 for out == 1
  const float sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.0f;
  const float sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.0f;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  if (out_pitch == Wo && Wo % 4 == 0 && al16(out) && out_bs % 4 == 0)
    interp_v4_kernel<<<dim3((Wo / 4 + 63) / 64, (Ho + 3) / 4, B * C), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, sh, sw,
                                                                                   out, out_bs, in_pitch);
  else
    interp_kernel<<<dim3((Wo + 63) / 64, (Ho + 3) / 4, B * C), 256, 0, s>>>(in, in_bs, C, H, W, Ho, Wo, sh, sw, out,
                                                                            out_bs, in_pitch, out_pitch);
  return sa::check_launch("sa_interp_bilinear_ac");
}

extern "C" int sa_interp_bilinear_ac(const float *in, long in_bs, int B, int C, int H, int W, int Ho, int Wo,
                                     float *out, long out_bs, void *stream) {
  return sa_interp_bilinear_ac_p(in, in_bs, W, B, C, H, W, Ho, Wo, out, out_bs, Wo, stream);
}

extern "C" int sa_relu_copy(const float *in, long in_bs, int B, int C, int HW, float *out, long out_bs,
                            void *stream) {
  SA_REQUIRE(in && out, "sa_relu_copy: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && C > 0 && HW > 0 && (long)C * HW < (1L << 31), "sa_relu_copy: bad shape");
  const unsigned per = (unsigned)((long)C * HW);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  relu_copy_kernel<<<dim3((per + 255) / 256, B), 256, 0, s>>>(in, in_bs, per, out, out_bs);
  return sa::check_launch("sa_relu_copy");
}

extern "C" int sa_flow_update(float *coords_x, const float *delta, long delta_bs, int B, int H, int W,
                              float *flow_a, long flow_a_bs, float *flow_b, long flow_b_bs, void *stream) {
  SA_REQUIRE(coords_x, "sa_flow_update: null coords");
  SA_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && (long)H * W < (1L << 31), "sa_flow_update: bad shape");
  const unsigned hw = (unsigned)((long)H * W);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  flow_update_kernel<<<dim3((hw + 255) / 256, B), 256, 0, s>>>(coords_x, delta, delta_bs, W, hw, flow_a, flow_a_bs,
                                                                flow_b, flow_b_bs);
  return sa::check_launch("sa_flow_update");
}
