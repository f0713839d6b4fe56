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

// pool2x / interp: grid y = one (image, channel) plane, grid x over a flat index of the
// plane's output vectors (VEC consecutive outputs of one row, one VEC-wide store), FLAT_K
// vectors per lane 256 apart (coalesced): every lane has work whatever the row width, and
// the plane base is uniform (scalar) with 32-bit in-plane offsets.  The row of a vector is
// umulhi(index, magic) (exact: index * nv < 2^32, checked on the host).  (The round-3
// kernels mapped 64 lanes to a row segment and 4 rows to a workgroup: at the tiled configs'
// widths, 70 / 140 / 280, up to half the lanes idled, at 1-1.5 TB/s.)
constexpr int FLAT_K = 4;

struct FlatGeo {
  long in_bs, out_bs;
  int C, H, W, Ho, Wo, in_p, out_p;
  unsigned nv, per, magic;  // vectors per row and per plane; ceil(2^32 / nv)
};

__device__ __forceinline__ void flat_row(const FlatGeo &g, unsigned i, unsigned &y, unsigned &xv) {
  y = g.nv == 1 ? i : __umulhi(i, g.magic);
  xv = i - y * g.nv;
}

template <int VEC>
__device__ __forceinline__ void st_vec(float *p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
  } else {
    *p = v[0];
  }
}

// F.avg_pool2d(x, 3, stride=2, padding=1), count_include_pad=True -> always / 9; each window
// row summed as (left + centre) + right (an absent column adds an exact 0), rows in order.
// VLOAD (W == 2 Wo, in_p % 4 == 0, 16-byte aligned planes): the window columns of a vector's
// outputs, 2 VEC x0 - 1 .. 2 VEC x0 + 2 VEC - 1, as one scalar and VEC / 2 float4 loads per row.
template <int VEC, bool VLOAD>
__device__ __forceinline__ void pool2x_flat_body(const float *__restrict__ in, float *__restrict__ out, const FlatGeo &g,
                                                 unsigned bx, unsigned plane) {
  const unsigned b = plane / (unsigned)g.C, c = plane - b * (unsigned)g.C;
  const float *p = in + b * g.in_bs + (long)c * g.H * g.in_p;
  float *o = out + b * g.out_bs + (long)c * g.Ho * g.out_p;
  const unsigned base = bx * (256u * FLAT_K) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < FLAT_K; ++k) {
    const unsigned i = base + k * 256u;
    if (i >= g.per) return;
    unsigned y, xv;
    flat_row(g, i, y, xv);
    const int x0 = 2 * VEC * (int)xv;
    float s[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) s[j] = 0.f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = 2 * (int)y + dy;
      if (yy < 0 || yy >= g.H) continue;
      const float *r = p + yy * g.in_p;
      if constexpr (VLOAD && VEC >= 2) {
        float w[2 * VEC + 1];
        w[0] = x0 > 0 ? r[x0 - 1] : 0.0f;
#pragma unroll
        for (int q = 0; q < VEC / 2; ++q) {
          const float4 t = *reinterpret_cast<const float4 *>(r + x0 + 4 * q);
          w[1 + 4 * q] = t.x; w[2 + 4 * q] = t.y; w[3 + 4 * q] = t.z; w[4 + 4 * q] = t.w;
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) s[j] += (w[2 * j] + w[2 * j + 1]) + w[2 * j + 2];
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int xx = x0 + 2 * j;
          const float l = xx > 0 ? r[xx - 1] : 0.0f;
          const float rt = xx + 1 < g.W ? r[xx + 1] : 0.0f;
          s[j] += (l + r[xx]) + rt;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s[j] = s[j] / 9.0f;
    st_vec<VEC>(o + y * g.out_p + VEC * xv, s);
  }
}

template <int VEC, bool VLOAD>
__global__ __launch_bounds__(256) void pool2x_flat_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                          FlatGeo g) {
  pool2x_flat_body<VEC, VLOAD>(in, out, g, blockIdx.x, blockIdx.y);
}

// F.interpolate(bilinear, align_corners=True) with upsample_bilinear2d's arithmetic:
// source coordinate scale * dst, floor, the +1 neighbour clamped at the last row / column,
// lambda weights, (lx0 * a + lx1 * b) per row, then the row blend.
template <int VEC>
__global__ __launch_bounds__(256) void interp_flat_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                          FlatGeo g, float sh, float sw) {
  const unsigned b = blockIdx.y / (unsigned)g.C, c = blockIdx.y - b * (unsigned)g.C;
  const float *p = in + b * g.in_bs + (long)c * g.H * g.in_p;
  float *o = out + b * g.out_bs + (long)c * g.Ho * g.out_p;
  const unsigned base = blockIdx.x * (256u * FLAT_K) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < FLAT_K; ++k) {
    const unsigned i = base + k * 256u;
    if (i >= g.per) return;
    unsigned y, xv;
    flat_row(g, i, y, xv);
    const float ry = sh * (float)y;
    const int y0 = (int)ry;
    const int yp = y0 < g.H - 1 ? 1 : 0;
    const float ly1 = ry - (float)y0, ly0 = 1.0f - ly1;
    const float *r0 = p + y0 * g.in_p, *r1 = p + (y0 + yp) * g.in_p;
    float v[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float rx = sw * (float)(VEC * (int)xv + j);
      const int x0 = (int)rx;
      const int xp = x0 < g.W - 1 ? 1 : 0;
      const float lx1 = rx - (float)x0, lx0 = 1.0f - lx1;
      v[j] = ly0 * (lx0 * r0[x0] + lx1 * r0[x0 + xp]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x0 + xp]);
    }
    st_vec<VEC>(o + y * g.out_p + VEC * xv, v);
  }
}

// The same resize as separable passes over a band of RB output rows of one plane: the
// horizontal blends (lx0 * a + lx1 * b) of every source row the band needs go to LDS once,
// then each output is ly0 * top + ly1 * bottom from two LDS rows -- the operations and their
// order of interp_flat_kernel, so bit-identical, with ~1.2 instead of 4 gathered loads per
// output.  grid: x = bands, y = planes; LDS: nr_cap rows x Wo (host-sized, <= 64 KiB).
// magic_o: ceil(2^32 / Wo) for the horizontal pass's flat (row, column) index.
template <int VEC>
__device__ __forceinline__ void interp_band_body(const float *__restrict__ in, float *__restrict__ out, const FlatGeo &g,
                                                 float sh, float sw, int RB, unsigned magic_o, unsigned bx,
                                                 unsigned plane, float *hrow) {
  const unsigned b = plane / (unsigned)g.C, c = plane - b * (unsigned)g.C;
  const float *p = in + b * g.in_bs + (long)c * g.H * g.in_p;
  float *o = out + b * g.out_bs + (long)c * g.Ho * g.out_p;
  const int ya = (int)bx * RB, yb = min(ya + RB, g.Ho);
  const int r0 = (int)(sh * (float)ya);
  const int yl = (int)(sh * (float)(yb - 1));
  const int nr = yl + (yl < g.H - 1 ? 1 : 0) - r0 + 1;
  const unsigned nh = (unsigned)(nr * g.Wo);
  for (unsigned i = threadIdx.x; i < nh; i += 256u) {
    const unsigned r = __umulhi(i, magic_o), x = i - r * (unsigned)g.Wo;
    const float *src = p + (r0 + (int)r) * g.in_p;
    const float rx = sw * (float)x;
    const int x0 = (int)rx;
    const int xp = x0 < g.W - 1 ? 1 : 0;
    const float lx1 = rx - (float)x0, lx0 = 1.0f - lx1;
    hrow[i] = lx0 * src[x0] + lx1 * src[x0 + xp];
  }
  __syncthreads();
  const unsigned nvec = (unsigned)(yb - ya) * g.nv;
  for (unsigned i = threadIdx.x; i < nvec; i += 256u) {
    unsigned yy, xv;
    flat_row(g, i, yy, xv);
    const int y = ya + (int)yy;
    const float ry = sh * (float)y;
    const int y0 = (int)ry;
    const int yp = y0 < g.H - 1 ? 1 : 0;
    const float ly1 = ry - (float)y0, ly0 = 1.0f - ly1;
    const float *h0 = hrow + (y0 - r0) * g.Wo + VEC * xv, *h1 = h0 + yp * g.Wo;
    float v[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = ly0 * h0[j] + ly1 * h1[j];
    st_vec<VEC>(o + y * g.out_p + VEC * xv, v);
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void interp_band_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                          FlatGeo g, float sh, float sw, int RB, unsigned magic_o) {
  extern __shared__ float hrow[];
  interp_band_body<VEC>(in, out, g, sh, sw, RB, magic_o, blockIdx.x, blockIdx.y, hrow);
}

// the flow planes of the motion encoder's input from the coordinates (sa_flow_update with only
// flow_b): out[b][0] = coords - x, out[b][1] = 0 (stereoanywhere.py:272-280, update.py:90)
__device__ __forceinline__ void flow_x_body(const float *__restrict__ cx, float *__restrict__ out, const FlatGeo &g,
                                            unsigned bx, unsigned b) {
  const unsigned base = bx * (256u * FLAT_K) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < FLAT_K; ++k) {
    const unsigned r = base + k * 256u;
    if (r >= g.per) return;
    unsigned y, x;
    flat_row(g, r, y, x);
    const float fx = cx[b * g.in_bs + r] - (float)x;
    out[b * g.out_bs + r] = fx;
    out[b * g.out_bs + g.per + r] = 0.0f;
  }
}

// Up to 4 independent pool2x / interp jobs in one launch (the update loop's plumbing between
// two conv launches: pool(h08) + interp(h32) before gru16, interp(h16) + pool(h16) before
// gru08): job j owns blocks [start[j], start[j + 1]), each block one (x-block, plane) of its
// job's own launch shape, so the small jobs' launch tails overlap.
struct ResampleJobDev {
  const float *in;  // (flow job: the coordinates)
  float *out;
  FlatGeo g;
  float sh, sw;
  int kind, vec, vload, RB;  // kind 0 pool2x, 1 interp, 2 flow planes
  unsigned magic_o, bx;  // x-blocks per plane
};
struct ResampleLaunch {
  ResampleJobDev job[4];
  unsigned start[5];
  int njobs;
};

__global__ __launch_bounds__(256) void resample_multi_kernel(ResampleLaunch L) {
  extern __shared__ float hrow[];
  int j = 0;
  while (j + 1 < L.njobs && blockIdx.x >= L.start[j + 1]) ++j;
  const ResampleJobDev &J = L.job[j];
  const unsigned local = blockIdx.x - L.start[j], plane = local / J.bx, bx = local - plane * J.bx;
  if (J.kind == 2) {
    flow_x_body(J.in, J.out, J.g, bx, plane);
  } else if (J.kind == 0) {
    if (J.vec == 4 && J.vload)
      pool2x_flat_body<4, true>(J.in, J.out, J.g, bx, plane);
    else if (J.vec == 4)
      pool2x_flat_body<4, false>(J.in, J.out, J.g, bx, plane);
    else if (J.vec == 2 && J.vload)
      pool2x_flat_body<2, true>(J.in, J.out, J.g, bx, plane);
    else if (J.vec == 2)
      pool2x_flat_body<2, false>(J.in, J.out, J.g, bx, plane);
    else
      pool2x_flat_body<1, false>(J.in, J.out, J.g, bx, plane);
  } else {
    if (J.vec == 4)
      interp_band_body<4>(J.in, J.out, J.g, J.sh, J.sw, J.RB, J.magic_o, bx, plane, hrow);
    else if (J.vec == 2)
      interp_band_body<2>(J.in, J.out, J.g, J.sh, J.sw, J.RB, J.magic_o, bx, plane, hrow);
    else
      interp_band_body<1>(J.in, J.out, J.g, J.sh, J.sw, J.RB, J.magic_o, bx, plane, hrow);
  }
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

// the widest store the output rows allow (Wo, the row pitch, the batch stride and the base
// all multiples of VEC floats)
static int flat_vec(const float *out, int Wo, int out_p, long out_bs) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(out);
  if (Wo % 4 == 0 && out_p % 4 == 0 && out_bs % 4 == 0 && (a & 15) == 0) return 4;
  if (Wo % 2 == 0 && out_p % 2 == 0 && out_bs % 2 == 0 && (a & 7) == 0) return 2;
  return 1;
}

static FlatGeo flat_geo(long in_bs, int in_p, int C, int H, int W, int Ho, int Wo, long out_bs, int out_p, int vec) {
  FlatGeo g{in_bs, out_bs, C, H, W, Ho, Wo, in_p, out_p, 0u, 0u, 0u};
  g.nv = (unsigned)(Wo / vec);
  g.per = (unsigned)Ho * g.nv;
  g.magic = g.nv > 1 ? (unsigned)(((1UL << 32) + g.nv - 1) / g.nv) : 0u;  // nv == 1: flat_row skips it
  return g;
}

// umulhi(i, ceil(2^32 / nv)) == i / nv for i < per when per * nv < 2^32 (the rounding error
// of the magic, < nv / 2^32 per unit of i, stays below 1 / nv)
static bool flat_ok(const FlatGeo &g) { return (unsigned long)g.per * g.nv < (1UL << 32); }

static dim3 flat_grid(const FlatGeo &g, int B) {
  return dim3((g.per + 256u * FLAT_K - 1) / (256u * FLAT_K), (unsigned)(B * g.C));
}

// The band interp's rows per block: RB output rows while their source rows' blends fit 64 KiB
// of LDS (nr_cap bounds the rows a band touches: ceil(sh (RB - 1)) + 2, + 1 for float
// rounding); false: the flat kernel (one output column, or rows too wide)
static bool band_shape(float sh, int Ho, int Wo, int &RB, size_t &lds) {
  if (Wo < 2) return false;
  for (RB = 16; RB >= 2; RB /= 2) {
    const int nr_cap = (int)ceilf(sh * (float)(RB - 1)) + 3;
    lds = (size_t)nr_cap * Wo * sizeof(float);
    if (lds <= 65536 && (unsigned long)nr_cap * Wo * Wo < (1UL << 32)) return true;
  }
  (void)Ho;
  return false;
}

extern "C" int sa_pool2x_p(const float *in, long in_bs, int in_pitch, int B, int C, int H, int W, float *out,
                           long out_bs, int out_pitch, void *stream) {
  SA_REQUIRE(in && out, "sa_pool2x: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && (long)B * C <= 65535, "sa_pool2x: bad shape");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  SA_REQUIRE(in_pitch >= W && out_pitch >= Wo, "sa_pool2x: row pitch below the width");
  SA_REQUIRE((long)H * in_pitch < (1L << 31) && (long)Ho * out_pitch < (1L << 31), "sa_pool2x: plane too large");
  const int vec = flat_vec(out, Wo, out_pitch, out_bs);
  // vector loads: W == 2 Wo (the window of the last vector ends at column W - 1), float4-aligned rows
  const bool vload = vec >= 2 && W == 2 * Wo && in_pitch % 4 == 0 && in_bs % 4 == 0 && al16(in);
  const FlatGeo g = flat_geo(in_bs, in_pitch, C, H, W, Ho, Wo, out_bs, out_pitch, vec);
  SA_REQUIRE(flat_ok(g), "sa_pool2x: output plane shape unsupported (plane too large)");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  if (vec == 4 && vload)
    pool2x_flat_kernel<4, true><<<flat_grid(g, B), 256, 0, s>>>(in, out, g);
  else if (vec == 4)
    pool2x_flat_kernel<4, false><<<flat_grid(g, B), 256, 0, s>>>(in, out, g);
  else if (vec == 2 && vload)
    pool2x_flat_kernel<2, true><<<flat_grid(g, B), 256, 0, s>>>(in, out, g);
  else if (vec == 2)
    pool2x_flat_kernel<2, false><<<flat_grid(g, B), 256, 0, s>>>(in, out, g);
  else
    pool2x_flat_kernel<1, false><<<flat_grid(g, B), 256, 0, s>>>(in, out, g);
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
  const int vec = flat_vec(out, Wo, out_pitch, out_bs);
  const FlatGeo g = flat_geo(in_bs, in_pitch, C, H, W, Ho, Wo, out_bs, out_pitch, vec);
  SA_REQUIRE(flat_ok(g), "sa_interp_bilinear_ac: output plane shape unsupported (plane too large)");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_PLUMBING, s);
  int RB;
  size_t lds;
  if (band_shape(sh, Ho, Wo, RB, lds)) {
    const unsigned magic_o = (unsigned)(((1UL << 32) + Wo - 1) / Wo);
    const dim3 grid((Ho + RB - 1) / RB, (unsigned)(B * C));
    if (vec == 4)
      interp_band_kernel<4><<<grid, 256, lds, s>>>(in, out, g, sh, sw, RB, magic_o);
    else if (vec == 2)
      interp_band_kernel<2><<<grid, 256, lds, s>>>(in, out, g, sh, sw, RB, magic_o);
    else
      interp_band_kernel<1><<<grid, 256, lds, s>>>(in, out, g, sh, sw, RB, magic_o);
    return sa::check_launch("sa_interp_bilinear_ac");
  }
  if (vec == 4)
    interp_flat_kernel<4><<<flat_grid(g, B), 256, 0, s>>>(in, out, g, sh, sw);
  else if (vec == 2)
    interp_flat_kernel<2><<<flat_grid(g, B), 256, 0, s>>>(in, out, g, sh, sw);
  else
    interp_flat_kernel<1><<<flat_grid(g, B), 256, 0, s>>>(in, out, g, sh, sw);
  return sa::check_launch("sa_interp_bilinear_ac");
}

// sa_resample_multi: validates every job as sa_pool2x_p / sa_interp_bilinear_ac_p do, then one
// launch; an interp job the band kernel cannot take runs on its own (flat kernel) first.
extern "C" int sa_resample_multi(int njobs, const SaResampleJob *jobs, void *stream) {
  SA_REQUIRE(njobs >= 1 && njobs <= 4 && jobs, "sa_resample_multi: 1..4 jobs");
  ResampleLaunch L{};
  size_t lds_max = 0;
  unsigned total = 0;
  int n = 0;
  hipStream_t s = sa::as_stream(stream);
  for (int i = 0; i < njobs; ++i) {
    const SaResampleJob &q = jobs[i];
    SA_REQUIRE(q.in && q.out, "sa_resample_multi: null pointer");
    SA_REQUIRE(q.kind == SA_RESAMPLE_POOL2X || q.kind == SA_RESAMPLE_BILINEAR_AC || q.kind == SA_RESAMPLE_FLOW_X,
               "sa_resample_multi: unknown kind");
    SA_REQUIRE(q.B > 0 && q.C > 0 && q.H > 0 && q.W > 0 && (long)q.B * q.C <= 65535, "sa_resample_multi: bad shape");
    int Ho = q.Ho, Wo = q.Wo;
    if (q.kind == SA_RESAMPLE_FLOW_X) {
      SA_REQUIRE(q.C == 1 && Ho == q.H && Wo == q.W && q.in_pitch == q.W && q.out_pitch == q.W &&
                     q.in_bs >= (long)q.H * q.W && q.out_bs >= 2L * q.H * q.W && (long)q.H * q.W < (1L << 31),
                 "sa_resample_multi: flow job needs dense [B,1,H,W] coordinates and [B,2,H,W] flow planes");
      ResampleJobDev &J = L.job[n];
      J.in = q.in;
      J.out = q.out;
      J.g = flat_geo(q.in_bs, q.W, 1, q.H, q.W, q.H, q.W, q.out_bs, q.W, 1);
      SA_REQUIRE(flat_ok(J.g), "sa_resample_multi: flow plane too large");
      J.kind = 2;
      J.vec = 1;
      J.bx = (J.g.per + 256u * FLAT_K - 1) / (256u * FLAT_K);
      L.start[n] = total;
      total += J.bx * (unsigned)q.B;
      ++n;
      continue;
    }
    if (q.kind == SA_RESAMPLE_POOL2X) {
      const int ho = (q.H + 2 - 3) / 2 + 1, wo = (q.W + 2 - 3) / 2 + 1;
      SA_REQUIRE(Ho == ho && Wo == wo, "sa_resample_multi: pool2x output size must be ((H-1)/2+1, (W-1)/2+1)");
    }
    SA_REQUIRE(Ho > 0 && Wo > 0 && q.in_pitch >= q.W && q.out_pitch >= Wo, "sa_resample_multi: row pitch below the width");
    SA_REQUIRE((long)q.H * q.in_pitch < (1L << 31) && (long)Ho * q.out_pitch < (1L << 31),
               "sa_resample_multi: plane too large");
    const int vec = flat_vec(q.out, Wo, q.out_pitch, q.out_bs);
    const FlatGeo g = flat_geo(q.in_bs, q.in_pitch, q.C, q.H, q.W, Ho, Wo, q.out_bs, q.out_pitch, vec);
    SA_REQUIRE(flat_ok(g), "sa_resample_multi: output plane shape unsupported (plane too large)");
    ResampleJobDev &J = L.job[n];
    J.in = q.in;
    J.out = q.out;
    J.g = g;
    J.kind = q.kind == SA_RESAMPLE_POOL2X ? 0 : 1;
    J.vec = vec;
    if (J.kind == 0) {
      J.vload = vec >= 2 && q.W == 2 * Wo && q.in_pitch % 4 == 0 && q.in_bs % 4 == 0 && al16(q.in);
      J.bx = (g.per + 256u * FLAT_K - 1) / (256u * FLAT_K);
    } else {
      J.sh = Ho > 1 ? (float)(q.H - 1) / (float)(Ho - 1) : 0.0f;
      J.sw = Wo > 1 ? (float)(q.W - 1) / (float)(Wo - 1) : 0.0f;
      size_t lds;
      if (!band_shape(J.sh, Ho, Wo, J.RB, lds)) {
        const int rc = sa_interp_bilinear_ac_p(q.in, q.in_bs, q.in_pitch, q.B, q.C, q.H, q.W, Ho, Wo, q.out, q.out_bs,
                                               q.out_pitch, stream);
        if (rc) return rc;
        continue;
      }
      J.magic_o = (unsigned)(((1UL << 32) + Wo - 1) / Wo);
      J.bx = (unsigned)((Ho + J.RB - 1) / J.RB);
      if (lds > lds_max) lds_max = lds;
    }
    L.start[n] = total;
    total += J.bx * (unsigned)(q.B * q.C);
    ++n;
  }
  if (n == 0) return 0;
  L.njobs = n;
  L.start[n] = total;
  sa::TimingScope ts(SA_K_PLUMBING, s);
  resample_multi_kernel<<<total, 256, lds_max, s>>>(L);
  return sa::check_launch("sa_resample_multi");
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
