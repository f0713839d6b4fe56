// K2 — the mono cost volume: surface normals of the 1/4-res mono maps, their all-pairs
// correlation, binned by the half-open depth masks, written straight into the 3-D
// hourglass's [B, nbins, W2, H, W1] layout.
//
// Reference: estimate_normals (utils.py:73-77, kornia spatial_gradient 'diff' —
// replicate pad, unnormalised central difference); mono volume
// 1.73 * CorrBlock1D.corr(n2, n3) (stereoanywhere.py:136, corr.py:117-132, /sqrt(3) in
// fp32); generate_masks (utils.py:48-54: bin n holds n/N <= m < (n+1)/N, so m == 1.0
// is in no bin); masked product (stereoanywhere.py:161) and the hourglass permute
// (hourglass.py:63).  The reference materialises [B,8,H,W1,W2] and then a permuted
// copy; here each output cell is computed once and written once (7 of 8 channels are
// zero because a pixel pair shares at most one bin).  Write-bound: 4·nbins bytes/cell.
// The fused hourglass does not read this volume: its two consumers (the stride-2 conv and
// the final up-cat conv, conv3d_fused.hip) evaluate the one-hot cells from per-pixel
// records (sa_mono_bin_records); the volume remains for the unfused (torch) hourglass.
#include "sa_common.h"

namespace {

__global__ __launch_bounds__(256) void normals_kernel(const float *__restrict__ mde, int H, int W,
                                                      float gain, long npix,
                                                      float *__restrict__ nrm) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long b = p / hw;
  const int y = (int)((p % hw) / W), x = (int)(p % W);
  const float *m = mde + b * hw;
  const int xl = max(x - 1, 0), xr = min(x + 1, W - 1);
  const int yu = max(y - 1, 0), yd = min(y + 1, H - 1);
  const float gx = gain * m[(long)y * W + xr] - gain * m[(long)y * W + xl];
  const float gy = gain * m[(long)yd * W + x] - gain * m[(long)yu * W + x];
  const float nx = -gx, ny = -gy, nz = 1.0f;
  const float norm = sqrtf(nx * nx + ny * ny + nz * nz);
  float *o = nrm + b * 3 * hw + (p % hw);
  o[0] = nx / norm;
  o[hw] = ny / norm;
  o[2 * hw] = nz / norm;
}

__device__ __forceinline__ int depth_bin(float m, int nbins) {
  // m*nbins is exact for power-of-two nbins; the general case compares like the reference
  for (int n = 0; n < nbins; ++n) {
    if (m < (float)(n + 1) / (float)nbins && m >= (float)n / (float)nbins) return n;
  }
  return -1;
}

// one thread = VEC consecutive j of one (b, k, h): VEC-wide stores into each of the nbins
// planes (VEC = 4 when W1 % 4 == 0, else 1)
template <int NB, int VEC>
__global__ __launch_bounds__(256) void masked_volume_kernel(
    const float *__restrict__ n2, const float *__restrict__ n3, const float *__restrict__ m2,
    const float *__restrict__ m3, int H, int W1, int W2, float gain, long nthreads,
    float *__restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const int q = W1 / VEC;
  const int j0 = (int)(t % q) * VEC;
  const long r1 = t / q;
  const int h = (int)(r1 % H);
  const long r2 = r1 / H;
  const int k = (int)(r2 % W2);
  const long b = r2 / W2;
  const long hw1 = (long)H * W1, hw2 = (long)H * W2;
  const float *nl = n2 + b * 3 * hw1 + (long)h * W1 + j0;
  const long pk = b * 3 * hw2 + (long)h * W2 + k;
  const float c0 = n3[pk], c1 = n3[pk + hw2], c2 = n3[pk + 2 * hw2];
  const int bk = depth_bin(m3[b * hw2 + (long)h * W2 + k], NB);
  float a0[VEC], a1[VEC], a2[VEC], ml[VEC];
  if constexpr (VEC == 4) {
    const float4 x0 = *reinterpret_cast<const float4 *>(nl);
    const float4 x1 = *reinterpret_cast<const float4 *>(nl + hw1);
    const float4 x2 = *reinterpret_cast<const float4 *>(nl + 2 * hw1);
    const float4 mm = *reinterpret_cast<const float4 *>(m2 + b * hw1 + (long)h * W1 + j0);
    a0[0] = x0.x; a0[1] = x0.y; a0[2] = x0.z; a0[3] = x0.w;
    a1[0] = x1.x; a1[1] = x1.y; a1[2] = x1.z; a1[3] = x1.w;
    a2[0] = x2.x; a2[1] = x2.y; a2[2] = x2.z; a2[3] = x2.w;
    ml[0] = mm.x; ml[1] = mm.y; ml[2] = mm.z; ml[3] = mm.w;
  } else {
    a0[0] = nl[0];
    a1[0] = nl[hw1];
    a2[0] = nl[2 * hw1];
    ml[0] = m2[b * hw1 + (long)h * W1 + j0];
  }
  const float sq3 = sqrtf(3.0f);
  float v[VEC];
  int bj[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    v[e] = gain * ((a0[e] * c0 + a1[e] * c1 + a2[e] * c2) / sq3);
    bj[e] = depth_bin(ml[e], NB);
  }
  float *o = out + ((b * NB) * W2 + k) * hw1 + (long)h * W1 + j0;
  const long plane = (long)W2 * hw1;
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    float r[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) r[e] = (bk == n && bj[e] == n) ? v[e] : 0.0f;
    if constexpr (VEC == 4) {
      *reinterpret_cast<float4 *>(o + n * plane) = make_float4(r[0], r[1], r[2], r[3]);
    } else {
      o[n * plane] = r[0];
    }
  }
}

// per-pixel record (n0, n1, n2, bin) of one view: the mono volume's one-hot structure
// without the volume (the hourglass's first convs evaluate cell (n, k, h, j) from the two
// records: value at channel n = bin iff both pixels are in bin n, else 0)
__global__ __launch_bounds__(256) void bin_records_kernel(const float *__restrict__ nrm, const float *__restrict__ m,
                                                          int hw, int nbins, long npix, float4 *__restrict__ rec) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long b = p / hw, q = p - b * hw;
  const float *n = nrm + b * 3 * hw + q;
  rec[p] = make_float4(n[0], n[hw], n[2 * hw], (float)depth_bin(m[p], nbins));
}

}  // namespace

extern "C" int sa_mono_bin_records(const float *normals, const float *m, int B, int H, int W, int nbins,
                                   float *rec, void *stream) {
  SA_REQUIRE(normals && m && rec, "sa_mono_bin_records: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0 && nbins > 0 && nbins <= 64, "sa_mono_bin_records: bad shape");
  SA_REQUIRE(((uintptr_t)rec & 15) == 0, "sa_mono_bin_records: records need 16-byte alignment");
  const long npix = (long)B * H * W;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  bin_records_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(normals, m, H * W, nbins, npix,
                                                                     reinterpret_cast<float4 *>(rec));
  return sa::check_launch("sa_mono_bin_records");
}

extern "C" int sa_mono_normals(const float *mde, int B, int H, int W, float gain, float *normals,
                               void *stream) {
  SA_REQUIRE(mde && normals, "sa_mono_normals: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W > 0, "sa_mono_normals: empty shape");
  const long npix = (long)B * H * W;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  normals_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(mde, H, W, gain, npix, normals);
  return sa::check_launch("sa_mono_normals");
}

extern "C" int sa_mono_masked_volume(const float *n2, const float *n3, const float *m2, const float *m3,
                                     int B, int H, int W1, int W2, int nbins, float gain, float *out,
                                     void *stream) {
  SA_REQUIRE(n2 && n3 && m2 && m3 && out, "sa_mono_masked_volume: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 0 && W2 > 0, "sa_mono_masked_volume: empty shape");
  SA_REQUIRE(nbins == 8, "sa_mono_masked_volume: only vol_n_masks == 8 is built (got %d)", nbins);
  const bool vec = W1 % 4 == 0 && ((uintptr_t)n2 | (uintptr_t)m2 | (uintptr_t)out) % 16 == 0;
  const long nthreads = (long)B * W2 * H * (vec ? W1 / 4 : W1);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MONO_VOLUME, s);
  const unsigned grid = (unsigned)((nthreads + 255) / 256);
  if (vec) {
    masked_volume_kernel<8, 4><<<grid, 256, 0, s>>>(n2, n3, m2, m3, H, W1, W2, gain, nthreads, out);
  } else {
    masked_volume_kernel<8, 1><<<grid, 256, 0, s>>>(n2, n3, m2, m3, H, W1, W2, gain, nthreads, out);
  }
  return sa::check_launch("sa_mono_masked_volume");
}
