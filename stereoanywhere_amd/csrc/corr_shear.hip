// K4 on a disparity-sheared pyramid: the correlation-pyramid lookup (CorrBlock1D.__call__,
// corr.py:93-115, through bilinear_sampler, utils.py:19-35) fused with the motion encoder's
// convc1 (update.py:75, 84), reading a copy of the pyramid laid out so that a wave's lanes
// (consecutive pixels j of one image row) read consecutive addresses.
//
// The row layout (corr_volume.hip: pixel row j holds its levels back to back) puts each
// pixel's 10-cell window in its own row, ~1.8 KB from its neighbour's: a wave touches 64
// separate cache lines per level, and the lookup moved 2.3x the bytes it uses.  Level l of
// image row (b, h) is sheared here into S_l[e][j] = C_l[j][(j >> l) - e + W_l - 1]:
//   e in [0, E_l), E_l = W_l + ((W1 - 1) >> l)   (all (j, k) pairs of the level, k = (j >> l) -
//   e + W_l - 1; the entries with k outside [0, W_l) are left unwritten: the lookup's tap test
//   selects the reference's zero padding there without reading them into the result)
// so pixel j's cell k sits at row e = (j >> l) - k + W_l - 1, column j.  Rows are P = W1 rounded
// up to 32 floats apart (sa_shear_row_pitch), so a 32-pixel row segment starting at a multiple
// of 32 is one whole 128-byte line: the producers write whole lines, never two halves from two
// blocks.  Neighbouring pixels
// at the same disparity read the same row e at neighbouring columns: one load instruction of
// the wave is one or two row segments.  Storage ~2x the row layout; written once per forward
// by sa_corr_pyramid_shear from the row-layout pyramid, read at every GRU iteration.
#include "sa_common.h"
#include "convc1_mfma.h"

namespace {

// the sheared slice of one image row (b, h): levels back to back, each E_l x W1 floats
struct ShGeo {
  int L, W1, W2, P;   // P: row pitch (floats)
  int wid[4], rows[4];
  long off[4];   // level offsets within a slice (floats)
  long slice;    // floats per slice, a multiple of 4
};

ShGeo shear_geo(int W1, int W2, int L) {
  ShGeo g{};
  g.L = L;
  g.W1 = W1;
  g.W2 = W2;
  g.P = sa::shear_pitch(W1);
  long off = 0;
  for (int l = 0; l < L; ++l) {
    g.wid[l] = sa_pyramid_level_width(W2, l);
    g.rows[l] = g.wid[l] + ((W1 - 1) >> l);
    g.off[l] = off;
    off += (long)g.rows[l] * g.P;
  }
  g.slice = off;   // (a multiple of 32)
  return g;
}

// one level of 32 consecutive pixel rows j of one slice: their W_l cells read once into LDS
// (row-contiguous loads), then every row e of the level written along j (128-byte segments)
constexpr int SH_J = 32;
__global__ __launch_bounds__(256) void shear_kernel(const float *__restrict__ pyr, long rs, int W1, int P, int off_l,
                                                    int Wl, int El, int lev, long slice_sz, long soff,
                                                    float *__restrict__ out) {
  extern __shared__ float tile[];   // [SH_J][Wl + 1]
  const long slice = blockIdx.z;
  const int j0 = blockIdx.x * SH_J;
  const int tid = threadIdx.x, pitch = Wl + 1;
  const int nj = min(SH_J, W1 - j0);
  for (int r = tid >> 6; r < nj; r += 4) {
    const float *src = pyr + (slice * W1 + j0 + r) * rs + off_l;
    for (int k = tid & 63; k < Wl; k += 64) tile[r * pitch + k] = src[k];
  }
  __syncthreads();
  // row e of column j holds cell k = (j >> lev) - e + Wl - 1 of row j; the cells with k outside
  // [0, Wl) are not written: the lookup's tap test on the grid index selects 0 for them
  // without using the loaded value (that halves this pass's writes)
  const int jl = tid % SH_J, j = j0 + jl;
  if (jl >= nj) return;
  float *dst = out + slice * slice_sz + soff + j;
  for (int e = tid / SH_J; e < El; e += 256 / SH_J) {
    const int k = (j >> lev) - e + Wl - 1;
    if (k >= 0 && k < Wl) dst[(long)e * P] = tile[jl * pitch + k];
  }
}

struct ShLGeo {
  int H, W1, P;
  long cbs;
  long slice;
  int wid[4], rows[4];
  int off[4];
};

// lookup_c1_vec_kernel (corr_lookup.hip) on the sheared pyramid: the same per-tap grid
// arithmetic, the window's cells gathered by one load each from the rows e of column j.
// DUAL: one thread takes its pixel in both volumes (grid.y = 1): the tap grid is computed once,
// both volumes' gathers are in flight together, and each convc1 weight is loaded once for both
// (half the waves, each with twice the independent work).
template <int L, int R, int COUT, bool MF = false, bool DUAL = false>
__global__ __launch_bounds__(256, (DUAL ? 2 : 1)) void lookup_c1_shear_kernel(const float *__restrict__ sa, const float *__restrict__ sb,
                                                              const float *__restrict__ cx, ShLGeo g, int npix,
                                                              const float *__restrict__ wt,
                                                              const float *__restrict__ bias, int nvol,
                                                              float *__restrict__ out) {
  constexpr int K = 2 * R + 1, NT = L * K, WIN = 2 * R + 4;   // cells x_-R - 1 .. x_-R + 2R + 2
  constexpr int NV = DUAL ? 2 : 1;
  static_assert(!MF || COUT == 64, "MFMA convc1: 64 outputs");
  __shared__ float c1lds[MF ? 4 : 1][MF ? NT * sa::C1_PITCH : 1];
  const int p0 = blockIdx.x * 256 + threadIdx.x;
  if (!MF && p0 >= npix) return;
  const int p = p0 < npix ? p0 : npix - 1;   // (MFMA: the whole wave takes part)
  const int v0 = DUAL ? 0 : blockIdx.y;
  const int hw = g.H * g.W1;
  const int b = p / hw, rem = p - b * hw;
  const int h = rem / g.W1, j = rem - h * g.W1;
  const float x = cx[(long)b * g.cbs + rem];
  const long soff = ((long)b * g.H + h) * g.slice + j;
  const float *__restrict__ S[NV];
  S[0] = (v0 ? sb : sa) + soff;
  if constexpr (DUAL) S[NV - 1] = sb + soff;
  float f[NV][NT];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int Wl = g.wid[l], El = g.rows[l];
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
      // (the wide clamp of lookup_c1_vec_kernel: consecutive taps stay within 1 of x_-R + t)
      xw = fminf(fmaxf(xw, -16777216.0f), 16777216.0f);
      xi[t + R] = (int)xw;
    }
    // cell k = xi[0] - 1 + c sits at row e = (j >> l) - k + Wl - 1 of column j
    const int e0 = (j >> l) - xi[0] + Wl;
    float cell[NV][WIN];
#pragma unroll
    for (int vv = 0; vv < NV; ++vv) {
      const float *__restrict__ lv = S[vv] + g.off[l];
#pragma unroll
      for (int c = 0; c < WIN; ++c) {
        const int e = e0 - c;
        cell[vv][c] = (unsigned)e < (unsigned)El ? lv[(long)e * g.P] : 0.0f;
      }
    }
#pragma unroll
    for (int vv = 0; vv < NV; ++vv)
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const int d = xi[t] - xi[0] - t;   // -1, 0 or +1 (fp32 rounding of the grid position)
        const float c0 = d == 0 ? cell[vv][t + 1] : d < 0 ? cell[vv][t] : cell[vv][t + 2];
        const float c1 = d == 0 ? cell[vv][t + 2] : d < 0 ? cell[vv][t + 1] : cell[vv][t + 3 < WIN ? t + 3 : WIN - 1];
        const float a0 = (xi[t] >= 0 && xi[t] <= Wl - 1) ? c0 : 0.0f;
        const float a1 = (xi[t] + 1 >= 0 && xi[t] + 1 <= Wl - 1) ? c1 : 0.0f;
        const float w = wgt[t];
        f[vv][l * K + t] = a0 * (1.0f - w) + a1 * w;
      }
  }
  if constexpr (MF) {
    const int lane = threadIdx.x & 63;
    sa::C1Weights<NT> w;
    sa::c1_load_weights<NT>(wt, bias, lane, w);
    const int wp0 = p0 - lane;
#pragma unroll
    for (int vv = 0; vv < NV; ++vv)
      sa::c1_mfma<NT>(f[vv], w, c1lds[threadIdx.x >> 6], lane, [&](int q, int gq, const auto &r) {
        sa::c1_store4(out, wp0 + 16 * q + 4 * (lane >> 4), 16 * gq + (lane & 15), hw, nvol, v0 + vv, npix, r);
      });
    return;
  }
  // (both volumes' channels c0 .. c0 + 7 together in DUAL: each weight is loaded once)
  float *__restrict__ o = out + ((long)b * nvol + v0) * COUT * hw + rem;
#pragma unroll(DUAL ? 2 : 4)
  for (int c0 = 0; c0 < COUT; c0 += 8) {
    float acc[NV][8];
#pragma unroll
    for (int vv = 0; vv < NV; ++vv)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[vv][c] = bias[c0 + c];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float wk = wt[k * COUT + c0 + c];
#pragma unroll
        for (int vv = 0; vv < NV; ++vv) acc[vv][c] = fmaf(wk, f[vv][k], acc[vv][c]);
      }
    }
#pragma unroll
    for (int vv = 0; vv < NV; ++vv)
#pragma unroll
      for (int c = 0; c < 8; ++c) o[((long)vv * COUT + c0 + c) * hw] = fmaxf(acc[vv][c], 0.0f);
  }
}

// The same lookup + convc1 with the work spread over a block's 256 threads for 64 pixels: phase 1
// gives each (volume, level) of a pixel to its own thread (4 or 8 tasks per pixel: 12 gathers and
// the 9 taps each), the taps go to LDS as [volume][tap][pixel]; phase 2 gives each thread 16 of the
// 64 convc1 outputs of one pixel in every volume (the same k-ordered fmaf chains, weights uniform
// per wave).  Four times the waves of lookup_c1_shear_kernel with a fraction of its registers:
// the gathers and the output stores of many more waves overlap.
template <int L, int R, int COUT, int NW = 4>
__global__ __launch_bounds__(64 * NW) void lookup_c1_shear_lds_kernel(const float *__restrict__ sa,
                                                                  const float *__restrict__ sb,
                                                                  const float *__restrict__ cx, ShLGeo g, int npix,
                                                                  const float *__restrict__ wt,
                                                                  const float *__restrict__ bias, int nvol,
                                                                  float *__restrict__ out) {
  constexpr int K = 2 * R + 1, NT = L * K, WIN = 2 * R + 4, PX = 64, CG = COUT / NW;
  constexpr int TPT = (2 * L + NW - 1) / NW;   // (volume, level) tasks per thread
  static_assert(COUT % NW == 0, "NW channel groups");
  __shared__ float ft[2][NT][PX];
  const int tid = threadIdx.x, px = tid & (PX - 1);
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar weight loads
  const int p0 = blockIdx.x * PX + px;
  const int p = p0 < npix ? p0 : npix - 1;
  const int hw = g.H * g.W1;
  const int b = p / hw, rem = p - b * hw;
  const int h = rem / g.W1, j = rem - h * g.W1;
  const float x = cx[(long)b * g.cbs + rem];
  const long soff = ((long)b * g.H + h) * g.slice + j;
  // phase 1: tasks (volume, level) = grp, grp + NW (wave-uniform; unrolled: a thread's tasks'
  // gathers in flight together)
#pragma unroll
  for (int tt = 0; tt < TPT; ++tt) {
    const int task = grp + NW * tt;
    if (task >= nvol * L) break;
    const int v = task / L, l = task % L;
    const int Wl = g.wid[l], El = g.rows[l];
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
      xw = fminf(fmaxf(xw, -16777216.0f), 16777216.0f);
      xi[t + R] = (int)xw;
    }
    const int e0 = (j >> l) - xi[0] + Wl;
    const float *__restrict__ lv = (v ? sb : sa) + soff + g.off[l];
    float cell[WIN];
#pragma unroll
    for (int c = 0; c < WIN; ++c) {
      const int e = e0 - c;
      cell[c] = (unsigned)e < (unsigned)El ? lv[(long)e * g.P] : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int d = xi[t] - xi[0] - t;
      const float c0 = d == 0 ? cell[t + 1] : d < 0 ? cell[t] : cell[t + 2];
      const float c1 = d == 0 ? cell[t + 2] : d < 0 ? cell[t + 1] : cell[t + 3 < WIN ? t + 3 : WIN - 1];
      const float a0 = (xi[t] >= 0 && xi[t] <= Wl - 1) ? c0 : 0.0f;
      const float a1 = (xi[t] + 1 >= 0 && xi[t] + 1 <= Wl - 1) ? c1 : 0.0f;
      const float w = wgt[t];
      ft[v][l * K + t][px] = a0 * (1.0f - w) + a1 * w;
    }
  }
  __syncthreads();
  if (p0 >= npix) return;
  // phase 2: channels CG * grp .. + CG - 1, one volume after the other (16 accumulators)
  const int c0 = CG * grp;
  for (int v = 0; v < nvol; ++v) {
    float acc[CG];
#pragma unroll
    for (int c = 0; c < CG; ++c) acc[c] = bias[c0 + c];
#pragma unroll 4
    for (int k = 0; k < NT; ++k) {
      const float f = ft[v][k][px];
#pragma unroll
      for (int c = 0; c < CG; ++c) acc[c] = fmaf(wt[k * COUT + c0 + c], f, acc[c]);
    }
    float *__restrict__ o = out + (((long)b * nvol + v) * COUT + c0) * hw + rem;
#pragma unroll
    for (int c = 0; c < CG; ++c) o[(long)c * hw] = fmaxf(acc[c], 0.0f);
  }
}

}  // namespace

extern "C" int sa_lookup_get_mfma();

namespace {
int g_shear_dual = 3;   // sheared lookup form: 0 one volume per thread, 1 both, 2 / 3 spread over a 4 / 8-wave block
}
extern "C" void sa_lookup_set_shear_dual(int on) { g_shear_dual = on < 0 ? 0 : on > 3 ? 3 : on; }
extern "C" int sa_lookup_get_shear_dual() { return g_shear_dual; }

extern "C" long sa_shear_row_pitch(int W1) { return W1 > 0 ? sa::shear_pitch(W1) : -1; }

extern "C" long sa_shear_slice_size(int W1, int W2, int num_levels) {
  if (W1 <= 0 || W2 <= 0 || num_levels < 1 || num_levels > 4) return -1;
  return shear_geo(W1, W2, num_levels).slice;
}

extern "C" long sa_shear_level_offset(int W1, int W2, int num_levels, int level) {
  if (level < 0 || level >= num_levels || num_levels > 4) return -1;
  return shear_geo(W1, W2, num_levels).off[level];
}

// 1 when the sheared pipeline (sa_corr_pyramid_shear + sa_corr_lookup_conv1x1_sheared) takes this
// geometry: one grid z-slice per image row (B * H <= 65535), a 32-row LDS tile of the widest
// level (W2 <= 511), a coarsest level of width >= 2 and a pixel count in int range
extern "C" int sa_corr_shear_supported(int B, int H, int W1, int W2, int num_levels) {
  if (B <= 0 || H <= 0 || W1 <= 0 || W2 <= 0 || num_levels != 4) return 0;
  if ((long)B * H > 65535) return 0;
  if ((long)SH_J * (W2 + 1) * 4 > 64 * 1024) return 0;
  if (sa_pyramid_level_width(W2, num_levels - 1) < 2) return 0;
  if ((long)B * H * W1 >= (1L << 31)) return 0;
  return 1;
}

extern "C" int sa_corr_pyramid_shear(const float *pyramid, long row_stride, int B, int H, int W1, int W2,
                                     int num_levels, float *sheared, void *stream) {
  SA_REQUIRE(pyramid && sheared, "sa_corr_pyramid_shear: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 0 && W2 > 0 && num_levels >= 1 && num_levels <= 4,
             "sa_corr_pyramid_shear: bad shape");
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels), "sa_corr_pyramid_shear: row_stride too small");
  SA_REQUIRE((long)B * H <= 65535, "sa_corr_pyramid_shear: more than 65535 image rows");
  const ShGeo g = shear_geo(W1, W2, num_levels);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_SHEAR, s);
  SA_REQUIRE((long)SH_J * (W2 + 1) * 4 <= 64 * 1024, "sa_corr_pyramid_shear: W2 %d too wide for the LDS tile", W2);
  for (int l = 0; l < num_levels; ++l) {
    const dim3 grid((unsigned)((W1 + SH_J - 1) / SH_J), 1u, (unsigned)(B * H));
    const size_t lds = (size_t)SH_J * (g.wid[l] + 1) * sizeof(float);
    shear_kernel<<<grid, 256, lds, s>>>(pyramid, row_stride, W1, g.P, sa_pyramid_level_offset(W2, l), g.wid[l], g.rows[l],
                                        l, g.slice, g.off[l], sheared);
  }
  return sa::check_launch("sa_corr_pyramid_shear");
}

extern "C" int sa_corr_lookup_conv1x1_sheared(const float *sheared_a, const float *sheared_b, int W2, int num_levels,
                                              int radius, const float *coords_x, long coords_bstride, int B, int H,
                                              int W1, const float *weight_kc, const float *bias, int Cout, float *out,
                                              void *stream) {
  SA_REQUIRE(sheared_a && coords_x && out && weight_kc && bias, "sa_corr_lookup_conv1x1_sheared: null pointer");
  SA_REQUIRE(B > 0 && H > 0 && W1 > 0 && W2 > 0, "sa_corr_lookup_conv1x1_sheared: empty shape");
  SA_REQUIRE(num_levels == 4 && radius == 4 && Cout == 64,
             "sa_corr_lookup_conv1x1_sheared: built for 4 levels, radius 4, 64 outputs (got %d, %d, %d)", num_levels,
             radius, Cout);
  SA_REQUIRE(sa_pyramid_level_width(W2, num_levels - 1) >= 2,
             "sa_corr_lookup_conv1x1_sheared: level %d of width %d is too narrow to sample", num_levels - 1,
             sa_pyramid_level_width(W2, num_levels - 1));
  const long npix = (long)B * H * W1;
  SA_REQUIRE(npix < (1L << 31), "sa_corr_lookup_conv1x1_sheared: too many pixels");
  const ShGeo sg = shear_geo(W1, W2, num_levels);
  ShLGeo g{};
  g.H = H;
  g.W1 = W1;
  g.P = sg.P;
  g.cbs = coords_bstride;
  g.slice = sg.slice;
  for (int l = 0; l < 4; ++l) {
    g.wid[l] = l < num_levels ? sg.wid[l] : 0;
    g.rows[l] = l < num_levels ? sg.rows[l] : 0;
    g.off[l] = l < num_levels ? (int)sg.off[l] : 0;
  }
  const int nvol = sheared_b ? 2 : 1;
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_LOOKUP, s);
  const float *sbb = sheared_b ? sheared_b : sheared_a;
  if (g_shear_dual >= 2 && !sa_lookup_get_mfma()) {
    if (g_shear_dual == 3)
      lookup_c1_shear_lds_kernel<4, 4, 64, 8><<<(unsigned)((npix + 63) / 64), 512, 0, s>>>(
          sheared_a, sbb, coords_x, g, (int)npix, weight_kc, bias, nvol, out);
    else
      lookup_c1_shear_lds_kernel<4, 4, 64><<<(unsigned)((npix + 63) / 64), 256, 0, s>>>(
          sheared_a, sbb, coords_x, g, (int)npix, weight_kc, bias, nvol, out);
    return sa::check_launch("sa_corr_lookup_conv1x1_sheared");
  }
  const bool dual = nvol == 2 && g_shear_dual;
  dim3 grid((unsigned)((npix + 255) / 256), dual ? 1 : nvol);
#define SA_LK(MF_, DU_) \
  lookup_c1_shear_kernel<4, 4, 64, MF_, DU_><<<grid, 256, 0, s>>>(sheared_a, sbb, coords_x, g, (int)npix, weight_kc, \
                                                                  bias, nvol, out)
  if (sa_lookup_get_mfma()) {
    if (dual) SA_LK(true, true);
    else SA_LK(true, false);
  } else {
    if (dual) SA_LK(false, true);
    else SA_LK(false, false);
  }
#undef SA_LK
  return sa::check_launch("sa_corr_lookup_conv1x1_sheared");
}
