// Stride-1 3x3x3 convolutions of the hourglass (final_agg[1..2]: 8 -> 8 at full resolution,
// down_layers[0][1] / agg_layers[1][1..2]: 16 -> 16 at half, down_layers[1][1]: 32 -> 32 at quarter
// resolution; hourglass.py:13-91,
// BasicConv3d submodule.py:25-53) as an implicit GEMM on v_mfma_f32_16x16x32_f16 with split
// operands.
//
// Precision: every activation v = T(x) (the producer's InstanceNorm + LeakyReLU applied on load)
// is split into f16 hi + lo (22 significant bits); every weight is scaled by 2^12 and split the
// same way.  Each MFMA K-step accumulates hi*hi + hi*lo + lo*hi in fp32: the f16 products are
// exact, so the sum carries ~2^-22 relative error per term - the fp32 kernels' accuracy.  No
// range guard is needed: an InstanceNorm'ed value satisfies sum(v^2) = n var / (var + eps) <= n
// over its n = D*H*W voxels, so |v| <= sqrt(n) < 2^15 for n < 2^30 (the host requires it), and
// LeakyReLU only shrinks it; weights with |w| * 2^12 >= 2^15 are refused by ops.py.
//
// GEMM mapping (one wave, one MFMA): M = 16 consecutive output columns w, N = 16 output
// channels x planes, K = 32 = 4 groups of 8 input channels at one input plane:
//   * 8 -> 8: N = (2 output planes dd, 8 co), K = 4 input planes e (the pair's 3-tap D windows
//     span 4 planes; B(e, dd) = W[kd = e - dd], zero outside 0..2): 9 K-steps per plane pair;
//   * 16 -> 16: N = 16 co, K = (2 planes x 2 channel halves): 2 K-steps per (kh, kw), the second
//     half-empty (its empty lanes read a zero block);
//   * 32 -> 32: N = 16 co (a block computes one half of the outputs), K = 4 channel quarters at one
//     plane: 3 K-steps per (kh, kw), 216 weight registers: 4 waves, one per SIMD.
// B (the weights) is stationary in registers for the whole kernel (72 / 144 / 216); A is read
// from LDS with one ds_read_b128 per lane per operand half, at immediate offsets from a per-step
// base: zero address arithmetic in the MFMA loop.
//
// Dataflow: a block owns a TH x 64 tile of (h, w) over a range of DR output planes and streams
// the volume along D through a ring of staged input planes in LDS (the input is read once per
// block plus a (TH+2)/TH halo in H, mostly served from L2 by the neighbouring tiles that the
// XCD-grouped block order keeps on the same XCD).  Planes for the next step are loaded into
// registers at the top of a step and transformed, split and written to LDS after its MFMAs.
// Layout [B, C, D, H, W] throughout (D = W2, W = W1), as conv3d_fused.hip.
#include <cmath>

#include "sa_common.h"

#pragma clang fp contract(fast)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr float kWScale = 4096.0f;   // 2^12: weights -> f16 range

// 8 -> 8 and 16 -> 16: 8 waves (two per SIMD); 32 -> 32: 4 waves, one per SIMD (its 216 weight
// VGPRs), each block one 16-channel half of the outputs (NCH = 2)
template <int CIN, int COUT>
struct MfCfg {
  static constexpr int DD = COUT == 8 ? 2 : 1;        // output planes per step (N = DD x co)
  static constexpr int NCO = 16 / DD;                  // output channels per block
  static constexpr int NCH = COUT / NCO;               // output-channel blocks
  static constexpr int NCG = CIN / 8;                  // 8-channel groups
  static constexpr int NG = (DD + 2) * NCG;            // K groups (plane, channel group) per (kh, kw)
  static constexpr int KS = (NG + 3) / 4;              // MFMA K-steps per (kh, kw)
  static constexpr bool ZERO = KS * 4 > NG;            // some lanes of the last K-step are empty
  static constexpr int TH = CIN == 8 ? 8 : 4;          // output rows per block
  static constexpr int TW = CIN == 32 ? 32 : 64;       // output columns per block
  static constexpr int NWAVE = CIN == 32 ? 4 : 8;
  static constexpr int NTHR = 64 * NWAVE;
  static constexpr int WPE = CIN == 32 ? 1 : 2;        // waves per SIMD (register budget)
  static constexpr int MT = TH * TW / 16 / NWAVE;      // 16-column tiles per wave
  static constexpr int WPR = NWAVE / TH;               // waves per output row
  static constexpr int ROWS = TH + 2, COLS = TW + 2;
  static constexpr int PLANE = (ROWS * COLS + 15) / 16 * 16;   // 16-B entries, a multiple of 256 B
  static constexpr int RING = 2 * DD + 2;              // planes in use (DD + 2) + filling (DD)
  static constexpr int SLOT = NCG * 2 * PLANE;         // entries per ring slot: [cg][hl][entry]
  static constexpr int ENTRIES = RING * SLOT + (ZERO ? 2 * PLANE : 0);
  static constexpr int JOBS = NCG * ROWS * COLS;       // 8-channel staging jobs per plane
  static constexpr int JPT = (JOBS * DD + NTHR - 1) / NTHR;   // jobs per thread per step
  static constexpr int TAB = 9 * KS * 2 * 64;          // B fragments (f16x8) per output-channel block
  static_assert(ENTRIES * 16 <= 150 * 1024, "LDS");
  static_assert(MT * WPR * 16 == TW, "tiling");
};

// n-th column of the B fragment -> (output plane offset, output channel in the block's NCO)
template <int COUT>
__host__ __device__ inline void n_split(int n, int &dd, int &co) {
  if (COUT == 8) {
    dd = n >> 3;
    co = n & 7;
  } else {
    dd = 0;
    co = n;
  }
}

// [Cin][27][Cout] fp32 (ops.conv3d layout) -> the per-lane B fragments
// [NCH][9 (kh,kw)][KS][hl][64][8]
template <int CIN, int COUT>
__global__ void mf_weights_kernel(const float *__restrict__ w, f16x8 *__restrict__ tab) {
  using C = MfCfg<CIN, COUT>;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // ((ch * 9 + khw) * KS + t) * 64 + lane
  if (i >= C::NCH * 9 * C::KS * 64) return;
  const int lane = i & 63, t = (i >> 6) % C::KS, khw = (i >> 6) / C::KS % 9, ch = (i >> 6) / C::KS / 9;
  const int n = lane & 15, G = 4 * t + (lane >> 4);
  int dd, co;
  n_split<COUT>(n, dd, co);
  co += ch * C::NCO;
  const int e = G / C::NCG, cg = G % C::NCG, kd = e - dd;
  f16x8 hi, lo;
  for (int j = 0; j < 8; ++j) {
    float v = 0.0f;
    if (G < C::NG && kd >= 0 && kd <= 2) v = w[((8 * cg + j) * 27 + kd * 9 + khw) * COUT + co] * kWScale;
    const _Float16 h = (_Float16)v;
    hi[j] = h;
    lo[j] = (_Float16)(v - (float)h);
  }
  tab[ch * C::TAB + ((khw * C::KS + t) * 2 + 0) * 64 + lane] = hi;
  tab[ch * C::TAB + ((khw * C::KS + t) * 2 + 1) * 64 + lane] = lo;
}

template <int CIN, int COUT>
__global__ __launch_bounds__((MfCfg<CIN, COUT>::NTHR), 1)
__attribute__((amdgpu_waves_per_eu(MfCfg<CIN, COUT>::WPE, MfCfg<CIN, COUT>::WPE))) void conv3d_mf_kernel(const float *__restrict__ in, int D, int H, int W,
                                                                const f16x8 *__restrict__ wtab,
                                                                const float *__restrict__ mean,
                                                                const float *__restrict__ rstd, float slope,
                                                                float *__restrict__ out, double *__restrict__ partial,
                                                                int tilesW, int tilesH, int tilesD, int DR) {
  using C = MfCfg<CIN, COUT>;
  __shared__ f16x8 lds[C::ENTRIES];
  __shared__ float2 nrm[CIN];
  __shared__ double red[C::NWAVE][C::NCO][2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wid_ = (int)sa::xcd_remap(blockIdx.x, gridDim.x);
  const int ch = wid_ % C::NCH, wid = wid_ / C::NCH;   // (an output-channel block's neighbours share its input)
  const int bx = wid % tilesW, by = (wid / tilesW) % tilesH, dz = (wid / (tilesW * tilesH)) % tilesD;
  const int b = wid / (tilesW * tilesH * tilesD);
  wtab += ch * C::TAB;
  const int w0 = bx * C::TW, h0 = by * C::TH, d0 = dz * DR, d1 = min(d0 + DR, D);
  const long HW = (long)H * W;

  // T(x) = lrelu(x * rstd - mean * rstd); the whole ring starts zeroed: entries outside H x W
  // (the zero padding) are never written again
  if (tid < CIN) {
    const float rs = rstd[b * CIN + tid];
    nrm[tid] = make_float2(rs, -mean[b * CIN + tid] * rs);
  }
  for (int i = tid; i < C::ENTRIES; i += C::NTHR) lds[i] = f16x8{};

  // B fragments for the whole kernel
  f16x8 bw[9][C::KS][2];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int t = 0; t < C::KS; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) bw[k][t][hl] = wtab[((k * C::KS + t) * 2 + hl) * 64 + lane];

  // the thread's staging jobs, the same for every group of DD planes: job J = tid + 512 k ->
  // (plane q of the group, channel group cg, entry (row, col) of the (TH+2) x 66 window at
  // (h0 - 1, w0 - 1)); jobs outside H x W are dropped
  // the image's volume through a buffer resource: 32-bit offsets (< 2^32 bytes per image, checked
  // by the host), channel j of a job's group as the scalar offset j * D*H*W*4
  const __amdgpu_buffer_rsrc_t src_img = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(in + (long)b * CIN * D * HW), (short)0, (int)((long)CIN * D * HW * 4), 0x00020000);
  const int chan_bytes = (int)(D * HW * 4);
  unsigned joff[C::JPT];
  int jdst[C::JPT], jq[C::JPT], jcg[C::JPT];
  bool jok[C::JPT];
#pragma unroll
  for (int k = 0; k < C::JPT; ++k) {
    const int J = tid + k * C::NTHR;
    const int q = J / C::JOBS, r_ = J % C::JOBS, cg = r_ / (C::ROWS * C::COLS), e = r_ % (C::ROWS * C::COLS);
    const int hh = h0 - 1 + e / C::COLS, ww = w0 - 1 + e % C::COLS;
    jok[k] = J < C::DD * C::JOBS && hh >= 0 && hh < H && ww >= 0 && ww < W;
    joff[k] = jok[k] ? (unsigned)((8 * cg * (long)D * HW + (long)hh * W + ww) * 4) : 0u;
    jdst[k] = cg * 2 * C::PLANE + e;
    jq[k] = q;
    jcg[k] = cg;
  }
  // planes p0 .. p0 + DD - 1: loads into registers, then transform + split into their ring slots
  auto stage_load = [&](int p0, float (&x)[C::JPT][8]) {
#pragma unroll
    for (int k = 0; k < C::JPT; ++k) {
      const int p = p0 + jq[k];
      if (jok[k] && p >= 0 && p < D) {
        const unsigned vo = joff[k] + (unsigned)(p * HW * 4);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          x[k][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(src_img, vo, j * chan_bytes, 0));
      }
    }
  };
  auto stage_put = [&](int p0, const float (&x)[C::JPT][8]) {
#pragma unroll
    for (int k = 0; k < C::JPT; ++k) {
      if (!jok[k]) continue;
      const int p = p0 + jq[k];
      f16x8 hi{}, lo{};
      if (p >= 0 && p < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 nr = nrm[8 * jcg[k] + j];
          float v = __builtin_fmaf(x[k][j], nr.x, nr.y);
          v = fmaxf(v, v * slope);   // LeakyReLU for 0 <= slope <= 1 (NaN stays NaN)
          const _Float16 h = (_Float16)v;
          hi[j] = h;
          lo[j] = (_Float16)(v - (float)h);
        }
      }
      const int dst = ((p + C::RING) % C::RING) * C::SLOT + jdst[k];
      lds[dst] = hi;
      lds[dst + C::PLANE] = lo;
    }
  };
  __syncthreads();   // nrm, ring zeroed

  // prologue: planes d0 - 1 .. d0 + DD
#pragma unroll 1
  for (int p0 = d0 - 1; p0 < d0 + C::DD + 1; p0 += C::DD) {
    float x[C::JPT][8];
    stage_load(p0, x);
    stage_put(p0, x);
  }
  __syncthreads();

  // this wave's output row and columns; the lane's A row (m) and K group (g)
  const int r = wv / C::WPR, mt0 = (wv % C::WPR) * C::MT;
  const int m = lane & 15, g = lane >> 4;
  const int h = h0 + r;
  int dd_l, co_l;
  n_split<COUT>(m, dd_l, co_l);   // the lane's accumulator column n = lane & 15
  const int wl = w0 + 16 * mt0 + 4 * g;   // + 16 mt + j: the lane's accumulator rows
  const bool vec = (W & 3) == 0;
  double s_acc = 0.0, q_acc = 0.0;

  // step i (output planes dout = d0 + DD i ..): its top issues the loads of step i + 2's new planes,
  // its end writes step i + 1's (loaded during step i - 1) into the ring: two steps of loads in
  // flight, alternating between two register sets
  const int nsteps = (d1 - d0 + C::DD - 1) / C::DD;
  float xa[C::JPT][8], xb[C::JPT][8];
  if (nsteps > 1) stage_load(d0 + C::DD + 1, xa);
  auto step = [&](const int i, float (&xload)[C::JPT][8], float (&xput)[C::JPT][8]) __attribute__((always_inline)) {
    const int dout = d0 + C::DD * i;
    if (i + 2 < nsteps) stage_load(dout + 2 * C::DD + 1, xload);

    // the lane's A bases per K-step: group G = 4 t + g -> (plane e, channel group cg)
    int base[C::KS];
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
      const int G = 4 * t + g, e = G / C::NCG, cg = G % C::NCG;
      const int slot = (dout - 1 + e + C::RING) % C::RING;
      base[t] = G < C::NG ? ((slot * C::NCG + cg) * 2) * C::PLANE : C::RING * C::SLOT;
      base[t] += r * C::COLS + 16 * mt0 + m;
    }
    f32x4 acc[C::MT];
#pragma unroll
    for (int u = 0; u < C::MT; ++u) acc[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // A fragments one (kh, kw, t) step ahead: the MFMAs of a step overlap the next step's reads
    constexpr int NK = 9 * C::KS;
    f16x8 ah[2][C::MT], al[2][C::MT];
    auto fetch = [&](int kk, f16x8 (&h_)[C::MT], f16x8 (&l_)[C::MT]) {
      const int t = kk % C::KS, k = kk / C::KS, kh = k / 3, kw = k % 3;
#pragma unroll
      for (int u = 0; u < C::MT; ++u) {
        const f16x8 *a = lds + base[t] + kh * C::COLS + kw + 16 * u;
        h_[u] = a[0];
        l_[u] = a[C::PLANE];
      }
    };
    fetch(0, ah[0], al[0]);
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * C::MT, 0);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const int cur = kk & 1;
      if (kk + 1 < NK) fetch(kk + 1, ah[cur ^ 1], al[cur ^ 1]);
      const int t = kk % C::KS, k = kk / C::KS;
#pragma unroll
      for (int u = 0; u < C::MT; ++u) {
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cur][u], bw[k][t][0], acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cur][u], bw[k][t][1], acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[cur][u], bw[k][t][0], acc[u], 0, 0, 0);
      }
      // (the default schedule sinks every read next to its MFMA and waits on it)
      if (kk + 1 < NK) __builtin_amdgcn_sched_group_barrier(0x100, 2 * C::MT, 0);   // DS reads
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * C::MT, 0);                     // MFMAs
    }

    // epilogue: the lane holds out[b][co][dout + dd][h][wl + 16 u + j], j = 0..3
    const int d = dout + dd_l;
    if (d < d1 && h < H) {
      float s = 0.0f, q = 0.0f;
      float *o = out + (((long)b * COUT + ch * C::NCO + co_l) * D + d) * HW + (long)h * W;
#pragma unroll
      for (int u = 0; u < C::MT; ++u) {
        const int w = wl + 16 * u;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[u][j] * (1.0f / kWScale);
        if (vec && w + 3 < W) {
          *reinterpret_cast<float4 *>(o + w) = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s += v[j];
            q += v[j] * v[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (w + j < W) {
              o[w + j] = v[j];
              s += v[j];
              q += v[j] * v[j];
            }
        }
      }
      s_acc += (double)s;
      q_acc += (double)q;
    }

    // step i + 1's planes -> LDS (their slots held planes only step i - 1 read)
    if (i + 1 < nsteps) stage_put(dout + C::DD + 1, xput);
    __syncthreads();
  };
#pragma unroll 1
  for (int i = 0; i < nsteps; i += 2) {
    step(i, xb, xa);
    if (i + 1 < nsteps) step(i + 1, xa, xb);
  }

  // InstanceNorm partials: lanes n, n + 16, n + 32, n + 48 (and n + 8 for the plane pairs)
  // share an output channel
  if (partial) {
#pragma unroll
    for (int o = C::DD == 2 ? 8 : 16; o < 64; o <<= 1) {
      s_acc += __shfl_xor(s_acc, o);
      q_acc += __shfl_xor(q_acc, o);
    }
    if (lane < C::NCO) {
      red[wv][lane][0] = s_acc;
      red[wv][lane][1] = q_acc;
    }
    __syncthreads();
    if (tid < C::NCO) {
      double a = 0.0, e = 0.0;
#pragma unroll
      for (int k = 0; k < C::NWAVE; ++k) {
        a += red[k][tid][0];
        e += red[k][tid][1];
      }
      const int nparts = tilesW * tilesH * tilesD;
      const int blk = (dz * tilesH + by) * tilesW + bx;
      double *p = partial + (((long)b * COUT + ch * C::NCO + tid) * nparts + blk) * 2;
      p[0] = a;
      p[1] = e;
    }
  }
}

int g_mf_dr = 0;   // sa_conv3d_mf_set_planes: 0 = automatic

struct MfGeo {
  int tilesW, tilesH, tilesD, DR;
};

inline bool mf_shape(int Cin, int Cout) {
  return (Cin == 8 && Cout == 8) || (Cin == 16 && Cout == 16) || (Cin == 32 && Cout == 32);
}

// (tile sizes and blocks per output-channel set of MfCfg<Cin, Cin>)
MfGeo mf_geo(int B, int Cin, int D, int H, int W) {
  const int th = Cin == 8 ? 8 : 4, tw = Cin == 32 ? 32 : 64, dd = Cin == 8 ? 2 : 1, nch = Cin == 32 ? 2 : 1;
  const int waves = Cin == 32 ? 4 : 8;
  MfGeo g{(W + tw - 1) / tw, (H + th - 1) / th, 1, 0};
  int dr = g_mf_dr > 0 ? g_mf_dr : D;
  if (g_mf_dr <= 0) {
    // halve the planes per block until the grid fills the chip ~8 times over (in waves: 8 per
    // block-of-8-waves) or reaches 8 planes
    const long per = (long)B * g.tilesW * g.tilesH * nch * waves / 8;
    while (dr > 8 && per * ((D + dr - 1) / dr) < 8 * 256) dr = (dr + 1) / 2;
  }
  dr = (dr + dd - 1) / dd * dd;
  g.DR = dr;
  g.tilesD = (D + dr - 1) / dr;
  return g;
}

}  // namespace

extern "C" void sa_conv3d_mf_set_planes(int planes) { g_mf_dr = planes; }
extern "C" int sa_conv3d_mf_get_planes() { return g_mf_dr; }

extern "C" long sa_conv3d_mf_weights_size(int Cin, int Cout) {
  if (!mf_shape(Cin, Cout)) return -1;
  const int tab = Cin == 8 ? MfCfg<8, 8>::NCH * MfCfg<8, 8>::TAB
                : Cin == 16 ? MfCfg<16, 16>::NCH * MfCfg<16, 16>::TAB : MfCfg<32, 32>::NCH * MfCfg<32, 32>::TAB;
  return (long)tab * 16;
}

extern "C" int sa_conv3d_mf_weights(const float *weight, int Cin, int Cout, void *table, void *stream) {
  SA_REQUIRE(weight && table, "sa_conv3d_mf_weights: null pointer");
  SA_REQUIRE(mf_shape(Cin, Cout), "sa_conv3d_mf_weights: built for 8 -> 8, 16 -> 16 and 32 -> 32 (got %d -> %d)", Cin,
             Cout);
  hipStream_t s = sa::as_stream(stream);
  f16x8 *t = reinterpret_cast<f16x8 *>(table);
#define SA_MFW(CI)                                                                                              \
  mf_weights_kernel<CI, CI><<<(MfCfg<CI, CI>::NCH * 9 * MfCfg<CI, CI>::KS * 64 + 255) / 256, 256, 0, s>>>(weight, t)
  if (Cin == 8) SA_MFW(8);
  else if (Cin == 16) SA_MFW(16);
  else SA_MFW(32);
#undef SA_MFW
  return sa::check_launch("sa_conv3d_mf_weights");
}

extern "C" long sa_conv3d_mf_stat_parts(int B, int Cin, int Cout, int D, int H, int W) {
  if (!mf_shape(Cin, Cout) || B <= 0 || D <= 0 || H <= 0 || W <= 0) return -1;
  const MfGeo g = mf_geo(B, Cin, D, H, W);
  return (long)g.tilesW * g.tilesH * g.tilesD;
}

extern "C" int sa_conv3d_mf(const float *in, int B, int Cin, int D, int H, int W, const void *table, int Cout,
                            const float *in_mean, const float *in_rstd, float slope, float *out,
                            double *stats_partial, void *stream) {
  SA_REQUIRE(in && table && out && in_mean && in_rstd, "sa_conv3d_mf: null pointer");
  SA_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, "sa_conv3d_mf: empty shape");
  SA_REQUIRE(mf_shape(Cin, Cout), "sa_conv3d_mf: built for 8 -> 8, 16 -> 16 and 32 -> 32 (got %d -> %d)", Cin, Cout);
  // |InstanceNorm'ed value| <= sqrt(voxels) < 2^15: the f16 hi part cannot overflow
  SA_REQUIRE((long)D * H * W < (1L << 30), "sa_conv3d_mf: a channel volume must hold < 2^30 voxels");
  SA_REQUIRE(slope >= 0.0f && slope <= 1.0f, "sa_conv3d_mf: LeakyReLU slope must lie in [0, 1]");
  SA_REQUIRE((long)Cin * D * H * W * 4 < (1L << 31), "sa_conv3d_mf: an image's volume must hold < 2^31 bytes");
  SA_REQUIRE((long)B * Cin * D * H * W < (1L << 62), "sa_conv3d_mf: size");
  const MfGeo g = mf_geo(B, Cin, D, H, W);
  const long blocks = (long)B * g.tilesW * g.tilesH * g.tilesD * (Cin == 32 ? 2 : 1);
  SA_REQUIRE(blocks < (1L << 31), "sa_conv3d_mf: grid");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  const f16x8 *t = reinterpret_cast<const f16x8 *>(table);
#define SA_MF(CI)                                                                                             \
  conv3d_mf_kernel<CI, CI><<<(unsigned)blocks, MfCfg<CI, CI>::NTHR, 0, s>>>(                                  \
      in, D, H, W, t, in_mean, in_rstd, slope, out, stats_partial, g.tilesW, g.tilesH, g.tilesD, g.DR)
  if (Cin == 8) SA_MF(8);
  else if (Cin == 16) SA_MF(16);
  else SA_MF(32);
#undef SA_MF
  return sa::check_launch("sa_conv3d_mf");
}
