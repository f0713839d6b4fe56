// The hourglass's stride-2 16 -> 32 3x3x3 convolution (down_layers[1][0]: hourglass.py:27-33,
// BasicConv3d submodule.py:25-53) as an implicit GEMM on v_mfma_f32_16x16x32_f16 with split
// operands, as conv3d_mfma.hip does for the stride-1 convs (same precision argument: InstanceNorm'ed
// activations satisfy |v| < 2^15, weights are scaled by 2^12 and refused beyond |w| >= 8 by ops.py;
// hi*hi + hi*lo + lo*hi per K-step, fp32 accumulation).
//
// GEMM mapping: M = 16 consecutive output columns, N = 16 output channels, K = 32 = two taps x 16
// input channels (tap 27 of the last K-step is empty: its weights are zero): 14 K-steps per output
// row and channel half.
// Tile = one output plane x 4 rows x 16 columns x 32 channels; a block of 4 waves stages the tile's
// input footprint (3 planes x 9 rows x 33 columns x 16 channels, the producer's InstanceNorm +
// LeakyReLU and the feature-attention gate gl[b,c,h,w] * gr[b,c,h,d] applied and split into
// f16 hi / lo while staging) in LDS as 16-byte entries of 8
// channels, [channel group][hl][plane][row][column]; wave w computes channel half w & 1 of rows
// 2 (w >> 1) and 2 (w >> 1) + 1 with its half's 28 B fragments resident in registers for the
// whole kernel.  The grid is persistent (two blocks per CU, each a contiguous run of tiles with the
// output plane fastest) so the weights are loaded once per block and the gate's (h, w) factors once
// per run of planes.  InstanceNorm partials (float64) per (image, channel, tile).
// Layout [B, C, D, H, W] (D = W2, W = W1), as conv3d_fused.hip.
#include "sa_common.h"

#pragma clang fp contract(fast)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr float kS2WScale = 4096.0f;                  // 2^12: weights -> f16 range
constexpr int S2_CIN = 16, S2_COUT = 32, S2_KS = 14;  // K-steps: 2 taps x 16 channels
constexpr int S2_TR = 4, S2_TC = 16;                  // output rows x columns per tile
constexpr int S2_PR = 2 * S2_TR + 1, S2_PC = 2 * S2_TC + 1;   // 9 x 33 input rows x columns
constexpr int S2_PPL = S2_PR * S2_PC;                 // entries per (channel group, hl, plane)
constexpr int S2_ENT = 2 * 2 * 3 * S2_PPL;            // 3564 entries, 57 KB
constexpr int S2_JOBS = 2 * 3 * S2_PPL;               // (channel group, plane, row, column) jobs
constexpr int S2_JPT = (S2_JOBS + 255) / 256;
constexpr int S2_TAB = 2 * S2_KS * 2 * 64;            // B fragments [half][K-step][hl][lane]

// [16][27][32] fp32 (ops.conv3d layout) -> the per-lane B fragments [half][K-step][hl][64]:
// lane l, element j: tap 2 s + (l >> 5), channel 8 ((l >> 4) & 1) + j, output 16 half + (l & 15)
__global__ void s2mf_weights_kernel(const float *__restrict__ w, f16x8 *__restrict__ tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * S2_KS * 64) return;
  const int lane = i & 63, s = (i >> 6) % S2_KS, nt = (i >> 6) / S2_KS;
  const int g = lane >> 4, tap = 2 * s + (g >> 1), cg = g & 1, co = 16 * nt + (lane & 15);
  f16x8 hi, lo;
  for (int j = 0; j < 8; ++j) {
    const float v = tap < 27 ? w[((8 * cg + j) * 27 + tap) * S2_COUT + co] * kS2WScale : 0.0f;
    const _Float16 h = (_Float16)v;
    hi[j] = h;
    lo[j] = (_Float16)(v - (float)h);
  }
  tab[((nt * S2_KS + s) * 2 + 0) * 64 + lane] = hi;
  tab[((nt * S2_KS + s) * 2 + 1) * 64 + lane] = lo;
}

__global__ __launch_bounds__(256, 2) void conv3d_s2mf_kernel(const float *__restrict__ in, int D, int H, int W,
                                                             int Do, int Ho, int Wo, const f16x8 *__restrict__ tab,
                                                             const float *__restrict__ mean,
                                                             const float *__restrict__ rstd, float slope,
                                                             const float *__restrict__ gl,
                                                             const float *__restrict__ gr,
                                                             float *__restrict__ out, double *__restrict__ partial,
                                                             int tilesW, int tilesH, int ntiles) {
  __shared__ f16x8 lds[S2_ENT];
  __shared__ float2 nrm[S2_CIN];
  // the tile's gate factors, staged once per tile: gl [ch][row][column], gr [ch][row][plane]
  __shared__ float gls[S2_CIN * S2_PPL], grs[S2_CIN * S2_PR * 3];
  __shared__ double red[2][2][16][2];   // [half][wave pair][channel][sum, sum of squares]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = wv & 1, rh = wv >> 1;   // channel half; rows 2 rh, 2 rh + 1 of the tile
  f16x8 bw[S2_KS][2];
#pragma unroll
  for (int s = 0; s < S2_KS; ++s)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) bw[s][hl] = tab[((nt * S2_KS + s) * 2 + hl) * 64 + lane];
  const long HW = (long)H * W, DHW = (long)D * HW;
  const int per_image = Do * tilesH * tilesW;
  const int m = lane & 15, g = lane >> 4, cgl = g & 1, tsel = g >> 1;
  // a block takes a contiguous run of tiles, output planes fastest: the gate factors (which do not
  // depend on the plane) are staged once per run of one (image, row tile, column tile); runs of
  // neighbouring blocks on one XCD (the XCD-grouped block id)
  const int chunk = (ntiles + gridDim.x - 1) / gridDim.x;
  const int t0 = (int)sa::xcd_remap(blockIdx.x, gridDim.x) * chunk, t1 = min(t0 + chunk, ntiles);
  int gkey = -1, prev = -2;
  for (int tile = t0; tile < t1; ++tile) {
    const int od = tile % Do, rest = tile / Do;
    // input plane id lives in LDS plane slot (id + 3) % 3: the next output plane of a run reuses
    // the last input plane of this one and stages only its two new planes
    const bool reuse = tile == prev + 1 && od > 0;
    prev = tile;
    const int tx = rest % tilesW, ty = (rest / tilesW) % tilesH;
    const int b = tile / per_image;
    const int id0 = 2 * od - 1, ih0 = 2 * ty * S2_TR - 1, iw0 = 2 * tx * S2_TC - 1;
    __syncthreads();   // the previous tile's LDS reads and reductions are done
    if (tid < S2_CIN) {
      const float rs = rstd[b * S2_CIN + tid];
      nrm[tid] = make_float2(rs, -mean[b * S2_CIN + tid] * rs);
    }
    if (gl && rest != gkey) {   // (block-uniform) gl: once per run of planes
      gkey = rest;
      for (int i = tid; i < S2_CIN * S2_PPL; i += 256) {
        const int ch = i / S2_PPL, rc = i % S2_PPL, ih = ih0 + rc / S2_PC, iw = iw0 + rc % S2_PC;
        const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < W;
        gls[i] = ok ? gl[(((long)b * S2_CIN + ch) * H + ih) * W + iw] : 0.0f;
      }
    }
    if (gl) {   // gr: the tile's 3 input planes
      for (int i = tid; i < S2_CIN * S2_PR * 3; i += 256) {
        const int ch = i / (S2_PR * 3), rp = i % (S2_PR * 3), ih = ih0 + rp / 3, id = id0 + rp % 3;
        const bool ok = ih >= 0 && ih < H && id >= 0 && id < D;
        grs[i] = ok ? gr[(((long)b * S2_CIN + ch) * H + ih) * D + id] : 0.0f;
      }
    }
    __syncthreads();
    // staging: T(x) = [gl gr] lrelu(x * rstd - mean * rstd), zero outside the volume (the padding)
    const int np = reuse ? 2 : 3, p0 = 3 - np, njobs = 2 * np * S2_PPL;
#pragma unroll
    for (int q = 0; q < S2_JPT; ++q) {
      const int job = tid + 256 * q;
      if (job < njobs) {
        const int c = job % S2_PC, r = (job / S2_PC) % S2_PR, p = p0 + (job / S2_PPL) % np, cg = job / (np * S2_PPL);
        const int id = id0 + p, ih = ih0 + r, iw = iw0 + c;
        const bool ok = id >= 0 && id < D && ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float *src = in + ((long)b * S2_CIN + 8 * cg) * DHW + (ok ? (long)id * HW + (long)ih * W + iw : 0);
        float x[8], gt[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = ok ? src[(long)j * DHW] : 0.0f;
        if (gl) {   // (block-uniform) the gate of (b, c, h, w) x (b, c, h, d), as InXform's pg
#pragma unroll
          for (int j = 0; j < 8; ++j)
            gt[j] = gls[(8 * cg + j) * S2_PPL + r * S2_PC + c] * grs[((8 * cg + j) * S2_PR + r) * 3 + p];
        }
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 nr = nrm[8 * cg + j];
          float v = fmaf(x[j], nr.x, nr.y);
          v = fmaxf(v, v * slope);
          if (gl) v = gt[j] * v;
          v = ok ? v : 0.0f;
          const _Float16 h = (_Float16)v;
          hi[j] = h;
          lo[j] = (_Float16)(v - (float)h);
        }
        const int sl = (id + 3) % 3;
        // columns stored even ones first, then odd ones: the stride-2 reads of a K-step hit
        // consecutive entries (2 m + kw -> m + kw / 2, or 17 + m for kw = 1)
        const int cs = (c & 1) ? 17 + (c >> 1) : (c >> 1);
        lds[((cg * 2 + 0) * 3 + sl) * S2_PPL + r * S2_PC + cs] = hi;
        lds[((cg * 2 + 1) * 3 + sl) * S2_PPL + r * S2_PC + cs] = lo;
      }
    }
    __syncthreads();
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int slot0 = (id0 + 3) % 3;   // LDS plane slot of the kd = 0 input plane (uniform)
#pragma unroll
    for (int s = 0; s < S2_KS; ++s) {
      const int tap = min(2 * s + tsel, 26);   // (tap 27: zero weights, any finite A)
      const int kh = (tap / 3) % 3, kw = tap % 3;
      const int sk = slot0 + (tsel ? min(2 * s + 1, 26) / 9 : (2 * s) / 9);
      const int pk = (sk >= 3 ? sk - 3 : sk) * S2_PPL;   // the tap's input plane slot
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int base = cgl * 2 * 3 * S2_PPL + pk + (2 * (2 * rh + mt) + kh) * S2_PC + m + (kw == 1 ? 17 : kw >> 1);
        const f16x8 ahi = lds[base], alo = lds[base + 3 * S2_PPL];
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bw[s][0], acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bw[s][1], acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bw[s][0], acc[mt], 0, 0, 0);
      }
    }
    // D lane layout: output columns 4 g .. 4 g + 3 of the M-tile, channel 16 nt + m
    const int co = 16 * nt + m, ow = tx * S2_TC + 4 * g;
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int oh = ty * S2_TR + 2 * rh + mt;
      if (oh >= Ho) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[mt][j] * (1.0f / kS2WScale);
      float *dst = out + (((long)b * S2_COUT + co) * Do + od) * (long)Ho * Wo + (long)oh * Wo + ow;
      if (ow + 3 < Wo && (Wo & 3) == 0) {
        *reinterpret_cast<float4 *>(dst) = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1 += v[j];
          s2 += v[j] * v[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ow + j < Wo) {
            dst[j] = v[j];
            s1 += v[j];
            s2 += v[j] * v[j];
          }
      }
    }
    if (partial) {
      double d1 = s1, d2 = s2;
      d1 += __shfl_xor(d1, 16);
      d2 += __shfl_xor(d2, 16);
      d1 += __shfl_xor(d1, 32);
      d2 += __shfl_xor(d2, 32);
      if (g == 0) {
        red[nt][rh][m][0] = d1;
        red[nt][rh][m][1] = d2;
      }
      __syncthreads();
      if (tid < 32) {
        const int n2 = tid >> 4, mm = tid & 15;
        double *pp = partial + (((long)b * S2_COUT + 16 * n2 + mm) * per_image + tile % per_image) * 2;
        pp[0] = red[n2][0][mm][0] + red[n2][1][mm][0];
        pp[1] = red[n2][0][mm][1] + red[n2][1][mm][1];
      }
    }
  }
}

}  // namespace

extern "C" long sa_conv3d_s2mf_weights_size() { return (long)S2_TAB * 16; }

// [16][27][32] (ops.conv3d layout) -> the kernel's B-fragment table (sa_conv3d_s2mf_weights_size
// bytes); the caller refuses weights with |w| >= 8 (ops.conv3d_s2mf_weights)
extern "C" int sa_conv3d_s2mf_weights(const float *weight, void *table, void *stream) {
  SA_REQUIRE(weight && table, "sa_conv3d_s2mf_weights: null pointer");
  hipStream_t s = sa::as_stream(stream);
  s2mf_weights_kernel<<<(2 * S2_KS * 64 + 255) / 256, 256, 0, s>>>(weight, static_cast<f16x8 *>(table));
  return sa::check_launch("sa_conv3d_s2mf_weights");
}

// InstanceNorm partials per (image, output channel): one per tile of the output plane range
extern "C" long sa_conv3d_s2mf_stat_parts(int Do, int Ho, int Wo) {
  if (Do <= 0 || Ho <= 0 || Wo <= 0) return -1;
  return (long)Do * ((Ho + S2_TR - 1) / S2_TR) * ((Wo + S2_TC - 1) / S2_TC);
}

// out = conv3d([gl * gr *] lrelu((x - mean) * rstd), W, stride 2, padding 1) for 16 -> 32 channels;
// x [B][16][D][H][W], mean / rstd [B*16] (the producer's InstanceNorm), optional gate maps
// gate_l [B*16][H][W] and gate_r [B*16][H][D] (sa_conv3d's), out [B][32][Do][Ho][Wo] with
// Do = (D - 1) / 2 + 1 etc.; partial: optional float64 (sum, sum of squares) per (b, co, tile)
extern "C" int sa_conv3d_s2mf(const float *in, int B, int D, int H, int W, const void *table, const float *mean,
                              const float *rstd, float slope, const float *gate_l, const float *gate_r, float *out,
                              double *partial, void *stream) {
  SA_REQUIRE(in && table && mean && rstd && out, "sa_conv3d_s2mf: null pointer");
  SA_REQUIRE((gate_l == nullptr) == (gate_r == nullptr), "sa_conv3d_s2mf: both gate maps or none");
  SA_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, "sa_conv3d_s2mf: empty shape");
  SA_REQUIRE((long)S2_CIN * D * H * W < (1L << 31) && (long)D * H * W < (1L << 30),
             "sa_conv3d_s2mf: volume too large (the split range needs D*H*W < 2^30)");
  SA_REQUIRE(slope >= 0.0f && slope <= 1.0f, "sa_conv3d_s2mf: LeakyReLU slope must be in [0, 1]");
  const int Do = (D - 1) / 2 + 1, Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int tilesW = (Wo + S2_TC - 1) / S2_TC, tilesH = (Ho + S2_TR - 1) / S2_TR;
  const long ntiles = (long)B * Do * tilesH * tilesW;
  SA_REQUIRE(ntiles < (1L << 31), "sa_conv3d_s2mf: too many tiles");
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV3D, s);
  const unsigned grid = (unsigned)std::min<long>(ntiles, 512);   // two persistent blocks per CU
  conv3d_s2mf_kernel<<<grid, 256, 0, s>>>(in, D, H, W, Do, Ho, Wo, static_cast<const f16x8 *>(table), mean, rstd,
                                          slope, gate_l, gate_r, out, partial, tilesW, tilesH, (int)ntiles);
  return sa::check_launch("sa_conv3d_s2mf");
}
