// Direct 2-D convolution for the motion encoder's flow stem (convf1 = Conv2d(2, 64, 7,
// padding=3) followed by ReLU, update.py:76, 85).
//
// With two input channels this conv is 1.6 GFLOP per 544x960 batch of four, but the
// library path lowered it to an NHWC implicit GEMM plus layout transposes (~1.7 ms per
// GRU iteration).  Here a 16x16-pixel block stages the (16+K-1)^2 halo of every input
// channel in LDS and each thread accumulates all COUT outputs of its pixel with
// wave-uniform (scalar) weights; bias and ReLU are applied in the epilogue.
#include "sa_common.h"

#include <cstdint>

// Convolution sums have no reference summation order to reproduce (MIOpen picks its own
// algorithm), so let a*b+c contract to (packed) FMA here; the library builds with
// -ffp-contract=off for the element-wise kernels that mirror torch expressions.
#pragma clang fp contract(fast)

namespace {

constexpr int T = 16;

template <int K, int COUT>
__global__ __launch_bounds__(256) void conv2d_small_kernel(const float *__restrict__ in, long in_bs, int Cin, int H,
                                                           int W, const float *__restrict__ wt,
                                                           const float *__restrict__ bias, int relu,
                                                           float *__restrict__ out, long out_bs) {
  constexpr int L = T + K - 1, P = K / 2;
  __shared__ float tile[L * L];
  const int tx = threadIdx.x & (T - 1), ty = threadIdx.x / T;
  const int x0 = blockIdx.x * T, y0 = blockIdx.y * T, b = blockIdx.z;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
  for (int ci = 0; ci < Cin; ++ci) {
    const float *src = in + (long)b * in_bs + (long)ci * H * W;
    __syncthreads();
    for (int i = threadIdx.x; i < L * L; i += 256) {
      const int yy = y0 - P + i / L, xx = x0 - P + i % L;
      tile[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? src[(long)yy * W + xx] : 0.0f;
    }
    __syncthreads();
    const float *wc = wt + (long)ci * K * K * COUT;  // weights pre-arranged [ci][ky][kx][co]
#pragma unroll 1
    for (int ky = 0; ky < K; ++ky)
#pragma unroll 1
      for (int kx = 0; kx < K; ++kx) {
        const float v = tile[(ty + ky) * L + tx + kx];
        const float *wp = wc + (ky * K + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] += wp[co] * v;
      }
  }
  const int x = x0 + tx, y = y0 + ty;
  if (x < W && y < H) {
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float r = acc[co] + (bias ? bias[co] : 0.0f);
      if (relu) r = fmaxf(r, 0.0f);
      out[(long)b * out_bs + (long)co * H * W + (long)y * W + x] = r;
    }
  }
}

// The flow stem (Cin 2, 7x7, 64 outputs) as an implicit GEMM on fp32 MFMA: M = pixels, N = 64
// output channels, K = 2 * 49 taps (padded to 100).  Block = 16 x 16 pixels, its halo staged in
// LDS once; wave w owns rows 4w .. 4w + 3 (four 16-pixel M-tiles).  v_mfma_f32_16x16x4_f32 lane
// (m = l % 16, k = l / 16) reads A = the tile pixel m's tap 4 j + k (one ds_read feeds the
// MFMAs of all four 16-channel blocks); the B operands (weights, tap 4 j + k, channel 16 cb +
// l % 16) stay in 100 VGPRs for the block's lifetime.  Accumulator lane l holds pixels
// 4 (l / 16) .. + 3 of channel l % 16: one float4 store per (M-tile, channel block).
// F1_CIN = 1: the model's call (round 6): the stereo flow's vertical channel is identically zero
// (sa_flow_update / the flow_x resample job write 0), so its 49 taps only add exact zeros; with
// them skipped (13 instead of 25 K steps) the sums are the same.
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int F1_K = 7, F1_L = T + F1_K - 1;

template <int F1_CIN>
__global__ __launch_bounds__(256) void conv2d_f1_mfma_kernel(const float *__restrict__ in, long in_bs, int H, int W,
                                                             const float *__restrict__ wt,
                                                             const float *__restrict__ bias, int relu,
                                                             float *__restrict__ out, long out_bs) {
  constexpr int F1_TAPS = F1_CIN * F1_K * F1_K, F1_KS = (F1_TAPS + 3) / 4;
  __shared__ float tile[2 * F1_L * F1_L + 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int x0 = blockIdx.x * T, y0 = blockIdx.y * T, b = blockIdx.z;
  const int m = lane & 15, kq = lane >> 4;
  // weights -> B operands: tap 4 j + kq, channel 16 cb + m (taps >= 98 are zero)
  float wb[F1_KS][4];
#pragma unroll
  for (int j = 0; j < F1_KS; ++j) {
    const int tap = 4 * j + kq;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) wb[j][cb] = tap < F1_TAPS ? wt[tap * 64 + 16 * cb + m] : 0.0f;
  }
  // LDS offsets of each tap (ci, ky, kx) relative to the pixel's window origin
  int toff[F1_KS];
#pragma unroll
  for (int j = 0; j < F1_KS; ++j) {
    const int tap = min(4 * j + kq, F1_TAPS - 1);
    const int ci = tap / (F1_K * F1_K), r = tap % (F1_K * F1_K);
    toff[j] = ci * F1_L * F1_L + (r / F1_K) * F1_L + r % F1_K;
  }
  const float *src = in + (long)b * in_bs;
  for (int i = threadIdx.x; i < F1_CIN * F1_L * F1_L; i += 256) {
    const int ci = i / (F1_L * F1_L), r = i % (F1_L * F1_L);
    const int yy = y0 - 3 + r / F1_L, xx = x0 - 3 + r % F1_L;
    tile[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? src[(long)ci * H * W + (long)yy * W + xx] : 0.0f;
  }
  __syncthreads();
  f32x4 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[t][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < F1_KS; ++j) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float a = tile[toff[j] + (4 * wv + t) * F1_L + m];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[j][cb], acc[t][cb], 0, 0, 0);
    }
  }
  // D lane layout: pixel 4 kq + i of the M-tile row, channel 16 cb + m
  const long hw = (long)H * W;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int y = y0 + 4 * wv + t, x = x0 + 4 * kq;
    if (y >= H) continue;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int co = 16 * cb + m;
      const float bv = bias ? bias[co] : 0.0f;
      f32x4 v = acc[t][cb];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += bv;
        if (relu) v[e] = fmaxf(v[e], 0.0f);
      }
      float *dst = out + (long)b * out_bs + co * hw + (long)y * W + x;
      if (x + 3 < W && (W & 3) == 0) {
        *reinterpret_cast<f32x4 *>(dst) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (x + e < W) dst[e] = v[e];
      }
    }
  }
}

// 3x3 / pad 1 conv with many inputs and very few outputs (flow_head.conv2: 256 -> 2,
// update.py:98-110), which the library runs at a few % of its arithmetic rate.  Memory
// bound.  A block is 62 output columns x NR rows x all outputs; its 8 waves split the input
// channels.  Per channel a lane loads one column (NR + 2 rows, coalesced across lanes) and
// takes its x-1 / x+1 neighbours from the adjacent lanes with DPP wave shifts (lanes 0 and
// 63 load the halo columns), so every input value is read from memory once per block;
// loads run UNR channels ahead.  The 8 partial sums are reduced through LDS in a fixed
// order; bias in the epilogue.  Weights in the module's own [Cout][Cin][3][3] layout
// (wave-uniform scalar loads).
constexpr int NW = 8, NR = 4, NCOL = 62;

__device__ __forceinline__ float lane_prev(float v) {   // lane i <- lane i - 1 (DPP wave_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_next(float v) {   // lane i <- lane i + 1 (DPP wave_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}

template <int COUT>
__global__ __launch_bounds__(512) void conv2d_k3_narrow_kernel(const float *__restrict__ in, long in_bs, int Cin,
                                                               int H, int W, const float *__restrict__ wt,
                                                               const float *__restrict__ bias,
                                                               float *__restrict__ out, long out_bs) {
  __shared__ float red[NW - 1][COUT][NR][64];
  const int lane = threadIdx.x & 63;
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long hw = (long)H * W;
  const int x = blockIdx.x * NCOL + lane - 1;   // the column this lane loads
  const int y0 = blockIdx.y * NR;
  const int b = blockIdx.z;
  const bool xin = x >= 0 && x < W;
  int roff[NR + 2];
  bool rok[NR + 2];
#pragma unroll
  for (int r = 0; r < NR + 2; ++r) {
    const int yy = y0 - 1 + r;
    rok[r] = xin && yy >= 0 && yy < H;
    roff[r] = rok[r] ? yy * W + x : 0;
  }
  const int per = Cin / NW, c0 = grp * per;
  float acc[NR][COUT];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[i][co] = 0.0f;
  const float *src = in + (long)b * in_bs + (long)c0 * hw;
  constexpr int UNR = 4;
  for (int cb = 0; cb < per; cb += UNR) {
    float col[UNR][NR + 2];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int r = 0; r < NR + 2; ++r) col[u][r] = (cb + u < per && rok[r]) ? src[(long)(cb + u) * hw + roff[r]] : 0.0f;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (cb + u >= per) break;
      float lft[NR + 2], rgt[NR + 2];
#pragma unroll
      for (int r = 0; r < NR + 2; ++r) {
        lft[r] = lane_prev(col[u][r]);
        rgt[r] = lane_next(col[u][r]);
      }
      const int ci = c0 + cb + u;
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        const float *w = wt + ((long)co * Cin + ci) * 9;
        float wk[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) wk[t] = w[t];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            acc[i][co] += wk[ky * 3 + 0] * lft[i + ky];
            acc[i][co] += wk[ky * 3 + 1] * col[u][i + ky];
            acc[i][co] += wk[ky * 3 + 2] * rgt[i + ky];
          }
        }
      }
    }
  }
  if (grp > 0) {
#pragma unroll
    for (int co = 0; co < COUT; ++co)
#pragma unroll
      for (int i = 0; i < NR; ++i) red[grp - 1][co][i][lane] = acc[i][co];
  }
  __syncthreads();
  if (grp == 0 && lane >= 1 && lane <= NCOL && x < W) {
#pragma unroll
    for (int co = 0; co < COUT; ++co)
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        if (y0 + i >= H) break;
        float r = acc[i][co];
#pragma unroll
        for (int g = 0; g < NW - 1; ++g) r += red[g][co][i][lane];
        out[(long)b * out_bs + co * hw + (long)(y0 + i) * W + x] = r + (bias ? bias[co] : 0.0f);
      }
  }
}

}  // namespace

extern "C" int sa_conv2d_k3_narrow(const float *in, long in_bs, int B, int Cin, int H, int W, const float *weight,
                                   const float *bias, int Cout, float *out, long out_bs, void *stream) {
  SA_REQUIRE(in && weight && out, "sa_conv2d_k3_narrow: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && Cin > 0 && Cin % NW == 0 && H > 0 && W > 0, "sa_conv2d_k3_narrow: bad shape");
  SA_REQUIRE((long)H * W < (1L << 31), "sa_conv2d_k3_narrow: plane too large");
  dim3 grid((unsigned)((W + NCOL - 1) / NCOL), (unsigned)((H + NR - 1) / NR), (unsigned)B);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_NARROW, s);
  if (Cout == 2) {
    conv2d_k3_narrow_kernel<2><<<grid, 512, 0, s>>>(in, in_bs, Cin, H, W, weight, bias, out, out_bs);
    return sa::check_launch("sa_conv2d_k3_narrow");
  }
  sa::set_error("sa_conv2d_k3_narrow: built for 2 outputs (got %d)", Cout);
  return SA_E_ARG;
}

extern "C" int sa_conv2d_small(const float *in, long in_bs, int B, int Cin, int H, int W, const float *weight,
                               const float *bias, int Cout, int ksize, int relu, float *out, long out_bs,
                               void *stream) {
  SA_REQUIRE(in && weight && out, "sa_conv2d_small: null pointer");
  SA_REQUIRE(B > 0 && Cin > 0 && Cin <= 8 && H > 0 && W > 0, "sa_conv2d_small: bad shape");
  SA_REQUIRE(ksize == 7 && Cout == 64, "sa_conv2d_small: built for 7x7 -> 64 channels (got %dx%d -> %d)", ksize,
             ksize, Cout);
  dim3 grid((W + T - 1) / T, (H + T - 1) / T, B);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_CONV_SMALL, s);
  const bool aligned = (reinterpret_cast<uintptr_t>(out) & 15) == 0 && out_bs % 4 == 0;
  if (Cin == 2 && aligned)
    conv2d_f1_mfma_kernel<2><<<grid, 256, 0, s>>>(in, in_bs, H, W, weight, bias, relu, out, out_bs);
  else if (Cin == 1 && aligned)
    conv2d_f1_mfma_kernel<1><<<grid, 256, 0, s>>>(in, in_bs, H, W, weight, bias, relu, out, out_bs);
  else
    conv2d_small_kernel<7, 64><<<grid, 256, 0, s>>>(in, in_bs, Cin, H, W, weight, bias, relu, out, out_bs);
  return sa::check_launch("sa_conv2d_small");
}
