// K1 — all-pairs 1-D correlation volume on fp32 MFMA, fused with the truncation
// volume and the 1-D average-pool pyramid.
//
// Reference: CorrBlock1D.corr (corr.py:117-132) = einsum('aijk,aijh->ajkh')/sqrt(C);
// truncate_corr_volume_v2 (utils.py:216-238) applied at stereoanywhere.py:253-254;
// CorrBlock1D.__init__ (corr.py:76-91) pyramid of avg_pool2d([1,2]).
//
// For every image row (b,h) the volume is a W1 x W2 GEMM with K = C (256):
// A[j][c] = fmap2[b,c,h,j] and B[c][k] = fmap3[b,c,h,k] are both contiguous along
// j / k in NCHW, i.e. exactly the k-major operand layout v_mfma_f32_32x32x2_f32 reads
// (A lane l: A[l&31][l>>5], B lane l: B[l>>5][l&31]).  A block computes a 64(j) x 128(k)
// tile with 4 waves (each 32 x 64 = two 32x32 accumulators), staging 32-channel slices
// of both panels through LDS with one register-prefetched stage in flight.
// f32-input MFMA is exact f32 (a k-ordered fmaf chain), so the sum differs from the
// CPU einsum only by accumulation order.
//
// Epilogue: divide by sqrt(C), multiply by the analytic truncation factor
// T = (1-m) + m (sigmoid((j-d)-k)(1-a) + a) (two per-pixel scalars, zero extra HBM
// bytes), then write level 0 and build levels 1..3 with lane shuffles: the accumulator
// column is the lane (col = lane&31), so pairs (k, k+1) sit in lanes (l, l^1).
#include "sa_common.h"

namespace {

constexpr int TJ = 64;    // tile rows (left pixels j)
constexpr int TK = 128;   // tile cols (right pixels k)
constexpr int KC = 32;    // channels per LDS stage

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Geo {
  int C, H, W1, W2, tilesJ, tilesK, nlev;
  long rs;
  int off[4], wid[4];
};

template <bool VEC, bool TRUNC>
__global__ __launch_bounds__(256) void corr_pyramid_kernel(
    const float *__restrict__ f2, const float *__restrict__ f3, Geo g, float sqrt_c,
    const float *__restrict__ tdisp, const float *__restrict__ tconf, float atten,
    float *__restrict__ pyr) {
  __shared__ float As[KC][TJ];
  __shared__ float Bs[KC][TK];

  const unsigned nwg = gridDim.x;
  const unsigned wid = sa::xcd_remap(blockIdx.x, nwg);
  const int tiles = g.tilesJ * g.tilesK;
  const int bh = wid / tiles, tile = wid % tiles;
  const int j0 = (tile / g.tilesK) * TJ, k0 = (tile % g.tilesK) * TK;
  const int b = bh / g.H, h = bh % g.H;
  const long cstride = (long)g.H * g.W1;  // fmap2 channel stride
  const long cstride3 = (long)g.H * g.W2;
  const long base2 = (long)b * g.C * cstride + (long)h * g.W1;
  const long base3 = (long)b * g.C * cstride3 + (long)h * g.W2;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wj = w & 1, wk = w >> 1;

  f32x16 acc0 = {0.f}, acc1 = {0.f};
  float4 ra[2], rb[4];

  auto load = [&](int c0) {
    // A panel
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = t + 256 * i;
      const int c = q >> 4, j = j0 + ((q & 15) << 2);
      const bool okc = (c0 + c) < g.C;
      const float *p = f2 + base2 + (long)(c0 + c) * cstride + j;
      if (VEC && okc && j + 3 < g.W1) {
        ra[i] = *reinterpret_cast<const float4 *>(p);
      } else {
        ra[i].x = (okc && j + 0 < g.W1) ? p[0] : 0.f;
        ra[i].y = (okc && j + 1 < g.W1) ? p[1] : 0.f;
        ra[i].z = (okc && j + 2 < g.W1) ? p[2] : 0.f;
        ra[i].w = (okc && j + 3 < g.W1) ? p[3] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + 256 * i;
      const int c = q >> 5, k = k0 + ((q & 31) << 2);
      const bool okc = (c0 + c) < g.C;
      const float *p = f3 + base3 + (long)(c0 + c) * cstride3 + k;
      if (VEC && okc && k + 3 < g.W2) {
        rb[i] = *reinterpret_cast<const float4 *>(p);
      } else {
        rb[i].x = (okc && k + 0 < g.W2) ? p[0] : 0.f;
        rb[i].y = (okc && k + 1 < g.W2) ? p[1] : 0.f;
        rb[i].z = (okc && k + 2 < g.W2) ? p[2] : 0.f;
        rb[i].w = (okc && k + 3 < g.W2) ? p[3] : 0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = t + 256 * i;
      *reinterpret_cast<float4 *>(&As[q >> 4][(q & 15) << 2]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + 256 * i;
      *reinterpret_cast<float4 *>(&Bs[q >> 5][(q & 31) << 2]) = rb[i];
    }
  };

  load(0);
  for (int c0 = 0; c0 < g.C; c0 += KC) {
    __syncthreads();  // previous stage fully consumed
    store();
    __syncthreads();
    if (c0 + KC < g.C) load(c0 + KC);  // prefetch next stage under the MFMAs
    const int arow = lane >> 5, col = lane & 31;
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      const float a = As[kk + arow][wj * 32 + col];
      const float b0 = Bs[kk + arow][wk * 64 + col];
      const float b1 = Bs[kk + arow][wk * 64 + 32 + col];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }
  }

  // ---------------------------------------------------------------- epilogue
  const int col = lane & 31, hi = lane >> 5;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * hi;
      const int j = j0 + wj * 32 + row;
      const int k = k0 + wk * 64 + n * 32 + col;
      float v = (n == 0 ? acc0[r] : acc1[r]) / sqrt_c;
      const bool jok = j < g.W1;
      if (TRUNC) {
        float d = 0.f, m = 0.f;
        if (jok) {
          const long pix = ((long)b * g.H + h) * g.W1 + j;
          d = tdisp[pix];
          m = tconf[pix];
        }
        const float center = (float)j - d;
        const float tv = center - (float)k;
        const float s = sa::sigmoidf_ref(tv);
        const float T = 1.0f * (1.0f - m) + m * (s * (1.0f - atten) + atten);
        v = T * v;
      }
      float *row_ptr = pyr + (((long)b * g.H + h) * g.W1 + j) * g.rs;
      if (jok && k < g.W2) row_ptr[k] = v;
      if (g.nlev > 1) {
        // level 1: (v[k] + v[k+1]) / 2 held by the even lane
        const float v1 = (v + __shfl_xor(v, 1)) * 0.5f;
        const int k1 = k >> 1;
        if (jok && (col & 1) == 0 && k1 < g.wid[1]) row_ptr[g.off[1] + k1] = v1;
        if (g.nlev > 2) {
          const float v2 = (v1 + __shfl_xor(v1, 2)) * 0.5f;
          const int k2 = k >> 2;
          if (jok && (col & 3) == 0 && k2 < g.wid[2]) row_ptr[g.off[2] + k2] = v2;
          if (g.nlev > 3) {
            const float v3 = (v2 + __shfl_xor(v2, 4)) * 0.5f;
            const int k3 = k >> 3;
            if (jok && (col & 7) == 0 && k3 < g.wid[3]) row_ptr[g.off[3] + k3] = v3;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K1 v2 — the same volume + truncation + pyramid for the common case (C % 16 == 0, W1 and W2
// multiples of 4, 16-byte aligned rows), built for W/4 of a few hundred pixels:
//   block = one image row (b, h), 64 left pixels j (4 waves x one 16-row MFMA tile) x up to 256
//           right pixels k; W1 = 240 takes 3.75 blocks per row with no padded j rows
//   wave  = 16 j x 256 k as 16 v_mfma_f32_16x16x4_f32 tiles whose columns interleave by 4:
//           tile (g, t) holds pixels k = 64 g + 4 n + t (n = the accumulator column), so a lane
//           owns 4 consecutive k of every row it holds -> level 0 is one float4 store, levels 1
//           and 2 are formed in registers and level 3 takes one lane shuffle
//   chunk = 16 channels of both panels (A [16][64], B [16][256]) copied global -> LDS by
//           LDS-DMA (no staging registers), double-buffered, one barrier per chunk; 40 KiB per
//           block, so four blocks (16 waves) share a CU and cover each other's waits
//   per K step (4 channels): one ds_read_b32 (A), four ds_read_b128 (B), 16 MFMAs
// Arithmetic per element is the v1 kernel's: one k-ordered chain of exact fp32 MFMA products
// and the same epilogue expressions.
constexpr int V2_J = 64, V2_K = 256, V2_KC = 16;
constexpr int V2_ABUF = V2_KC * V2_J, V2_BBUF = V2_KC * V2_K, V2_BUF = V2_ABUF + V2_BBUF;

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void v2_dma16(__amdgpu_buffer_rsrc_t r, float *lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds, 16, voff, 0, 0, 0);
}

// The disparity-sheared output (corr_shear.hip): per image row (b, h) a slice of `slice` floats,
// level l at off[l] as rows[l] x W1 floats, S_l[e][j] = C_l[j][(j >> l) - e + W_l - 1]
struct ShOut {
  float *base;
  long slice;
  int pitch;   // row pitch (floats, a multiple of 32)
  long off[4];
  int rows[4];
};

// The sheared rows of one 32-pixel round: level l's cells of pixels [jr0, jr0 + 32) and cells
// [K, KE) staged in LDS as Tl[jl][kk - K] (pitch pl, odd: the lane reads Tl[jl][(jr0 + jl >> l) - e
// + W_l - 1 - K] fall in distinct banks), written as rows e of the level: lanes 0-31 row e,
// lanes 32-63 row e + 1, each a whole 128-byte line (the row pitch is a multiple of 32 floats and
// jr0 of 32).  Only the rows holding a cell of [K, KE) are visited; cells outside the level are
// not written (the sheared lookup's tap test never uses them).
__device__ __forceinline__ void sh_write_round(const ShOut &so, float *sl, const float *Tl, int pl, int l, int Wl,
                                               int K, int KE, int W1, int jr0, int wv, int nw, int lane) {
  const int jh = lane & 31, j = jr0 + jh;
  const int jr1 = min(jr0 + 32, W1);
  int emin = (jr0 >> l) - (KE - 1) + Wl - 1, emax = ((jr1 - 1) >> l) - K + Wl - 1;
  emin = max(emin, 0);
  emax = min(emax, so.rows[l] - 1);
  const int jsh = j >> l;
  float *dst = sl + so.off[l] + j;
  const float *src = Tl + jh * pl - K;
#pragma unroll 2
  for (int e = emin + 2 * wv + (lane >> 5); e <= emax; e += 2 * nw) {
    const int kk = jsh - e + Wl - 1;
    if (j < jr1 && kk >= K && kk < KE) dst[(long)e * so.pitch] = src[kk];
  }
}

template <bool TRUNC, bool POW2, bool SHEAR = false>
// (the sheared epilogue holds the cells while it stages them: 3 blocks per CU, no spill)
__global__ __launch_bounds__(256, (SHEAR ? 3 : 4)) void corr_pyramid_v2_kernel(const float *__restrict__ f2, const float *__restrict__ f3,
                                                              Geo g, int jblocks, int kblocks, int kstep, float sqrt_c,
                                                              float inv_c, const float *__restrict__ tdisp,
                                                              const float *__restrict__ tconf, float atten,
                                                              float *__restrict__ pyr, int f2_bytes, int f3_bytes,
                                                              ShOut so) {
  __shared__ __attribute__((aligned(16))) float smem[2 * V2_BUF];
  const unsigned nwg = gridDim.x;
  const unsigned wid = sa::xcd_remap(blockIdx.x, nwg);
  // consecutive ids: the j blocks of one (row, k block) -> they share the B panel in L2
  const int jb = wid % jblocks, rest = wid / jblocks, kb = rest % kblocks, bh = rest / kblocks;
  const int b = bh / g.H, h = bh % g.H;
  // k range [k0, kend): kstep (a multiple of 64, <= 256) splits W2 into near-equal blocks
  const int j0 = jb * V2_J, k0 = kb * kstep, kend = min(k0 + kstep, g.W2);
  const int ngroups = (kend - k0 + 63) >> 6;   // 64-wide column groups with work (wave-uniform)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(f2), (short)0, f2_bytes,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(f3), (short)0, f3_bytes,
                                                                      0x00020000);
  // DMA sources: wave w fills A rows 4w..4w+3 (lane: channel 4w + lane/16, j0 + 4 (lane%16)) and
  // B rows 4w..4w+3 (one channel each, k0 + 4 lane); out-of-range groups read 0
  const long plane1 = (long)g.H * g.W1, plane2 = (long)g.H * g.W2;
  const int ja = j0 + 4 * (lane & 15);
  int aoff = (ja < g.W1) ? (int)((((long)b * g.C + 4 * w + (lane >> 4)) * plane1 + (long)h * g.W1 + ja) * 4) : 0x7ffffff0;
  const int kbq = k0 + 4 * lane;
  int boff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    boff[q] = (kbq < kend) ? (int)((((long)b * g.C + 4 * w + q) * plane2 + (long)h * g.W2 + kbq) * 4) : 0x7ffffff0;
  const int astep = (int)(V2_KC * plane1 * 4), bstep = (int)(V2_KC * plane2 * 4);
  auto issue = [&](int kc, int buf) __attribute__((always_inline)) {
    float *pa = smem + buf * V2_BUF, *pb = pa + V2_ABUF;
    v2_dma16(ra, pa + w * 256, aoff == 0x7ffffff0 ? aoff : aoff + kc * astep);
#pragma unroll
    for (int q = 0; q < 4; ++q) v2_dma16(rb, pb + (4 * w + q) * V2_K, boff[q] == 0x7ffffff0 ? boff[q] : boff[q] + kc * bstep);
  };

  f32x4v acc[4][4];
#pragma unroll
  for (int gg = 0; gg < 4; ++gg)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[gg][t] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int nchunks = g.C / V2_KC;
  const int ar = (lane >> 4) * V2_J + 16 * w + (lane & 15);   // A[c = lane/16][16 w + lane%16]
  const int br = (lane >> 4) * V2_K + 4 * (lane & 15);         // B[c = lane/16][4 n .. 4 n + 3]
  const bool active = j0 + 16 * w < g.W1;                       // wave-uniform: rows left to compute
  // (round 6 built split-f16 products for this loop: the B panel split in place in LDS once per block,
  // the A value per lane, v_mfma_f32_16x16x16_f16 with hi / lo pairs; measured 1.09x SLOWER at cfg2,
  // 226 vs 208 us row layout, 243 vs 224 us sheared, and 1.25x at the booster batch: the in-place
  // split pass, its extra barrier per chunk and the B-operand register copies cost more than the
  // halved MFMA time.  Removed)
  issue(0, 0);
#pragma unroll 1
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = kc & 1;
    __syncthreads();   // chunk kc landed (vmcnt(0) precedes the barrier); buffer cur ^ 1 is free
    if (kc + 1 < nchunks) issue(kc + 1, cur ^ 1);
    if (!active) continue;
    const float *pa = smem + cur * V2_BUF + ar, *pb = smem + cur * V2_BUF + V2_ABUF + br;
#pragma unroll
    for (int s = 0; s < V2_KC / 4; ++s) {
      const float a = pa[s * 4 * V2_J];
      f32x4v bv[4];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) bv[gg] = *reinterpret_cast<const f32x4v *>(pb + s * 4 * V2_K + 64 * gg);
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        if (gg < ngroups) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[gg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[gg][t], acc[gg][t], 0, 0, 0);
        }
    }
  }

  // ---------------------------------------------------------------- epilogue
  const int n = lane & 15;
  auto cell = [&](int gg, int i, int t, int j, int P, float dji, float mji) __attribute__((always_inline)) {
    float x = POW2 ? acc[gg][t][i] * inv_c : acc[gg][t][i] / sqrt_c;
    if (TRUNC) {
      const float center = (float)j - dji;
      const float tv = center - (float)(P + t);
      const float s = sa::sigmoidf_fast(tv);
      const float T = 1.0f * (1.0f - mji) + mji * (s * (1.0f - atten) + atten);
      x = T * x;
    }
    return x;
  };
  float dj[4], mj[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = j0 + 16 * w + 4 * (lane >> 4) + i;
    dj[i] = mj[i] = 0.f;
    if (TRUNC && j < g.W1) {
      const long pix = ((long)b * g.H + h) * g.W1 + j;
      dj[i] = tdisp[pix];
      mj[i] = tconf[pix];
    }
  }
  if constexpr (SHEAR) {
    // two rounds of 32 pixels (waves 2r, 2r + 1 hold pixels 32r .. 32r + 31) through the (now
    // free) panel buffers: the round's level-0 cells staged and written as whole-line sheared rows
    // (sh_write_round), then its level 1..3 cells formed from the staged ones (the row path's
    // averaging order) into the same space and written the same way
    constexpr int P0 = 257, P1 = 129, P2 = 65, P3 = 33;   // LDS pitches (odd)
    constexpr int O2 = 32 * P1, O3 = O2 + 32 * P2;
    static_assert(32 * P0 <= 2 * V2_BUF && O3 + 32 * P3 <= 32 * P0, "round tiles fit the panel buffers");
    float *T = smem;
    float *sl = so.base + ((long)b * g.H + h) * so.slice;
    const int tid = threadIdx.x, pj = tid & 31, pc = tid >> 5;   // level pass: pixel pj, cells 32 pc ..
    // the cells in place (the truncation's per-pixel inputs die here)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[gg][t][i] = cell(gg, i, t, j0 + 16 * w + 4 * (lane >> 4) + i, k0 + 64 * gg + 4 * n, dj[i], mj[i]);
#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
      const int jr0 = j0 + 32 * r;
      if (jr0 >= g.W1) break;   // block-uniform
      __syncthreads();   // the panels / the previous round's tiles are free
      if ((w >> 1) == r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jl = 16 * (w & 1) + 4 * (lane >> 4) + i;
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            if (gg >= ngroups) break;
#pragma unroll
            for (int t = 0; t < 4; ++t)
              T[jl * P0 + 64 * gg + 4 * n + t] = acc[gg][t][i];
          }
        }
      }
      __syncthreads();
      sh_write_round(so, sl, T, P0, 0, g.wid[0], k0, min(kend, g.wid[0]), g.W1, jr0, w, 4, lane);
      if (g.nlev < 2) continue;
      float c1[16], c2[8], c3[4];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float *t0 = T + pj * P0 + 32 * pc + 2 * u;
        c1[u] = (t0[0] + t0[1]) * 0.5f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) c2[u] = (c1[2 * u] + c1[2 * u + 1]) * 0.5f;
#pragma unroll
      for (int u = 0; u < 4; ++u) c3[u] = (c2[2 * u] + c2[2 * u + 1]) * 0.5f;
      __syncthreads();   // level-0 rows read
#pragma unroll
      for (int u = 0; u < 16; ++u) T[pj * P1 + 16 * pc + u] = c1[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) T[O2 + pj * P2 + 8 * pc + u] = c2[u];
#pragma unroll
      for (int u = 0; u < 4; ++u) T[O3 + pj * P3 + 4 * pc + u] = c3[u];
      __syncthreads();
#pragma unroll 1
      for (int l = 1; l < g.nlev; ++l) {
        const int pl = l == 1 ? P1 : l == 2 ? P2 : P3, ol = l == 1 ? 0 : l == 2 ? O2 : O3;
        sh_write_round(so, sl, T + ol, pl, l, g.wid[l], k0 >> l, min(kend >> l, g.wid[l]), g.W1, jr0, w, 4, lane);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = j0 + 16 * w + 4 * (lane >> 4) + i;
    const bool jok = j < g.W1;
    float *row_ptr = pyr + (((long)b * g.H + h) * g.W1 + j) * g.rs;
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int P = k0 + 64 * gg + 4 * n;
      float v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = cell(gg, i, t, j, P, dj[i], mj[i]);
      if (P >= kend) continue;   // (kend - k0 is a multiple of 8 unless kend == W2)
      if (jok) {
        if (P + 3 < kend) {
          *reinterpret_cast<f32x4v *>(row_ptr + P) = f32x4v{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (P + t < kend) row_ptr[P + t] = v[t];
        }
      }
      if (g.nlev > 1) {
        const float l1a = (v[0] + v[1]) * 0.5f, l1b = (v[2] + v[3]) * 0.5f;
        const int k1 = P >> 1;
        if (jok && k1 < g.wid[1]) row_ptr[g.off[1] + k1] = l1a;
        if (jok && k1 + 1 < g.wid[1]) row_ptr[g.off[1] + k1 + 1] = l1b;
        if (g.nlev > 2) {
          const float l2 = (l1a + l1b) * 0.5f;
          const int k2 = P >> 2;
          if (jok && k2 < g.wid[2]) row_ptr[g.off[2] + k2] = l2;
          if (g.nlev > 3) {
            const float l3 = (l2 + __shfl_xor(l2, 1)) * 0.5f;
            const int k3 = P >> 3;
            if (jok && (n & 1) == 0 && k3 < g.wid[3]) row_ptr[g.off[3] + k3] = l3;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // one (row, group) at a time: bounds the registers
    }
  }
}

// Pyramid from an existing volume (mono path, stereoanywhere.py:257-259): one wave per
// row; each lane takes 8 consecutive level-0 values and emits the 4+2+1 coarser cells.
__global__ __launch_bounds__(256) void pyramid_from_volume_kernel(const float *__restrict__ vol,
                                                                  long rows, int W2, long in_rs,
                                                                  Geo g, float *__restrict__ pyr) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const float *src = vol + row * in_rs;
  float *dst = pyr + row * g.rs;
  // 8 consecutive level-0 values per lane-iteration -> one level-3 value
  for (int base = lane * 8; base < W2; base += 64 * 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (base + i < W2) ? src[base + i] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (base + i < W2) dst[base + i] = v[i];
    float l1[4], l2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      l1[i] = (v[2 * i] + v[2 * i + 1]) * 0.5f;
      const int k1 = base / 2 + i;
      if (g.nlev > 1 && k1 < g.wid[1]) dst[g.off[1] + k1] = l1[i];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      l2[i] = (l1[2 * i] + l1[2 * i + 1]) * 0.5f;
      const int k2 = base / 4 + i;
      if (g.nlev > 2 && k2 < g.wid[2]) dst[g.off[2] + k2] = l2[i];
    }
    const float l3 = (l2[0] + l2[1]) * 0.5f;
    const int k3 = base / 8;
    if (g.nlev > 3 && k3 < g.wid[3]) dst[g.off[3] + k3] = l3;
  }
}

// The same pyramid from a volume stored with W1 contiguous and W2 strided (the hourglass's
// [B, ., W2, H, W1] layout, a5 -> a8 with use_aggregate_mono_vol), without materialising the
// [B, H, W1, W2] permute: a block stages 64 pixels x a 256-wide W2 chunk of one (b, h) in LDS
// with loads coalesced along W1, then writes each pixel's pyramid row segment from LDS.  Any
// W2 is handled chunk by chunk: a chunk starts at a multiple of 8, so every level-1/2/3 cell
// (a pair / quad / octet of level-0 cells) lies inside one chunk.
constexpr int PT_J = 64, PT_CHUNK = 256, PT_PITCH = PT_CHUNK + 4;   // 16-byte aligned rows

__global__ __launch_bounds__(256) void pyramid_from_strided_kernel(const float *__restrict__ vol, long sb, long sh,
                                                                   long sk, int H, int W1, int W2, Geo g,
                                                                   float *__restrict__ pyr) {
  __shared__ __attribute__((aligned(16))) float tile[PT_J * PT_PITCH];
  const int j0 = blockIdx.x * PT_J, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float *src = vol + b * sb + h * sh + j0;
  // loads: thread t takes 4 consecutive pixels j = 4 (t % 16) .. + 3 of cell k = 16 i + t / 16
  // (one float4; W1 % 4 == 0, so a group is wholly inside or outside), 16 cells per pass, all
  // of a chunk's loads in flight before the transposing LDS writes.  LDS rows are XOR-swizzled
  // by 4-cell groups (swz) so the writes of 16 pixels of one cell spread over the banks.
  const int tq = threadIdx.x & 15, tk = threadIdx.x >> 4;
  const int jq = 4 * tq;
  const bool qok = j0 + jq < W1;
  auto swz = [](int j) { return ((j >> 2) & 7) << 2; };
  for (int c0 = 0; c0 < W2; c0 += PT_CHUNK) {
    const int cw = min(PT_CHUNK, W2 - c0);
    if (c0 > 0) __syncthreads();  // the previous chunk's rows have been read
    float4 q[PT_CHUNK / 16];
#pragma unroll
    for (int i = 0; i < PT_CHUNK / 16; ++i) {
      const int k = 16 * i + tk;
      q[i] = (qok && k < cw) ? *reinterpret_cast<const float4 *>(src + (long)(c0 + k) * sk + jq)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PT_CHUNK / 16; ++i) {
      const int k = 16 * i + tk;
      tile[(jq + 0) * PT_PITCH + (k ^ swz(jq + 0))] = q[i].x;
      tile[(jq + 1) * PT_PITCH + (k ^ swz(jq + 1))] = q[i].y;
      tile[(jq + 2) * PT_PITCH + (k ^ swz(jq + 2))] = q[i].z;
      tile[(jq + 3) * PT_PITCH + (k ^ swz(jq + 3))] = q[i].w;
    }
    __syncthreads();
    // a lane per 4 consecutive cells: level 0 as one float4, levels 1-2 in registers, level 3
    // from the neighbour lane
    const int lb = 4 * lane, base = c0 + lb;
    for (int jj = wv; jj < PT_J; jj += 4) {
      const int j = j0 + jj;
      if (j >= W1) break;
      float *dst = pyr + (((long)b * H + h) * W1 + j) * g.rs;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (lb < cw) {
        const float4 q = *reinterpret_cast<const float4 *>(tile + jj * PT_PITCH + (lb ^ swz(jj)));
        v[0] = q.x;
        v[1] = base + 1 < W2 ? q.y : 0.f;
        v[2] = base + 2 < W2 ? q.z : 0.f;
        v[3] = base + 3 < W2 ? q.w : 0.f;
        if (base + 3 < W2) {
          *reinterpret_cast<float4 *>(dst + base) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (base + i < W2) dst[base + i] = v[i];
        }
      }
      const float l1a = (v[0] + v[1]) * 0.5f, l1b = (v[2] + v[3]) * 0.5f;
      const float l2 = (l1a + l1b) * 0.5f;
      const float l3 = (l2 + __shfl_xor(l2, 1)) * 0.5f;
      if (lb < cw) {
        const int k1 = base / 2;
        if (g.nlev > 1 && k1 < g.wid[1]) dst[g.off[1] + k1] = l1a;
        if (g.nlev > 1 && k1 + 1 < g.wid[1]) dst[g.off[1] + k1 + 1] = l1b;
        if (g.nlev > 2 && base / 4 < g.wid[2]) dst[g.off[2] + base / 4] = l2;
        if (g.nlev > 3 && (lane & 1) == 0 && base / 8 < g.wid[3]) dst[g.off[3] + base / 8] = l3;
      }
    }
  }
}

// The same pyramid written in the disparity-sheared layout (ShOut): a block stages 32 pixels x a
// 256-cell W2 chunk of one (b, h) in LDS (loads coalesced along W1), writes the chunk's level-0
// cells as whole-line sheared rows (sh_write_round), forms its level 1..3 cells from the staged
// ones (the row path's averaging order) into the same LDS space and writes those rows.  Any W2,
// chunk by chunk (a chunk starts at a multiple of 8: every coarser cell lies inside one).
constexpr int PS_J = 32, PS_CHUNK = 256;
__global__ __launch_bounds__(256) void pyramid_from_strided_sheared_kernel(const float *__restrict__ vol, long sb,
                                                                           long sh, long sk, int H, int W1, int W2,
                                                                           Geo g, ShOut so) {
  constexpr int P0 = 257, P1 = 129, P2 = 65, P3 = 33;   // LDS pitches (odd: conflict-free row reads)
  constexpr int O2 = 32 * P1, O3 = O2 + 32 * P2;
  static_assert(O3 + 32 * P3 <= 32 * P0, "the level tiles reuse the level-0 tile");
  __shared__ float T[32 * P0];
  const int jr0 = blockIdx.x * PS_J, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float *src = vol + b * sb + h * sh + jr0;
  float *sl = so.base + ((long)b * H + h) * so.slice;
  // loads: thread t takes pixels 4 (t % 8) .. + 3 of cells 32 i + t / 8 (W1 % 4 == 0: a quad is
  // wholly inside or outside)
  const int tq = tid & 7, tk = tid >> 3, jq = 4 * tq;
  const bool qok = jr0 + jq < W1;
  // level pass: thread t forms pixel t % 32's coarser cells from level-0 cells 32 (t / 32) .. + 31
  const int pj = tid & 31, pc = tid >> 5;
  for (int c0 = 0; c0 < W2; c0 += PS_CHUNK) {
    const int cw = min(PS_CHUNK, W2 - c0);
    if (c0 > 0) __syncthreads();   // the previous chunk's rows are written
    float4 q[PS_CHUNK / 32];
#pragma unroll
    for (int i = 0; i < PS_CHUNK / 32; ++i) {
      const int k = 32 * i + tk;
      q[i] = (qok && k < cw) ? *reinterpret_cast<const float4 *>(src + (long)(c0 + k) * sk + jq)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PS_CHUNK / 32; ++i) {
      const int k = 32 * i + tk;
      T[(jq + 0) * P0 + k] = q[i].x;
      T[(jq + 1) * P0 + k] = q[i].y;
      T[(jq + 2) * P0 + k] = q[i].z;
      T[(jq + 3) * P0 + k] = q[i].w;
    }
    __syncthreads();
    sh_write_round(so, sl, T, P0, 0, g.wid[0], c0, min(c0 + cw, g.wid[0]), W1, jr0, wv, 4, lane);
    if (g.nlev < 2) continue;
    float c1[16], c2[8], c3[4];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float *t0 = T + pj * P0 + 32 * pc + 2 * u;
      c1[u] = (t0[0] + t0[1]) * 0.5f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) c2[u] = (c1[2 * u] + c1[2 * u + 1]) * 0.5f;
#pragma unroll
    for (int u = 0; u < 4; ++u) c3[u] = (c2[2 * u] + c2[2 * u + 1]) * 0.5f;
    __syncthreads();   // level-0 rows read
#pragma unroll
    for (int u = 0; u < 16; ++u) T[pj * P1 + 16 * pc + u] = c1[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) T[O2 + pj * P2 + 8 * pc + u] = c2[u];
#pragma unroll
    for (int u = 0; u < 4; ++u) T[O3 + pj * P3 + 4 * pc + u] = c3[u];
    __syncthreads();
    for (int l = 1; l < g.nlev; ++l) {
      const int pl = l == 1 ? P1 : l == 2 ? P2 : P3, ol = l == 1 ? 0 : l == 2 ? O2 : O3;
      sh_write_round(so, sl, T + ol, pl, l, g.wid[l], c0 >> l, min((c0 + cw) >> l, g.wid[l]), W1, jr0, wv, 4, lane);
    }
  }
}

Geo make_geo(int C, int H, int W1, int W2, int nlev, long rs) {
  Geo g{};
  g.C = C;
  g.H = H;
  g.W1 = W1;
  g.W2 = W2;
  g.tilesJ = (W1 + TJ - 1) / TJ;
  g.tilesK = (W2 + TK - 1) / TK;
  g.nlev = nlev;
  g.rs = rs;
  for (int i = 0; i < 4; ++i) {
    g.off[i] = sa_pyramid_level_offset(W2, i);
    g.wid[i] = sa_pyramid_level_width(W2, i);
  }
  return g;
}

}  // namespace

namespace {
ShOut make_shout(float *sheared, int W1, int W2, int nlev);

// sheared == nullptr: the row layout into pyramid / row_stride; else the sheared layout into
// sheared (the v2 kernel's preconditions required)
int corr_volume_pyramid_impl(const float *fmap2, const float *fmap3, int B, int C, int H, int W1, int W2,
                             float sqrt_c, const float *trunc_disp, const float *trunc_conf, float atten,
                             int num_levels, float *pyramid, long row_stride, float *sheared, void *stream) {
  if (sheared) {
    pyramid = sheared;   // (only for the checks below; the kernel writes through ShOut)
    row_stride = sa_pyramid_level_offset(W2, num_levels);
    row_stride = (row_stride + 3) / 4 * 4;
  }
  SA_REQUIRE(fmap2 && fmap3 && pyramid, "sa_corr_volume_pyramid: null pointer");
  SA_REQUIRE(B > 0 && C > 0 && H > 0 && W1 > 0 && W2 > 0, "sa_corr_volume_pyramid: empty shape");
  SA_REQUIRE(num_levels >= 1 && num_levels <= 4, "sa_corr_volume_pyramid: num_levels must be 1..4");
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels),
             "sa_corr_volume_pyramid: row_stride %ld too small", row_stride);
  SA_REQUIRE((trunc_disp == nullptr) == (trunc_conf == nullptr),
             "sa_corr_volume_pyramid: trunc_disp and trunc_conf go together");
  SA_REQUIRE((long)B * H * ((W1 + TJ - 1) / TJ) * ((W2 + TK - 1) / TK) < (1L << 31),
             "sa_corr_volume_pyramid: grid too large");
  Geo g = make_geo(C, H, W1, W2, num_levels, row_stride);
  const bool vec = (W1 % 4 == 0) && (W2 % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(fmap2) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(fmap3) % 16 == 0);
  hipStream_t s = sa::as_stream(stream);
  const long f2_bytes = (long)B * C * H * W1 * 4, f3_bytes = (long)B * C * H * W2 * 4;
  if (vec && C % V2_KC == 0 && row_stride % 4 == 0 && reinterpret_cast<uintptr_t>(pyramid) % 16 == 0 &&
      f2_bytes < (1L << 31) - 64 && f3_bytes < (1L << 31) - 64) {
    const int jblocks = (W1 + V2_J - 1) / V2_J, kblocks = (W2 + V2_K - 1) / V2_K;
    const int kstep = ((W2 + kblocks - 1) / kblocks + 63) / 64 * 64;   // <= V2_K
    const long nb = (long)B * H * jblocks * kblocks;
    SA_REQUIRE(nb < (1L << 31), "sa_corr_volume_pyramid: grid too large");
    int ex = 0;
    const float mant = frexpf(sqrt_c, &ex);
    const bool pow2 = mant == 0.5f;
    const float inv = pow2 ? 1.0f / sqrt_c : 0.0f;
    sa::TimingScope ts(SA_K_CORR_PYRAMID, s);
    const bool tr = trunc_disp != nullptr;
    const unsigned nbu = (unsigned)nb;
    const int a2 = (int)f2_bytes, a3 = (int)f3_bytes;
    const ShOut so = sheared ? make_shout(sheared, W1, W2, num_levels) : ShOut{};
#define SA_V2(TR_, P2_, SH_)                                                                                        \
  corr_pyramid_v2_kernel<TR_, P2_, SH_><<<nbu, 256, 0, s>>>(fmap2, fmap3, g, jblocks, kblocks, kstep, sqrt_c, inv, \
                                                            TR_ ? trunc_disp : nullptr, TR_ ? trunc_conf : nullptr, \
                                                            atten, pyramid, a2, a3, so)
    if (sheared) {
      if (tr && pow2) SA_V2(true, true, true);
      else if (tr) SA_V2(true, false, true);
      else if (pow2) SA_V2(false, true, true);
      else SA_V2(false, false, true);
    } else {
      if (tr && pow2) SA_V2(true, true, false);
      else if (tr) SA_V2(true, false, false);
      else if (pow2) SA_V2(false, true, false);
      else SA_V2(false, false, false);
    }
#undef SA_V2
    return sa::check_launch("sa_corr_volume_pyramid");
  }
  SA_REQUIRE(!sheared, "sa_corr_volume_pyramid_sheared: needs C %% 16 == 0, W1 and W2 %% 4 == 0, 16-byte aligned "
                       "feature maps under 2 GiB");
  const unsigned nblk = (unsigned)((long)B * H * g.tilesJ * g.tilesK);
  sa::TimingScope ts(SA_K_CORR_PYRAMID, s);
  const bool tr = trunc_disp != nullptr;
  if (vec && tr)
    corr_pyramid_kernel<true, true><<<nblk, 256, 0, s>>>(fmap2, fmap3, g, sqrt_c, trunc_disp, trunc_conf, atten, pyramid);
  else if (vec)
    corr_pyramid_kernel<true, false><<<nblk, 256, 0, s>>>(fmap2, fmap3, g, sqrt_c, nullptr, nullptr, atten, pyramid);
  else if (tr)
    corr_pyramid_kernel<false, true><<<nblk, 256, 0, s>>>(fmap2, fmap3, g, sqrt_c, trunc_disp, trunc_conf, atten, pyramid);
  else
    corr_pyramid_kernel<false, false><<<nblk, 256, 0, s>>>(fmap2, fmap3, g, sqrt_c, nullptr, nullptr, atten, pyramid);
  return sa::check_launch("sa_corr_volume_pyramid");
}
}  // namespace

extern "C" int sa_corr_volume_pyramid(const float *fmap2, const float *fmap3, int B, int C, int H,
                                      int W1, int W2, float sqrt_c, const float *trunc_disp,
                                      const float *trunc_conf, float atten, int num_levels,
                                      float *pyramid, long row_stride, void *stream) {
  return corr_volume_pyramid_impl(fmap2, fmap3, B, C, H, W1, W2, sqrt_c, trunc_disp, trunc_conf, atten, num_levels,
                                  pyramid, row_stride, nullptr, stream);
}

extern "C" int sa_corr_volume_pyramid_sheared(const float *fmap2, const float *fmap3, int B, int C, int H, int W1,
                                              int W2, float sqrt_c, const float *trunc_disp, const float *trunc_conf,
                                              float atten, int num_levels, float *sheared, void *stream) {
  SA_REQUIRE(sheared, "sa_corr_volume_pyramid_sheared: null pointer");
  return corr_volume_pyramid_impl(fmap2, fmap3, B, C, H, W1, W2, sqrt_c, trunc_disp, trunc_conf, atten, num_levels,
                                  nullptr, 0, sheared, stream);
}

extern "C" int sa_corr_pyramid_from_volume(const float *volume, long rows, int W2, long in_row_stride,
                                           int num_levels, float *pyramid, long row_stride,
                                           void *stream) {
  SA_REQUIRE(volume && pyramid, "sa_corr_pyramid_from_volume: null pointer");
  SA_REQUIRE(rows > 0 && W2 > 0 && in_row_stride >= W2, "sa_corr_pyramid_from_volume: bad shape");
  SA_REQUIRE(num_levels >= 1 && num_levels <= 4, "sa_corr_pyramid_from_volume: num_levels must be 1..4");
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels),
             "sa_corr_pyramid_from_volume: row_stride too small");
  Geo g = make_geo(1, 1, 1, W2, num_levels, row_stride);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MONO_PYRAMID, s);
  pyramid_from_volume_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(volume, rows, W2, in_row_stride, g, pyramid);
  return sa::check_launch("sa_corr_pyramid_from_volume");
}

extern "C" int sa_corr_pyramid_from_volume_strided(const float *volume, int B, int H, int W1, int W2, long sb, long sh,
                                                   long sk, int num_levels, float *pyramid, long row_stride,
                                                   void *stream) {
  SA_REQUIRE(volume && pyramid, "sa_corr_pyramid_from_volume_strided: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && H > 0 && H <= 65535 && W1 > 0 && W2 > 0,
             "sa_corr_pyramid_from_volume_strided: bad shape");
  SA_REQUIRE(num_levels >= 1 && num_levels <= 4, "sa_corr_pyramid_from_volume_strided: num_levels must be 1..4");
  SA_REQUIRE(row_stride >= sa_pyramid_level_offset(W2, num_levels),
             "sa_corr_pyramid_from_volume_strided: row_stride too small");
  SA_REQUIRE(row_stride % 4 == 0 && reinterpret_cast<uintptr_t>(pyramid) % 16 == 0,
             "sa_corr_pyramid_from_volume_strided: pyramid rows must be 16-byte aligned");
  SA_REQUIRE(W1 % 4 == 0 && sb % 4 == 0 && sh % 4 == 0 && sk % 4 == 0 && reinterpret_cast<uintptr_t>(volume) % 16 == 0,
             "sa_corr_pyramid_from_volume_strided: needs W1 %% 4 == 0 and 16-byte aligned volume rows");
  Geo g = make_geo(1, 1, 1, W2, num_levels, row_stride);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MONO_PYRAMID, s);
  pyramid_from_strided_kernel<<<dim3((unsigned)((W1 + PT_J - 1) / PT_J), (unsigned)H, (unsigned)B), 256, 0, s>>>(
      volume, sb, sh, sk, H, W1, W2, g, pyramid);
  return sa::check_launch("sa_corr_pyramid_from_volume_strided");
}

namespace {
ShOut make_shout(float *sheared, int W1, int W2, int nlev) {
  ShOut so{};
  so.base = sheared;
  so.slice = sa_shear_slice_size(W1, W2, nlev);
  so.pitch = (int)sa_shear_row_pitch(W1);
  for (int l = 0; l < 4; ++l) {
    so.off[l] = l < nlev ? sa_shear_level_offset(W1, W2, nlev, l) : 0;
    so.rows[l] = l < nlev ? sa_pyramid_level_width(W2, l) + ((W1 - 1) >> l) : 0;
  }
  return so;
}
}  // namespace

extern "C" int sa_corr_pyramid_from_volume_strided_sheared(const float *volume, int B, int H, int W1, int W2, long sb,
                                                           long sh, long sk, int num_levels, float *sheared,
                                                           void *stream) {
  SA_REQUIRE(volume && sheared, "sa_corr_pyramid_from_volume_strided_sheared: null pointer");
  SA_REQUIRE(B > 0 && B <= 65535 && H > 0 && H <= 65535 && W1 > 0 && W2 > 0,
             "sa_corr_pyramid_from_volume_strided_sheared: bad shape");
  SA_REQUIRE(num_levels >= 1 && num_levels <= 4,
             "sa_corr_pyramid_from_volume_strided_sheared: num_levels must be 1..4");
  SA_REQUIRE(W1 % 4 == 0 && sb % 4 == 0 && sh % 4 == 0 && sk % 4 == 0 && reinterpret_cast<uintptr_t>(volume) % 16 == 0,
             "sa_corr_pyramid_from_volume_strided_sheared: needs W1 %% 4 == 0 and 16-byte aligned volume rows");
  Geo g = make_geo(1, 1, 1, W2, num_levels, 0);
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MONO_PYRAMID, s);
  pyramid_from_strided_sheared_kernel<<<dim3((unsigned)((W1 + PS_J - 1) / PS_J), (unsigned)H, (unsigned)B), 256, 0,
                                        s>>>(volume, sb, sh, sk, H, W1, W2, g, make_shout(sheared, W1, W2, num_levels));
  return sa::check_launch("sa_corr_pyramid_from_volume_strided_sheared");
}
