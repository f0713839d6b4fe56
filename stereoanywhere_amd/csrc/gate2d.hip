// The DoubleFeatureAtt gates of the fused hourglass (submodule.py:113-140, used at
// hourglass.py:66-91): per branch g = sigmoid(conv1x1(leaky(IN(conv3x3(feat))))) with a
// one-channel feature plane, 32 hidden channels (BasicConv: conv without bias, InstanceNorm2d
// without affine, LeakyReLU 0.01) and C outputs (bias).  Until round 6 these ran as torch/MIOpen
// launches on the mono side stream (8 Winograd 3x3 convs, their InstanceNorm as batch_norm
// statistics + transform, 6 GEMMs, 8 sigmoids: ~0.43 ms at cfg2, ~2.3 ms per cfg5 image).
// Every branch of a forward goes out in two launches:
//   feature_gate_stats — a block per 1024-pixel tile of a (job, image) plane forms the tile's 32
//     hidden values per pixel and writes per-channel partial sums (shifted by the value at the
//     plane's centre, so the variance does not cancel) as fp64 to its own slot (no atomics: the
//     next launch sums them in a fixed order, so every run gives the same bits);
//   feature_gate_apply — each block sums its plane's partials in tile order, forms mean and
//     1 / sqrt(var + 1e-5) (biased variance, as InstanceNorm), recomputes the hidden values,
//     normalises, LeakyReLU, the 1x1 conv with bias and the sigmoid, and writes the C planes.
#include "sa_common.h"

namespace {

constexpr int GT_HID = 32, GT_TPB = 256, GT_PPT = 4, GT_TILE = GT_TPB * GT_PPT, GT_MAXC = 64;

struct GateLaunch {
  SaFeatureGateJob j[SA_GATE_MAX_JOBS];
  double *part[SA_GATE_MAX_JOBS];    // job i's per-(image, tile) partial sums in the workspace
  int first[SA_GATE_MAX_JOBS + 1];   // first block of job i (blocks: B x tiles per job)
  int njobs;
};

__device__ __forceinline__ int gt_job(const GateLaunch &L, int blk) {
  int i = 0;
#pragma unroll
  for (int k = 1; k < SA_GATE_MAX_JOBS; ++k) i += (k < L.njobs && blk >= L.first[k]) ? 1 : 0;
  return i;
}

// the 3x3 neighbourhood of pixel (y, x) with zero padding
__device__ __forceinline__ void gt_patch(const float *__restrict__ p, int H, int W, int y, int x, float (&nb)[9]) {
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = y + dy, xx = x + dx;
      const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
      const float v = p[min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1)];   // (clamped, then selected)
      nb[(dy + 1) * 3 + dx + 1] = in ? v : 0.0f;
    }
}

// hidden channel k at a pixel: conv3x3 (no bias) in the reference's tap order
__device__ __forceinline__ float gt_hidden(const float *w3, int k, const float (&nb)[9]) {
  float v = 0.0f;
#pragma unroll
  for (int q = 0; q < 9; ++q) v = fmaf(w3[k * 9 + q], nb[q], v);
  return v;
}

__global__ __launch_bounds__(GT_TPB) void feature_gate_stats_kernel(const GateLaunch L) {
  const int blk = blockIdx.x, ji = gt_job(L, blk);
  const SaFeatureGateJob &J = L.j[ji];
  const int tiles = (J.H * J.W + GT_TILE - 1) / GT_TILE;
  const int r = blk - L.first[ji], b = r / tiles, tile = r - b * tiles;
  __shared__ float w3[GT_HID * 9], shift[GT_HID];
  __shared__ double part[GT_TPB / 64][2 * GT_HID];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float *p = J.in + (long)b * J.in_bs;
  for (int i = t; i < GT_HID * 9; i += GT_TPB) w3[i] = J.w3[i];
  __syncthreads();
  if (t < GT_HID) {   // the shift: hidden value at the plane's centre (the same in every block)
    float nb[9];
    gt_patch(p, J.H, J.W, J.H / 2, J.W / 2, nb);
    shift[t] = gt_hidden(w3, t, nb);
  }
  __syncthreads();
  float s1[GT_HID], s2[GT_HID];
#pragma unroll
  for (int k = 0; k < GT_HID; ++k) s1[k] = s2[k] = 0.0f;
  const int npx = J.H * J.W;
#pragma unroll
  for (int e = 0; e < GT_PPT; ++e) {
    const int px = tile * GT_TILE + e * GT_TPB + t;
    if (px >= npx) continue;
    float nb[9];
    gt_patch(p, J.H, J.W, px / J.W, px % J.W, nb);
#pragma unroll
    for (int k = 0; k < GT_HID; ++k) {
      const float d = gt_hidden(w3, k, nb) - shift[k];
      s1[k] += d;
      s2[k] = fmaf(d, d, s2[k]);
    }
  }
  // per channel: the wave's sum (fp32, 64 lanes x <= 4 pixels), then the block's in fp64
#pragma unroll
  for (int k = 0; k < GT_HID; ++k) {
    const float a = sa::wave_sum_dpp(s1[k]), c = sa::wave_sum_dpp(s2[k]);
    if (lane == 0) {
      part[wv][k] = (double)a;
      part[wv][GT_HID + k] = (double)c;
    }
  }
  __syncthreads();
  if (t < 2 * GT_HID) {
    double s = part[0][t];
#pragma unroll
    for (int w = 1; w < GT_TPB / 64; ++w) s += part[w][t];
    L.part[ji][((long)b * tiles + tile) * (2 * GT_HID) + t] = s;
  }
}

__global__ __launch_bounds__(GT_TPB) void feature_gate_apply_kernel(const GateLaunch L) {
  const int blk = blockIdx.x, ji = gt_job(L, blk);
  const SaFeatureGateJob &J = L.j[ji];
  const int tiles = (J.H * J.W + GT_TILE - 1) / GT_TILE;
  const int r = blk - L.first[ji], b = r / tiles, tile = r - b * tiles;
  __shared__ float w3[GT_HID * 9], w1[GT_MAXC * GT_HID], b1[GT_MAXC], mean[GT_HID], rstd[GT_HID];
  __shared__ double tot[2 * GT_HID];
  const int t = threadIdx.x, C = J.C;
  const float *p = J.in + (long)b * J.in_bs;
  for (int i = t; i < GT_HID * 9; i += GT_TPB) w3[i] = J.w3[i];
  for (int i = t; i < C * GT_HID; i += GT_TPB) w1[i] = J.w1[i];
  for (int i = t; i < C; i += GT_TPB) b1[i] = J.b1 ? J.b1[i] : 0.0f;
  if (t < 2 * GT_HID) {   // the plane's sums, tiles in order
    const double *q = L.part[ji] + (long)b * tiles * (2 * GT_HID) + t;
    double s = 0.0;
    for (int i = 0; i < tiles; ++i) s += q[(long)i * (2 * GT_HID)];
    tot[t] = s;
  }
  __syncthreads();
  if (t < GT_HID) {
    float nb[9];
    gt_patch(p, J.H, J.W, J.H / 2, J.W / 2, nb);
    const double n = (double)J.H * J.W, m1 = tot[t] / n;
    const double var = fmax(tot[GT_HID + t] / n - m1 * m1, 0.0);
    mean[t] = (float)((double)gt_hidden(w3, t, nb) + m1);
    rstd[t] = 1.0f / sqrtf((float)var + 1e-5f);
  }
  __syncthreads();
  const int npx = J.H * J.W;
  float *ob = J.out + (long)b * J.out_bs;
  for (int e = 0; e < GT_PPT; ++e) {
    const int px = tile * GT_TILE + e * GT_TPB + t;
    if (px >= npx) continue;
    float nb[9], a[GT_HID];
    gt_patch(p, J.H, J.W, px / J.W, px % J.W, nb);
#pragma unroll
    for (int k = 0; k < GT_HID; ++k) {
      const float y = (gt_hidden(w3, k, nb) - mean[k]) * rstd[k];
      a[k] = y >= 0.0f ? y : y * 0.01f;   // LeakyReLU (negative_slope 0.01)
    }
    for (int c = 0; c < C; ++c) {
      float v = b1[c];
#pragma unroll
      for (int k = 0; k < GT_HID; ++k) v = fmaf(w1[c * GT_HID + k], a[k], v);
      ob[(long)c * npx + px] = sa::sigmoidf_ref(v);
    }
  }
}

bool gt_prepare(int njobs, const SaFeatureGateJob *jobs, GateLaunch &L, long *ws_need) {
  if (njobs < 1 || njobs > SA_GATE_MAX_JOBS || !jobs) return false;
  L.njobs = njobs;
  int blocks = 0;
  long ws = 0;
  for (int i = 0; i < njobs; ++i) {
    const SaFeatureGateJob &J = jobs[i];
    if (J.B < 1 || J.H < 1 || J.W < 1 || J.C < 1 || J.C > GT_MAXC || !J.in || !J.w3 || !J.w1 || !J.out) return false;
    if (J.in_bs < (long)J.H * J.W || J.out_bs < (long)J.C * J.H * J.W) return false;
    const long tiles = ((long)J.H * J.W + GT_TILE - 1) / GT_TILE;
    L.j[i] = J;
    L.first[i] = blocks;
    blocks += (int)(J.B * tiles);
    ws += J.B * tiles * 2 * GT_HID;
  }
  L.first[njobs] = blocks;
  for (int i = njobs + 1; i <= SA_GATE_MAX_JOBS; ++i) L.first[i] = blocks;
  if (ws_need) *ws_need = ws * (long)sizeof(double);
  return true;
}

}  // namespace

extern "C" long sa_feature_gates_ws_size(int njobs, const SaFeatureGateJob *jobs) {
  GateLaunch L;
  long ws = 0;
  return gt_prepare(njobs, jobs, L, &ws) ? ws : -1;
}

extern "C" int sa_feature_gates(int njobs, const SaFeatureGateJob *jobs, void *ws, void *stream) {
  GateLaunch L;
  long need = 0;
  SA_REQUIRE(gt_prepare(njobs, jobs, L, &need), "sa_feature_gates: bad jobs (1..8 jobs, C <= 64, strides)");
  SA_REQUIRE(ws, "sa_feature_gates: null workspace");
  double *w = static_cast<double *>(ws);
  for (int i = 0; i < njobs; ++i) {   // each job's partials in its own range of the workspace
    L.part[i] = w;
    const long tiles = ((long)L.j[i].H * L.j[i].W + GT_TILE - 1) / GT_TILE;
    w += L.j[i].B * tiles * 2 * GT_HID;
  }
  hipStream_t s = sa::as_stream(stream);
  sa::TimingScope ts(SA_K_MISC, s);
  const unsigned blocks = (unsigned)L.first[njobs];
  feature_gate_stats_kernel<<<blocks, GT_TPB, 0, s>>>(L);
  int rc = sa::check_launch("sa_feature_gates (stats)");
  if (rc) return rc;
  feature_gate_apply_kernel<<<blocks, GT_TPB, 0, s>>>(L);
  return sa::check_launch("sa_feature_gates (apply)");
}
