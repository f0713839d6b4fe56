// Box-state probe for bench.py: the shader clock the chip holds under a dense MFMA
// load, read in-kernel (MI355X_MICROARCH.md 'DVFS give-back' item 6: delta s_memtime / delta
// s_memrealtime x 100 MHz), next to sysfs's pp_dpm_sclk which does not show the give-back.  Every
// wave runs chains of v_mfma_f32_16x16x16_f16 on non-trivial operands between the two stamps; lane 0
// stores the two deltas with a vector store.  Not on the hot path.
#include <algorithm>
#include <vector>

#include "sa_common.h"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x4 = __attribute__((ext_vector_type(4))) _Float16;

__global__ __launch_bounds__(256) void clock_probe_kernel(int iters, float *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  // random-looking operands (zeros would let the chip hold a higher clock than real work does)
  const float s = 0.37f + 0.011f * (float)lane + 0.003f * (float)(wave & 31);
  f16x4 a = f16x4{(_Float16)s, (_Float16)(1.0f - s), (_Float16)(0.5f * s), (_Float16)(s - 0.25f)};
  f16x4 b = f16x4{(_Float16)(0.9f - s), (_Float16)(0.3f * s), (_Float16)(s + 0.1f), (_Float16)(0.7f * s)};
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(b, b, c3, 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  const f32x4 t = (c0 + c1) + (c2 + c3);
  if (lane == 0) {
    out[3 * wave] = (float)(t1 - t0);
    out[3 * wave + 1] = (float)(r1 - r0);
    out[3 * wave + 2] = t.x + t.y + t.z + t.w;   // keeps the chains live
  }
}

}  // namespace

extern "C" int sa_clock_probe(int blocks, int iters, double *mhz, double *ms) {
  SA_REQUIRE(blocks > 0 && blocks <= 65536 && iters > 0 && mhz && ms, "sa_clock_probe: bad arguments");
  const int nw = blocks * 4;
  float *d = nullptr;
  if (hipMalloc(&d, sizeof(float) * 3 * nw) != hipSuccess) {
    sa::set_error("sa_clock_probe: hipMalloc failed");
    return SA_E_RUNTIME;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, nullptr);
  clock_probe_kernel<<<blocks, 256, 0, nullptr>>>(iters, d);
  (void)hipEventRecord(e1, nullptr);
  std::vector<float> h(3 * nw);
  const bool ok = hipMemcpy(h.data(), d, sizeof(float) * 3 * nw, hipMemcpyDeviceToHost) == hipSuccess;
  float ev = 0.0f;
  (void)hipEventElapsedTime(&ev, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d);
  if (!ok) {
    sa::set_error("sa_clock_probe: copy failed");
    return SA_E_RUNTIME;
  }
  std::vector<double> f(nw);
  for (int w = 0; w < nw; ++w) f[w] = h[3 * w + 1] > 0.0f ? (double)h[3 * w] / (double)h[3 * w + 1] * 100.0 : 0.0;
  std::nth_element(f.begin(), f.begin() + nw / 2, f.end());
  *mhz = f[nw / 2];
  *ms = ev;
  return sa::check_launch("sa_clock_probe");
}
