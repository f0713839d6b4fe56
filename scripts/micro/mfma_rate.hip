// Back-to-back MFMA issue rate per SIMD (4 waves per CU, one per SIMD; 4 independent
// accumulators per wave): v_mfma_f32_16x16x4_f32, v_mfma_f32_16x16x16_f16 and
// v_mfma_f32_16x16x32_f16, reported as wall ns per MFMA per SIMD and cycles at the clock
// the s_memtime counter reports.  Build: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int IT = 4096;
template <int K>
__global__ __launch_bounds__(256) void k(float *out, unsigned long long *cyc) {
  f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  const float x = threadIdx.x * 1e-3f;
  const f16x4 h4 = {(_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x};
  const f16x8 h8 = {(_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x, (_Float16)x};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < IT; ++i) {
    if constexpr (K == 0) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a3, 0, 0, 0);
    } else if constexpr (K == 1) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, a3, 0, 0, 0);
    } else {
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, a3, 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const f32x4 s = a0 + a1 + a2 + a3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float *out;
  unsigned long long *cyc;
  const int nb = 1024;
  hipMalloc(&out, nb * 256 * 4);
  hipMalloc(&cyc, nb * 8);
  const char *names[3] = {"16x16x4_f32", "16x16x16_f16", "16x16x32_f16"};
  for (int kk = 0; kk < 3; ++kk) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      if (kk == 0) k<0><<<nb, 256>>>(out, cyc);
      else if (kk == 1) k<1><<<nb, 256>>>(out, cyc);
      else k<2><<<nb, 256>>>(out, cyc);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      // 1024 blocks of 4 waves over 256 CUs x 4 SIMDs: 4 waves per SIMD in sequence (or 1 at a time)
      const double per_simd = (double)nb * 4 / 1024 * IT * 4;
      if (rep) printf("%-14s %.3f ms  %.2f ns per MFMA per SIMD  %.1f memtime cycles per MFMA (one wave)\n", names[kk], ms,
                      ms * 1e6 / per_simd, (double)c / (IT * 4));
    }
  }
  return 0;
}
