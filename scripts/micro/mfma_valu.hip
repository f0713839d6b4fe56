// Microbenchmark: does f32 MFMA (v_mfma_f32_16x16x4_f32) overlap with f32 VALU work on one
// SIMD?  Each wave runs ITER x (16 independent MFMAs + NV independent VALU FMAs); time per
// iteration per SIMD vs NV, at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int NV>
__global__ void k(float *out, int iters, float a0) {
  f32x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0, 0, 0, 0};
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = a0 + threadIdx.x * 0.001f + i;
  float a = a0 + threadIdx.x, b = a0 * 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV / 16; ++j) v[j & 7] = fmaf(v[j & 7], 1.0001f, 0.5f);
    }
    a += 1.0f;
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV>
void run(int threads) {
  float *out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  const int iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<NV><<<256, threads>>>(out, 10, 1.0f);
  hipEventRecord(e0);
  k<NV><<<256, threads>>>(out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int wps = threads / 256;   // waves per SIMD
  // cycles per (16 MFMA + NV VALU) per wave at 2.4 GHz
  printf("threads %3d (waves/SIMD %d) NV %3d: %.3f ms, %.1f cycles per iteration per SIMD (MFMA floor %d)\n", threads,
         wps, NV, ms, ms * 1e-3 * 2.4e9 / iters, 16 * 32 * wps);
  hipFree(out);
}

int main() {
  for (int t : {256, 512}) {
    run<0>(t);
    run<16>(t);
    run<32>(t);
    run<64>(t);
    run<128>(t);
  }
  return 0;
}
