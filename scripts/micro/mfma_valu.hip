// Microbenchmark of the fp32 MFMA issue model on one SIMD (cycles from s_memtime-style clock64
// per wave).  Each wave runs ITER x (16 independent MFMAs + NV VALU FMAs); variants:
//   kind 0: 16x16x4 f32, VALU on independent registers
//   kind 1: 32x32x2 f32 (8 per iteration: same flops), VALU independent
//   kind 2: 16x16x4 f32, the MFMA A operand produced by the VALU op just before it
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int NV, int KIND>
__global__ void k(float *out, long long *cyc, int iters, float a0) {
  f32x4 acc[16];
  f32x16 acc32[8];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) acc32[i] = f32x16{0};
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = a0 + threadIdx.x * 0.001f + i;
  float a = a0 + threadIdx.x, b = a0 * 0.5f;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (KIND == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc32[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc32[i], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NV / 8; ++j) v[j & 7] = fmaf(v[j & 7], 1.0001f, 0.5f);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
#pragma unroll
        for (int j = 0; j < NV / 16; ++j) v[(i + j) & 7] = fmaf(v[(i + j) & 7], 1.0001f, 0.5f);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(KIND == 2 ? v[i & 7] : a, b, acc[i], 0, 0, 0);
      }
    }
    a += 1.0f;
  }
  const long long t1 = clock64();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += acc32[i][0] + acc32[i][5];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int NV, int KIND>
void run(int threads) {
  float *out;
  long long *cyc;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  hipMalloc(&cyc, 256 * 16 * sizeof(long long));
  const int iters = 2000;
  k<NV, KIND><<<256, threads>>>(out, cyc, 10, 1.0f);
  k<NV, KIND><<<256, threads>>>(out, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  long long h[256 * 16];
  hipMemcpy(h, cyc, sizeof(long long) * 256 * (threads / 64), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256 * (threads / 64); ++i) m += h[i];
  m /= 256 * (threads / 64);
  const int wps = threads / 256;
  printf("kind %d waves/SIMD %d NV %3d: %.1f cycles per iteration per SIMD (MFMA floor %d)\n", KIND, wps, NV,
         m / iters, 16 * 32 * wps);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int t : {256, 512}) {
    run<0, 0>(t);
    run<16, 0>(t);
    run<32, 0>(t);
    run<64, 0>(t);
    run<0, 1>(t);
    run<16, 1>(t);
    run<32, 1>(t);
    run<64, 1>(t);
    run<16, 2>(t);
    run<32, 2>(t);
  }
  return 0;
}
