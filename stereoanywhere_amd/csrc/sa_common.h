// Shared runtime pieces of libsa_hip.so: error reporting, launch helpers, the
// live per-kernel timing used by bench.py, and small device math helpers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/stereoanywhere_hip.h"

namespace sa {

void set_error(const char *fmt, ...);

// Event-bracketed timing (sa_timing_enable). begin/end are no-ops when disabled.
struct TimingScope {
  int id;
  hipStream_t stream;
  bool on;
  TimingScope(int kernel_id, hipStream_t s);
  ~TimingScope();
};

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SA_E_LAUNCH;
  }
  return SA_OK;
}

#define SA_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      ::sa::set_error(__VA_ARGS__);    \
      return SA_E_ARG;                 \
    }                                  \
  } while (0)

// Bijective XCD-grouping remap of a linear block id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): consecutive work items land on one XCD so
// blocks sharing an operand panel share that XCD's L2.
__device__ __forceinline__ unsigned xcd_remap(unsigned orig, unsigned nwg) {
  const unsigned q = nwg / 8u, r = nwg % 8u, xcd = orig % 8u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
}

// torch.sigmoid / F.sigmoid on CPU: 1 / (1 + exp(-x)).
__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// The same to a few ulp with the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32): for
// epilogues that evaluate one sigmoid per output element (the truncation volume).  Relative
// error <= ~1e-6 for |x| <= 100, <= ~2e-5 up to |x| ~ 700 (the exponent's product rounding),
// where the value is ~0 or ~1 anyway.
__device__ __forceinline__ float sigmoidf_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * 1.44269504088896341f));
}

}  // namespace sa
