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

// row pitch of the disparity-sheared pyramid (corr_shear.hip): W1 rounded up to 32 floats, so a
// 32-pixel row segment starting at a multiple of 32 is one 128-byte line
inline int shear_pitch(int W1) { return (W1 + 31) / 32 * 32; }

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

// Wave-wide reductions on DPP lane moves (quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror,
// row_mirror, then row_bcast:15 / row_bcast:31 carry the 16-lane row totals up to lane 63).
// __shfl_xor compiles to ds_bpermute: an LDS round trip per butterfly step.  Lanes of masked
// rows receive the identity.  The total is valid in lane 63 (wave_*_dpp return it wave-uniform).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f32(float identity, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, identity),
                                                               __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {   // identity 0.0 (both halves 0)
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, ROW_MASK, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(-INFINITY, v));
  v = fmaxf(v, dpp_f32<0x4E>(-INFINITY, v));
  v = fmaxf(v, dpp_f32<0x141>(-INFINITY, v));
  v = fmaxf(v, dpp_f32<0x140>(-INFINITY, v));
  v = fmaxf(v, dpp_f32<0x142, 0xA>(-INFINITY, v));
  v = fmaxf(v, dpp_f32<0x143, 0xC>(-INFINITY, v));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(0.0f, v);
  v += dpp_f32<0x4E>(0.0f, v);
  v += dpp_f32<0x141>(0.0f, v);
  v += dpp_f32<0x140>(0.0f, v);
  v += dpp_f32<0x142, 0xA>(0.0f, v);
  v += dpp_f32<0x143, 0xC>(0.0f, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
// N independent reductions with their DPP steps interleaved (the same tree per value: results equal
// wave_max_dpp / wave_sum_dpp bit for bit), so the N dependency chains hide each other's latency
template <int N>
__device__ __forceinline__ void wave_max_dpp_n(float (&v)[N]) {
#define SA_DPP_STEP(CTRL, RM)                                                     \
  _Pragma("unroll") for (int i = 0; i < N; ++i) v[i] = fmaxf(v[i], dpp_f32<CTRL, RM>(-INFINITY, v[i]));
  SA_DPP_STEP(0xB1, 0xF) SA_DPP_STEP(0x4E, 0xF) SA_DPP_STEP(0x141, 0xF) SA_DPP_STEP(0x140, 0xF)
  SA_DPP_STEP(0x142, 0xA) SA_DPP_STEP(0x143, 0xC)
#undef SA_DPP_STEP
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[i]), 63));
}
template <int N>
__device__ __forceinline__ void wave_sum_dpp_n(float (&v)[N]) {
#define SA_DPP_STEP(CTRL, RM) \
  _Pragma("unroll") for (int i = 0; i < N; ++i) v[i] += dpp_f32<CTRL, RM>(0.0f, v[i]);
  SA_DPP_STEP(0xB1, 0xF) SA_DPP_STEP(0x4E, 0xF) SA_DPP_STEP(0x141, 0xF) SA_DPP_STEP(0x140, 0xF)
  SA_DPP_STEP(0x142, 0xA) SA_DPP_STEP(0x143, 0xC)
#undef SA_DPP_STEP
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[i]), 63));
}
// Butterfly forms (gfx950): the four in-row DPP steps as above (every lane valid, so each folds into
// the operation's DPP source), then v_permlane16_swap and v_permlane32_swap: each exchanges half
// of the lanes between two copies of the value, so one operation on the pair completes the next
// level and the total ends up in every lane (no row_bcast masks, identity moves or v_readlane).
// A different addition order than wave_sum_dpp (not the same bits).
template <int CTRL>
__device__ __forceinline__ float dpp_all(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <bool MAX>
__device__ __forceinline__ float bfly_op(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }
template <bool MAX, int N>
__device__ __forceinline__ void wave_reduce_bfly_n(float (&v)[N]) {
#define SA_BF_STEP(CTRL) _Pragma("unroll") for (int i = 0; i < N; ++i) v[i] = bfly_op<MAX>(v[i], dpp_all<CTRL>(v[i]));
  SA_BF_STEP(0xB1) SA_BF_STEP(0x4E) SA_BF_STEP(0x141) SA_BF_STEP(0x140)
#undef SA_BF_STEP
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const unsigned u = __builtin_bit_cast(unsigned, v[i]);
    const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    v[i] = bfly_op<MAX>(__builtin_bit_cast(float, (unsigned)p[0]), __builtin_bit_cast(float, (unsigned)p[1]));
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const unsigned u = __builtin_bit_cast(unsigned, v[i]);
    const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    v[i] = bfly_op<MAX>(__builtin_bit_cast(float, (unsigned)p[0]), __builtin_bit_cast(float, (unsigned)p[1]));
  }
}

// fp64 sum; the total is in lane 63 only
__device__ __forceinline__ double wave_sum_dpp_lane63(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  v += dpp_f64<0x142, 0xA>(v);
  v += dpp_f64<0x143, 0xC>(v);
  return v;
}

}  // namespace sa
