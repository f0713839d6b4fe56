// Error reporting, pyramid geometry and live event timing for libsa_hip.so.
#include <cstring>
#include <mutex>
#include <vector>

#include "sa_common.h"

namespace sa {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {
struct KernelTimes {
  std::vector<hipEvent_t> pool;  // pairs: start, stop
  size_t used = 0;
};
std::mutex g_mu;
bool g_timing = false;
KernelTimes g_times[SA_K_COUNT];
const char *g_names[SA_K_COUNT] = {"corr_volume_pyramid", "corr_lookup", "mono_masked_volume",
                                   "softargmin_conf",     "weighted_lsq", "gru_zr",
                                   "gru_out",             "convex_upsample", "misc",
                                   "conv3d_fused",        "norm_act",
                                   "conv2d_wino", "conv2d_direct", "conv2d_wino4", "corr_shear",
                                   "mono_pyramid", "gru_plumbing", "conv2d_small", "conv2d_narrow",
                                   "conv1x1"};
}  // namespace

TimingScope::TimingScope(int kernel_id, hipStream_t s) : id(kernel_id), stream(s), on(false) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_timing) return;
  KernelTimes &t = g_times[id];
  if (t.used + 2 > t.pool.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      t.pool.push_back(e);
    }
  }
  (void)hipEventRecord(t.pool[t.used], stream);
  on = true;
}

TimingScope::~TimingScope() {
  if (!on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  KernelTimes &t = g_times[id];
  (void)hipEventRecord(t.pool[t.used + 1], stream);
  t.used += 2;
}

}  // namespace sa

extern "C" {

const char *sa_last_error(void) { return sa::g_err; }

int sa_pyramid_level_width(int w2, int level) {
  int w = w2;
  for (int i = 0; i < level; ++i) w /= 2;
  return w;
}

int sa_pyramid_level_offset(int w2, int level) {
  int off = 0, w = w2;
  for (int i = 0; i < level; ++i) {
    off += w;
    w /= 2;
  }
  return off;
}

long sa_pyramid_row_stride(int w2, int num_levels) {
  long s = sa_pyramid_level_offset(w2, num_levels);
  return (s + 3) / 4 * 4;
}

int sa_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(sa::g_mu);
  sa::g_timing = on != 0;
  for (auto &t : sa::g_times) t.used = 0;
  return SA_OK;
}

int sa_timing_read(int kernel_id, double *total_ms, long *count) {
  if (kernel_id < 0 || kernel_id >= SA_K_COUNT || !total_ms || !count) {
    sa::set_error("sa_timing_read: bad arguments");
    return SA_E_ARG;
  }
  std::lock_guard<std::mutex> lk(sa::g_mu);
  auto &t = sa::g_times[kernel_id];
  double tot = 0.0;
  for (size_t i = 0; i + 1 < t.used; i += 2) {
    if (hipEventSynchronize(t.pool[i + 1]) != hipSuccess) {
      sa::set_error("sa_timing_read: hipEventSynchronize failed");
      return SA_E_RUNTIME;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t.pool[i], t.pool[i + 1]) != hipSuccess) {
      sa::set_error("sa_timing_read: hipEventElapsedTime failed");
      return SA_E_RUNTIME;
    }
    tot += ms;
  }
  *total_ms = tot;
  *count = (long)(t.used / 2);
  t.used = 0;
  return SA_OK;
}

const char *sa_kernel_name(int kernel_id) {
  if (kernel_id < 0 || kernel_id >= SA_K_COUNT) return "?";
  return sa::g_names[kernel_id];
}

}  // extern "C"

extern "C" int sa_abi_version(void) { return SA_ABI_VERSION; }   // (1 through round 5)

extern "C" long sa_struct_size(int which) {
  switch (which) {
    case SA_STRUCT_WINO_PROBLEM: return (long)sizeof(SaWinoProblem);
    case SA_STRUCT_GATE_EPILOGUE: return (long)sizeof(SaGateEpilogue);
    case SA_STRUCT_RESAMPLE_JOB: return (long)sizeof(SaResampleJob);
    case SA_STRUCT_FEATURE_GATE_JOB: return (long)sizeof(SaFeatureGateJob);
    default: return -1;
  }
}
