// Launch counters behind hv_diag_launch_counts (include/hv_tuning.h): host code only.
#include <atomic>

#include "hv_common.h"

namespace {
std::atomic<long long> g_counts[HV_KF_COUNT];
}

void hv_diag_count(int family) {
  if (family >= 0 && family < HV_KF_COUNT) g_counts[family].fetch_add(1, std::memory_order_relaxed);
}

extern "C" void hv_diag_launch_counts(long long* out) {
  for (int i = 0; i < HV_KF_COUNT; ++i) out[i] = g_counts[i].load(std::memory_order_relaxed);
}

extern "C" void hv_diag_reset_counts(void) {
  for (int i = 0; i < HV_KF_COUNT; ++i) g_counts[i].store(0, std::memory_order_relaxed);
}
