// Library-level ABI entry points: version, build target and thread-local error reporting.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include <mutex>
#include <set>
#include <utility>

#include "common.h"

namespace sv {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(SV_ERR_LAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
  return SV_OK;
}

namespace {
constexpr int kMaxDevices = 64;
std::mutex g_dev_mu;
int g_cus[kMaxDevices] = {};                       // 0 = not queried yet
std::set<std::pair<const void*, int>> g_lds_attr;  // (kernel, device) pairs whose LDS limit is raised
}  // namespace

int stream_device(hipStream_t s) {
  int dev = 0;
  if (!s || hipStreamGetDevice(s, &dev) != hipSuccess) hipGetDevice(&dev);
  return dev;
}

int device_cus(hipStream_t s) {
  const int dev = stream_device(s);
  if (dev < 0 || dev >= kMaxDevices) return 256;
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (!g_cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_cus[dev] = n;
  }
  return g_cus[dev];
}

void ensure_lds_attr(const void* kernel, int bytes, hipStream_t s) {
  if (bytes <= 65536) return;
  const int dev = stream_device(s);
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (g_lds_attr.insert({kernel, dev}).second) {
    int cur = -1;
    hipGetDevice(&cur);
    if (cur != dev) hipSetDevice(dev);
    hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (cur != dev) hipSetDevice(cur);
  }
}

int policy_grid(const sv_gemm_policy* pol, int total, int per_cu_default, hipStream_t s) {
  int grid = total;
  const int wpc = pol && pol->wg_per_cu > 0 ? (pol->wg_per_cu > 2 ? 2 : pol->wg_per_cu) : per_cu_default;
  if (wpc > 0) {
    const int slots = wpc * device_cus(s);
    if (grid > slots) grid = slots;
  }
  if (pol && pol->grid_cap > 0 && grid > pol->grid_cap) grid = pol->grid_cap;  // persistent over the rest
  return grid;
}

}  // namespace sv

extern "C" {

int sv_version(void) { return 3; }

const char* sv_last_error_string(void) { return sv::g_err; }

const char* sv_build_target(void) {
#ifdef SV_OFFLOAD_ARCH
  return SV_OFFLOAD_ARCH;
#else
  return "gfx950";
#endif
}

}  // extern "C"
