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

int sv_stream_create_cu_reserved(int32_t device, const int32_t* reserved, int32_t n_reserved, sv_stream_t* out) {
  SV_REQUIRE(out && (n_reserved == 0 || reserved) && n_reserved >= 0, "sv_stream_create_cu_reserved: bad arguments");
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
    return sv::set_error(SV_ERR_INVALID_ARG, "sv_stream_create_cu_reserved: no device %d", device);
  SV_REQUIRE(n_reserved < ncu, "sv_stream_create_cu_reserved: reserving %d of %d CUs", n_reserved, ncu);
  const int words = (ncu + 31) / 32;
  uint32_t mask[64];
  SV_REQUIRE(words <= 64, "sv_stream_create_cu_reserved: %d CUs", ncu);
  for (int w = 0; w < words; ++w) mask[w] = 0xffffffffu;
  if (ncu % 32) mask[words - 1] = (1u << (ncu % 32)) - 1u;
  for (int i = 0; i < n_reserved; ++i) {
    SV_REQUIRE(reserved[i] >= 0 && reserved[i] < ncu, "sv_stream_create_cu_reserved: CU %d out of range", reserved[i]);
    mask[reserved[i] / 32] &= ~(1u << (reserved[i] % 32));
  }
  int cur = 0;
  hipGetDevice(&cur);
  if (cur != device) hipSetDevice(device);
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (cur != device) hipSetDevice(cur);
  if (e != hipSuccess)
    return sv::set_error(SV_ERR_LAUNCH, "sv_stream_create_cu_reserved: %s", hipGetErrorString(e));
  *out = (sv_stream_t)s;
  return SV_OK;
}

const char* sv_build_target(void) {
#ifdef SV_OFFLOAD_ARCH
  return SV_OFFLOAD_ARCH;
#else
  return "gfx950";
#endif
}

}  // extern "C"
