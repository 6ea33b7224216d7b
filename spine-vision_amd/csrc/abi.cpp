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

}  // namespace sv

// The per-device context (sv_ctx): everything the launches are sized by, queried once per device, under one mutex.
struct sv_ctx {
  int device = -1;
  int cus = 0;  // 0 = not queried yet
  int lds = 0;
  int refs = 0;
  char arch[32] = "";
  std::set<const void*> lds_raised;  // kernels whose dynamic-LDS limit is raised on this device
};

namespace sv {

namespace {
constexpr int kMaxDevices = 64;
std::mutex g_dev_mu;
sv_ctx g_ctx[kMaxDevices];

// the device's context with its properties queried (caller holds g_dev_mu)
sv_ctx& ctx_locked(int dev) {
  sv_ctx& c = g_ctx[dev];
  if (!c.cus) {
    c.device = dev;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    c.cus = n;
    int l = 0;
    if (hipDeviceGetAttribute(&l, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || l <= 0) l = 163840;
    c.lds = l;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) snprintf(c.arch, sizeof(c.arch), "%s", prop.gcnArchName);
  }
  return c;
}
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
  return ctx_locked(dev).cus;
}

int stream_cus(hipStream_t s) {
  const int all = device_cus(s);
  uint32_t mask[32] = {};
  const int words = (all + 31) / 32;
  if (words > 32 || hipExtStreamGetCUMask(s, (uint32_t)words, mask) != hipSuccess) return all;
  int n = 0;
  for (int w = 0; w < words; ++w) n += __builtin_popcount(mask[w]);
  return n > 0 && n < all ? n : all;
}

int ensure_lds_attr(const void* kernel, int bytes, hipStream_t s) {
  if (bytes <= 65536) return SV_OK;
  const int dev = stream_device(s);
  if (dev < 0 || dev >= kMaxDevices) return SV_OK;
  std::lock_guard<std::mutex> lk(g_dev_mu);
  sv_ctx& c = ctx_locked(dev);
  if (c.lds_raised.count(kernel)) return SV_OK;
  int cur = -1;
  hipGetDevice(&cur);
  if (cur != dev) hipSetDevice(dev);
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (cur != dev) hipSetDevice(cur);
  if (e != hipSuccess)
    return set_error(SV_ERR_LAUNCH, "hipFuncSetAttribute(MaxDynamicSharedMemorySize = %d) failed on device %d: %s", bytes,
                     dev, hipGetErrorString(e));
  c.lds_raised.insert(kernel);  // remembered only once raised: a failed attempt is retried at the next launch
  return SV_OK;
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

int sv_version(void) { return 9; }

int sv_ctx_create(int32_t device, sv_ctx** out) {
  SV_REQUIRE(out, "sv_ctx_create: null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  SV_REQUIRE(device >= 0 && device < n && device < sv::kMaxDevices, "sv_ctx_create: no device %d (%d visible)",
             (int)device, n);
  std::lock_guard<std::mutex> lk(sv::g_dev_mu);
  sv_ctx& c = sv::ctx_locked(device);
  ++c.refs;
  *out = &c;
  return SV_OK;
}

int sv_ctx_destroy(sv_ctx* ctx) {
  SV_REQUIRE(ctx && ctx >= sv::g_ctx && ctx < sv::g_ctx + sv::kMaxDevices, "sv_ctx_destroy: not a context");
  std::lock_guard<std::mutex> lk(sv::g_dev_mu);
  SV_REQUIRE(ctx->refs > 0, "sv_ctx_destroy: context of device %d already released", ctx->device);
  if (--ctx->refs == 0) {  // forget the cached state; the LDS limits stay raised in the runtime (harmless)
    const int dev = ctx->device;
    *ctx = sv_ctx{};
    ctx->device = dev;
  }
  return SV_OK;
}

int sv_ctx_get_info(const sv_ctx* ctx, sv_ctx_info* out) {
  SV_REQUIRE(ctx && out && ctx >= sv::g_ctx && ctx < sv::g_ctx + sv::kMaxDevices, "sv_ctx_get_info: bad arguments");
  std::lock_guard<std::mutex> lk(sv::g_dev_mu);
  sv_ctx& c = sv::ctx_locked((int)(ctx - sv::g_ctx));
  out->device = c.device;
  out->compute_units = c.cus;
  out->lds_bytes_per_wg = c.lds;
  out->xcds = c.cus % 8 == 0 ? 8 : 1;
  out->lds_raised_kernels = (int32_t)c.lds_raised.size();
  out->refs = c.refs;
  snprintf(out->arch, sizeof(out->arch), "%s", c.arch);
  return SV_OK;
}

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
