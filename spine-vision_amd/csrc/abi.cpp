// Library-level ABI entry points: version, build target and thread-local error reporting.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

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

extern "C" {

int sv_version(void) { return 2; }

const char* sv_last_error_string(void) { return sv::g_err; }

const char* sv_build_target(void) {
#ifdef SV_OFFLOAD_ARCH
  return SV_OFFLOAD_ARCH;
#else
  return "gfx950";
#endif
}

}  // extern "C"
