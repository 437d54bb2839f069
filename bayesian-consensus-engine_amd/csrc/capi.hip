// capi.hip -- library-level C ABI: version, errors, device queries.
#include <stdarg.h>
#include <stdio.h>

#include "bce_internal.hpp"

namespace bce {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", what, hipGetErrorString(e));
    return BCE_EHIP;
  }
  return BCE_OK;
}

int cu_count() {
  static int cached = 0;
  if (!cached) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cached = n;
    else
      cached = 256;
  }
  return cached;
}

}  // namespace bce

extern "C" int bce_abi_version(void) { return BCE_ABI_VERSION; }
extern "C" const char* bce_last_error(void) { return bce::g_err; }
extern "C" int bce_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
