// capi.hip -- library-level C ABI: version, errors, device queries.
#include <stdarg.h>
#include <stdio.h>

#include "bce_internal.hpp"
#include "consensus_common.hpp"

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

int* fault_word() {
  static int* words[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!words[dev]) {
    int* p = nullptr;
    if (hipMalloc((void**)&p, sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, sizeof(int)) != hipSuccess) return nullptr;
    words[dev] = p;
  }
  return words[dev];
}

static int g_spin_cap = 1 << 22;
int spin_cap() { return g_spin_cap; }

static const char* fault_text(int code) {
  switch (code) {
    case kFaultSpinLoader: return "consensus_pipe_kernel: loader wave timed out waiting for a free slot";
    case kFaultSpinCompute: return "consensus_pipe_kernel: compute wave timed out waiting for its tile";
    case kFaultSid: return "consensus: a sid is >= n_sources (its row read was clamped)";
    case kFaultTooLong: return "consensus: a market is longer than the launch's max_len (left unprocessed)";
    case kFaultSpinChain: return "consensus_wide_kernel: exact-mode chain hand-off timed out";
    default: return "unknown device fault";
  }
}

}  // namespace bce

extern "C" int bce_fault_check(void* stream) {
  int* w = bce::fault_word();
  if (!w) {
    bce::set_error("bce_fault_check: no fault word on this device");
    return BCE_EHIP;
  }
  hipStream_t st = bce::as_stream(stream);
  int h = 0;
  BCE_HIP(hipMemcpyAsync(&h, w, sizeof h, hipMemcpyDeviceToHost, st));
  BCE_HIP(hipStreamSynchronize(st));
  if (h == 0) return BCE_OK;
  BCE_HIP(hipMemsetAsync(w, 0, sizeof(int), st));
  BCE_HIP(hipStreamSynchronize(st));
  bce::set_error("device fault %d: %s", h, bce::fault_text(h));
  return BCE_EHIP;
}

extern "C" int bce_debug_set_spin_cap(int cap) {
  bce::g_spin_cap = (cap > 0) ? cap : (1 << 22);
  return BCE_OK;
}

extern "C" int bce_abi_version(void) { return BCE_ABI_VERSION; }
extern "C" const char* bce_last_error(void) { return bce::g_err; }
extern "C" int bce_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
