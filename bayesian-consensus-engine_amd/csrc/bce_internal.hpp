// bce_internal.hpp -- host-side plumbing shared by the engine's translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/bce.h"

namespace bce {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch that was just enqueued.
int check_launch(const char* what);

// Device properties cached per device (CU count for grid sizing).  Thread-safe.
int cu_count();

// Resident workgroups per CU of `fn` at `threads` threads and `lds` dynamic LDS bytes,
// cached per (device, kernel, shape); `fallback` when the query fails.  Thread-safe.
int blocks_per_cu(const void* fn, int threads, size_t lds, int fallback, const char* name = nullptr);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel).  Thread-safe.
int ensure_dynamic_lds(const void* fn, int bytes);

// The planned launch's side streams (kSideStreams per device): side_fork records a fork
// event on `st`, makes the first k side streams wait on it and takes the device's fork lock,
// which the caller holds until side_join has made `st` wait on their work -- so two host
// threads planning on different streams never wait on each other's fork/join events.
constexpr int kSideStreams = 1;
int side_fork(hipStream_t st, int k, hipStream_t* sides, std::unique_lock<std::mutex>* lock);
int side_join(hipStream_t st, int k);

}  // namespace bce

#define BCE_REQUIRE(cond, ...)        \
  do {                                \
    if (!(cond)) {                    \
      ::bce::set_error(__VA_ARGS__);  \
      return BCE_EINVAL;              \
    }                                 \
  } while (0)

#define BCE_HIP(call)                                                        \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::bce::set_error("%s failed: %s", #call, hipGetErrorString(e_));       \
      return BCE_EHIP;                                                       \
    }                                                                        \
  } while (0)
