// bce_internal.hpp -- host-side plumbing shared by the engine's translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bce.h"

namespace bce {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch that was just enqueued.
int check_launch(const char* what);

// Device properties cached per process (CU count for grid sizing).
int cu_count();

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
