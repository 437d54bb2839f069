// errors.cpp -- the library's thread-local error string (bce_last_error), host C++ only, so the
// host-side translation units (jsonl.cpp) also build without HIP for the sanitizer target.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/bce.h"

namespace bce {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

}  // namespace bce

extern "C" const char* bce_last_error(void) { return bce::g_err; }
