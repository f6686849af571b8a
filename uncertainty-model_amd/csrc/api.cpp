// Error state and version for the umamd C ABI (host-only).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace umamd {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace umamd

extern "C" {
const char* um_last_error(void) { return umamd::g_err; }
int um_version(void) { return 1; }
}
