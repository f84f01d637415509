// C-ABI plumbing: thread-local error message and version.  (Kernels live in *.hip.)
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace clskd {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
static thread_local char g_kernel[160] = "";
void note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kernel, sizeof(g_kernel), fmt, ap);
  va_end(ap);
}
}  // namespace clskd

extern "C" const char* clskd_last_error(void) { return clskd::g_err; }
extern "C" const char* clskd_conv_last_kernel(void) { return clskd::g_kernel; }
extern "C" int clskd_version(void) { return 1; }
