// C-ABI plumbing: version, thread-local error message, launch checks.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

static thread_local char g_err[512] = "";

void fv_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fv_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fv_set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return FV_OK;
}

extern "C" {
int fv_abi_version(void) { return FV_ABI_VERSION; }
const char* fv_last_error(void) { return g_err; }
}
