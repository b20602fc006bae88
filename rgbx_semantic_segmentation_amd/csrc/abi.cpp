// C-ABI housekeeping: version, thread-local error string, launch checks.
#include "cmx_common.h"
#include <stdarg.h>
#include <stdio.h>

static thread_local char g_err[1024] = {0};

void cmx_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int cmx_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cmx_set_error("%s: %s", what, hipGetErrorString(e));
    return CMX_ERR_LAUNCH;
  }
  return CMX_OK;
}

extern "C" int cmx_abi_version(void) { return CMX_ABI_VERSION; }
extern "C" const char* cmx_last_error(void) { return g_err; }
