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

// Host -> device copy of a packed launch-record table (cmx_*_pack) on the caller's stream.
// `src` must be pinned host memory that stays unmodified until the copy has run (inside a
// HIP-graph capture: for the graph's lifetime, since every replay re-reads it).
extern "C" int cmx_upload(void* dst, const void* src, size_t nbytes, hipStream_t s) {
  CMX_REQUIRE(dst && src, CMX_ERR_ARG, "upload: null pointer");
  const hipError_t e = hipMemcpyAsync(dst, src, nbytes, hipMemcpyHostToDevice, s);
  CMX_REQUIRE(e == hipSuccess, CMX_ERR_LAUNCH, "upload: %s", hipGetErrorString(e));
  return CMX_OK;
}
