// C-ABI housekeeping: version, thread-local error string, launch checks.
#include "cmx_common.h"
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

// Launch-policy knobs (tile policy, split-K, k-group waves, SRA path thresholds): each starts at
// its CMX_<NAME> environment value or built-in default and can be changed in-process with
// cmx_tune, so A/B measurements interleave the variants in one process instead of comparing
// separate runs.  A knob is read when a launch is planned (eager call or graph capture), never
// by a replayed graph.
namespace {
struct Knob {
  char name[32];
  int value;
};
Knob g_knobs[64];
int g_nknobs = 0;

int find_knob(const char* name) {
  for (int i = 0; i < g_nknobs; ++i)
    if (!strcmp(g_knobs[i].name, name)) return i;
  return -1;
}
}  // namespace

int& cmx_knob(const char* name, int def) {
  int i = find_knob(name);
  if (i < 0) {
    if (g_nknobs == 64) { static int spill; spill = def; return spill; }
    i = g_nknobs++;
    snprintf(g_knobs[i].name, sizeof(g_knobs[i].name), "%s", name);
    char env[48];
    snprintf(env, sizeof(env), "CMX_%s", name);
    const char* e = getenv(env);
    g_knobs[i].value = e ? atoi(e) : def;
  }
  return g_knobs[i].value;
}

extern "C" int cmx_tune(const char* name, int value) {
  CMX_REQUIRE(name, CMX_ERR_ARG, "tune: null name");
  CMX_REQUIRE(strlen(name) < sizeof(g_knobs[0].name) && (find_knob(name) >= 0 || g_nknobs < 64), CMX_ERR_ARG,
              "tune: knob name '%s' too long or table full", name);
  cmx_knob(name, value) = value;          // a knob tuned before its first launch keeps this value
  return CMX_OK;
}

extern "C" int cmx_tune_get(const char* name) {
  const int i = find_knob(name);
  return i < 0 ? -1 : g_knobs[i].value;
}
