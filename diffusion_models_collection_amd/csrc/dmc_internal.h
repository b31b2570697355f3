// Host-side helpers shared by the C-ABI entry points (error reporting, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "dmc.h"

namespace dmc {
void set_error(const char* fmt, ...);
inline hipStream_t as_stream(void* s) { return (hipStream_t)s; }
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}
inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
}  // namespace dmc

// Launch-plan options (A/B switches for measurement and tests). Read ONCE per process from the environment
// (DMC_* variables, at the first planner call) into one table; afterwards only dmc_set_option() /
// dmc_reset_options() change it. The planners read plain fields, never the environment.
namespace dmc {
enum Opt {
  OPT_NO_NARROW, OPT_NO_GLDS, OPT_NO_SPLITK, OPT_NO_BUFLDS, OPT_NO_HALO, OPT_HALO_PRO, OPT_GN_STATS_SPLIT,
  OPT_GN_BWD_SPLIT, OPT_ATTN_STAGED, OPT_ATTN_HG, OPT_WG_BLOCKS, OPT_GN_STATS_ONE_MAX, OPT_GN_BWD_ONE_MAX,
  OPT_NO_XCD, OPT_NO_EPI_STATS, OPT_WG_MINPIX, OPT_GN_BWD_SLICES, OPT_NO_SKGN, OPT_WG_HALO_TARGET, OPT_SK_TARGET,
  OPT_SK_MAX, OPT_NO_NHALO, OPT_GN_BWD_FUSED, OPT_GN_BWD_FUSED_MAXHW, OPT_GN_BWD_NT,
  OPT_REG_EPI, OPT_GEMM1X1, OPT_WG_PIPE, OPT_IMG_MASK, OPT_IMG_GN, OPT_WG_IMG4, OPT_COUNT
};
long opt(Opt o);
}  // namespace dmc

#define DMC_REQUIRE(cond, ...)       \
  do {                               \
    if (!(cond)) {                   \
      dmc::set_error(__VA_ARGS__);   \
      return 1;                      \
    }                                \
  } while (0)
