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

// A/B switches for measurement (read once per process, never on the device).
#include <stdlib.h>
inline bool getenv_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] && v[0] != '0';
}

#define DMC_REQUIRE(cond, ...)       \
  do {                               \
    if (!(cond)) {                   \
      dmc::set_error(__VA_ARGS__);   \
      return 1;                      \
    }                                \
  } while (0)
