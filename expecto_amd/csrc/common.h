// Shared helpers for the expecto HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "../../include/expecto_hip.h"

namespace expecto {

void set_error(const std::string& msg);

#define EXPECTO_HIP_CHECK(expr)                                                        \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      ::expecto::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));         \
      return EXPECTO_EHIP;                                                             \
    }                                                                                  \
  } while (0)

#define EXPECTO_REQUIRE(cond, msg)                                                     \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      ::expecto::set_error(msg);                                                       \
      return EXPECTO_EINVAL;                                                           \
    }                                                                                  \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return EXPECTO_EHIP;
  }
  return EXPECTO_OK;
}

}  // namespace expecto
