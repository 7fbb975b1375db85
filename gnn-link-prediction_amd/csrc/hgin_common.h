// Shared helpers for libhgin.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/hgin.h"

namespace hgin {

constexpr int kWave = 64;  // CDNA wavefront

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Launch bookkeeping: returns 0 or the hipError_t of the launch (after recording a message).
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return HGIN_OK;
}

// Async memset whose status is folded into the call's return value.
inline int memset_async(void* p, int v, size_t bytes, hipStream_t s, const char* what) {
  hipError_t e = hipMemsetAsync(p, v, bytes, s);
  if (e != hipSuccess) {
    set_error("%s: hipMemsetAsync failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return HGIN_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace hgin

#define HGIN_ARG_CHECK(cond, ...)     \
  do {                                \
    if (!(cond)) {                    \
      ::hgin::set_error(__VA_ARGS__); \
      return HGIN_E_ARG;              \
    }                                 \
  } while (0)
