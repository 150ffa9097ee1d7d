// Shared host/device helpers for libhbk.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "hbk.h"

namespace hbk {

// Thread-local last-error text; set by every failing entry point.
void set_error(const char* fmt, ...);

// Return value helpers for the C ABI.
inline int arg_error(const char* what) {
  set_error("hbk: invalid argument: %s", what);
  return HBK_ERR_ARG;
}

int hip_error(hipError_t e, const char* where);

#define HBK_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hbk::hip_error(e_, #call); \
  } while (0)

// Check for a launch failure right after a kernel launch.
#define HBK_LAUNCH_CHECK(name)                                  \
  do {                                                          \
    hipError_t e_ = hipGetLastError();                          \
    if (e_ != hipSuccess) return hbk::hip_error(e_, name);      \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- device ----
struct cf {  // complex float, kept in two VGPRs
  float x, y;
};

__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
  return {fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x)};
}
// multiply by -i
__device__ __forceinline__ cf cmul_mi(cf a) { return {a.y, -a.x}; }

}  // namespace hbk
