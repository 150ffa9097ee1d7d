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

// Grid of a persistent (grid-stride) kernel: blocks_per_cu x the CUs the
// stream may use (its CU mask when created by hbk_stream_create_cu_mask, else
// the device's): a grid sized for more CUs than the stream owns leaves a tail
// wave of workgroups running alone.
int64_t persistent_blocks(int blocks_per_cu, const void* stream);

// ---------------------------------------------------------------- device ----
// Complex float as a 2-lane vector so adds / multiplies lower to the packed
// v_pk_{add,mul,fma}_f32 (two f32 per lane per instruction on gfx950).
typedef float cf __attribute__((ext_vector_type(2)));

__device__ __forceinline__ cf cadd(cf a, cf b) { return a + b; }
__device__ __forceinline__ cf csub(cf a, cf b) { return a - b; }
// (a.x b.x - a.y b.y, a.x b.y + a.y b.x) = a.x * b + a.y * (-b.y, b.x)
__device__ __forceinline__ cf cmul(cf a, cf b) {
  const cf bs = {-b.y, b.x};
  return __builtin_elementwise_fma(cf{a.y, a.y}, bs, cf{a.x, a.x} * b);
}
// max that propagates NaN (torch / numpy max-pool semantics; fmaxf drops NaN)
__device__ __forceinline__ float nan_max(float a, float b) { return (b > a || b != b) ? b : a; }

// a conj(b) = a.x (b.x, -b.y) + a.y (b.y, b.x)
__device__ __forceinline__ cf cmul_conj(cf a, cf b) {
  return __builtin_elementwise_fma(cf{a.y, a.y}, cf{b.y, b.x}, cf{a.x, a.x} * cf{b.x, -b.y});
}

// multiply by -i
__device__ __forceinline__ cf cmul_mi(cf a) { return cf{a.y, -a.x}; }

}  // namespace hbk
