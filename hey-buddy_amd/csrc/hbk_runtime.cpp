// Library identity, thread-local error reporting and device queries.
#include <stdarg.h>

#include "hbk_common.h"

namespace hbk {

static thread_local char g_last_error[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int hip_error(hipError_t e, const char* where) {
  set_error("hbk: HIP error %d (%s) at %s", static_cast<int>(e), hipGetErrorString(e), where);
  return HBK_ERR_HIP;
}

int64_t persistent_blocks(int blocks_per_cu, const void* stream) {
  static thread_local int cached_dev = -1;
  static thread_local int cached_cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return int64_t(256) * blocks_per_cu;
  if (dev != cached_dev) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      cached_cus = cus;
    cached_dev = dev;
  }
  int cus = cached_cus;
  if (stream) {
    uint32_t mask[32] = {};
    if (hipExtStreamGetCUMask(static_cast<hipStream_t>(const_cast<void*>(stream)), 32, mask) == hipSuccess) {
      int n = 0;
      for (uint32_t w : mask) n += __builtin_popcount(w);
      if (n > 0 && n < cus) cus = n;
    } else {
      (void)hipGetLastError();
    }
  }
  return int64_t(cus) * blocks_per_cu;
}

__device__ int32_t g_profile_mark[64];

// One wave; the store keeps the launch from being optimised into nothing.
__global__ void hbk_profile_mark_kernel(int32_t tag) { g_profile_mark[threadIdx.x] = tag; }

}  // namespace hbk

extern "C" {

const char* hbk_version(void) { return "hbk 0.1.0 gfx950"; }

const char* hbk_last_error(void) { return hbk::g_last_error; }

int hbk_device_count(int* count) {
  if (!count) return hbk::arg_error("count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) {
    (void)hipGetLastError();
    *count = 0;
    return HBK_OK;
  }
  if (e != hipSuccess) return hbk::hip_error(e, "hipGetDeviceCount");
  *count = n;
  return HBK_OK;
}

int hbk_stream_create_cu_mask(const uint32_t* cu_mask, int n_words, void** stream) {
  if (!cu_mask || n_words <= 0 || !stream) return hbk::arg_error("cu_mask / n_words / stream");
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(n_words), cu_mask);
  if (e != hipSuccess) return hbk::hip_error(e, "hipExtStreamCreateWithCUMask");
  *stream = s;
  return HBK_OK;
}

int hbk_profile_mark(int32_t tag, void* stream) {
  hipLaunchKernelGGL(hbk::hbk_profile_mark_kernel, dim3(1), dim3(64), 0, hbk::as_stream(stream), tag);
  HBK_LAUNCH_CHECK("hbk_profile_mark_kernel");
  return HBK_OK;
}

int hbk_stream_destroy(void* stream) {
  if (!stream) return hbk::arg_error("stream is NULL");
  hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? HBK_OK : hbk::hip_error(e, "hipStreamDestroy");
}

}  // extern "C"
