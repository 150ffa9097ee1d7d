// Per-CU streaming bandwidth probe (tuning aid, not a product kernel): each
// workgroup sums `per_wg` float4s from its own region (distinct: HBM-streamed)
// or from one shared region (shared: L2-resident after the first touch), with
// `depth` 16-B loads per thread in flight.
#include <hip/hip_runtime.h>
#include <cstdint>

template <int DEPTH>
__global__ void __launch_bounds__(256) bw_kernel(const float4* __restrict__ src, int64_t per_wg, int shared,
                                                 int64_t region, float* out) {
  const int64_t base = shared ? 0 : int64_t(blockIdx.x) * per_wg;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = threadIdx.x; i < per_wg; i += 256 * DEPTH) {
    float4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      int64_t j = i + 256 * d;
      j = j < per_wg ? j : per_wg - 1;
      v[d] = src[(base + j) % region];
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc.x += v[d].x;
      acc.y += v[d].y;
      acc.z += v[d].z;
      acc.w += v[d].w;
    }
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[threadIdx.x] = acc.x;
}

extern "C" int bw_run(const void* src, int64_t per_wg, int shared, int64_t region, float* out, int blocks, int depth,
                      void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float4* p = static_cast<const float4*>(src);
  switch (depth) {
    case 1: hipLaunchKernelGGL(bw_kernel<1>, dim3(blocks), dim3(256), 0, s, p, per_wg, shared, region, out); break;
    case 4: hipLaunchKernelGGL(bw_kernel<4>, dim3(blocks), dim3(256), 0, s, p, per_wg, shared, region, out); break;
    case 8: hipLaunchKernelGGL(bw_kernel<8>, dim3(blocks), dim3(256), 0, s, p, per_wg, shared, region, out); break;
    default: hipLaunchKernelGGL(bw_kernel<16>, dim3(blocks), dim3(256), 0, s, p, per_wg, shared, region, out);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
