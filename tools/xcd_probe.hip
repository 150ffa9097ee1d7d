// Which XCD (and CU) does each workgroup of a launch land on? Reads the XCC_ID and HW_ID
// hardware registers (s_getreg_b32: reads only) into a device buffer, one entry per block.
// Used by tools/xcd_probe.py to map hipExtStreamCreateWithCUMask bits to XCDs.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void xcd_probe_kernel(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    // HW_REG_XCC_ID (id 20) bits [3:0]; HW_REG_HW_ID (id 4): CU_ID bits [11:8], SH_ID [12], SE_ID [15:13]
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
    // keep the block resident a little so that the dispatcher spreads the grid
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(10);
  }
}

extern "C" int xcd_probe(uint32_t* out, int blocks, int spin, void* stream) {
  hipLaunchKernelGGL(xcd_probe_kernel, dim3(blocks), dim3(64), 0, static_cast<hipStream_t>(stream), out, spin);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
