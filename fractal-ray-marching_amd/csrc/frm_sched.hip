// frm_sched.hip — tile scheduling for the persistent kernel: most expensive tiles first.
//
// A pixel's march is strictly sequential (up to 2 x max_steps DEs of up to N+1 bodies),
// so a frame cannot end before its longest pixel. Fetched last, such pixels run alone
// after the work queue drains (measured: 8 of 20 ms at 4K). The kernel records per tile
// the critical-path cost (max bodies of any of its pixels); the next frame fetches tiles
// in descending order of that cost (hipcub radix sort). Ordering never changes a pixel's
// bytes — every pixel is computed by the same deterministic function.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "frm_internal.h"

namespace frm {

__global__ void iota_kernel(uint32_t* out, uint32_t n) {
  uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = i;
}

size_t schedule_temp_bytes(uint32_t tiles) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                               (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)tiles);
  return bytes;
}

hipError_t schedule_tiles(uint32_t tiles, bool has_history, uint32_t* cost, uint32_t* cost_sorted,
                          uint32_t* order, uint32_t* iota, void* temp, size_t temp_bytes, hipStream_t stream) {
  const dim3 grid((tiles + 255u) / 256u);
  hipLaunchKernelGGL(iota_kernel, grid, dim3(256), 0, stream, iota, tiles);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (has_history) {
    e = hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, cost, cost_sorted, iota, order,
                                                     (int)tiles, 0, 32, stream);
  } else {
    e = hipMemcpyAsync(order, iota, tiles * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
  }
  if (e != hipSuccess) return e;
  return hipMemsetAsync(cost, 0, tiles * sizeof(uint32_t), stream);
}

}  // namespace frm
