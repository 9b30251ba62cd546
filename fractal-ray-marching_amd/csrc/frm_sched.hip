// frm_sched.hip — pixel scheduling for the persistent kernel: most expensive pixels first.
//
// A pixel's march is strictly sequential (up to 2 x max_steps DEs of up to N+1 bodies),
// so a frame cannot end before its longest pixel, and pixels still running when the work
// queue drains decide the frame's tail. The kernel records for every pixel an 8-bit
// log-scale key of its cost (Mandelbulb bodies, frm_kernels.hip cost_key); the next launch
// of the same geometry fetches pixels in descending key order (longest-processing-time-
// first list scheduling over all lanes of the GPU).
// The sort is stable and 8 bits wide: one radix pass over npix (key, pixel) pairs.
// Ordering never changes a pixel's bytes — every pixel is computed by the same
// deterministic function, whichever lane runs it and whenever.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "frm_internal.h"

namespace frm {

__global__ void iota_kernel(uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = i;
}

size_t schedule_temp_bytes(uint32_t npix) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const uint8_t*)nullptr, (uint8_t*)nullptr,
                                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)npix, 0, 8);
  return bytes;
}

// Resample of a whole-frame key map (sw x sh, row-major) to dw x dh: the history a resized
// frame starts from. A new pixel takes the largest key of the source pixels its footprint
// covers, widened by one source pixel on every side (at most 8 x 8 of them). Costs are not
// smooth on a fractal (grazing rays along silhouettes are the expensive ones, and they move
// between resolutions), and for longest-first list scheduling an over-estimate only starts a
// cheap pixel early while an under-estimate leaves an expensive one for the tail.
__global__ void rescale_keys_kernel(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw,
                                    uint32_t dh) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= dw * dh) return;
  const uint32_t y = i / dw, x = i - y * dw;
  const uint32_t x0 = (uint32_t)(((uint64_t)x * sw) / dw), y0 = (uint32_t)(((uint64_t)y * sh) / dh);
  const uint32_t x1 = (uint32_t)(((uint64_t)(x + 1) * sw + dw - 1) / dw);
  const uint32_t y1 = (uint32_t)(((uint64_t)(y + 1) * sh + dh - 1) / dh);
  const uint32_t xa = x0 > 0 ? x0 - 1 : 0, ya = y0 > 0 ? y0 - 1 : 0;
  const uint32_t xb = min(min(x1 + 1, sw), xa + 8), yb = min(min(y1 + 1, sh), ya + 8);
  uint32_t k = 0;
  for (uint32_t sy = ya; sy < yb; ++sy)
    for (uint32_t sx = xa; sx < xb; ++sx) k = max(k, (uint32_t)src[(size_t)sy * sw + sx]);
  dst[i] = (uint8_t)k;
}

hipError_t rescale_keys(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh,
                        hipStream_t stream) {
  const uint32_t n = dw * dh;
  hipLaunchKernelGGL(rescale_keys_kernel, dim3((n + 255u) / 256u), dim3(256), 0, stream, src, sw, sh, dst, dw, dh);
  return hipGetLastError();
}

hipError_t fill_iota(uint32_t* out, uint32_t n, hipStream_t stream) {
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255u) / 256u), dim3(256), 0, stream, out, n);
  return hipGetLastError();
}

hipError_t schedule_pixels(uint32_t npix, bool has_history, const uint8_t* key, uint8_t* key_sorted,
                           const uint32_t* iota, uint32_t* order, void* temp, size_t temp_bytes,
                           hipStream_t stream) {
  if (has_history)
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, key, key_sorted, iota, order, (int)npix,
                                                        0, 8, stream);
  return hipMemcpyAsync(order, iota, (size_t)npix * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
}

}  // namespace frm
