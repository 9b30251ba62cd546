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

// ---- history across a camera move (the reference's frame loop moves the camera and the time
// every frame, initialized_app.rs:43-48) -------------------------------------------------------
// The cost keys of a frame belong to its pixels' rays. Seen from the next frame's camera, an
// expensive region (a grazing silhouette, a deep crevice with a long shadow march) lands on
// other pixels: tens of pixels per 60 Hz frame for the HEADLINE_FLY orbit at 4K. Fetching by the
// stale keys starts the moved spikes late, and the frame's tail is theirs. The previous launch's
// records hold, per pixel, whether the primary ray hit and at which distance t (ShadeGeom), so
// its keys are forward-projected: a hit pixel's surface point o + t d is projected into the new
// camera, a missed ray's direction (a point at infinity) likewise, and its key lands on the
// 2 x 2 new pixels around the projected point (largest key wins: an over-estimate only starts a
// cheap pixel early). New pixels nothing lands on keep their old key. Keys order fetches only.

__device__ __forceinline__ uint32_t band_row_to_global_s(const BandGeometry& g, uint32_t lr) {
  const uint32_t b = lr / g.band_rows;
  return (g.first_band + b * g.band_stride) * g.band_rows + (lr - b * g.band_rows);
}

// global row y -> local row of this launch's bands, or UINT32_MAX when another rank owns it
__device__ __forceinline__ uint32_t global_to_band_row(const BandGeometry& g, uint32_t y, uint32_t valid_rows) {
  const uint32_t b = y / g.band_rows;
  if (b < g.first_band || (b - g.first_band) % g.band_stride != 0u) return 0xFFFFFFFFu;
  const uint32_t lr = ((b - g.first_band) / g.band_stride) * g.band_rows + (y - b * g.band_rows);
  return lr < valid_rows ? lr : 0xFFFFFFFFu;
}

__global__ void reproject_keys_kernel(ReprojectArgs a, const uint8_t* __restrict__ keys, uint32_t* __restrict__ map) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= a.npix) return;
  const uint32_t w = a.prev.width;
  const uint32_t lr = i / w, x = i - lr * w;
  const uint32_t y = band_row_to_global_s(a.g, lr);
  const uint32_t key = keys[i];
  const ShadeTail tl = a.tails[i];
  const v3 d = camera_ray(a.prev, x, y);
  v3 v;
  if (tl.word & kRecHit) {  // the surface point, relative to the new camera
    const float t = a.geom[i].t;
    v = mk(fmaf(t, d.x, a.prev.origin.x) - a.next.origin.x, fmaf(t, d.y, a.prev.origin.y) - a.next.origin.y,
           fmaf(t, d.z, a.prev.origin.z) - a.next.origin.z);
  } else {
    v = d;  // a point at infinity: only the rotation moves it
  }
  // camera coordinates: the inverse of the (orthonormal) rotation rows, c_i = sum_j row[j][i] v_j
  const float (&R)[3][4] = a.next.row;
  const float cx = R[0][0] * v.x + R[1][0] * v.y + R[2][0] * v.z;
  const float cy = R[0][1] * v.x + R[1][1] * v.y + R[2][1] * v.z;
  const float cz = R[0][2] * v.x + R[1][2] * v.y + R[2][2] * v.z;
  if (!(cz > 1e-6f)) return;
  // the ray of pixel (sx, sy) is normalize(sx * aspect_x, sy * aspect_y, CAMERA_DIRECTION_Z)
  const float sx = cx / cz * (kCameraDirectionZ / a.next.aspect_x);
  const float sy = cy / cz * (kCameraDirectionZ / a.next.aspect_y);
  const float px = (sx + 1.0f) * (0.5f * (float)w) - 0.5f;
  const float py = (1.0f - sy) * (0.5f * (float)a.next.height) - 0.5f;
  if (!(px > -1.0f && px < (float)w && py > -1.0f && py < (float)a.next.height)) return;
  const int x0 = (int)floorf(px), y0 = (int)floorf(py);
  for (int yy = y0; yy <= y0 + 1; ++yy) {
    if (yy < 0 || yy >= (int)a.next.height) continue;
    const uint32_t nl = global_to_band_row(a.g, (uint32_t)yy, a.valid_rows);
    if (nl == 0xFFFFFFFFu) continue;
    for (int xx = x0; xx <= x0 + 1; ++xx)
      if (xx >= 0 && xx < (int)w) atomicMax(&map[(size_t)nl * w + (uint32_t)xx], key + 1u);
  }
}

__global__ void reproject_fill_kernel(uint32_t npix, const uint32_t* __restrict__ map, uint8_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= npix) return;
  const uint32_t m = map[i];
  if (m) keys[i] = (uint8_t)(m - 1u);
}

hipError_t reproject_keys(const ReprojectArgs& a, uint8_t* keys, uint32_t* scratch, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(scratch, 0, (size_t)a.npix * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  const dim3 grid((a.npix + 255u) / 256u);
  hipLaunchKernelGGL(reproject_keys_kernel, grid, dim3(256), 0, stream, a, (const uint8_t*)keys, scratch);
  hipLaunchKernelGGL(reproject_fill_kernel, grid, dim3(256), 0, stream, a.npix, (const uint32_t*)scratch, keys);
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
