// frm_kernels.hip — gfx950 kernels of the fractal ray-marcher.
//
// render_simple<FAM>: one thread per pixel, one wave64 per 8x8 pixel tile (so the 64
//   lanes of a wave march spatially coherent rays), 256-thread blocks = 16x16 pixels.
//   Literal restatement of fragment_main (fragment.wgsl:327-349): primary march, on hit
//   the four normal taps, the shadow march toward the sun and the shading; sRGB encode
//   and a packed 32-bit RGBA8 store. Work counters are reduced per wave in registers and
//   added with one 64-bit atomic per wave and counter.
// unshuffle_bands: rank-major band buffers -> row-major frame (multi-GPU gather).
#include <hip/hip_runtime.h>

#include "frm_internal.h"
#include "frm_srgb_table.h"

namespace frm {

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ uint32_t band_row_to_global(const BandGeometry& g, uint32_t lr) {
  uint32_t b = lr / g.band_rows;
  return (g.first_band + b * g.band_stride) * g.band_rows + (lr - b * g.band_rows);
}

template <uint32_t FAM, bool ITERS>
__global__ __launch_bounds__(256) void render_simple(KernelArgs a) {
  __shared__ float table[256];
  table[threadIdx.x] = kSrgbThresholds[threadIdx.x];
  __syncthreads();

  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t x = blockIdx.x * 16u + (wave & 1u) * 8u + (lane & 7u);
  const uint32_t lr = blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
  const uint32_t width = a.f.width;

  uint32_t n_pix = 0;
  PixelCount pc = {0u, 0u, 0u, 0u, {0u, 0u}};
  if (x < width && lr < a.g.local_rows) {
    const uint32_t y = band_row_to_global(a.g, lr);
    if (y < a.f.height) {
      n_pix = 1;
      v3 color = shade_pixel<FAM, ITERS>(a.f, a.s, x, y, pc);
      a.out[(size_t)lr * width + x] = pack_rgba(color, table);
    }
  }

  unsigned long long v[7] = {n_pix, pc.hit, pc.primary, pc.shadow, pc.normal, pc.de.bodies, pc.de.bailouts};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    unsigned long long s = wave_sum(v[k]);
    if (lane == 0 && s) atomicAdd(&a.counters[k], s);
  }
}

// dst row y <- band b = y / band_rows, held by rank b % ranks as its (b / ranks)-th band.
// T = uint4 when rows and rank strides are 16-byte multiples, else uint32_t.
template <typename T>
__global__ __launch_bounds__(256) void unshuffle_bands(const T* __restrict__ src, size_t rank_stride,
                                                       T* __restrict__ dst, uint32_t row_words,
                                                       uint32_t height, uint32_t band_rows,
                                                       uint32_t ranks) {
  const uint32_t y = blockIdx.y;
  if (y >= height) return;
  const uint32_t b = y / band_rows, r = y - b * band_rows;
  const uint32_t rank = b % ranks, j = b / ranks;
  const T* s = src + rank * rank_stride + (size_t)(j * band_rows + r) * row_words;
  T* d = dst + (size_t)y * row_words;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < row_words; i += gridDim.x * 256u) d[i] = s[i];
}

// ---- diagnostics -------------------------------------------------------------------
template <uint32_t FAM, bool ITERS>
__global__ __launch_bounds__(256) void eval_scene(SceneUniforms s, const float* pts, uint32_t n,
                                                  float* dist, float* color) {
  uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  DeCount cnt = {0u, 0u};
  v3 p = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
  dist[i] = scene_de<FAM, ITERS>(s, p, cnt);
  v3 c = scene_color<FAM>(p);
  color[3 * i] = c.x;
  color[3 * i + 1] = c.y;
  color[3 * i + 2] = c.z;
}

__global__ __launch_bounds__(256) void eval_math(int fn, const float* a, const float* b, uint32_t n,
                                                 float* out) {
  uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  float x = a[i], y = b ? b[i] : 0.0f, r;
  switch (fn) {
    case 0: r = sin_(x); break;
    case 1: r = cos_(x); break;
    case 2: r = acos_(x); break;
    case 3: r = atan2_(x, y); break;
    case 4: r = log_(x); break;
    case 5: r = log2_(x); break;
    case 6: r = exp2_(x); break;
    case 7: r = pow_(x, y); break;
    case 8: r = sqrt_(x); break;
    default: r = x / y; break;
  }
  out[i] = r;
}

template <uint32_t FAM, bool ITERS>
static void eval_scene_one(const SceneUniforms& s, const float* pts, uint32_t n, float* dist, float* color,
                           hipStream_t stream) {
  hipLaunchKernelGGL((eval_scene<FAM, ITERS>), dim3((n + 255u) / 256u), dim3(256), 0, stream, s, pts, n, dist,
                     color);
}

template <uint32_t FAM>
static void eval_scene_fam(const SceneUniforms& s, const float* pts, uint32_t n, float* dist, float* color,
                           hipStream_t stream) {
  if (s.n) eval_scene_one<FAM, true>(s, pts, n, dist, color, stream);
  else eval_scene_one<FAM, false>(s, pts, n, dist, color, stream);
}

hipError_t launch_eval_scene(const SceneUniforms& s, const float* pts, uint32_t n, float* dist, float* color,
                             hipStream_t stream) {
  switch (s.family) {
    case kMenger: eval_scene_fam<kMenger>(s, pts, n, dist, color, stream); break;
    case kSierpinski: eval_scene_fam<kSierpinski>(s, pts, n, dist, color, stream); break;
    case kKoch: eval_scene_fam<kKoch>(s, pts, n, dist, color, stream); break;
    case kMandelbulb: eval_scene_fam<kMandelbulb>(s, pts, n, dist, color, stream); break;
    default: eval_scene_fam<kSphere>(s, pts, n, dist, color, stream); break;
  }
  return hipGetLastError();
}

hipError_t launch_eval_math(int fn, const float* a, const float* b, uint32_t n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(eval_math, dim3((n + 255u) / 256u), dim3(256), 0, stream, fn, a, b, n, out);
  return hipGetLastError();
}

template <uint32_t FAM>
static hipError_t launch_family(const KernelArgs& args, KernelKind kind, int cu_count,
                                hipStream_t stream) {
  (void)kind;
  (void)cu_count;
  dim3 grid((args.f.width + 15u) / 16u, (args.g.local_rows + 15u) / 16u);
  if (args.s.n)
    hipLaunchKernelGGL((render_simple<FAM, true>), grid, dim3(256), 0, stream, args);
  else
    hipLaunchKernelGGL((render_simple<FAM, false>), grid, dim3(256), 0, stream, args);
  return hipGetLastError();
}

hipError_t launch_render(const KernelArgs& args, KernelKind kind, int cu_count, hipStream_t stream) {
  switch (args.s.family) {
    case kMenger: return launch_family<kMenger>(args, kind, cu_count, stream);
    case kSierpinski: return launch_family<kSierpinski>(args, kind, cu_count, stream);
    case kKoch: return launch_family<kKoch>(args, kind, cu_count, stream);
    case kMandelbulb: return launch_family<kMandelbulb>(args, kind, cu_count, stream);
    default: return launch_family<kSphere>(args, kind, cu_count, stream);
  }
}

hipError_t launch_unshuffle(const uint8_t* src, size_t rank_stride, uint8_t* dst, uint32_t width,
                            uint32_t height, uint32_t band_rows, uint32_t ranks,
                            hipStream_t stream) {
  if (width % 4u == 0 && rank_stride % 16u == 0) {
    const uint32_t words = width / 4u;
    dim3 grid((words + 255u) / 256u, height);
    hipLaunchKernelGGL(unshuffle_bands<uint4>, grid, dim3(256), 0, stream, (const uint4*)src,
                       rank_stride / 16u, (uint4*)dst, words, height, band_rows, ranks);
  } else {
    dim3 grid((width + 255u) / 256u, height);
    hipLaunchKernelGGL(unshuffle_bands<uint32_t>, grid, dim3(256), 0, stream, (const uint32_t*)src,
                       rank_stride / 4u, (uint32_t*)dst, width, height, band_rows, ranks);
  }
  return hipGetLastError();
}

}  // namespace frm
