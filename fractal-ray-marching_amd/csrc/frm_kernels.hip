// frm_kernels.hip — gfx950 kernels of the fractal ray-marcher.
//
// render_persistent<FAM>: see below (the default).
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

// ---- persistent ray-regeneration kernel -------------------------------------------
// One lane = one pixel at a time, driven by a per-lane state machine over the phases of
// fragment_main (primary march -> 4 normal taps -> shadow march -> shade). Every loop
// iteration advances every live lane by exactly one unit of DE work: one Mandelbulb loop
// body (the DE is resumable: z, dr, magnitude, body index live in registers), or one
// whole DE for the fixed-trip-count families. A lane whose pixel is finished takes the
// next pixel from a wave-local pool, refilled with one atomic per 8x8 tile from a global
// queue, so lanes never wait for the slowest ray of their wave (SIMD utilisation) and the
// Mandelbulb bailout no longer serialises the wave on its longest DE. Per-pixel arithmetic
// is the same sequence of operations as shade_pixel<>, so the bytes are identical.
constexpr uint32_t kIdle = 0xFFFFFFFFu;
constexpr uint32_t kTile = 64u;  // pixels per queue entry (one 8x8 tile)

enum Phase : uint32_t { kPrimary = 0, kTap0 = 1, kTap3 = 4, kShadow = 5 };

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <uint32_t FAM, bool ITERS>
__global__ __launch_bounds__(256) void render_persistent(KernelArgs a) {
  __shared__ float table[256];
  table[threadIdx.x] = kSrgbThresholds[threadIdx.x];
  __syncthreads();

  const FrameUniforms& f = a.f;
  const SceneUniforms& su = a.s;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lane_bit = 1ull << lane;
  const uint32_t total = a.tiles_total * kTile;
  const uint32_t n_iter = iterations<ITERS>(su.n);

  // wave-uniform pixel pool [pool_next, pool_end)
  uint32_t pool_next = 0, pool_end = 0;
  bool exhausted = false;

  // per-lane state
  uint32_t pix = kIdle;        // local pixel index (x + lr * width) being shaded
  uint32_t phase = kPrimary;
  bool need_point = false;     // start a DE at the phase's next sample point
  bool done = false;           // the current DE has its result
  v3 o = mk(0.f, 0.f, 0.f), d = o, hp = o, color = o, nsum = o, q = o, z = o;
  float t = 0.f, closeness = 0.f, spec = 0.f, dr = 1.f, mag = 0.f, de = 0.f;
  uint32_t it = 0, psteps = 0, body = 0;
  uint32_t c_pix = 0, c_hit = 0, c_prim = 0, c_shadow = 0;
  DeCount cnt = {0u, 0u};

  for (;;) {
    // 1. refill idle lanes from the pool (one global atomic per 8x8 tile)
    uint64_t want = __ballot(pix == kIdle);
    if (want == 0 && exhausted) break;  // unreachable: live lanes keep the wave going
    if (want != 0 && !exhausted) {
      if (pool_next == pool_end) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(a.queue, kTile);
        base = uniform(__shfl(base, 0, 64));
        if (base >= total) {
          exhausted = true;
        } else {
          pool_next = base;
          pool_end = base + kTile;
        }
      }
      if (!exhausted || pool_next != pool_end) {
        const uint32_t avail = pool_end - pool_next;
        const uint32_t rank = __popcll(want & (lane_bit - 1ull));
        if ((want & lane_bit) && rank < avail) {
          // tile-major pixel order: consecutive indices form 8x8 tiles
          const uint32_t idx = pool_next + rank, tile = idx >> 6, in = idx & 63u;
          const uint32_t x = (tile % a.tiles_x) * 8u + (in & 7u);
          const uint32_t lr = (tile / a.tiles_x) * 8u + (in >> 3);
          if (x < f.width && lr < a.g.local_rows) {
            const uint32_t y = band_row_to_global(a.g, lr);
            if (y < f.height) {
              pix = lr * f.width + x;
              c_pix++;
              d = camera_ray(f, x, y);
              o = f.origin;
              t = 0.f;
              it = 0;
              phase = kPrimary;
              need_point = true;
            }
          }
        }
        pool_next += min(avail, (uint32_t)__popcll(want));
      }
    }

    // 2. start the next DE of every lane that needs one
    if (need_point) {
      need_point = false;
      q = (phase - kTap0 <= kTap3 - kTap0) ? normal_tap_pos(hp, (int)(phase - kTap0)) : ray_at(o, t, d);
      if constexpr (FAM == kMandelbulb) {
        z = q;
        dr = 1.f;
        body = 0;
        mag = length(q);
        done = mag > su.mb_bailout;
        if (done) cnt.bailouts++;
      } else {
        de = scene_de<FAM, ITERS>(su, q, cnt);
        done = true;
      }
    }

    // 3. one Mandelbulb body for every lane with a DE in flight
    if constexpr (FAM == kMandelbulb) {
      if (pix != kIdle && !done) {
        mb_body(su, q, mag, z, dr);
        cnt.bodies++;
        body++;
        if (body > n_iter) {
          done = true;  // N+1 bodies: the distance uses the last loop-top magnitude
        } else {
          mag = length(z);
          if (mag > su.mb_bailout) {
            done = true;
            cnt.bailouts++;
          }
        }
      }
    }

    // 4. consume finished DEs: march / normal / shadow bookkeeping, shading
    if (pix != kIdle && done) {
      done = false;
      if constexpr (FAM == kMandelbulb) de = mb_distance(mag, dr);
      bool finished = false;
      float sun_distance = 0.f;
      if (phase == kPrimary) {
        c_prim++;
        if (de <= kMinDistance) {  // hit: object_result.distance = t >= 0
          c_hit++;
          hp = q;
          color = scene_color<FAM>(q);
          psteps = it;
          phase = kTap0;
          need_point = true;
        } else {
          t = t + de;
          it++;
          if (it < f.max_steps && t < kMaxTotalDistance) {
            need_point = true;
          } else {  // miss: BACKGROUND_COLOR
            a.out[pix] = 255u << 24;
            pix = kIdle;
          }
        }
      } else if (phase != kShadow) {  // normal taps k.xyy, k.yyx, k.yxy, k.xxx
        if (phase == kTap0) nsum = mk(de, -de, -de);
        else if (phase == kTap0 + 1) nsum = mk(nsum.x - de, nsum.y - de, nsum.z + de);
        else if (phase == kTap0 + 2) nsum = mk(nsum.x - de, nsum.y + de, nsum.z - de);
        else nsum = mk(nsum.x + de, nsum.y + de, nsum.z + de);
        if (phase == kTap3) {
          v3 n = normalize(nsum);
          color = shade_hit_pre(f, color, d, n, psteps, &spec);
          o = shadow_origin(hp, n);
          d = to_sun();
          t = 0.f;
          it = 0;
          closeness = kInfinity;
          phase = kShadow;
        } else {
          phase++;
        }
        need_point = true;
      } else {  // shadow march toward the sun
        c_shadow++;
        closeness = min_(closeness, de / t);
        if (de <= kMinDistance) {
          finished = true;
          sun_distance = t;
        } else {
          t = t + de;
          it++;
          if (it < f.max_steps && t < kMaxTotalDistance) need_point = true;
          else {
            finished = true;
            sun_distance = -kInfinity;
          }
        }
      }
      if (finished) {
        a.out[pix] = pack_rgba(shade_hit_post(color, spec, sun_distance, closeness), table);
        pix = kIdle;
      }
    }

    if (exhausted && __ballot(pix != kIdle) == 0) break;
  }

  unsigned long long v[7] = {c_pix, c_hit, c_prim, c_shadow, 4ull * c_hit, cnt.bodies, cnt.bailouts};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    unsigned long long sum = wave_sum(v[k]);
    if (lane == 0 && sum) atomicAdd(&a.counters[k], sum);
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

template <uint32_t FAM, bool ITERS>
static hipError_t launch_persistent(const KernelArgs& args, int cu_count, hipStream_t stream) {
  static int blocks_per_cu = 0;  // occupancy of this instantiation (per process)
  if (blocks_per_cu == 0) {
    int n = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, render_persistent<FAM, ITERS>, 256, 0);
    if (e != hipSuccess) return e;
    blocks_per_cu = n > 0 ? n : 1;
  }
  // every wave starts with one 8x8 tile; never launch more waves than tiles
  uint32_t blocks = (uint32_t)(blocks_per_cu * cu_count);
  const uint32_t max_blocks = (args.tiles_total + 3u) / 4u;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL((render_persistent<FAM, ITERS>), dim3(blocks), dim3(256), 0, stream, args);
  return hipGetLastError();
}

template <uint32_t FAM>
static hipError_t launch_family(const KernelArgs& args, KernelKind kind, int cu_count,
                                hipStream_t stream) {
  if (kind == kKernelPersistent)
    return args.s.n ? launch_persistent<FAM, true>(args, cu_count, stream)
                    : launch_persistent<FAM, false>(args, cu_count, stream);
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
