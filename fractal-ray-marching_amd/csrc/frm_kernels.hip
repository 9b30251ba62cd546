// frm_kernels.hip — gfx950 kernels of the fractal ray-marcher and their launchers.
//
// The render kernels (render_simple, march_persistent, shade_pass) live in
// frm_render_kernels.h so frm_reload can recompile them at run time; this file adds the
// multi-GPU unshuffle, the presentation blit, the diagnostics kernels (eval_scene,
// eval_math) and the host launchers, which take a reloaded module's kernels when one is
// active (frm_reload.hip).
#include <hip/hip_runtime.h>

#include <cstring>

#include "frm_render_kernels.h"

namespace frm {

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
    case 9: r = x / y; break;
#if defined(__HIP_DEVICE_COMPILE__)  // frm_fast.h is device-only
    case 10: r = sqrt_nosmall(x); break;
    case 11: r = div_tame(x, y); break;
    case 12: r = div_tame_nz(x, y); break;
    case 13: { float c; sincos_small(x, &r, &c); } break;
    case 14: { float s; sincos_small(x, &s, &r); } break;
    case 15: r = acos_dev(x); break;
    case 16: r = atan2_tame(x, y); break;
    case 17: r = log2_tame(x); break;
    case 18: r = exp2_tame(x); break;
    case 19: r = log_posnormal(x); break;
    default: r = (float)encode_srgb(x, kSrgbThresholds); break;
#else
    default: r = x; break;
#endif
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
    case kMandelbulbHw: eval_scene_fam<kMandelbulbHw>(s, pts, n, dist, color, stream); break;
    default: eval_scene_fam<kSphere>(s, pts, n, dist, color, stream); break;
  }
  return hipGetLastError();
}

// Per-pixel trace of the geometric inputs of the shading, from the records of a persistent launch
// (parity tooling, frm_debug_trace; the layout of the oracle's om_render_trace): hit, primary
// steps, normal xyz, sun hit, sun closeness, object colour xyz (hits), zeros for misses.
template <uint32_t FAM>
__global__ __launch_bounds__(256) void trace_pass(KernelArgs a, float* __restrict__ out) {
  const uint32_t width = a.f.width;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= a.npix) return;
  const uint32_t lr = idx / width, x = idx - lr * width;
  const uint32_t y = band_row_to_global(a.g, lr);
  const uint2 r1 = *reinterpret_cast<const uint2*>(&a.tails[idx]);
  float t[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r1.y & kRecHit) {
    const float4 r0 = *reinterpret_cast<const float4*>(&a.geom[idx]);
    const v3 hp = ray_at(a.f.origin, r0.x, camera_ray(a.f, x, y));
    const v3 c = scene_color<FAM>(hp);
    t[0] = 1.f;
    t[1] = (float)(r1.y & kRecStepsMask);
    t[2] = r0.y, t[3] = r0.z, t[4] = r0.w;
    t[5] = (r1.y & kRecSunMiss) ? 0.f : 1.f;
    t[6] = __uint_as_float(r1.x);
    t[7] = c.x, t[8] = c.y, t[9] = c.z;
  }
  for (int k = 0; k < 10; ++k) out[(size_t)idx * 10u + k] = t[k];
}

hipError_t launch_trace(const KernelArgs& a, float* out, hipStream_t stream) {
  const dim3 grid((a.npix + 255u) / 256u);
  switch (a.s.family) {
    case kMenger: hipLaunchKernelGGL(trace_pass<kMenger>, grid, dim3(256), 0, stream, a, out); break;
    case kSierpinski: hipLaunchKernelGGL(trace_pass<kSierpinski>, grid, dim3(256), 0, stream, a, out); break;
    case kKoch: hipLaunchKernelGGL(trace_pass<kKoch>, grid, dim3(256), 0, stream, a, out); break;
    case kMandelbulb: hipLaunchKernelGGL(trace_pass<kMandelbulb>, grid, dim3(256), 0, stream, a, out); break;
    case kMandelbulbHw: hipLaunchKernelGGL(trace_pass<kMandelbulbHw>, grid, dim3(256), 0, stream, a, out); break;
    default: hipLaunchKernelGGL(trace_pass<kSphere>, grid, dim3(256), 0, stream, a, out); break;
  }
  return hipGetLastError();
}

hipError_t launch_eval_math(int fn, const float* a, const float* b, uint32_t n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(eval_math, dim3((n + 255u) / 256u), dim3(256), 0, stream, fn, a, b, n, out);
  return hipGetLastError();
}

static int blocks_override() {  // experiments: FRM_BLOCKS_PER_CU
  const char* env = getenv("FRM_BLOCKS_PER_CU");
  const int v = env ? atoi(env) : 0;
  return v >= 1 && v <= 64 ? v : 0;
}

// A reloaded module's kernel (frm_reload.hip) takes the same KernelArgs by value.
static hipError_t module_launch(hipFunction_t fn, dim3 grid, dim3 block, hipStream_t stream, const KernelArgs& args) {
  void* params[] = {const_cast<KernelArgs*>(&args)};
  return hipModuleLaunchKernel(fn, grid.x, grid.y, grid.z, block.x, block.y, block.z, 0, stream, params, nullptr);
}

// KernelArgs::first_t / first_info: step 0 of each frame's primary rays, evaluated here once per
// frame instead of once per pixel (fragment.wgsl:289-300 at total_distance 0: ray_at(o, 0, d) =
// fma(0, d, o) = o bit for bit, unless a component of o is -0, whose sum with 0 * d would follow
// d's sign). The DE is the kernels' own scene_de built for the host (the exact builtins; the
// device's tame paths give the same bits, tests/native and test_gpu_de), with the power the march
// uses (ANIM: the frame's power, power - 1). The pixels skip the step only when it neither hits
// nor ends the march (distance in (MIN_DISTANCE, MAX_TOTAL_DISTANCE), max_steps >= 2): they then
// start at step 1 with t = 0 + distance, it = 1, the step's bodies in their cost and the step
// counted (primary DE, bodies, bailout) as its consumption would. Not for hardware math (no host
// equivalent) or runtime-reloaded kernels (edited sources).
template <uint32_t FAM, bool ITERS>
static void first_steps(KernelArgs& a, bool anim) {
  a.first_counts[0] = a.first_counts[1] = a.first_counts[2] = 0;
  if constexpr (FAM == kMandelbulbHw) {
    (void)anim;
  } else {
    for (uint32_t k = 0; k < a.batch && k < kMaxBatch; ++k) {
      const v3 o = a.cams[k].origin;
      SceneUniforms u = a.s;
      if (anim) {
        u.mb_power = a.mb_powers[k];
        u.mb_power_m1 = u.mb_power - 1.0f;
      }
      DeCount cnt = {0u, 0u};
      const float de = scene_de<FAM, ITERS>(u, o, cnt);
      uint32_t ob[3];
      memcpy(ob, &o, sizeof(ob));
      const bool neg0 = ob[0] == 0x80000000u || ob[1] == 0x80000000u || ob[2] == 0x80000000u;
      const bool skip = !neg0 && a.f.max_steps >= 2u && de > kMinDistance && de < kMaxTotalDistance;
      a.first_t[k] = 0.0f + de;
      a.first_info[k] = skip ? ((is_mandelbulb(FAM) ? cnt.bodies : 1u) | (cnt.bailouts ? kFirstBail : 0u) | kFirstSkip) : 0u;
      if (skip) {  // every local pixel of the frame is fetched once by this launch
        a.first_counts[0] += a.npix;
        if (is_mandelbulb(FAM)) {
          a.first_counts[1] += (unsigned long long)a.npix * cnt.bodies;
          a.first_counts[2] += cnt.bailouts ? a.npix : 0u;
        }
      }
    }
  }
}

// Every built-in persistent launch, a single frame included, runs the multi-frame instantiation
// (a single frame is a batch of one, its camera in cams[0]): the single-frame one needs 82 VGPRs
// on ROCm 7.2 (5 waves/SIMD), the multi-frame one 80 (6 waves/SIMD).
template <uint32_t FAM, bool ITERS>
static hipError_t launch_persistent(const KernelArgs& args, int cu_count, hipStream_t stream,
                                    const ReloadedKernels* rk, int blocks_cap) {
  // occupancy of each built-in instantiation (per process); reloaded modules query their own
  // (frm_reload.hip)
  static int blocks_per_cu = 0, blocks_per_cu_anim = 0;
  if (blocks_per_cu == 0) {
    int n = 0;
    hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, march_persistent<FAM, ITERS, true>, kMarchBlock, 0);
    if (e != hipSuccess) return e;
    blocks_per_cu = n > 0 ? n : 1;
    blocks_per_cu_anim = blocks_per_cu;
    if constexpr (is_mandelbulb(FAM) && ITERS) {
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, march_persistent<FAM, ITERS, true, true>, kMarchBlock, 0);
      if (e != hipSuccess) return e;
      blocks_per_cu_anim = n > 0 ? n : 1;
    }
  }
  int bpc = rk ? rk->persistent_blocks_per_cu[FAM][ITERS] : (args.anim ? blocks_per_cu_anim : blocks_per_cu);
  if (blocks_cap > 0 && bpc > blocks_cap) bpc = blocks_cap;
  if (const int v = blocks_override()) bpc = v;
  // every wave starts with one chunk of 64 pixels; never launch more waves than chunks
  uint32_t blocks = (uint32_t)(bpc * cu_count);
  const uint32_t positions = args.batch > 1 ? args.batch * ((args.npix + kChunk - 1u) / kChunk) * kChunk : args.npix;
  const uint32_t max_blocks = ((positions + kChunk - 1u) / kChunk + kMarchWaves - 1u) / kMarchWaves;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) blocks = 1;
  const uint32_t pixels = args.g.local_rows * args.f.width;
  const uint32_t shade_blocks = (pixels + kShadeBlockPixels - 1u) / kShadeBlockPixels;
  if (rk) {
    hipError_t e = module_launch(rk->persistent[FAM][ITERS], dim3(blocks), dim3(kMarchBlock), stream, args);
    if (e != hipSuccess) return e;
    return module_launch(rk->shade[FAM], dim3(shade_blocks, args.batch), dim3(256), stream, args);
  }
  KernelArgs m = args;  // + the frames' step 0
  constexpr bool kAnimKernel = is_mandelbulb(FAM) && ITERS;  // the ANIM instantiation exists
  first_steps<FAM, ITERS>(m, kAnimKernel && args.anim);
  if constexpr (kAnimKernel) {
    if (args.anim) {
      hipLaunchKernelGGL((march_persistent<FAM, ITERS, true, true>), dim3(blocks), dim3(kMarchBlock), 0, stream, m);
    } else {
      hipLaunchKernelGGL((march_persistent<FAM, ITERS, true>), dim3(blocks), dim3(kMarchBlock), 0, stream, m);
    }
  } else {
    hipLaunchKernelGGL((march_persistent<FAM, ITERS, true>), dim3(blocks), dim3(kMarchBlock), 0, stream, m);
  }
  hipLaunchKernelGGL((shade_pass<FAM>), dim3(shade_blocks, args.batch), dim3(256), 0, stream, args);
  if (args.key_hist)  // fused scheduling: the slot's next fetch order
    hipLaunchKernelGGL(rank_pass, dim3((args.npix + kShadeBlockPixels - 1u) / kShadeBlockPixels), dim3(256), 0, stream,
                       args.pixel_key, args.npix, args.key_hist, args.order_out);
  return hipGetLastError();
}

template <uint32_t FAM>
static hipError_t launch_family(const KernelArgs& args, KernelKind kind, int cu_count, hipStream_t stream,
                                const ReloadedKernels* rk, int blocks_cap) {
  if (kind == kKernelPersistent)
    return args.s.n ? launch_persistent<FAM, true>(args, cu_count, stream, rk, blocks_cap)
                    : launch_persistent<FAM, false>(args, cu_count, stream, rk, blocks_cap);
  dim3 grid((args.f.width + 15u) / 16u, (args.g.local_rows + 15u) / 16u);
  if (rk) return module_launch(rk->simple[FAM][args.s.n ? 1 : 0], grid, dim3(256), stream, args);
  if (args.s.n)
    hipLaunchKernelGGL((render_simple<FAM, true>), grid, dim3(256), 0, stream, args);
  else
    hipLaunchKernelGGL((render_simple<FAM, false>), grid, dim3(256), 0, stream, args);
  return hipGetLastError();
}

// A resident ring grid (frm_api.hip resident_render): the occupancy limit of the RES instantiation
// (the Mandelbulb's with per-lane powers: ring frames differ in time) over every CU, the first
// args.ring.service_waves workgroups serving the ring (frm_render_kernels.h ring_service).
template <uint32_t FAM, bool ITERS>
static hipError_t launch_ring_fam(const KernelArgs& args, int cu_count, hipStream_t stream, int* out_blocks) {
  constexpr bool kAnim = is_mandelbulb(FAM);
  static int blocks_per_cu = 0;
  if (blocks_per_cu == 0) {
    int n = 0;
    hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, march_persistent<FAM, ITERS, false, kAnim, true>, kMarchBlock, 0);
    if (e != hipSuccess) return e;
    blocks_per_cu = n > 0 ? n : 1;
  }
  int bpc = blocks_per_cu;
  if (const int v = blocks_override()) bpc = v;
  const uint32_t blocks = (uint32_t)(bpc * cu_count);
  if (out_blocks) *out_blocks = (int)blocks;
  if (getenv("FRM_RING_DEBUG")) fprintf(stderr, "frm ring grid: %d blocks per CU (occupancy %d), %u blocks\n", bpc, blocks_per_cu, blocks);
  if (args.ring.service_waves >= blocks) return hipErrorInvalidValue;
  hipLaunchKernelGGL((march_persistent<FAM, ITERS, false, kAnim, true>), dim3(blocks), dim3(kMarchBlock), 0, stream, args);
  return hipGetLastError();
}

template <uint32_t FAM>
static hipError_t launch_ring_family(const KernelArgs& args, int cu_count, hipStream_t stream, int* out_blocks) {
  return args.s.n ? launch_ring_fam<FAM, true>(args, cu_count, stream, out_blocks)
                  : launch_ring_fam<FAM, false>(args, cu_count, stream, out_blocks);
}

hipError_t launch_ring(const KernelArgs& args, int cu_count, hipStream_t stream, int* out_blocks) {
  switch (args.s.family) {
    case kMenger: return launch_ring_family<kMenger>(args, cu_count, stream, out_blocks);
    case kSierpinski: return launch_ring_family<kSierpinski>(args, cu_count, stream, out_blocks);
    case kKoch: return launch_ring_family<kKoch>(args, cu_count, stream, out_blocks);
    case kMandelbulb: return launch_ring_family<kMandelbulb>(args, cu_count, stream, out_blocks);
    case kMandelbulbHw: return launch_ring_family<kMandelbulbHw>(args, cu_count, stream, out_blocks);
    default: return launch_ring_family<kSphere>(args, cu_count, stream, out_blocks);
  }
}

hipError_t launch_render(const KernelArgs& args, KernelKind kind, int cu_count, hipStream_t stream,
                         const ReloadedKernels* rk, int blocks_cap) {
  switch (args.s.family) {
    case kMenger: return launch_family<kMenger>(args, kind, cu_count, stream, rk, blocks_cap);
    case kSierpinski: return launch_family<kSierpinski>(args, kind, cu_count, stream, rk, blocks_cap);
    case kKoch: return launch_family<kKoch>(args, kind, cu_count, stream, rk, blocks_cap);
    case kMandelbulb: return launch_family<kMandelbulb>(args, kind, cu_count, stream, rk, blocks_cap);
    case kMandelbulbHw: return launch_family<kMandelbulbHw>(args, kind, cu_count, stream, rk, blocks_cap);
    default: return launch_family<kSphere>(args, kind, cu_count, stream, rk, blocks_cap);
  }
}

// Presentation resample: the reference's blit pass draws the render
// texture on the window surface (blit.wgsl:6-11) through a clamp-to-edge sampler with linear
// magnification and nearest minification (persistent_graphics.rs:55-64). The texture is
// Rgba8UnormSrgb, so texels are decoded to linear light before filtering; the surface's
// format decides the output encoding (FRM_BLIT_SRGB) and byte order (FRM_BLIT_BGRA).
// One thread per output column of four pixels (rows 16 apart), 16 x 64 output pixels per block.
__device__ __forceinline__ float blit_mix(float a, float b, float t) { return a * (1.0f - t) + b * t; }

__device__ __forceinline__ uint32_t blit_channel(float c, bool srgb, const float* table) {
  if (srgb) return encode_srgb(c, table);                            // exact, NaN -> 0
  return (uint32_t)rintf(fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f);      // unorm, NaN -> 0
}

constexpr uint32_t kBlitRows = 4;  // output rows per thread (16 x 64 output pixels per block)

__global__ __launch_bounds__(256) void blit_kernel(const uint32_t* __restrict__ src, uint32_t sw, uint32_t sh,
                                                   uint32_t* __restrict__ dst, uint32_t dw, uint32_t dh,
                                                   uint32_t flags, uint32_t magnify) {
  __shared__ float dec_t[256], enc[256];
  const uint32_t t = threadIdx.y * 16u + threadIdx.x;
  dec_t[t] = kSrgbDecode[t];
  enc[t] = kSrgbThresholds[t];
  __syncthreads();
  auto dec = [](uint32_t i) { return dec_t[i]; };
  const uint32_t x = blockIdx.x * 16u + threadIdx.x;
  if (x >= dw) return;
  const bool srgb = (flags & 1u) != 0;
  // the quad's varyings (vertex.wgsl:11-13) at this pixel centre, then blit.wgsl:8-9
  const float u = (screen_x(x, dw) + 1.0f) * 0.5f;
  for (uint32_t j = 0; j < kBlitRows; ++j) {
    const uint32_t y = (blockIdx.y * kBlitRows + j) * 16u + threadIdx.y;
    if (y >= dh) return;
    const float v = 1.0f - (screen_y(y, dh) + 1.0f) * 0.5f;
    float r, g, b;
    if (magnify) {  // FilterMode::Linear: 2x2 texels around (u*W - 1/2, v*H - 1/2), clamp to edge
      const float tu = u * (float)sw - 0.5f, tv = v * (float)sh - 0.5f;
      const float fu = floorf(tu), fv = floorf(tv);
      const float a = tu - fu, c = tv - fv;
      const int iu = (int)fu, iv = (int)fv;
      const uint32_t x0 = (uint32_t)min(max(iu, 0), (int)sw - 1), x1 = (uint32_t)min(max(iu + 1, 0), (int)sw - 1);
      const uint32_t y0 = (uint32_t)min(max(iv, 0), (int)sh - 1), y1 = (uint32_t)min(max(iv + 1, 0), (int)sh - 1);
      const uint32_t t00 = src[y0 * sw + x0], t10 = src[y0 * sw + x1], t01 = src[y1 * sw + x0], t11 = src[y1 * sw + x1];
      float ch[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t sh8 = 8u * k;
        const float top = blit_mix(dec((t00 >> sh8) & 255u), dec((t10 >> sh8) & 255u), a);
        const float bot = blit_mix(dec((t01 >> sh8) & 255u), dec((t11 >> sh8) & 255u), a);
        ch[k] = blit_mix(top, bot, c);
      }
      r = ch[0], g = ch[1], b = ch[2];
    } else {  // FilterMode::Nearest
      const uint32_t ix = (uint32_t)min(max((int)floorf(u * (float)sw), 0), (int)sw - 1);
      const uint32_t iy = (uint32_t)min(max((int)floorf(v * (float)sh), 0), (int)sh - 1);
      const uint32_t tx = src[iy * sw + ix];
      r = dec(tx & 255u), g = dec((tx >> 8) & 255u), b = dec((tx >> 16) & 255u);
    }
    const uint32_t cr = blit_channel(r, srgb, enc), cg = blit_channel(g, srgb, enc), cb = blit_channel(b, srgb, enc);
    dst[y * dw + x] = (flags & 2u) ? (cb | (cg << 8) | (cr << 16) | (255u << 24)) : (cr | (cg << 8) | (cb << 16) | (255u << 24));
  }
}

hipError_t launch_blit(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh,
                       uint32_t flags, hipStream_t stream) {
  // mag vs min: texels per output pixel along the more compressed axis (the sampler's LOD)
  const bool magnify = (float)sw / (float)dw <= 1.0f && (float)sh / (float)dh <= 1.0f;
  hipLaunchKernelGGL(blit_kernel, dim3((dw + 15u) / 16u, (dh + 16u * kBlitRows - 1u) / (16u * kBlitRows)), dim3(16, 16), 0, stream,
                     (const uint32_t*)src, sw, sh, (uint32_t*)dst, dw, dh, flags, magnify ? 1u : 0u);
  return hipGetLastError();
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

#ifdef FRM_STAMPS
extern "C" int frm_debug_waves(uint64_t* out, size_t slots) {
  if (slots > frm::kWaveDebugSlots) slots = frm::kWaveDebugSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(frm::g_wave_debug), slots * 128) == hipSuccess ? (int)slots : -1;
}
#endif
