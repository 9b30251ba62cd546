/*
 * frm.h — C ABI of the MI355X-native offscreen fractal ray-marcher (libfrm.so).
 *
 * This is the drop-in boundary that replaces the reference's wgpu graphics layer
 * (MariusDoe/fractal-ray-marching: src/graphics.rs, src/persistent_graphics.rs,
 * src/reloadable_graphics.rs, src/blit_graphics.rs) for the one hot path the
 * reference has: the per-pixel sphere tracer `fragment_main` in src/fragment.wgsl:327-349.
 * The caller keeps the reference's own `Parameters` uniform (src/parameters.rs:6-15)
 * byte for byte; `frm_parameters` below is that struct.
 *
 * Conventions
 *   - Every entry point returns an `int` status (FRM_OK = 0). Nothing aborts, throws
 *     or panics across the ABI. The message of the last failure on a context is
 *     available from frm_last_error(); failures before a context exists are available
 *     from frm_last_error(NULL) (thread-local).
 *   - A context drives one GPU, or with frm_config.device_count a group of GPUs row-tiling
 *     each frame, and is not thread-safe (one context per host thread), mirroring the
 *     reference's single winit event-loop thread (src/app.rs).
 *   - Rendering is stream-ordered. frm_render() with a NULL stats pointer is
 *     asynchronous; frm_read_frame()/frm_synchronize() wait for it. With
 *     frames_in_flight > 1, consecutive frm_render() calls run on rotating streams and
 *     may overlap on the GPU; frm_read_frame()/frm_present() see the last one.
 *   - Plain pointers and sizes only; `void* stream` is a hipStream_t (NULL = the
 *     context's own stream).
 */
#ifndef FRM_H
#define FRM_H

#if !defined(__HIPCC_RTC__) /* hiprtc (frm_reload) defines the fixed-width types itself */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define FRM_ABI_VERSION 5u  /* 2: frm_config.frames_in_flight (was reserved); 3: frm_render_bands_batch
                               takes dst_bytes, frm_set_parameters bounds the fractal loop work;
                               4: asynchronous readback (frm_read_frame_async, frm_present_async,
                               frm_frame_pixels); 5: frm_config.device_count / devices (one context
                               row-tiles every frame over several GPUs, RCCL gather) */

/* ---- status codes -------------------------------------------------------- */
enum {
  FRM_OK = 0,
  FRM_ERR_INVALID_ARGUMENT = 1, /* NULL pointer, zero size, out-of-range value       */
  FRM_ERR_NO_DEVICE = 2,        /* no HIP device / device index out of range          */
  FRM_ERR_HIP = 3,              /* a HIP runtime call failed (message has the name)   */
  FRM_ERR_OUT_OF_MEMORY = 4,    /* device allocation failed                           */
  FRM_ERR_NOT_READY = 5,        /* frm_render before frm_resize / frm_set_parameters  */
  FRM_ERR_BUFFER_TOO_SMALL = 6, /* destination smaller than the frame or band set      */
  FRM_ERR_UNSUPPORTED = 7,      /* an operation this build does not support            */
  FRM_ERR_COMPILE = 8           /* frm_reload: the sources failed to compile (log in last_error) */
};

/* ---- the reference's uniform, byte for byte -------------------------------
 * src/parameters.rs:6-15 (#[repr(C)], bytemuck Pod) mirrored in WGSL at
 * src/fragment.wgsl:108-116. Offsets: camera_matrix 0, aspect_scale 64, time 72,
 * num_iterations 76, scene_index 80, padding 84; sizeof == 96.
 * camera_matrix holds the TRANSPOSE of the cgmath camera matrix in column-major
 * order (parameters.rs:23-25), i.e. camera_matrix[4*j + i] = C[row j][col i]; the
 * kernel computes C·v exactly like `(v * camera_matrix)` in fragment.wgsl:315-317. */
typedef struct frm_parameters {
  float camera_matrix[16];
  float aspect_scale[2];
  float time;
  uint32_t num_iterations;
  uint32_t scene_index;
  uint8_t padding[12];
} frm_parameters;

#if defined(__HIPCC_RTC__)
static_assert(sizeof(frm_parameters) == 96, "frm_parameters must be 96 bytes");
#elif defined(__cplusplus)
static_assert(sizeof(frm_parameters) == 96, "frm_parameters must be 96 bytes");
static_assert(offsetof(frm_parameters, aspect_scale) == 64, "aspect_scale @64");
static_assert(offsetof(frm_parameters, time) == 72, "time @72");
static_assert(offsetof(frm_parameters, num_iterations) == 76, "num_iterations @76");
static_assert(offsetof(frm_parameters, scene_index) == 80, "scene_index @80");
#else
_Static_assert(sizeof(frm_parameters) == 96, "frm_parameters must be 96 bytes");
#endif

#define FRM_NUM_SCENES 19u            /* parameters.rs:35 (NUM_SCENES)                 */
#define FRM_DEFAULT_MAX_STEPS 5000u   /* fragment.wgsl:4 (MAX_ITERATIONS)              */
/* Largest fractal loop trip count (Menger/Koch/Sierpinski folds, Mandelbulb bodies - 1) that
 * frm_set_parameters accepts without FRM_FLAG_UNBOUNDED_ITERATIONS. num_iterations is any u32
 * in the reference (update_num_iterations saturates, parameters.rs:31-33), and every DE runs
 * O(num_iterations) loop bodies (fragment.wgsl:181,207,226,245), so a frame near 2^32 runs for
 * days; such parameters get FRM_ERR_UNSUPPORTED unless the context opted out. Sierpinski's
 * i32 loop runs no fold for N >= 2^31 (fragment.wgsl:181), which is cheap and always accepted.
 * The Mandelbulb's `i <= N` loop (fragment.wgsl:245) never ends for N = 0xffffffff (the u32
 * counter wraps first; the reference hangs too): refused even with the opt-out. */
#define FRM_MAX_NUM_ITERATIONS 65536u
#define FRM_MAX_DIMENSION 32768u      /* width/height limit per frame                  */

/* config flags */
#define FRM_FLAG_SCENE_SPHERE 0x1u  /* build-only extension scene for BASELINE config C1:
                                       DE = length(p) - 0.5, colour = colorize(p). Not in
                                       the reference (its out-of-range scene ids map to 0). */
#define FRM_FLAG_SIMPLE_KERNEL 0x2u /* use the one-thread-per-pixel kernel instead of the
                                       persistent ray-regeneration kernel (same bytes). */
#define FRM_FLAG_PERSISTENT_KERNEL 0x4u /* always use the persistent kernel. With neither
                                       kernel flag the context picks per launch: simple
                                       below one resident persistent grid of pixels
                                       (frm_kernel_for_pixels), persistent above. */
#define FRM_FLAG_UNBOUNDED_ITERATIONS 0x8u /* accept num_iterations above FRM_MAX_NUM_ITERATIONS
                                       (the caller accepts frames whose cost grows with it) */
#define FRM_FLAG_HW_MATH 0x10u      /* OPT-IN, NOT BIT-EXACT: the Mandelbulb (scene 18) body, magnitude
                                       and distance on the GPU's hardware transcendentals (v_log,
                                       v_exp, v_sin, v_cos, v_sqrt, v_rcp), as a Vulkan driver lowers
                                       fragment.wgsl's builtins (WGSL leaves their precision to the
                                       implementation). Faster; frames differ from the oracle's and
                                       are checked by the classified comparison against precise
                                       builtins. Other scenes and the shading
                                       are unchanged (exact). Never the default. */

/* kernels (frm_kernel_for_pixels) */
#define FRM_KERNEL_PERSISTENT 0u
#define FRM_KERNEL_SIMPLE 1u

typedef struct frm_config {
  int32_t device;     /* HIP device ordinal (replaces the wgpu adapter request,
                         persistent_graphics.rs:43-50)                                 */
  uint32_t max_steps; /* march() step cap; 0 = FRM_DEFAULT_MAX_STEPS, at most
                         FRM_MAX_STEPS_LIMIT. It also feeds the ambient-occlusion term
                         (fragment.wgsl:289,342)                                         */
  uint32_t flags;     /* FRM_FLAG_*                                                    */
  uint32_t frames_in_flight; /* frames a context may have in flight on the GPU at once,
                         1..FRM_MAX_FRAMES_IN_FLIGHT (0 = 1). Each render launch (frm_render,
                         frm_render_bands) takes the next of this many slots of device scratch
                         (pixel records, scheduling arrays, work queue; frm_render: also a
                         framebuffer and a stream), so frame k+1 runs while frame k's longest
                         pixels finish instead of after them. No reference counterpart: the
                         reference renders one frame per submit (graphics.rs:91-110).        */
  uint32_t device_count; /* 0: one GPU, `device` (every field above as before). 1..FRM_MAX_DEVICES:
                         a GROUP context over devices[0..device_count-1] (`device` ignored): every
                         frm_render row-tiles the frame over those GPUs (device r renders the
                         interleaved bands r, r+N, ..., as frm_render_bands with first_band r and
                         band_stride N), gathers the bands on devices[0] with RCCL point-to-point
                         transfers over xGMI (grouped ncclSend/ncclRecv; device-to-device copies
                         when a device is listed twice, e.g. to rehearse N ranks on one GPU) and
                         reassembles the frame there; frm_read_frame, frm_present and their async
                         forms then see the whole frame, exactly as on one GPU. The per-rank band
                         entry points (frm_render_bands*, frm_unshuffle_bands, frm_debug_trace,
                         frm_debug_*_pixel_keys) are FRM_ERR_UNSUPPORTED on a group. No reference
                         counterpart (the reference is single-device, graphics.rs:25-37).       */
  int32_t devices[16];  /* HIP device ordinals of a group (FRM_MAX_DEVICES)                        */
} frm_config;

#define FRM_MAX_FRAMES_IN_FLIGHT 8u
#define FRM_MAX_DEVICES 16u
/* Band height a group context uses for a frame of `height` rows over `devices` GPUs: the smallest
 * height >= 16 that splits the frame into a multiple of `devices` bands (else 16), so the
 * interleaved bands balance the devices' work. */
int frm_group_band_rows(uint32_t height, uint32_t devices, uint32_t* out_band_rows);
/* largest frm_config.max_steps: the persistent kernel packs a pixel's primary step count
   into 22 bits of its 8-byte record (the reference's MAX_ITERATIONS is 5000) */
#define FRM_MAX_STEPS_LIMIT 4194303u

/* Work counters of one render (exact; equal to the CPU oracle's counts). */
typedef struct frm_stats {
  uint64_t pixels;          /* pixels shaded                                           */
  uint64_t hit_pixels;      /* primary march hits (distance >= 0, fragment.wgsl:334)   */
  uint64_t primary_steps;   /* scene() evaluations inside the primary march loop       */
  uint64_t shadow_steps;    /* scene() evaluations inside the shadow march loop        */
  uint64_t normal_evals;    /* scene() evaluations in calculate_normal (4 per hit)     */
  uint64_t fractal_bodies;  /* Mandelbulb loop bodies that ran to completion           */
  uint64_t fractal_bailouts;/* Mandelbulb loop exits by bailout                        */
  uint64_t march_steps;     /* primary_steps + shadow_steps (the headline unit)        */
  uint64_t wom_ops;         /* algorithmic VALU lane-ops of the frame */
  double kernel_ms;         /* device time of the render kernel(s) (HIP events)        */
} frm_stats;

typedef struct frm_ctx frm_ctx;

/* ---- lifecycle (replaces Graphics::init, graphics.rs:25-37) ------------------ */
int frm_create(frm_ctx** out_ctx, const frm_config* config);
int frm_destroy(frm_ctx* ctx);
const char* frm_last_error(const frm_ctx* ctx);
uint32_t frm_abi_version(void);
int frm_device_count(int32_t* out_count);

/* ---- frame size (replaces BlitGraphics::init / update_render_texture_size,
 *      graphics.rs:54-57, render_texture_config.rs:1-22). Sizes the device RGBA8
 *      framebuffer(s), pitch = 4*width. The caller sets aspect_scale with
 *      frm_parameters_update_aspect(width, height) semantics (parameters.rs:18-21).
 *      Asynchronous: frames in flight finish at their own size and their pending
 *      readbacks (frm_read_frame_async tickets) keep their bytes; the buffers of the new
 *      size are allocated in stream order (no host wait), as a wgpu texture re-creation
 *      does not stall the frames already submitted. */
int frm_resize(frm_ctx* ctx, uint32_t width, uint32_t height);

/* ---- uniform upload (replaces Graphics::update_parameters_buffer,
 *      graphics.rs:59-61 → queue.write_buffer, persistent_graphics.rs:167-173).
 *      The struct is copied; it reaches the kernel by value. FRM_ERR_UNSUPPORTED (the previous
 *      parameters stay) when the scene's fractal loop would exceed FRM_MAX_NUM_ITERATIONS trips
 *      on a context without FRM_FLAG_UNBOUNDED_ITERATIONS, or never end (see above). */
int frm_set_parameters(frm_ctx* ctx, const frm_parameters* parameters);

/* ---- draw (replaces Graphics::render, graphics.rs:91-110). One full frame into
 *      the context framebuffer. stats == NULL: asynchronous. stats != NULL: waits
 *      for every frame in flight, then for this one, and fills the counters and
 *      kernel time. */
int frm_render(frm_ctx* ctx, frm_stats* stats);

/* ---- readback (replaces the blit pass + present, graphics.rs:101-108). Copies the
 *      whole RGBA8 sRGB frame (row 0 = top, 4*width*height bytes) to host memory. */
int frm_read_frame(frm_ctx* ctx, uint8_t* dst, size_t dst_bytes);

/* Present the last rendered frame at out_width x out_height into host dst (RGBA8 or BGRA8,
 * pitch 4*out_width): the reference's blit pass, which draws the render texture on the
 * window surface (blit.wgsl:6-11; graphics.rs:91-110) through a clamp-to-edge sampler with
 * linear magnification and nearest minification (persistent_graphics.rs:55-64), texels
 * read as linear light (the texture is Rgba8UnormSrgb, blit_graphics.rs:14). The surface
 * format is platform-chosen (persistent_graphics.rs:95): FRM_BLIT_SRGB encodes the output
 * as sRGB (an ...UnormSrgb surface) instead of linear unorm, FRM_BLIT_BGRA writes B,G,R,A.
 * Synchronous. Same size + FRM_BLIT_SRGB reproduces frm_read_frame's bytes. */
#define FRM_BLIT_SRGB 0x1u
#define FRM_BLIT_BGRA 0x2u
int frm_present(frm_ctx* ctx, uint32_t out_width, uint32_t out_height, uint32_t flags, uint8_t* dst,
                size_t dst_bytes);
int frm_synchronize(frm_ctx* ctx);

/* ---- asynchronous readback: presentation with a frame of latency, as the reference's
 *      surface has it. The reference configures its surface with wgpu's default
 *      (persistent_graphics.rs:158-162, Surface::get_default_config:
 *      desired_maximum_frame_latency = 2): present() and submit() return before the GPU has
 *      drawn the frame, so the CPU prepares frame k+1 while frame k renders. With
 *      frames_in_flight >= 2 the same loop on libfrm is
 *          frm_render(k); frm_read_frame_async(&t[k]);      (both return at once)
 *          frm_frame_pixels(t[k-1], &pixels);                (waits for frame k-1 only)
 *      so frame k is already queued behind frame k-1 and fills the GPU while frame k-1's
 *      longest pixels finish.
 * frm_read_frame_async: enqueues the copy of the last frm_render's frame (frm_read_frame's
 *      bytes) into a library-owned pinned host image of that frame's slot; returns a ticket.
 * frm_present_async: the same for frm_present's blit output (out size, FRM_BLIT_* flags).
 * frm_frame_pixels: waits for a ticket's copy and returns its pixels (4*w*h bytes, row 0 =
 *      top). The image belongs to the render slot: it stays valid until frames_in_flight
 *      further frm_render calls have been made (a later async readback of the same slot
 *      replaces it); an expired or unknown ticket gives FRM_ERR_INVALID_ARGUMENT. */
int frm_read_frame_async(frm_ctx* ctx, uint64_t* out_ticket);
int frm_present_async(frm_ctx* ctx, uint32_t out_width, uint32_t out_height, uint32_t flags,
                      uint64_t* out_ticket);
int frm_frame_pixels(frm_ctx* ctx, uint64_t ticket, const uint8_t** out_pixels, size_t* out_bytes);

/* The kernel (FRM_KERNEL_*) a render or band launch of `pixels` pixels runs on this
 * context: the FRM_FLAG_*_KERNEL flag when set, otherwise FRM_KERNEL_SIMPLE when pixels
 * is below one resident persistent grid (1536 lanes per CU) and FRM_KERNEL_PERSISTENT
 * from there on. No reference counterpart (the reference has one fragment pipeline). */
int frm_kernel_for_pixels(const frm_ctx* ctx, uint64_t pixels, uint32_t* out_kernel);

/* Runtime kernel reload (the reference's `r` key: graphics.rs:39-48, reloadable_graphics.rs:
 * 15-52). Recompiles the render kernels with hiprtc from source_dir, a directory holding an
 * edited copy of this package's csrc/ headers (frm_render_kernels.h and the headers it
 * includes: scenes, distance estimators, builtins, shading), and renders every later frame
 * of this context with them. On failure (FRM_ERR_COMPILE, log in frm_last_error) the
 * previous kernels stay active, as the reference keeps its pipeline. source_dir = NULL
 * returns to the built-in kernels. Waits for the context's stream. */
int frm_reload(frm_ctx* ctx, const char* source_dir);

/* ---- row-tiled rendering for multi-GPU (no reference counterpart: the reference
 *      is single-device). Band b covers frame rows [b*band_rows, (b+1)*band_rows).
 *      This call renders bands first_band, first_band+band_stride, ... (below
 *      num_bands(H)) and stores them back to back, band-major, at dev_dst (device
 *      memory of this context's GPU), each row 4*width bytes. `stream` is a
 *      hipStream_t (NULL = context stream). dev_counters, if not NULL, is device
 *      memory of FRM_NUM_COUNTERS uint64 to which the work counters are ADDED.
 *      Asynchronous. With frames_in_flight = F the launch uses the next of F scratch
 *      slots; a slot last used on another stream is awaited on the device, so a caller
 *      that rotates F streams (and F destination buffers) overlaps F launches. */
#define FRM_NUM_COUNTERS 8u
int frm_band_rows_for(uint32_t height, uint32_t band_rows, uint32_t first_band,
                      uint32_t band_stride, uint32_t* out_rows);
int frm_render_bands(frm_ctx* ctx, uint8_t* dev_dst, size_t dst_bytes, uint32_t band_rows,
                     uint32_t first_band, uint32_t band_stride, void* stream,
                     uint64_t* dev_counters);
/* Multi-frame launch: renders `count` frames (1..FRM_MAX_BATCH) of the context's size in ONE
 * launch, frame k with params[k], each as frm_render_bands would render it (this rank's bands,
 * band-major) into dev_dst + k * frame_stride_bytes. The frames' pixels share one work queue
 * (each frame's pixels longest first, the frames interleaved), so one frame's longest pixels
 * run beside the other frames' work instead of ending a launch with idle lanes: for short
 * launches (a rank's share of a row-split frame) the persistent kernel's tail is paid once
 * per batch. The frames may differ in camera, and the Mandelbulb's (scene 18) in time too (its
 * power is its one time-derived constant, fragment.wgsl:75; each lane then carries its frame's
 * power): otherwise params[k] must give the same scene, num_iterations, time-derived scene
 * constants and aspect as params[0] (FRM_ERR_INVALID_ARGUMENT otherwise). A scripted
 * fly-through (the CLI's, bench.py's HEADLINE_FLY) so renders several of its frames per launch. The context's parameters become params[count-1].
 * Counters are added over all frames. Bytes per frame are those of frm_render_bands; dev_dst
 * holds dst_bytes bytes, at least (count - 1) * frame_stride_bytes + one frame's bands
 * (FRM_ERR_BUFFER_TOO_SMALL otherwise); frame_stride_bytes is a multiple of 4 below 16 GiB. */
#define FRM_MAX_BATCH 32u
int frm_render_bands_batch(frm_ctx* ctx, uint32_t count, const frm_parameters* params,
                           uint8_t* dev_dst, size_t dst_bytes, size_t frame_stride_bytes, uint32_t band_rows,
                           uint32_t first_band, uint32_t band_stride, void* stream,
                           uint64_t* dev_counters);
/* Reassemble a frame from per-rank band buffers laid out rank-major in dev_src
 * (rank r's buffer starts at r*rank_stride_bytes, as written by frm_render_bands with
 * first_band = r, band_stride = ranks) into row-major dev_dst. Asynchronous. */
int frm_unshuffle_bands(frm_ctx* ctx, const uint8_t* dev_src, size_t rank_stride_bytes,
                        uint8_t* dev_dst, size_t dst_bytes, uint32_t band_rows,
                        uint32_t ranks, void* stream);
/* Convert FRM_NUM_COUNTERS raw counters (host copy) to frm_stats for the context's
 * current parameters (fills wom_ops; kernel_ms = 0). */
int frm_stats_from_counters(const frm_ctx* ctx, const uint64_t* counters, frm_stats* out);

/* ---- diagnostics (parity tooling; synchronous, host pointers) -------------------
 * frm_eval_scene: evaluates the current scene's distance estimator and object colour
 * (scene(position), fragment.wgsl:18-78) at n points (xyz interleaved) on the GPU.
 * frm_eval_math: evaluates one frm builtin on the GPU, element-wise; fn = FRM_MATH_*. */
enum {
  FRM_MATH_SIN = 0, FRM_MATH_COS = 1, FRM_MATH_ACOS = 2, FRM_MATH_ATAN2 = 3,
  FRM_MATH_LOG = 4, FRM_MATH_LOG2 = 5, FRM_MATH_EXP2 = 6, FRM_MATH_POW = 7,
  FRM_MATH_SQRT = 8, FRM_MATH_DIV = 9,
  /* device fast paths (bit-identical to the builtin above on their stated domain, used by
     the Mandelbulb body when a whole wave qualifies; csrc/frm_fast.h) */
  FRM_MATH_SQRT_NOSMALL = 10, FRM_MATH_DIV_TAME = 11, FRM_MATH_DIV_TAME_NZ = 12,
  FRM_MATH_SIN_SMALL = 13, FRM_MATH_COS_SMALL = 14, FRM_MATH_ACOS_DEV = 15,
  FRM_MATH_ATAN2_TAME = 16, FRM_MATH_LOG2_TAME = 17, FRM_MATH_EXP2_TAME = 18,
  FRM_MATH_LOG_POSNORMAL = 19,
  /* the Rgba8UnormSrgb store's 8-bit code of a linear value (as a float; csrc/frm_scene.h) */
  FRM_MATH_SRGB_ENCODE = 20
};
int frm_eval_scene(frm_ctx* ctx, const float* points, uint32_t n, float* out_distance,
                   float* out_color);
int frm_eval_math(frm_ctx* ctx, int32_t fn, const float* a, const float* b, uint32_t n,
                  float* out);
/* frm_debug_pixel_keys: the 8-bit scheduling cost keys (16 log2(bodies + 1), csrc/frm_sched.hip)
 * the context's last persistent launch recorded per local pixel, row-major; copies
 * min(n, pixels) bytes and returns that count, or a negative frm_status. */
int frm_debug_pixel_keys(frm_ctx* ctx, uint8_t* out, size_t n);
/* frm_debug_set_pixel_keys: replaces the keys the next persistent launch orders its pixels by
 * (n = width x height; the next slot must hold a whole frame of the current size). */
int frm_debug_set_pixel_keys(frm_ctx* ctx, const uint8_t* keys, size_t n);

/* frm_debug_trace: the geometric inputs of the shading of every pixel of the last frm_render (a
 * whole frame on the persistent kernel, with the size and parameters that render used; refused
 * with FRM_ERR_NOT_READY when a later launch has reused its slot), 10 floats per
 * pixel, row-major, in the layout of the oracle's per-pixel trace: hit, primary steps, normal xyz,
 * sun hit, sun closeness, object colour xyz (hits; zeros for misses). Parity tooling for frames
 * that are not bit-exact by design (FRM_FLAG_HW_MATH). n_floats >= 10 x width x height. */
int frm_debug_trace(frm_ctx* ctx, float* out, size_t n_floats);

/* ---- host-side mirrors of the reference's Parameters mutators (src/parameters.rs).
 *      These let a C/C++/Python host drive the same uniform without Rust. */
void frm_parameters_default(frm_parameters* p);                               /* #[derive(Default)] */
void frm_parameters_update_aspect(frm_parameters* p, uint32_t w, uint32_t h); /* parameters.rs:18-21 */
void frm_parameters_update_time(frm_parameters* p, float delta);             /* parameters.rs:27-29 */
void frm_parameters_update_num_iterations(frm_parameters* p, int32_t delta); /* parameters.rs:31-33 */
void frm_parameters_update_scene_index(frm_parameters* p, int32_t delta);    /* parameters.rs:37-40 */
/* parameters.rs:23-25 with Camera::to_matrix (camera.rs:26-44):
 * camera_matrix = transpose(T(position) * Ry(yaw) * Rx(pitch)), column-major. */
void frm_parameters_update_camera(frm_parameters* p, const float position[3], float yaw,
                                  float pitch);

/* ---- animation driver: host-side restatement of the reference's Camera (src/camera.rs)
 *      and Timing (src/timing.rs), for scripted fly-throughs without a window (SURVEY
 *      §8(f) row 2). Keyboard/mouse input becomes explicit arguments: held keys as a
 *      FRM_KEY_* bit set (held_keys.rs), the frame time as seconds (timing.rs uses
 *      Instant::now). All arithmetic is f32 in cgmath's operation order. */
#define FRM_KEY_MOVE_FORWARD (1u << 0)  /* held_keys.rs:6-17 */
#define FRM_KEY_MOVE_BACKWARD (1u << 1)
#define FRM_KEY_MOVE_RIGHT (1u << 2)
#define FRM_KEY_MOVE_LEFT (1u << 3)
#define FRM_KEY_MOVE_UP (1u << 4)
#define FRM_KEY_MOVE_DOWN (1u << 5)
#define FRM_KEY_PITCH_UP (1u << 6)
#define FRM_KEY_PITCH_DOWN (1u << 7)
#define FRM_KEY_YAW_RIGHT (1u << 8)
#define FRM_KEY_YAW_LEFT (1u << 9)

enum { /* camera.rs:16-23 */
  FRM_LOCK_YAW_NONE = 0,
  FRM_LOCK_YAW_INWARDS = 1,
  FRM_LOCK_YAW_RIGHT = 2,
  FRM_LOCK_YAW_OUTWARDS = 3,
  FRM_LOCK_YAW_LEFT = 4
};

typedef struct frm_camera { /* camera.rs:5-14 */
  float position[3];
  float pitch;                  /* radians, clamped to [-pi/2, pi/2]          */
  float yaw;                    /* radians, kept in (-2pi, 2pi) by fmod        */
  float movement_per_second;
  float orbit_angle_per_second; /* radians per second about the y axis         */
  int32_t lock_yaw_mode;        /* FRM_LOCK_YAW_*                              */
  int32_t lock_pitch;           /* bool                                        */
} frm_camera;

void frm_camera_default(frm_camera* c);                                  /* camera.rs:176-188 */
void frm_camera_update(frm_camera* c, uint32_t held_keys, float seconds); /* camera.rs:100-147 */
void frm_camera_update_speed(frm_camera* c, float delta);                /* camera.rs:60-62 */
void frm_camera_update_orbit_speed(frm_camera* c, float delta);          /* camera.rs:64-69 */
void frm_camera_reset_orbit_speed(frm_camera* c);                        /* camera.rs:71-73 */
void frm_camera_toggle_lock_pitch(frm_camera* c);                        /* camera.rs:75-77 */
void frm_camera_cycle_lock_yaw_mode(frm_camera* c, int32_t backwards);   /* camera.rs:79-98 */
void frm_camera_rotate_from_cursor(frm_camera* c, float yaw_pixels,
                                   float pitch_pixels);                  /* camera.rs:151-154 */
void frm_parameters_update_camera_from(frm_parameters* p, const frm_camera* c); /* parameters.rs:23-25 */

typedef struct frm_timing { /* timing.rs:5-10, minus the wall clock and the FPS log */
  float time_factor;
} frm_timing;

void frm_timing_init(frm_timing* t);                                     /* timing.rs:13-21 */
/* parameters.time += time_factor * delta_seconds (timing.rs:23-30); returns delta_seconds */
float frm_timing_update(frm_timing* t, frm_parameters* p, float delta_seconds);
void frm_timing_update_time_factor(frm_timing* t, float delta);          /* timing.rs:32-34 */
void frm_timing_stop_time(frm_timing* t);                                /* timing.rs:36-38 */

#ifdef __cplusplus
}
#endif
#endif /* FRM_H */
