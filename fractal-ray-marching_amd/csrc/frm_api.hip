// frm_api.hip — the C ABI of include/frm.h: context lifetime, device buffers, uniform
// upload, frame dispatch and readback. Replaces the reference's wgpu host layer
// (graphics.rs:25-164, persistent_graphics.rs:33-173, blit_graphics.rs:16-62).
// Errors never cross the ABI as exceptions/aborts: every HIP failure becomes a status
// code plus a message retrievable with frm_last_error().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>

#include <new>
#include <string>
#include <vector>

#include "frm.h"
#include "frm_internal.h"

using namespace frm;

// Mandelbulb persistent kernel: lanes that must be waiting before a wave runs its service
// pass (tuning knob; FRM_SERVICE_MIN overrides it for experiments).
static constexpr uint32_t kDefaultServiceMin = 24;  // swept 16..36 on MI355X (round 1: 20); round-2 kernel: headline 16/20/24/28 = 11.43/11.36/11.18/11.24 ms, C2 flat
// Kernel choice without a FRM_FLAG_*_KERNEL flag: below one resident persistent grid
// (6 blocks of 256 lanes per CU for the Mandelbulb) a launch has fewer pixels than lanes,
// and the persistent kernel's fixed costs (pixel sort, grid, separate shading pass) outweigh
// its load balancing: 256x256 runs 23 G steps/s simple vs 10 persistent, 1920x1080 8 vs 20.
static constexpr uint64_t kSimplePixelsPerCu = 1536;
// Queue positions a launch may claim beyond its pixels (2 chunks per wave of a grid of up to
// 2^17 waves); launches are limited to 2^32 - 1 - this many fetch positions.
static constexpr uint64_t kQueueHeadroom = 1ull << 24;
// Persistent grid of a single-frame launch on a context with frames in flight (launch()), for
// launches of up to kInflightCapPixels pixels (four 4K frames: 8K): the capped grids of two frames
// fill the CUs side by side (8K drop-in loop 37.6 -> 36.2 ms/frame). A larger frame's boundary is
// a small part of its time and the cap costs more than it gains (C5, 16384^2: 3 in flight 533-547
// ms/frame capped against 489-491 at the occupancy limit, 2 in flight 578 against 511;
// profiles/round5/c5cap, c4cap, final/configs).
// 16 = half the 8-wave kernel's occupancy (sweep 12/14/16/32 on the drop-in loop: 8.22 / 8.03 /
// 7.90 / 8.55 ms fixed, 8.96 / 8.82 / 8.71 / 9.87 moving; profiles/round5/dropin_bpc8; with the
// round-5 7-wave kernel 12 was best, profiles/round5/dropin_bpc).
// With F frames in flight the cap is the kernel's occupancy (32 workgroups per CU) over F, so the F
// grids fit side by side (round 6, one rank's 8-way share of the headline, one frame per launch:
// 3 in flight 1.49 ms at 16 per CU, 1.21 at 10-11; 4 in flight 1.09 at 8; 2 in flight 16 stays best,
// 1.53-1.56 at 12-20; profiles/round6/share/). F = 2 gives the 16 above.
static constexpr int kInflightBlocksPerCu = 16;
static int inflight_blocks_per_cu(uint32_t frames_in_flight) {
  return frames_in_flight <= 2u ? kInflightBlocksPerCu : (int)(2u * kInflightBlocksPerCu / frames_in_flight);
}
static constexpr uint64_t kInflightCapPixels = 4ull * 3840u * 2160u;
// Single-frame launches with one frame in flight: 7 waves/SIMD (28 one-wave workgroups per CU)
// rather than the kernel's 8. A lone frame ends with its costliest pixels' marches, which an
// eighth wave per SIMD slows when they were not fetched first (render-and-wait loop, moving camera:
// 12.85-12.91 ms at 28 per CU, 13.11-13.29 at 32; fixed pose 9.55-9.60 against 9.38-9.46;
// profiles/round5/dropin_bpc8); multi-frame launches interleave their frames' tails and take 8.
static constexpr int kLoneFrameBlocksPerCu = 28;

// One frame in flight: the device state a render launch owns until it completes. A context
// has config.frames_in_flight slots and launches round-robin over them, so frame k+1 can
// start (its own scratch, queue and framebuffer) while frame k's last pixels finish.
struct Slot {
  hipStream_t stream = nullptr;  // frm_render's stream for this slot (slot 0: the context stream)
  hipEvent_t done = nullptr;     // recorded after the slot's last launch (any stream)
  bool pending = false;          // `done` has been recorded since the slot was last waited for
  hipStream_t last_stream = nullptr;  // stream of the slot's last launch
  // frm_render's framebuffers for this slot (context pool), used alternately: a frame's
  // asynchronous readback (copy stream) overlaps the slot's next render, which writes the other
  // one; fb is the current one. Capacity: a smaller frame size keeps the larger buffer.
  uint8_t* fbs[2] = {nullptr, nullptr};
  size_t fbs_cap[2] = {0, 0};
  hipEvent_t fb_read[2] = {nullptr, nullptr};  // after the last asynchronous readback of fbs[i]
  bool fb_read_pending[2] = {false, false};
  uint32_t fb_idx = 0;
  uint8_t* fb = nullptr;
  unsigned int* queue = nullptr;
  uint8_t* records = nullptr;  // persistent kernel scratch (ShadeGeom[cap] then ShadeTail[cap]), grown on demand
  size_t records_cap = 0;
  // pixel scheduling state (frm_sched.hip), sched_cap entries each: 0..cap-1, the fetch
  // order, the cost keys the slot's last launch recorded per pixel and the sort's key output
  uint32_t* sched_iota = nullptr;
  uint32_t* sched_order = nullptr;
  uint8_t* sched_keys = nullptr;  // 2 x sched_cap: keys, sorted keys
  void* sched_temp = nullptr;
  size_t sched_cap = 0, sched_temp_bytes = 0;
  uint64_t sched_key = 0;  // geometry the recorded keys belong to
  bool sched_history = false;
  uint32_t sched_w = 0, sched_h = 0;  // frame size of the recorded keys when they cover a whole frame
  bool sched_whole = false;
  // another slot's launch copied this slot's keys as its scheduling history (on keys_reader):
  // this slot's next launch, which rewrites them, waits for that copy
  hipEvent_t keys_read = nullptr;
  hipStream_t keys_reader = nullptr;
  uint64_t seq = 0;  // launch sequence number of the slot's last launch (frm_ctx::launch_seq)
  // fused scheduling (KernelArgs::key_hist): two launches' histogram + cursor words, used
  // alternately; order_ready: the slot's last launch ranked its pixels into sched_order and zeroed
  // the queue and the other half of rank_words for geometry order_key
  uint32_t* rank_words = nullptr;
  uint32_t rank_half = 0;
  bool order_ready = false;
  uint64_t order_key = 0;
  // asynchronous readback (frm_read_frame_async / frm_present_async): the frame's bytes (or its
  // blit) copied into a pinned host image after the render, on `rb_stream`: the render's own stream
  // when frames are in flight (another slot's stream renders the next frame meanwhile), else the
  // slot's copy stream after `done`, so that a lone slot's stream goes straight on to the next frame.
  // One stream per slot keeps a context within HIP's default 4 hardware queues per process: with a
  // copy stream per slot as well, 2 frames in flight used 4 streams, queues were shared and a
  // frame's render queued behind the previous frame's copy (drop-in loop at
  // GPU_MAX_HW_QUEUES=4). `copied` is recorded after the copy; the slot's next frm_render waits for
  // it before its launch rewrites the framebuffer.
  hipStream_t copy_stream = nullptr;  // owned (one slot only)
  hipStream_t rb_stream = nullptr;    // the stream of the last readback's copy
  uint8_t* host_img = nullptr;
  size_t host_cap = 0;
  uint8_t* present_dev = nullptr;  // frm_present_async's blit output (device, context pool), grown on demand
  size_t present_dev_cap = 0;
  hipEvent_t copied = nullptr;
  uint64_t copy_ticket = 0;  // 0: no readback held
  size_t copy_bytes = 0;
};

// A group context (frm_config.device_count): the context itself renders rank 0's bands on
// devices[0] and holds the frames; sub[r] (r >= 1) renders rank r's bands on devices[r]. Per frame
// slot: rank r's band buffer on its device, and on device 0 the rank-major gather buffer (rank 0's
// bands are rendered straight into its first part) that frm_unshuffle_bands' kernel reassembles
// into the slot's framebuffer.
struct GroupSlot {
  uint8_t* bands[FRM_MAX_DEVICES] = {};  // r >= 1 (device r's pool)
  size_t bands_cap[FRM_MAX_DEVICES] = {};
  hipEvent_t sent[FRM_MAX_DEVICES] = {};  // r >= 1, device r: after the slot's last gather read bands[r]
  hipEvent_t rendered[FRM_MAX_DEVICES] = {};  // r >= 1, device r: the bands are written (copy transport)
  hipEvent_t copied = nullptr;            // device 0: after the copy transport's gather
  bool gather_pending = false;
  uint8_t* gathered = nullptr;  // device 0 (context pool): ranks x stride bytes
  size_t gathered_cap = 0;
};
struct Group {
  uint32_t n = 0;
  frm_ctx* sub[FRM_MAX_DEVICES] = {};  // sub[0] unused: rank 0 is the group context itself
  ncclComm_t comm[FRM_MAX_DEVICES] = {};
  bool rccl = false;  // RCCL point-to-point gather (distinct devices); else device-to-device copies
  hipEvent_t comm_done[FRM_MAX_DEVICES] = {};  // device r: after the last gather's RCCL operations
  bool comm_pending = false;
  uint32_t band_rows = 0;
  size_t stride = 0;  // bytes of rank 0's bands (the largest share): the gather buffer's rank stride
  GroupSlot slots[FRM_MAX_FRAMES_IN_FLIGHT];
};

// The resident frame ring of a context (frm_internal.h RingArgs; resident_render below).
struct Ring {
  uint32_t slots = 0;         // R (2 or 4); 0: never set up
  RingHost* host = nullptr;   // pinned, coherent
  RingDev* dev = nullptr;
  // buffers of the ring's frame size (R frames each): records, framebuffers, fetch orders, cost keys,
  // and the scheduling scratch of its first orders
  uint8_t* records = nullptr;
  uint32_t* out = nullptr;
  uint32_t* order = nullptr;
  uint8_t* keys = nullptr;
  uint32_t* iota = nullptr;
  uint8_t* keys_sorted = nullptr;
  void* sched_temp = nullptr;
  size_t sched_temp_bytes = 0;
  size_t cap = 0;             // pixels per frame the buffers hold
  bool keys_valid = false;    // keys hold a frame of keys_w x keys_h
  uint32_t keys_w = 0, keys_h = 0;
  // zero-copy readback: two pinned host images per slot (frame g: image (g - 1) / R & 1 of its slot),
  // each the frame it holds (or will hold) and the ticket handed out for it
  uint32_t* img[kRingSlots][2] = {};
  size_t img_cap = 0;
  uint32_t img_seq[kRingSlots][2] = {};
  uint64_t img_ticket[kRingSlots][2] = {};
  size_t img_bytes[kRingSlots][2] = {};
  bool zero_copy = false;     // frm_read_frame_async has been called: frames carry a host image
  // images replaced by larger ones (a resize) while a ticket still named them: kept until destroy
  struct Retired {
    uint64_t ticket;
    uint32_t* img;
    uint32_t seq, slot;
    size_t bytes;
  };
  std::vector<Retired> retired;
  // the generation the ring is set up for (a frame with other scene uniforms, size, aspect or step
  // cap needs another grid and a fresh ring)
  bool gen_valid = false;
  SceneUniforms su{};
  uint32_t w = 0, h = 0, max_steps = 0;
  float aspect[2] = {0.f, 0.f};
  uint32_t next_seq = 1;      // seq of the next posted frame
  uint32_t last_seq = 0;      // the last posted frame
  uint32_t grid_id = 0;       // the last launched grid (0: none yet)
  uint32_t service_waves = 128;
};

struct frm_ctx {
  int device = 0;
  Group* group = nullptr;   // a group context (frm_config.device_count >= 1)
  bool bands_only = false;  // a group's rank r >= 1: renders bands, holds no frame
  uint32_t max_steps = FRM_DEFAULT_MAX_STEPS;
  uint32_t flags = 0;
  int cu_count = 0;
  hipStream_t stream = nullptr;  // the context stream (= slots[0].stream)
  // Stream-ordered pool of the buffers that follow the frame size (framebuffers, persistent-kernel
  // records, scheduling arrays, presentation output): they are released and re-allocated on the
  // stream that uses them, so frm_resize never drains the frames in flight. Freed blocks stay in
  // the pool (release threshold: never) for the next size change.
  hipMemPool_t pool = nullptr;
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  uint32_t width = 0, height = 0;
  Slot slots[FRM_MAX_FRAMES_IN_FLIGHT];
  uint32_t nslots = 1;
  uint32_t next_slot = 0;  // slot of the next launch
  uint32_t last_slot = 0;  // slot of the last frm_render (the frame read_frame/present see)
  uint64_t launch_seq = 0;  // render launches so far (Slot::seq)
  uint64_t render_seq = 0;  // launch_seq of the last frm_render
  uint64_t ticket_seq = 0;  // asynchronous readbacks so far
  frm_parameters render_params{};  // the parameters of the last frm_render (frm_debug_trace)
  SceneUniforms render_scene{};
  ReloadedKernels* reloaded = nullptr;  // frm_reload: kernels compiled from edited sources
  uint8_t* present_buf = nullptr;  // frm_present output, grown on demand
  size_t present_cap = 0;
  unsigned long long* counters = nullptr;  // FRM_NUM_COUNTERS
  uint32_t service_min = kDefaultServiceMin;
  bool fused_sched = true;  // KernelArgs::key_hist; FRM_SCHED=sort: every launch sorts (experiments)
  frm_parameters params{};
  bool has_params = false;
  SceneUniforms scene{};
  Ring ring;
  bool ring_enabled = false;  // FRM_RING=1: the resident frame ring (opt-in: slower)
  bool last_is_ring = false; // the last frm_render posted a ring frame (ring.last_seq)
  std::string error;
};

namespace {

thread_local std::string g_error;  // failures without a context

int fail(frm_ctx* ctx, int code, const char* fmt, ...) {
  char buf[8192];  // room for a compiler log (frm_reload)
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->error = buf;
  g_error = buf;
  return code;
}

int hip_fail(frm_ctx* ctx, hipError_t e, const char* what) {
  int code = (e == hipErrorOutOfMemory) ? FRM_ERR_OUT_OF_MEMORY : FRM_ERR_HIP;
  return fail(ctx, code, "%s failed: %s (%d)", what, hipGetErrorString(e), (int)e);
}

#define FRM_HIP(ctx, call)                              \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

#define FRM_NCCL(ctx, call)                                                                         \
  do {                                                                                              \
    ncclResult_t r_ = (call);                                                                       \
    if (r_ != ncclSuccess) return fail(ctx, FRM_ERR_HIP, "%s failed: %s", #call, ncclGetErrorString(r_)); \
  } while (0)

// A failure of a group's member context, reported on the group context.
int relay(frm_ctx* ctx, const frm_ctx* member, int rc) {
  return member == ctx ? rc : fail(ctx, rc, "device %d: %s", member->device, member->error.c_str());
}

int not_on_group(frm_ctx* ctx, const char* what) {
  return fail(ctx, FRM_ERR_UNSUPPORTED, "%s: not available on a group context (frm_config.device_count)", what);
}

// Device memory of the context pool, allocated / released in the order of stream s: a block
// released on s is reused only by work ordered after everything enqueued on s before the release.
int dev_alloc(frm_ctx* ctx, void** p, size_t bytes, hipStream_t s) {
  FRM_HIP(ctx, hipMallocFromPoolAsync(p, bytes, ctx->pool, s));
  return FRM_OK;
}
int dev_release(frm_ctx* ctx, void* p, hipStream_t s) {
  if (p) FRM_HIP(ctx, hipFreeAsync(p, s));
  return FRM_OK;
}
// Slot sl's framebuffer for a frame of `bytes`, grown on the slot stream (renders and synchronous
// readback use it there; an asynchronous readback on the copy stream is awaited first).
int ensure_fb(frm_ctx* ctx, Slot& sl, size_t bytes) {
  const uint32_t i = sl.fb_idx;
  sl.fb = sl.fbs[i];
  if (sl.fbs_cap[i] >= bytes) return FRM_OK;
  int rc = dev_release(ctx, sl.fbs[i], sl.stream);  // after its readback: frm_render / frm_resize wait
  if (rc) return rc;
  sl.fbs[i] = sl.fb = nullptr;
  sl.fbs_cap[i] = 0;
  if ((rc = dev_alloc(ctx, (void**)&sl.fbs[i], bytes, sl.stream))) return rc;
  sl.fbs_cap[i] = bytes;
  sl.fb = sl.fbs[i];
  return FRM_OK;
}
// Makes fbs[i] the slot's current framebuffer, its last asynchronous readback ordered before
// everything enqueued on the slot stream from here on.
int select_fb(frm_ctx* ctx, Slot& sl, uint32_t i) {
  sl.fb_idx = i;
  sl.fb = sl.fbs[i];
  if (sl.fb_read_pending[i]) {
    FRM_HIP(ctx, hipStreamWaitEvent(sl.stream, sl.fb_read[i], 0));
    sl.fb_read_pending[i] = false;
  }
  return FRM_OK;
}

uint32_t num_bands(uint32_t height, uint32_t band_rows) { return (height + band_rows - 1) / band_rows; }

// Rows produced by bands first, first+stride, ... below num_bands (the last band of the
// frame may be short, but a band buffer always reserves band_rows rows for it).
uint32_t band_local_rows(uint32_t height, uint32_t band_rows, uint32_t first, uint32_t stride) {
  uint32_t nb = num_bands(height, band_rows);
  if (first >= nb) return 0;
  uint32_t count = (nb - 1 - first) / stride + 1;
  return count * band_rows;
}

// Local rows that hold frame rows: all but the missing rows of a short last band, which
// can only be this launch's last band (its local rows are then a prefix).
uint32_t band_valid_rows(uint32_t height, const BandGeometry& g) {
  if (g.local_rows == 0) return 0;
  const uint32_t last = g.first_band + (g.local_rows / g.band_rows - 1u) * g.band_stride;
  const uint32_t end = (last + 1u) * g.band_rows;  // one past its last global row
  return end > height ? g.local_rows - (end - height) : g.local_rows;
}

// The fractal loop work a frame's parameters ask for (include/frm.h FRM_MAX_NUM_ITERATIONS):
// trips of the DE's loop per evaluation, after the reference's own loop semantics
// (Sierpinski's i32 loop runs none for N >= 2^31: compute_scene_uniforms sets n = 0).
int check_parameters(frm_ctx* ctx, const SceneUniforms& su, const frm_parameters& p) {
  if (is_mandelbulb(su.family) && su.n == 0xFFFFFFFFu)
    return fail(ctx, FRM_ERR_UNSUPPORTED,
                "num_iterations 0xffffffff: the Mandelbulb's `i <= num_iterations` loop (fragment.wgsl:245) "
                "never ends; parameters not changed");
  const uint32_t trips = su.family == kSphere ? 0u : su.n;
  if (trips > FRM_MAX_NUM_ITERATIONS && !(ctx->flags & FRM_FLAG_UNBOUNDED_ITERATIONS))
    return fail(ctx, FRM_ERR_UNSUPPORTED,
                "num_iterations %u (scene %u) above FRM_MAX_NUM_ITERATIONS = %u: every DE runs that many "
                "loop bodies; create the context with FRM_FLAG_UNBOUNDED_ITERATIONS to allow it; "
                "parameters not changed",
                p.num_iterations, p.scene_index, FRM_MAX_NUM_ITERATIONS);
  return FRM_OK;
}

int ensure_ready(frm_ctx* ctx) {
  if (!ctx) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx is NULL");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  if (!ctx->has_params) return fail(ctx, FRM_ERR_NOT_READY, "frm_set_parameters has not been called");
  return FRM_OK;
}

KernelArgs make_args(frm_ctx* ctx, uint8_t* dst, unsigned long long* counters, uint32_t band_rows,
                     uint32_t first, uint32_t stride, uint32_t local_rows) {
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  compute_frame_uniforms(ctx->params, ctx->width, ctx->height, ctx->max_steps, &a.f);
  a.s = ctx->scene;
  a.g.band_rows = band_rows;
  a.g.first_band = first;
  a.g.band_stride = stride;
  a.g.local_rows = local_rows;
  a.out = (uint32_t*)dst;
  a.counters = counters;
  a.npix = band_valid_rows(ctx->height, a.g) * ctx->width;
  a.service_min = ctx->service_min;
  a.batch = 1;
  a.rec_stride = local_rows * ctx->width;
  a.out_stride = local_rows * ctx->width;
  memcpy(a.cams[0].row, a.f.row, sizeof(a.f.row));  // a single frame is a batch of one
  a.cams[0].origin = a.f.origin;
  return a;
}

KernelKind kernel_for(const frm_ctx* ctx, uint64_t pixels) {
  if (ctx->flags & FRM_FLAG_SIMPLE_KERNEL) return kKernelSimple;
  if (ctx->flags & FRM_FLAG_PERSISTENT_KERNEL) return kKernelPersistent;
  return pixels < kSimplePixelsPerCu * (uint64_t)ctx->cu_count ? kKernelSimple : kKernelPersistent;
}

// Waits (host) until the slot's last launch has completed.
int wait_slot(frm_ctx* ctx, Slot& sl) {
  if (sl.pending) {
    FRM_HIP(ctx, hipEventSynchronize(sl.done));
    sl.pending = false;
  }
  return FRM_OK;
}

int synchronize_all(frm_ctx* ctx) {
  for (uint32_t i = 0; i < ctx->nslots; ++i) {
    Slot& sl = ctx->slots[i];
    if (sl.stream) FRM_HIP(ctx, hipStreamSynchronize(sl.stream));
    int rc = wait_slot(ctx, sl);
    if (rc) return rc;
  }
  return FRM_OK;
}

// The stream frm_render uses for slot i (created on first use: a context with one frame in
// flight never creates more than the context stream).
// Slots > 0 need a hardware queue of their own to overlap: HIP maps streams onto at most
// GPU_MAX_HW_QUEUES queues per process (4 by default) and hands the least-used one out again,
// and two frames whose streams share a queue never overlap. Plain
// non-blocking streams get distinct queues while the pool has room (bench.py raises the limit to
// 16); FRM_SLOT_STREAMS=cumask asks for CU-masked streams, which the runtime never pools.
hipStream_t own_queue_stream(int device) {
  hipDeviceProp_t prop;
  // default: a pooled non-blocking stream. "cumask": a CU-masked stream, which gets a hardware queue
  // of its own but is a BLOCKING stream (hipExtStreamCreateWithCUMask takes no flags): it
  // synchronises with the legacy null stream (torch's default stream, synchronous hipMemcpy), so
  // it is opt-in for hosts that never use that stream
  const char* kind = getenv("FRM_SLOT_STREAMS");
  const bool cumask = kind && strcmp(kind, "cumask") == 0;
  if (cumask && hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) {
    const uint32_t words = (uint32_t)(prop.multiProcessorCount + 31) / 32u;
    uint32_t mask[64];
    if (words <= 64u) {
      for (uint32_t w = 0; w < words; ++w) mask[w] = 0xFFFFFFFFu;
      hipStream_t s = nullptr;
      if (hipExtStreamCreateWithCUMask(&s, words, mask) == hipSuccess) return s;
    }
  }
  hipStream_t s = nullptr;
  return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? s : nullptr;
}

int slot_stream(frm_ctx* ctx, uint32_t i, hipStream_t* out) {
  Slot& sl = ctx->slots[i];
  if (!sl.stream && !(sl.stream = own_queue_stream(ctx->device)))
    return fail(ctx, FRM_ERR_HIP, "stream creation failed for render slot %u", i);
  *out = sl.stream;
  return FRM_OK;
}

// Enqueues one render launch on stream s with the scratch of the context's next slot.
// Stream order covers a slot reused on the same stream; a slot last used on another
// stream is awaited on the device (hipStreamWaitEvent), so callers may rotate streams.
int launch(frm_ctx* ctx, KernelArgs a, hipStream_t s, uint32_t* out_slot = nullptr) {
  if (a.g.local_rows == 0) return FRM_OK;
  const uint32_t si = ctx->next_slot;
  Slot& sl = ctx->slots[si];
  if (sl.pending && sl.last_stream != s) FRM_HIP(ctx, hipStreamWaitEvent(s, sl.done, 0));
  if (sl.keys_reader) {  // another slot's launch read this slot's keys: they are rewritten below
    if (sl.keys_reader != s) FRM_HIP(ctx, hipStreamWaitEvent(s, sl.keys_read, 0));
    sl.keys_reader = nullptr;
  }
  const KernelKind kind = kernel_for(ctx, a.npix);
  a.queue = sl.queue;
  if (kind == kKernelPersistent) {
    const size_t need = (size_t)a.g.local_rows * a.f.width * a.batch;
    if (need > sl.records_cap) {  // grows outside the steady state (first frame of a size)
      // stream-ordered: s runs after the slot's last launch (awaited above when on another stream)
      int rc = dev_release(ctx, sl.records, s);
      if (rc) return rc;
      sl.records = nullptr;
      sl.records_cap = 0;
      if ((rc = dev_alloc(ctx, (void**)&sl.records, need * kRecordBytes, s))) return rc;
      sl.records_cap = need;
    }
    a.geom = reinterpret_cast<ShadeGeom*>(sl.records);
    a.tails = reinterpret_cast<ShadeTail*>(sl.records + sl.records_cap * sizeof(ShadeGeom));
    // pixel scheduling: fetch this launch's pixels by the cost the slot recorded last time
    // for the same geometry (most expensive first)
    const uint32_t npix = a.npix;
    const uint64_t key = ((uint64_t)a.f.width << 40) ^ ((uint64_t)a.g.local_rows << 20) ^
                         ((uint64_t)a.g.band_rows << 8) ^ ((uint64_t)a.g.first_band << 4) ^ a.g.band_stride ^
                         ((uint64_t)a.f.height << 52);
    // a whole frame (not a rank's bands): its keys can seed a resized whole frame's order
    const bool whole = a.g.first_band == 0 && a.g.band_stride == 1 && npix == a.f.width * a.f.height;
    const bool same = sl.sched_history && key == sl.sched_key;
    const bool rescale = !same && sl.sched_history && sl.sched_whole && whole;
    // a slot without history of this geometry takes another slot's keys: with frames in
    // flight, every slot's first launch would otherwise fetch in row-major order
    int donor = -1;
    if (!same && !rescale)
      for (uint32_t j = 0; j < ctx->nslots && donor < 0; ++j) {
        const Slot& o = ctx->slots[j];
        if (j != si && o.sched_history && o.sched_key == key && o.sched_cap >= npix) donor = (int)j;
      }
    if (npix > sl.sched_cap) {
      // stream-ordered like the records; a donor's copy of these keys was awaited above
      uint8_t* old_keys = sl.sched_keys;  // kept until a resize has resampled it
      int rc = FRM_OK;
      for (void* b : {(void*)sl.sched_iota, (void*)sl.sched_order, sl.sched_temp})
        if ((rc = dev_release(ctx, b, s))) return rc;
      if (!rescale && (rc = dev_release(ctx, old_keys, s))) return rc;
      sl.sched_iota = sl.sched_order = nullptr;
      sl.sched_keys = nullptr;
      sl.sched_temp = nullptr;
      sl.sched_cap = 0;
      sl.sched_temp_bytes = schedule_temp_bytes(npix);
      if ((rc = dev_alloc(ctx, (void**)&sl.sched_iota, (size_t)npix * sizeof(uint32_t), s)) ||
          (rc = dev_alloc(ctx, (void**)&sl.sched_order, (size_t)npix * sizeof(uint32_t), s)) ||
          (rc = dev_alloc(ctx, (void**)&sl.sched_keys, (size_t)npix * 2, s)) ||
          (rc = dev_alloc(ctx, &sl.sched_temp, sl.sched_temp_bytes ? sl.sched_temp_bytes : 16, s)))
        return rc;
      FRM_HIP(ctx, fill_iota(sl.sched_iota, npix, s));
      sl.sched_cap = npix;
      if (rescale) {
        FRM_HIP(ctx, rescale_keys(old_keys, sl.sched_w, sl.sched_h, sl.sched_keys, a.f.width, a.f.height, s));
        if ((rc = dev_release(ctx, old_keys, s))) return rc;  // after the resample reads it
      }
    } else if (rescale) {
      // resample into the sort's output half, then back (the map is read and written)
      uint8_t* tmp = sl.sched_keys + sl.sched_cap;
      FRM_HIP(ctx, rescale_keys(sl.sched_keys, sl.sched_w, sl.sched_h, tmp, a.f.width, a.f.height, s));
      FRM_HIP(ctx, hipMemcpyAsync(sl.sched_keys, tmp, npix, hipMemcpyDeviceToDevice, s));
    }
    if (donor >= 0) {  // keys order fetches only, never a pixel's bytes
      Slot& dn = ctx->slots[donor];
      if (dn.pending && dn.last_stream != s) FRM_HIP(ctx, hipStreamWaitEvent(s, dn.done, 0));
      // an earlier reader's copy on another stream: order this copy after it, so the one
      // keys_read event recorded below covers every copy the donor's next launch must await
      if (dn.keys_reader && dn.keys_reader != s) FRM_HIP(ctx, hipStreamWaitEvent(s, dn.keys_read, 0));
      FRM_HIP(ctx, hipMemcpyAsync(sl.sched_keys, dn.sched_keys, npix, hipMemcpyDeviceToDevice, s));
      FRM_HIP(ctx, hipEventRecord(dn.keys_read, s));  // the donor's next launch waits for this copy
      dn.keys_reader = s;
    }
    // the steady state: the slot's last launch (same geometry) has already ranked its pixels and
    // reset this launch's counters in its shading pass, so nothing runs between the two launches
    const bool fused = same && sl.order_ready && sl.order_key == key;
    uint32_t* half = sl.rank_words + sl.rank_half * kRankWords;
    if (!fused) {
      const bool history = same || rescale || donor >= 0;
      FRM_HIP(ctx, schedule_pixels(npix, history, sl.sched_keys, sl.sched_keys + sl.sched_cap,
                                   sl.sched_iota, sl.sched_order, sl.sched_temp, sl.sched_temp_bytes, s));
      FRM_HIP(ctx, hipMemsetAsync(sl.queue, 0, kQueueDebugWord * sizeof(unsigned int), s));
      FRM_HIP(ctx, hipMemsetAsync(half, 0, kRankWords * sizeof(uint32_t), s));
    }
    // runtime-reloaded kernels may not rank (edited sources): the next launch sorts again
    const bool rank = ctx->reloaded == nullptr && ctx->fused_sched;
    a.key_hist = rank ? half : nullptr;
    a.key_hist_next = sl.rank_words + (sl.rank_half ^ 1u) * kRankWords;
    a.order_out = sl.sched_order;
    sl.order_ready = false;  // set below once the launch is enqueued
    sl.order_key = key;
    a.pixel_order = sl.sched_order;
    a.pixel_key = sl.sched_keys;
    sl.sched_key = key;
    sl.sched_history = true;
    sl.sched_whole = whole;
    sl.sched_w = a.f.width;
    sl.sched_h = a.f.height;
    unsigned int* dbg = sl.queue + kQueueDebugWord;
    a.debug = (unsigned long long*)dbg;  // the diagnostic words after the partition counters
#ifdef FRM_STAMPS
    FRM_HIP(ctx, hipMemsetAsync(dbg, 0, 16, s));
    FRM_HIP(ctx, hipMemsetAsync(dbg + 4, 0xff, 16, s));  // atomicMin slots
    FRM_HIP(ctx, hipMemsetAsync(dbg + 8, 0, 8, s));
#endif
  }
  if (kind != kKernelPersistent) sl.order_ready = false;
  // Single-frame persistent launches with frames in flight run a grid of 4 waves per SIMD (16
  // one-wave workgroups per CU) instead of the occupancy limit (8 for the Mandelbulb): two frames'
  // grids then share the GPU, each frame's shading and ranking find room beside the next frame's
  // grid, and one frame's tail runs beside the other's bulk. Measured (profiles/round5/dropin_bpc):
  // the drop-in loop 9.11-9.18 -> 8.57-8.60 ms (fixed pose), 10.08-10.13 -> 9.29-9.32 (HEADLINE_FLY);
  // multi-frame launches (one queue for all their frames) keep the full grid (8-way rank share
  // 1.098 ms/frame full, 1.117 at 12).
  int blocks_cap = 0;
  if (a.batch == 1) {
    if (ctx->nslots >= 2 && a.npix <= kInflightCapPixels)
      blocks_cap = inflight_blocks_per_cu(ctx->nslots);
    else if (ctx->nslots == 1)
      blocks_cap = kLoneFrameBlocksPerCu;
  }
  FRM_HIP(ctx, launch_render(a, kind, ctx->cu_count, s, ctx->reloaded, blocks_cap));
  if (a.key_hist) {
    sl.order_ready = true;
    sl.rank_half ^= 1u;
  }
  FRM_HIP(ctx, hipEventRecord(sl.done, s));
  sl.seq = ++ctx->launch_seq;
  sl.pending = true;
  sl.last_stream = s;
  ctx->next_slot = (si + 1u) % ctx->nslots;
  if (out_slot) *out_slot = si;
  return FRM_OK;
}

// Band height of a group's row split: the smallest height >= 16 that splits the frame into a
// multiple of n bands (else 16), so interleaved bands balance the devices (frm/tiling.py).
uint32_t group_band_rows(uint32_t height, uint32_t n) {
  for (uint32_t br = 16; br <= height; ++br)
    if (height % br == 0 && (height / br) % n == 0) return br;
  return 16;
}

frm_ctx* member(frm_ctx* ctx, uint32_t r) { return r == 0 ? ctx : ctx->group->sub[r]; }

// One frame of a group context: every device renders its interleaved bands on the stream of its
// next frame slot (frames in flight overlap as on one device), the bands meet on device 0 (RCCL
// grouped send/receive over xGMI, or device-to-device copies for a repeated device), and device 0
// reassembles the frame into the slot's framebuffer on the same stream; the slot's `done` event
// then covers the whole frame for frm_read_frame / frm_present and their async forms.
int group_render(frm_ctx* ctx, frm_stats* stats) {
  Group& G = *ctx->group;
  const uint32_t n = G.n;
  int rc = FRM_OK;
  if (stats)  // the counters must hold this frame alone
    for (uint32_t r = 0; r < n; ++r) {
      frm_ctx* c = member(ctx, r);
      FRM_HIP(ctx, hipSetDevice(c->device));
      if ((rc = synchronize_all(c))) return relay(ctx, c, rc);
    }
  const uint32_t si = ctx->next_slot;
  Slot& sl = ctx->slots[si];
  GroupSlot& gs = G.slots[si];
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st[FRM_MAX_DEVICES];
  if ((rc = slot_stream(ctx, si, &st[0]))) return rc;
  const hipStream_t s0 = st[0];
  if ((rc = select_fb(ctx, sl, sl.fb_idx ^ 1u))) return rc;
  const size_t fb_bytes = (size_t)ctx->width * ctx->height * 4u;
  if ((rc = ensure_fb(ctx, sl, fb_bytes + fb_bytes / 4u))) return rc;
  const size_t gather_bytes = (size_t)n * G.stride;
  if (gather_bytes > gs.gathered_cap) {  // its last use (this slot's last frame) is ordered before, on s0
    if ((rc = dev_release(ctx, gs.gathered, s0))) return rc;
    gs.gathered = nullptr;
    gs.gathered_cap = 0;
    if ((rc = dev_alloc(ctx, (void**)&gs.gathered, gather_bytes, s0))) return rc;
    gs.gathered_cap = gather_bytes;
  }
  if (stats) {
    FRM_HIP(ctx, hipMemsetAsync(ctx->counters, 0, FRM_NUM_COUNTERS * sizeof(unsigned long long), s0));
    FRM_HIP(ctx, hipEventRecord(ctx->ev_start, s0));
  }
  uint32_t rows[FRM_MAX_DEVICES];
  for (uint32_t r = 0; r < n; ++r) rows[r] = band_local_rows(ctx->height, G.band_rows, r, n);
  // ranks 1..n-1 on their devices
  for (uint32_t r = 1; r < n; ++r) {
    frm_ctx* c = G.sub[r];
    if (rows[r] == 0) continue;  // a frame of fewer bands than devices
    FRM_HIP(ctx, hipSetDevice(c->device));
    if ((rc = slot_stream(c, c->next_slot, &st[r]))) return relay(ctx, c, rc);
    // the band buffer's last gather (this slot's last frame) has read it
    if (gs.gather_pending)
      FRM_HIP(ctx, hipStreamWaitEvent(st[r], G.rccl ? gs.sent[r] : gs.copied, 0));
    if (gs.bands_cap[r] < G.stride) {
      if ((rc = dev_release(c, gs.bands[r], st[r]))) return relay(ctx, c, rc);
      gs.bands[r] = nullptr;
      gs.bands_cap[r] = 0;
      if ((rc = dev_alloc(c, (void**)&gs.bands[r], G.stride, st[r]))) return relay(ctx, c, rc);
      gs.bands_cap[r] = G.stride;
    }
    if (stats) FRM_HIP(ctx, hipMemsetAsync(c->counters, 0, FRM_NUM_COUNTERS * sizeof(unsigned long long), st[r]));
    KernelArgs a = make_args(c, gs.bands[r], c->counters, G.band_rows, r, n, rows[r]);
    if ((rc = launch(c, a, st[r]))) return relay(ctx, c, rc);
  }
  // rank 0, into the first part of the gather buffer
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  KernelArgs a0 = make_args(ctx, gs.gathered, ctx->counters, G.band_rows, 0, n, rows[0]);
  if ((rc = launch(ctx, a0, s0))) return rc;
  // gather on device 0, rank-major
  if (G.rccl) {
    // one communicator, so its operations run in issue order on every device: each frame's
    // transfers wait for the previous frame's (frames in flight use other streams)
    if (G.comm_pending)
      for (uint32_t r = 0; r < n; ++r) {
        if (r > 0 && rows[r] == 0) continue;
        FRM_HIP(ctx, hipSetDevice(member(ctx, r)->device));
        FRM_HIP(ctx, hipStreamWaitEvent(st[r], G.comm_done[r], 0));
      }
    FRM_NCCL(ctx, ncclGroupStart());
    for (uint32_t r = 1; r < n; ++r) {
      const size_t bytes = (size_t)rows[r] * ctx->width * 4u;
      if (!bytes) continue;
      FRM_HIP(ctx, hipSetDevice(G.sub[r]->device));
      FRM_NCCL(ctx, ncclSend(gs.bands[r], bytes, ncclUint8, 0, G.comm[r], st[r]));
      FRM_HIP(ctx, hipSetDevice(ctx->device));
      FRM_NCCL(ctx, ncclRecv(gs.gathered + (size_t)r * G.stride, bytes, ncclUint8, (int)r, G.comm[0], s0));
    }
    FRM_NCCL(ctx, ncclGroupEnd());
    for (uint32_t r = 0; r < n; ++r) {
      if (r > 0 && rows[r] == 0) continue;
      FRM_HIP(ctx, hipSetDevice(member(ctx, r)->device));
      FRM_HIP(ctx, hipEventRecord(G.comm_done[r], st[r]));
      if (r > 0) FRM_HIP(ctx, hipEventRecord(gs.sent[r], st[r]));
    }
    G.comm_pending = true;
  } else {
    for (uint32_t r = 1; r < n; ++r) {
      const size_t bytes = (size_t)rows[r] * ctx->width * 4u;
      if (!bytes) continue;
      FRM_HIP(ctx, hipSetDevice(G.sub[r]->device));
      FRM_HIP(ctx, hipEventRecord(gs.rendered[r], st[r]));
      FRM_HIP(ctx, hipSetDevice(ctx->device));
      FRM_HIP(ctx, hipStreamWaitEvent(s0, gs.rendered[r], 0));
      FRM_HIP(ctx, hipMemcpyAsync(gs.gathered + (size_t)r * G.stride, gs.bands[r], bytes, hipMemcpyDeviceToDevice, s0));
    }
    FRM_HIP(ctx, hipSetDevice(ctx->device));
    FRM_HIP(ctx, hipEventRecord(gs.copied, s0));
  }
  gs.gather_pending = true;
  // reassemble; the slot's `done` now covers render, gather and reassembly
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  FRM_HIP(ctx, launch_unshuffle(gs.gathered, G.stride, sl.fb, ctx->width, ctx->height, G.band_rows, n, s0));
  FRM_HIP(ctx, hipEventRecord(sl.done, s0));
  ctx->last_slot = si;
  ctx->render_seq = sl.seq;
  ctx->render_params = ctx->params;
  ctx->render_scene = ctx->scene;
  if (stats) {
    FRM_HIP(ctx, hipEventRecord(ctx->ev_stop, s0));
    uint64_t sum[FRM_NUM_COUNTERS] = {};
    for (uint32_t r = 0; r < n; ++r) {
      if (r > 0 && rows[r] == 0) continue;
      frm_ctx* c = member(ctx, r);
      uint64_t host[FRM_NUM_COUNTERS];
      FRM_HIP(ctx, hipSetDevice(c->device));
      FRM_HIP(ctx, hipMemcpyAsync(host, c->counters, sizeof(host), hipMemcpyDeviceToHost, st[r]));
      FRM_HIP(ctx, hipStreamSynchronize(st[r]));
      for (uint32_t k = 0; k < FRM_NUM_COUNTERS; ++k) sum[k] += host[k];
    }
    FRM_HIP(ctx, hipSetDevice(ctx->device));
    FRM_HIP(ctx, hipStreamSynchronize(s0));
    float ms = 0.0f;
    FRM_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
    if ((rc = frm_stats_from_counters(ctx, sum, stats))) return rc;
    stats->kernel_ms = ms;  // device 0's view: from its render's start to the reassembled frame
  }
  return FRM_OK;
}

// ---- resident frame ring --------------------------------------------------------------------
// Single-frame frm_render calls without stats on a context with frames in flight post their frames
// to the context's ring (frm_internal.h RingArgs) instead of launching a grid each: one persistent
// grid marches the posted frames in order (a wave moves on to the next frame when one's queue
// drains, as a multi-frame launch interleaves its frames) and its service waves shade, rank and
// publish each frame as its last pixel finishes, so a frame's tail overlaps the next frame's bulk as
// it does inside frm_render_bands_batch. The grid lives as long as frames keep arriving: a march wave
// that finds nothing left closes it (the last frame it serves is then fixed), and the host launches
// the next grid when it sees the closed flag after posting (the post and the flag are ordered by
// sequentially consistent accesses on both sides, so a frame is either seen by the closing grid or
// served by the next one). frm_read_frame_async tickets of ring frames are zero-copy: the shading also
// writes the frame into a pinned host image. Anything else on the context first drains the ring
// (ring_quiesce).

uint32_t ring_size(const frm_ctx* ctx) { return ctx->nslots >= 3 ? 4u : 2u; }

// Whether frm_render(ctx, NULL) goes through the ring.
bool ring_eligible(const frm_ctx* ctx) {
  if (!ctx->ring_enabled || ctx->group || ctx->bands_only || ctx->reloaded || ctx->nslots < 2) return false;
  const uint64_t npix = (uint64_t)ctx->width * ctx->height;
  if (kernel_for(ctx, npix) != kKernelPersistent || npix > (1ull << 28)) return false;
  // a ring's service waves give up after kRingWatchdogTicks (2 s) without progress: keep the
  // costliest possible pixel (2 marches of max_steps DEs of N + 1 bodies) well inside that
  const uint64_t trips = (ctx->scene.family == kSphere ? 0u : (uint64_t)ctx->scene.n) + 2u;
  return 2ull * ctx->max_steps * trips <= (1ull << 21);
}

bool ring_same_gen(const frm_ctx* ctx) {
  const Ring& R = ctx->ring;
  if (!R.gen_valid || R.w != ctx->width || R.h != ctx->height || R.max_steps != ctx->max_steps ||
      R.aspect[0] != ctx->params.aspect_scale[0] || R.aspect[1] != ctx->params.aspect_scale[1] ||
      R.slots != ring_size(ctx))
    return false;
  SceneUniforms a = R.su, b = ctx->scene;
  if (is_mandelbulb(a.family)) {  // ring frames carry their own power (march_persistent<..., ANIM, RES>)
    a.mb_power = b.mb_power = 0.f;
    a.mb_power_m1 = b.mb_power_m1 = 0.f;
  }
  return memcmp(&a, &b, sizeof(a)) == 0;
}

// Waits (host) until ring frame `seq` (slot s) is done. A grid that ended without it (a service
// wave's watchdog) is reported instead of waited for.
int ring_wait(frm_ctx* ctx, uint32_t s, uint32_t seq) {
  Ring& R = ctx->ring;
  for (uint64_t spin = 1;; ++spin) {
    if (__atomic_load_n(&R.host->done[s][0], __ATOMIC_ACQUIRE) >= seq) return FRM_OK;
    if ((spin & 255u) == 0) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(&R.host->done[s][0], __ATOMIC_ACQUIRE) >= seq) return FRM_OK;
        return fail(ctx, FRM_ERR_HIP, "resident frame ring: frame %u never completed (its grid ended)", seq);
      }
      if (e != hipErrorNotReady) return hip_fail(ctx, e, "hipStreamQuery");
      sched_yield();
    }
  }
}

// Every posted ring frame done and the ring's grids ended (the last one closes once nothing is
// left to claim). The context stream is then idle.
int ring_quiesce(frm_ctx* ctx) {
  Ring& R = ctx->ring;
  if (!R.grid_id) return FRM_OK;
  const uint32_t first = R.last_seq >= R.slots ? R.last_seq - R.slots + 1u : 1u;
  for (uint32_t q = first; q <= R.last_seq && q >= 1u; ++q)
    if (int rc = ring_wait(ctx, (q - 1u) & (R.slots - 1u), q)) return rc;
  FRM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return FRM_OK;
}

void ring_free_buffers(Ring& R) {
  for (void* b : {(void*)R.records, (void*)R.out, (void*)R.order, (void*)R.keys, (void*)R.iota, (void*)R.keys_sorted,
                  R.sched_temp})
    if (b) (void)hipFree(b);
  R.records = nullptr;
  R.out = R.order = R.iota = nullptr;
  R.keys = R.keys_sorted = nullptr;
  R.sched_temp = nullptr;
  R.cap = 0;
  R.keys_valid = false;
}

void ring_free_images(Ring& R) {
  for (uint32_t s = 0; s < kRingSlots; ++s)
    for (uint32_t par = 0; par < 2; ++par) {
      uint32_t*& p = R.img[s][par];
      if (p && R.img_ticket[s][par])  // a ticket still names it (frm_frame_pixels)
        R.retired.push_back({R.img_ticket[s][par], p, R.img_seq[s][par], s, R.img_bytes[s][par]});
      else if (p)
        (void)hipHostFree(p);
      p = nullptr;
    }
  memset(R.img_seq, 0, sizeof(R.img_seq));
  memset(R.img_ticket, 0, sizeof(R.img_ticket));
  R.img_cap = 0;
}

// A fresh ring for the context's current size, scene and step cap, after every earlier ring frame
// (synchronous: rare, between generations). Each slot's counters carry the epoch of the first new
// frame that will use it; each slot's first fetch order comes from the ring's cost keys of a frame
// of the same size (row-major without).
int ring_setup(frm_ctx* ctx) {
  Ring& R = ctx->ring;
  int rc = ring_quiesce(ctx);
  if (rc) return rc;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (!R.host) {
    FRM_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&R.host), sizeof(RingHost), hipHostMallocCoherent));
    memset(R.host, 0, sizeof(RingHost));
  }
  if (!R.dev) FRM_HIP(ctx, hipMalloc(&R.dev, sizeof(RingDev)));
  const uint32_t slots = ring_size(ctx);
  const size_t npix = (size_t)ctx->width * ctx->height;
  if (npix > R.cap || slots != R.slots) {
    ring_free_buffers(R);
    const size_t n = npix * slots;
    FRM_HIP(ctx, hipMalloc(&R.records, n * kRecordBytes));
    FRM_HIP(ctx, hipMalloc(&R.out, n * 4u));
    FRM_HIP(ctx, hipMalloc(&R.order, n * 4u));
    FRM_HIP(ctx, hipMalloc(&R.keys, n));
    FRM_HIP(ctx, hipMalloc(&R.iota, npix * 4u));
    FRM_HIP(ctx, hipMalloc(&R.keys_sorted, npix));
    R.sched_temp_bytes = schedule_temp_bytes((uint32_t)npix);
    FRM_HIP(ctx, hipMalloc(&R.sched_temp, R.sched_temp_bytes ? R.sched_temp_bytes : 16));
    R.cap = npix;
  }
  if (slots != R.slots) ring_free_images(R);
  R.slots = slots;
  // slot s's next frame: the first seq >= next_seq with (seq - 1) % R == s
  const uint32_t k0 = R.next_seq;
  RingDev* img = new (std::nothrow) RingDev();
  if (!img) return fail(ctx, FRM_ERR_OUT_OF_MEMORY, "host allocation failed");
  img->base = k0;
  memset(img->trace, 0xff, sizeof(img->trace));
  memset(img->grid_trace, 0xff, sizeof(img->grid_trace));
  for (auto& t : img->trace) t[2] = 0;  // max field
  // the counter sets of the first `slots` frames (the later ones are set up by the frame that
  // completes `slots` frames before them, ring_finish)
  for (uint32_t seq = k0; seq < k0 + slots; ++seq) {
    const unsigned long long ep = (unsigned long long)seq << 32;
    RingFrameCtl& c = img->set[(seq - 1u) & (2u * slots - 1u)];
    for (uint32_t x = 0; x <= kQueueParts; ++x) c.queue[x * (kQueuePartWords / 2u)] = ep;
    c.pix_done[0] = c.shade_next[0] = c.shade_done[0] = c.rank_next[0] = c.rank_done[0] = ep;
    const uint32_t s = (seq - 1u) & (slots - 1u);
    const uint32_t prev = seq > slots ? seq - slots : 0u;  // the slot's last frame: done (quiesced)
    img->done_seq[s][0] = prev;
    __atomic_store_n(&R.host->done[s][0], prev, __ATOMIC_RELAXED);
  }
  const hipError_t e = hipMemcpy(R.dev, img, sizeof(RingDev), hipMemcpyHostToDevice);
  delete img;
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpy(ring state)");
  const bool history = R.keys_valid && R.keys_w == ctx->width && R.keys_h == ctx->height;
  FRM_HIP(ctx, fill_iota(R.iota, (uint32_t)npix, ctx->stream));
  for (uint32_t s = 0; s < slots; ++s)
    FRM_HIP(ctx, schedule_pixels((uint32_t)npix, history, R.keys + s * npix, R.keys_sorted, R.iota, R.order + s * npix,
                                 R.sched_temp, R.sched_temp_bytes, ctx->stream));
  FRM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  R.keys_valid = true;  // every ring frame's shading writes them
  R.keys_w = ctx->width;
  R.keys_h = ctx->height;
  R.gen_valid = true;
  R.su = ctx->scene;
  R.w = ctx->width;
  R.h = ctx->height;
  R.max_steps = ctx->max_steps;
  R.aspect[0] = ctx->params.aspect_scale[0];
  R.aspect[1] = ctx->params.aspect_scale[1];
  return FRM_OK;
}

// A new grid for the ring, serving frames from `first` on (or from where its predecessor stopped).
int ring_launch(frm_ctx* ctx, uint32_t first) {
  Ring& R = ctx->ring;
  const uint32_t id = R.grid_id + 1u;
  __atomic_store_n(&R.host->grid_stop[id % kRingGridIds][0], 0xFFFFFFFFu, __ATOMIC_SEQ_CST);
  FRM_HIP(ctx, hipMemsetAsync(&R.dev->grid, 0, sizeof(RingGridCtl), ctx->stream));
  KernelArgs a = make_args(ctx, nullptr, ctx->counters, ctx->height, 0, 1, ctx->height);
  const size_t n = R.cap * R.slots;
  a.geom = reinterpret_cast<ShadeGeom*>(R.records);
  a.tails = reinterpret_cast<ShadeTail*>(R.records + n * sizeof(ShadeGeom));
  a.ring.host = R.host;
  a.ring.dev = R.dev;
  a.ring.slots = R.slots;
  a.ring.grid_id = id;
  a.ring.first_seq = first;
  a.ring.service_waves = R.service_waves;
  a.ring.out = R.out;
  a.ring.order = R.order;
  a.ring.keys = R.keys;
  int blocks = 0;
  FRM_HIP(ctx, launch_ring(a, ctx->cu_count, ctx->stream, &blocks));
  R.grid_id = id;
  return FRM_OK;
}

// frm_render(ctx, NULL) through the ring: post the frame, launching a grid if none will take it.
int ring_render(frm_ctx* ctx) {
  Ring& R = ctx->ring;
  int rc = FRM_OK;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (!ring_same_gen(ctx) && (rc = ring_setup(ctx))) return rc;
  const uint32_t k = R.next_seq;
  const uint32_t s = (k - 1u) & (R.slots - 1u);
  if ((rc = ring_wait(ctx, s, k > R.slots ? k - R.slots : 0u))) return rc;  // the slot's last frame
  FrameUniforms fu;
  compute_frame_uniforms(ctx->params, ctx->width, ctx->height, ctx->max_steps, &fu);
  RingFrame& F = R.host->frames[s];
  memcpy(F.row, fu.row, sizeof(F.row));
  F.ox = fu.origin.x;
  F.oy = fu.origin.y;
  F.oz = fu.origin.z;
  F.mb_power = ctx->scene.mb_power;
  F.seq = k;
  uint32_t* img = nullptr;
  if (R.zero_copy) {
    const size_t bytes = (size_t)ctx->width * ctx->height * 4u;
    if (bytes > R.img_cap) {  // images of another size: none of them is pending (ring_setup drained)
      ring_free_images(R);
      R.img_cap = bytes + bytes / 4u;  // headroom for the reference's +-1 render-texture steps
    }
    const uint32_t par = ((k - 1u) / R.slots) & 1u;
    if (!R.img[s][par])
      FRM_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&R.img[s][par]), R.img_cap, hipHostMallocCoherent));
    img = R.img[s][par];
    R.img_seq[s][par] = k;
    R.img_ticket[s][par] = 0;  // its earlier frame's ticket expires
    R.img_bytes[s][par] = bytes;
  }
  F.host_img = img;
  __atomic_store_n(&R.host->posted, k, __ATOMIC_SEQ_CST);  // after the frame's data
  // the running grid takes the frame unless it has closed (then it may or may not have seen it: a
  // new grid starts where the closed one stopped)
  if (R.grid_id == 0 || __atomic_load_n(&R.host->closed, __ATOMIC_SEQ_CST) == R.grid_id)
    if ((rc = ring_launch(ctx, k))) return rc;
  R.next_seq = k + 1u;
  R.last_seq = k;
  ctx->last_is_ring = true;
  ctx->render_params = ctx->params;
  ctx->render_scene = ctx->scene;
  return FRM_OK;
}

// The last frm_render was a ring frame: drain the ring and copy that frame into slot 0's framebuffer,
// so the single-frame paths (frm_read_frame, frm_present, their async forms) see it as before.
int ring_materialize(frm_ctx* ctx) {
  if (!ctx->last_is_ring) return FRM_OK;
  Ring& R = ctx->ring;
  int rc = ring_quiesce(ctx);
  if (rc) return rc;
  Slot& sl = ctx->slots[0];
  const size_t bytes = (size_t)ctx->width * ctx->height * 4u;
  if ((rc = select_fb(ctx, sl, sl.fb_idx)) || (rc = ensure_fb(ctx, sl, bytes + bytes / 4u))) return rc;
  const uint32_t s = (R.last_seq - 1u) & (R.slots - 1u);
  FRM_HIP(ctx, hipMemcpyAsync(sl.fb, R.out + (size_t)s * R.w * R.h, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  FRM_HIP(ctx, hipEventRecord(sl.done, ctx->stream));
  sl.pending = true;
  sl.last_stream = ctx->stream;
  sl.seq = ++ctx->launch_seq;
  ctx->last_slot = 0;
  ctx->render_seq = sl.seq;
  ctx->last_is_ring = false;
  return FRM_OK;
}

// frm_read_frame_async of a ring frame: a ticket for its zero-copy image. The frame before the first
// such call was posted without an image: it is waited for and copied once, and from then on every
// ring frame carries one.
int ring_read_async(frm_ctx* ctx, uint64_t* out_ticket) {
  Ring& R = ctx->ring;
  R.zero_copy = true;
  const uint32_t k = R.last_seq, s = (k - 1u) & (R.slots - 1u), par = ((k - 1u) / R.slots) & 1u;
  const size_t bytes = (size_t)R.w * R.h * 4u;
  if (!(R.img[s][par] && R.img_seq[s][par] == k)) {
    int rc = ring_quiesce(ctx);
    if (rc) return rc;
    if (bytes > R.img_cap) {
      ring_free_images(R);
      R.img_cap = bytes + bytes / 4u;
    }
    if (!R.img[s][par])
      FRM_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&R.img[s][par]), R.img_cap, hipHostMallocCoherent));
    FRM_HIP(ctx, hipMemcpy(R.img[s][par], R.out + (size_t)s * R.w * R.h, bytes, hipMemcpyDeviceToHost));
    R.img_seq[s][par] = k;
    R.img_bytes[s][par] = bytes;
  }
  R.img_ticket[s][par] = *out_ticket = ++ctx->ticket_seq;
  return FRM_OK;
}

// Drains the ring before anything that is not a ring frame uses the context.
int ring_leave(frm_ctx* ctx) {
  if (ctx->last_is_ring) return ring_materialize(ctx);
  return ring_quiesce(ctx);
}

int group_synchronize(frm_ctx* ctx) {
  for (uint32_t r = 1; r < ctx->group->n; ++r) {
    frm_ctx* c = ctx->group->sub[r];
    FRM_HIP(ctx, hipSetDevice(c->device));
    if (int rc = synchronize_all(c)) return relay(ctx, c, rc);
  }
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  return synchronize_all(ctx);
}

}  // namespace

extern "C" {

uint32_t frm_abi_version(void) { return FRM_ABI_VERSION; }

const char* frm_last_error(const frm_ctx* ctx) { return ctx ? ctx->error.c_str() : g_error.c_str(); }

int frm_device_count(int32_t* out_count) {
  if (!out_count) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "out_count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *out_count = 0;
    return hip_fail(nullptr, e, "hipGetDeviceCount");
  }
  *out_count = n;
  return FRM_OK;
}

// One single-device context on `device` (frm_create's checks done).
static int create_one(const frm_config* config, int device, frm_ctx** out_ctx);
static int create_group(const frm_config* config, frm_ctx** out_ctx);

int frm_create(frm_ctx** out_ctx, const frm_config* config) {
  if (!out_ctx || !config) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "out_ctx/config is NULL");
  *out_ctx = nullptr;
  if (config->frames_in_flight > FRM_MAX_FRAMES_IN_FLIGHT)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "config.frames_in_flight %u above %u", config->frames_in_flight,
                FRM_MAX_FRAMES_IN_FLIGHT);
  if (config->max_steps > FRM_MAX_STEPS_LIMIT)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "config.max_steps %u above %u", config->max_steps,
                FRM_MAX_STEPS_LIMIT);
  const uint32_t kernels = FRM_FLAG_SIMPLE_KERNEL | FRM_FLAG_PERSISTENT_KERNEL;
  if ((config->flags & ~(kernels | FRM_FLAG_SCENE_SPHERE | FRM_FLAG_UNBOUNDED_ITERATIONS | FRM_FLAG_HW_MATH)) ||
      (config->flags & kernels) == kernels)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "config.flags 0x%x: unknown flag or both kernel flags",
                config->flags);
  if (config->device_count > FRM_MAX_DEVICES)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "config.device_count %u above %u", config->device_count,
                FRM_MAX_DEVICES);
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(nullptr, FRM_ERR_NO_DEVICE, "no HIP device available (%s)", hipGetErrorString(e));
  if (config->device_count == 0) {
    if (config->device < 0 || config->device >= n)
      return fail(nullptr, FRM_ERR_NO_DEVICE, "device %d out of range [0, %d)", config->device, n);
    return create_one(config, config->device, out_ctx);
  }
  for (uint32_t r = 0; r < config->device_count; ++r)
    if (config->devices[r] < 0 || config->devices[r] >= n)
      return fail(nullptr, FRM_ERR_NO_DEVICE, "devices[%u] = %d out of range [0, %d)", r, config->devices[r], n);
  return create_group(config, out_ctx);
}

static int create_one(const frm_config* config, int device, frm_ctx** out_ctx) {
  hipError_t e = hipSuccess;
  frm_ctx* ctx = new (std::nothrow) frm_ctx();
  if (!ctx) return fail(nullptr, FRM_ERR_OUT_OF_MEMORY, "host allocation failed");
  ctx->device = device;
  ctx->max_steps = config->max_steps ? config->max_steps : FRM_DEFAULT_MAX_STEPS;
  ctx->flags = config->flags;
  ctx->nslots = config->frames_in_flight ? config->frames_in_flight : 1u;
  if (const char* env = getenv("FRM_SCHED")) ctx->fused_sched = strcmp(env, "sort") != 0;
  if (const char* env = getenv("FRM_RING")) ctx->ring_enabled = strcmp(env, "0") != 0;  // opt-in ring
  if (const char* env = getenv("FRM_RING_SERVICE")) {  // service waves of a ring grid (tuning)
    long v = strtol(env, nullptr, 10);
    if (v >= 1 && v <= 1024) ctx->ring.service_waves = (uint32_t)v;
  }
  if (const char* env = getenv("FRM_SERVICE_MIN")) {
    long v = strtol(env, nullptr, 10);
    if (v >= 1 && v <= 64) ctx->service_min = (uint32_t)v;
  }
  int rc = FRM_OK;
  do {
    if ((e = hipSetDevice(ctx->device)) != hipSuccess) { rc = hip_fail(ctx, e, "hipSetDevice"); break; }
    if ((e = hipDeviceGetAttribute(&ctx->cu_count, hipDeviceAttributeMultiprocessorCount, ctx->device)) != hipSuccess) {
      rc = hip_fail(ctx, e, "hipDeviceGetAttribute"); break;
    }
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) { rc = hip_fail(ctx, e, "hipStreamCreate"); break; }
    hipMemPoolProps props;
    memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = ctx->device;
    if ((e = hipMemPoolCreate(&ctx->pool, &props)) != hipSuccess) { rc = hip_fail(ctx, e, "hipMemPoolCreate"); break; }
    uint64_t keep = UINT64_MAX;
    if ((e = hipMemPoolSetAttribute(ctx->pool, hipMemPoolAttrReleaseThreshold, &keep)) != hipSuccess) {
      rc = hip_fail(ctx, e, "hipMemPoolSetAttribute"); break;
    }
    if ((e = hipEventCreate(&ctx->ev_start)) != hipSuccess) { rc = hip_fail(ctx, e, "hipEventCreate"); break; }
    if ((e = hipEventCreate(&ctx->ev_stop)) != hipSuccess) { rc = hip_fail(ctx, e, "hipEventCreate"); break; }
    if ((e = hipMalloc(&ctx->counters, FRM_NUM_COUNTERS * sizeof(unsigned long long))) != hipSuccess) { rc = hip_fail(ctx, e, "hipMalloc(counters)"); break; }
    ctx->slots[0].stream = ctx->stream;
    for (uint32_t i = 0; i < ctx->nslots && rc == FRM_OK; ++i) {
      Slot& sl = ctx->slots[i];
      if ((e = hipEventCreateWithFlags(&sl.done, hipEventDisableTiming)) != hipSuccess) rc = hip_fail(ctx, e, "hipEventCreate");
      else if ((e = hipEventCreateWithFlags(&sl.keys_read, hipEventDisableTiming)) != hipSuccess)
        rc = hip_fail(ctx, e, "hipEventCreate");
      else if ((e = hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming)) != hipSuccess)
        rc = hip_fail(ctx, e, "hipEventCreate");
      else if ((e = hipEventCreateWithFlags(&sl.fb_read[0], hipEventDisableTiming)) != hipSuccess ||
               (e = hipEventCreateWithFlags(&sl.fb_read[1], hipEventDisableTiming)) != hipSuccess)
        rc = hip_fail(ctx, e, "hipEventCreate");
      else if ((e = hipMalloc(&sl.queue, kQueueBytes)) != hipSuccess) rc = hip_fail(ctx, e, "hipMalloc(queue)");
      else if ((e = hipMalloc(&sl.rank_words, 2 * kRankWords * sizeof(uint32_t))) != hipSuccess)
        rc = hip_fail(ctx, e, "hipMalloc(rank words)");
    }
  } while (0);
  if (rc != FRM_OK) {
    g_error = ctx->error;
    frm_destroy(ctx);
    return rc;
  }
  *out_ctx = ctx;
  return FRM_OK;
}

// A group: the context on devices[0] plus one band-rendering context per further device, the
// RCCL communicator over them (ncclCommInitAll: one process, one rank per device) when the
// devices are distinct, and the per-slot gather events.
static int create_group(const frm_config* config, frm_ctx** out_ctx) {
  const uint32_t n = config->device_count;
  frm_ctx* ctx = nullptr;
  int rc = create_one(config, config->devices[0], &ctx);
  if (rc) return rc;
  Group* G = new (std::nothrow) Group();
  if (!G) {
    frm_destroy(ctx);
    return fail(nullptr, FRM_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  ctx->group = G;
  G->n = n;
  bool distinct = true;
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t q = 0; q < r; ++q) distinct = distinct && config->devices[q] != config->devices[r];
  const char* gather = getenv("FRM_GATHER");  // experiments: "copy" = device-to-device copies
  G->rccl = n > 1 && distinct && !(gather && strcmp(gather, "copy") == 0);
  hipError_t e = hipSuccess;
  for (uint32_t r = 1; r < n && rc == FRM_OK; ++r) {
    if ((rc = create_one(config, config->devices[r], &G->sub[r]))) {
      // the member's message (create_one left it in g_error) onto the group context, whose error
      // the failure path below reports
      const std::string why = g_error;
      rc = fail(ctx, rc, "devices[%u] = %d: %s", r, config->devices[r], why.c_str());
      break;
    }
    G->sub[r]->bands_only = true;
  }
  for (uint32_t r = 0; r < n && rc == FRM_OK; ++r) {
    const int dev = config->devices[r];
    if ((e = hipSetDevice(dev)) != hipSuccess) { rc = hip_fail(ctx, e, "hipSetDevice"); break; }
    if ((e = hipEventCreateWithFlags(&G->comm_done[r], hipEventDisableTiming)) != hipSuccess) {
      rc = hip_fail(ctx, e, "hipEventCreate");
      break;
    }
    for (uint32_t i = 0; i < ctx->nslots && rc == FRM_OK; ++i) {
      GroupSlot& gs = G->slots[i];
      if (r == 0) {
        if ((e = hipEventCreateWithFlags(&gs.copied, hipEventDisableTiming)) != hipSuccess) rc = hip_fail(ctx, e, "hipEventCreate");
      } else if ((e = hipEventCreateWithFlags(&gs.sent[r], hipEventDisableTiming)) != hipSuccess ||
                 (e = hipEventCreateWithFlags(&gs.rendered[r], hipEventDisableTiming)) != hipSuccess) {
        rc = hip_fail(ctx, e, "hipEventCreate");
      }
    }
  }
  if (rc == FRM_OK && G->rccl) {
    int devs[FRM_MAX_DEVICES];
    for (uint32_t r = 0; r < n; ++r) devs[r] = config->devices[r];
    const ncclResult_t nr = ncclCommInitAll(G->comm, (int)n, devs);
    if (nr != ncclSuccess) {
      for (uint32_t r = 0; r < n; ++r) G->comm[r] = nullptr;
      rc = fail(ctx, FRM_ERR_HIP, "ncclCommInitAll over %u devices failed: %s", n, ncclGetErrorString(nr));
    }
  }
  if (rc == FRM_OK) {
    e = hipSetDevice(ctx->device);
    if (e != hipSuccess) rc = hip_fail(ctx, e, "hipSetDevice");
  }
  if (rc != FRM_OK) {
    g_error = ctx->error;
    frm_destroy(ctx);
    return rc;
  }
  *out_ctx = ctx;
  return FRM_OK;
}

int frm_destroy(frm_ctx* ctx) {
  if (!ctx) return FRM_OK;
  if (Group* G = ctx->group) {  // the members first (best effort, statuses ignored)
    for (uint32_t r = 1; r < G->n; ++r) {
      frm_ctx* c = G->sub[r];
      if (!c) continue;
      (void)hipSetDevice(c->device);
      (void)synchronize_all(c);
      for (uint32_t i = 0; i < FRM_MAX_FRAMES_IN_FLIGHT; ++i) {
        GroupSlot& gs = G->slots[i];
        if (gs.bands[r] && c->stream) (void)hipFreeAsync(gs.bands[r], c->stream);
        for (hipEvent_t ev : {gs.sent[r], gs.rendered[r]})
          if (ev) (void)hipEventDestroy(ev);
      }
      if (G->comm_done[r]) (void)hipEventDestroy(G->comm_done[r]);
      if (G->comm[r]) (void)ncclCommDestroy(G->comm[r]);
      frm_destroy(c);
    }
    (void)hipSetDevice(ctx->device);
    (void)synchronize_all(ctx);
    for (uint32_t i = 0; i < FRM_MAX_FRAMES_IN_FLIGHT; ++i) {
      GroupSlot& gs = G->slots[i];
      if (gs.gathered && ctx->stream) (void)hipFreeAsync(gs.gathered, ctx->stream);
      if (gs.copied) (void)hipEventDestroy(gs.copied);
    }
    if (G->comm_done[0]) (void)hipEventDestroy(G->comm_done[0]);
    if (G->comm[0]) (void)ncclCommDestroy(G->comm[0]);
    delete G;
    ctx->group = nullptr;
  }
  // Teardown is best effort: statuses are ignored so every resource gets released.
  (void)hipSetDevice(ctx->device);
  {
    Ring& R = ctx->ring;
    if (R.grid_id) (void)ring_quiesce(ctx);
    if (getenv("FRM_RING_DEBUG")) {
      fprintf(stderr, "frm ring: %u frames posted, %u grids launched, %u service waves\n", R.last_seq, R.grid_id,
              R.service_waves);
      // FRM_RING_TRACE builds: the device timeline of the last frames (us from the first event shown)
      RingDev* d = R.dev ? new (std::nothrow) RingDev() : nullptr;
      if (d && hipMemcpy(d, R.dev, sizeof(RingDev), hipMemcpyDeviceToHost) == hipSuccess && d->trace[1][1] &&
          d->trace[1][1] != ~0ull) {
        const uint32_t first = R.last_seq > 40u ? R.last_seq - 40u : 1u;
        const unsigned long long t0 = d->trace[first & 63u][0];
        for (uint32_t q = first; q <= R.last_seq; ++q) {
          const unsigned long long* t = d->trace[q & 63u];
          fprintf(stderr, "frm ring trace: frame %u seen %.1f claims %.1f..%.1f marched %.1f shaded %.1f done %.1f\n", q,
                  (double)(long long)(t[0] - t0) / 100.0, (double)(long long)(t[1] - t0) / 100.0,
                  (double)(long long)(t[2] - t0) / 100.0, (double)(long long)(t[3] - t0) / 100.0,
                  (double)(long long)(t[4] - t0) / 100.0, (double)(long long)(t[5] - t0) / 100.0);
        }
        for (uint32_t id = R.grid_id > 30u ? R.grid_id - 30u : 1u; id <= R.grid_id; ++id)
          fprintf(stderr, "frm ring trace: grid %u start %.1f close %.1f\n", id,
                  (double)(long long)(d->grid_trace[id & 63u][0] - t0) / 100.0,
                  (double)(long long)(d->grid_trace[id & 63u][1] - t0) / 100.0);
      }
      delete d;
    }
    ring_free_buffers(R);
    ring_free_images(R);
    for (const Ring::Retired& r : R.retired) (void)hipHostFree(r.img);
    R.retired.clear();
    if (R.dev) (void)hipFree(R.dev);
    if (R.host) (void)hipHostFree(R.host);
  }
  for (uint32_t i = 0; i < ctx->nslots; ++i) {
    Slot& sl = ctx->slots[i];
    if (sl.stream) (void)hipStreamSynchronize(sl.stream);
    if (sl.copy_stream) (void)hipStreamSynchronize(sl.copy_stream);
    if (sl.pending) (void)hipEventSynchronize(sl.done);
  }
  for (uint32_t i = 0; i < ctx->nslots; ++i) {
    Slot& sl = ctx->slots[i];
    // pool blocks back to the pool (every stream is idle), then the pool itself below
    if (ctx->stream)
      for (void* b : {(void*)sl.fbs[0], (void*)sl.fbs[1], (void*)sl.records, (void*)sl.sched_iota, (void*)sl.sched_order,
                      (void*)sl.sched_keys, sl.sched_temp, (void*)sl.present_dev})
        if (b) (void)hipFreeAsync(b, ctx->stream);
    if (sl.queue) (void)hipFree(sl.queue);
    if (sl.rank_words) (void)hipFree(sl.rank_words);
    if (sl.done) (void)hipEventDestroy(sl.done);
    if (sl.keys_read) (void)hipEventDestroy(sl.keys_read);
    if (sl.copied) (void)hipEventDestroy(sl.copied);
    for (hipEvent_t ev : sl.fb_read)
      if (ev) (void)hipEventDestroy(ev);
    if (sl.host_img) (void)hipHostFree(sl.host_img);
    if (i > 0 && sl.stream) (void)hipStreamDestroy(sl.stream);
    if (sl.copy_stream) (void)hipStreamDestroy(sl.copy_stream);
  }
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->pool) (void)hipMemPoolDestroy(ctx->pool);
  if (ctx->present_buf) (void)hipFree(ctx->present_buf);
  unload_reloaded(ctx->reloaded);
  if (ctx->counters) (void)hipFree(ctx->counters);
  if (ctx->ev_start) (void)hipEventDestroy(ctx->ev_start);
  if (ctx->ev_stop) (void)hipEventDestroy(ctx->ev_stop);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return FRM_OK;
}

int frm_resize(frm_ctx* ctx, uint32_t width, uint32_t height) {
  if (!ctx) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx is NULL");
  if (width == 0 || height == 0 || width > FRM_MAX_DIMENSION || height > FRM_MAX_DIMENSION)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "frame size %ux%u outside [1, %u]^2", width, height,
                FRM_MAX_DIMENSION);
  if (Group* G = ctx->group) {  // every member follows; the band geometry of the new size
    for (uint32_t r = 1; r < G->n; ++r)
      if (int rc = frm_resize(G->sub[r], width, height)) return relay(ctx, G->sub[r], rc);
    G->band_rows = group_band_rows(height, G->n);
    G->stride = (size_t)band_local_rows(height, G->band_rows, 0, G->n) * width * 4u;
  }
  if (ctx->bands_only) {  // a group member: its band buffers belong to the group's frame slots
    ctx->width = width;
    ctx->height = height;
    return FRM_OK;
  }
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  // ring frames in flight finish first (a ring serves one size); their tickets keep their images
  if (int rc = ring_quiesce(ctx)) return rc;
  if (width != ctx->width || height != ctx->height) ctx->last_is_ring = false;
  if (ctx->slots[0].fb && width == ctx->width && height == ctx->height) return FRM_OK;
  if (!ctx->slots[0].stream) return fail(ctx, FRM_ERR_HIP, "context stream missing");
  // No drain: frames in flight finish at their own size. Every buffer that follows the size grows
  // in its stream's order when a launch of the new size needs it (ensure_fb, launch); slot 0's
  // framebuffer (what frm_read_frame sees before the next frm_render) grows here.
  const size_t bytes = (size_t)width * height * 4u;
  Slot& s0 = ctx->slots[0];
  int rc = select_fb(ctx, s0, s0.fb_idx);
  if (rc || (rc = ensure_fb(ctx, s0, bytes + bytes / 4u))) return rc;  // headroom for the reference's +-1 steps
  ctx->width = width;
  ctx->height = height;
  ctx->last_slot = 0;
  // no frame of the new size yet: frm_read_frame_async / frm_present_async refuse until the next
  // frm_render (tickets issued before keep their frames)
  ctx->render_seq = 0;
  return FRM_OK;
}

int frm_set_parameters(frm_ctx* ctx, const frm_parameters* parameters) {
  if (!ctx || !parameters) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/parameters is NULL");
  SceneUniforms su;
  compute_scene_uniforms(*parameters, ctx->flags, &su);
  int rc = check_parameters(ctx, su, *parameters);
  if (rc) return rc;
  ctx->params = *parameters;
  ctx->scene = su;
  ctx->has_params = true;
  if (Group* G = ctx->group)  // the members render the same frame (same flags, same uniforms)
    for (uint32_t r = 1; r < G->n; ++r) {
      G->sub[r]->params = *parameters;
      G->sub[r]->scene = su;
      G->sub[r]->has_params = true;
    }
  return FRM_OK;
}

int frm_render(frm_ctx* ctx, frm_stats* stats) {
  int rc = ensure_ready(ctx);
  if (rc) return rc;
  if (ctx->group) return group_render(ctx, stats);
  if (!stats && ring_eligible(ctx)) return ring_render(ctx);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if ((rc = ring_quiesce(ctx))) return rc;  // a frame outside the ring: the ring's frames first
  ctx->last_is_ring = false;
  if (stats && (rc = synchronize_all(ctx))) return rc;  // the counters must hold this frame alone
  const uint32_t si = ctx->next_slot;
  Slot& sl = ctx->slots[si];
  hipStream_t s;
  if ((rc = slot_stream(ctx, si, &s))) return rc;
  // the other framebuffer of the slot: the last one may still be read back (copy stream); this
  // one's readback (two renders of the slot ago) is awaited on the slot stream, long done
  if ((rc = select_fb(ctx, sl, sl.fb_idx ^ 1u))) return rc;
  const size_t fb_bytes = (size_t)ctx->width * ctx->height * 4u;
  if ((rc = ensure_fb(ctx, sl, fb_bytes + fb_bytes / 4u))) return rc;
  KernelArgs a = make_args(ctx, sl.fb, ctx->counters, ctx->height, 0, 1, ctx->height);
  if (stats) {
    FRM_HIP(ctx, hipMemsetAsync(ctx->counters, 0, FRM_NUM_COUNTERS * sizeof(unsigned long long), s));
    FRM_HIP(ctx, hipEventRecord(ctx->ev_start, s));
  }
  rc = launch(ctx, a, s);
  if (rc) return rc;
  ctx->last_slot = si;
  ctx->render_seq = sl.seq;
  ctx->render_params = ctx->params;
  ctx->render_scene = ctx->scene;
  if (stats) {
    FRM_HIP(ctx, hipEventRecord(ctx->ev_stop, s));
    uint64_t host[FRM_NUM_COUNTERS];
    FRM_HIP(ctx, hipMemcpyAsync(host, ctx->counters, sizeof(host), hipMemcpyDeviceToHost, s));
    FRM_HIP(ctx, hipStreamSynchronize(s));
    float ms = 0.0f;
    FRM_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
    rc = frm_stats_from_counters(ctx, host, stats);
    if (rc) return rc;
    stats->kernel_ms = ms;
  }
  return FRM_OK;
}

int frm_read_frame(frm_ctx* ctx, uint8_t* dst, size_t dst_bytes) {
  if (!ctx || !dst) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/dst is NULL");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  size_t need = (size_t)ctx->width * ctx->height * 4u;
  if (dst_bytes < need)
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "dst holds %zu bytes, frame needs %zu", dst_bytes, need);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = ring_materialize(ctx)) return rc;
  const Slot& sl = ctx->slots[ctx->last_slot];  // the frame of the last frm_render
  FRM_HIP(ctx, hipMemcpyAsync(dst, sl.fb, need, hipMemcpyDeviceToHost, sl.stream));
  FRM_HIP(ctx, hipStreamSynchronize(sl.stream));
  return FRM_OK;
}

int frm_present(frm_ctx* ctx, uint32_t out_width, uint32_t out_height, uint32_t flags, uint8_t* dst,
                size_t dst_bytes) {
  if (!ctx || !dst) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/dst is NULL");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  if (out_width == 0 || out_height == 0 || out_width > FRM_MAX_DIMENSION || out_height > FRM_MAX_DIMENSION)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "bad output size %ux%u", out_width, out_height);
  if (flags & ~(FRM_BLIT_SRGB | FRM_BLIT_BGRA)) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "unknown flags 0x%x", flags);
  const size_t need = (size_t)out_width * out_height * 4u;
  if (dst_bytes < need)
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "dst holds %zu bytes, output needs %zu", dst_bytes, need);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = ring_materialize(ctx)) return rc;
  const Slot& sl = ctx->slots[ctx->last_slot];  // the frame of the last frm_render
  if (need > ctx->present_cap) {
    FRM_HIP(ctx, hipStreamSynchronize(sl.stream));
    if (ctx->present_buf) FRM_HIP(ctx, hipFree(ctx->present_buf));
    ctx->present_buf = nullptr;
    ctx->present_cap = 0;
    FRM_HIP(ctx, hipMalloc(&ctx->present_buf, need));
    ctx->present_cap = need;
  }
  FRM_HIP(ctx, launch_blit(sl.fb, ctx->width, ctx->height, ctx->present_buf, out_width, out_height, flags,
                           sl.stream));
  FRM_HIP(ctx, hipMemcpyAsync(dst, ctx->present_buf, need, hipMemcpyDeviceToHost, sl.stream));
  FRM_HIP(ctx, hipStreamSynchronize(sl.stream));
  return FRM_OK;
}

// The slot's copy stream, ordered after the slot's last launch (its render).
static int copy_stream_after_render(frm_ctx* ctx, Slot& sl) {
  if (ctx->nslots >= 2 && sl.last_stream) {  // stream order: after the render
    sl.rb_stream = sl.last_stream;
    return FRM_OK;
  }
  if (!sl.copy_stream) FRM_HIP(ctx, hipStreamCreateWithFlags(&sl.copy_stream, hipStreamNonBlocking));
  FRM_HIP(ctx, hipStreamWaitEvent(sl.copy_stream, sl.done, 0));
  sl.rb_stream = sl.copy_stream;
  return FRM_OK;
}

// Enqueues the copy of `bytes` device bytes of the last frm_render's slot into its pinned host
// image (on sl.rb_stream, after copy_stream_after_render) and hands out a ticket for it.
static int readback_async(frm_ctx* ctx, Slot& sl, const uint8_t* src, size_t bytes, uint64_t* out_ticket) {
  if (bytes > sl.host_cap) {
    // the image's previous contents belong to an expired ticket (an earlier frame of this slot);
    // only its copy may still be running
    if (sl.copy_ticket) FRM_HIP(ctx, hipEventSynchronize(sl.copied));
    if (sl.host_img) FRM_HIP(ctx, hipHostFree(sl.host_img));
    sl.host_img = nullptr;
    sl.host_cap = 0;
    sl.copy_ticket = 0;
    // headroom: a +-1 step of the reference's render-texture factor (4 % per axis) reuses it
    const size_t cap = bytes + bytes / 4u;
    FRM_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&sl.host_img), cap, hipHostMallocDefault));
    sl.host_cap = cap;
  }
  FRM_HIP(ctx, hipMemcpyAsync(sl.host_img, src, bytes, hipMemcpyDeviceToHost, sl.rb_stream));
  FRM_HIP(ctx, hipEventRecord(sl.copied, sl.rb_stream));
  // the framebuffer is read (by this copy, or by frm_present_async's blit before it) until here
  FRM_HIP(ctx, hipEventRecord(sl.fb_read[sl.fb_idx], sl.rb_stream));
  sl.fb_read_pending[sl.fb_idx] = true;
  sl.copy_ticket = ++ctx->ticket_seq;
  sl.copy_bytes = bytes;
  *out_ticket = sl.copy_ticket;
  return FRM_OK;
}

int frm_read_frame_async(frm_ctx* ctx, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/out_ticket is NULL");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->last_is_ring) return ring_read_async(ctx, out_ticket);
  if (!ctx->render_seq) return fail(ctx, FRM_ERR_NOT_READY, "no frm_render since the context was created");
  Slot& sl = ctx->slots[ctx->last_slot];  // the frame of the last frm_render
  int rc = copy_stream_after_render(ctx, sl);
  if (rc) return rc;
  return readback_async(ctx, sl, sl.fb, (size_t)ctx->width * ctx->height * 4u, out_ticket);
}

int frm_present_async(frm_ctx* ctx, uint32_t out_width, uint32_t out_height, uint32_t flags, uint64_t* out_ticket) {
  if (!ctx || !out_ticket) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/out_ticket is NULL");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  if (!ctx->render_seq) return fail(ctx, FRM_ERR_NOT_READY, "no frm_render since the context was created");
  if (out_width == 0 || out_height == 0 || out_width > FRM_MAX_DIMENSION || out_height > FRM_MAX_DIMENSION)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "bad output size %ux%u", out_width, out_height);
  if (flags & ~(FRM_BLIT_SRGB | FRM_BLIT_BGRA)) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "unknown flags 0x%x", flags);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = ring_materialize(ctx)) return rc;
  Slot& sl = ctx->slots[ctx->last_slot];
  const size_t need = (size_t)out_width * out_height * 4u;
  int rc = copy_stream_after_render(ctx, sl);
  if (rc) return rc;
  if (need > sl.present_dev_cap) {  // its last use (an earlier frame of this slot) is ordered before
    if (sl.copy_ticket && sl.rb_stream) FRM_HIP(ctx, hipEventSynchronize(sl.copied));  // maybe on another stream
    if ((rc = dev_release(ctx, sl.present_dev, sl.rb_stream))) return rc;
    sl.present_dev = nullptr;
    sl.present_dev_cap = 0;
    if ((rc = dev_alloc(ctx, (void**)&sl.present_dev, need, sl.rb_stream))) return rc;
    sl.present_dev_cap = need;
  }
  FRM_HIP(ctx, launch_blit(sl.fb, ctx->width, ctx->height, sl.present_dev, out_width, out_height, flags,
                           sl.rb_stream));
  return readback_async(ctx, sl, sl.present_dev, need, out_ticket);
}

int frm_frame_pixels(frm_ctx* ctx, uint64_t ticket, const uint8_t** out_pixels, size_t* out_bytes) {
  if (!ctx || !out_pixels) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "ctx/out_pixels is NULL");
  if (ticket) {  // a ring frame's zero-copy image: wait for the frame (its shading wrote the image)
    Ring& R = ctx->ring;
    for (uint32_t s = 0; s < kRingSlots; ++s)
      for (uint32_t par = 0; par < 2; ++par)
        if (R.img_ticket[s][par] == ticket) {
          if (int rc = ring_wait(ctx, s, R.img_seq[s][par])) return rc;
          *out_pixels = reinterpret_cast<const uint8_t*>(R.img[s][par]);
          if (out_bytes) *out_bytes = R.img_bytes[s][par];
          return FRM_OK;
        }
    for (const Ring::Retired& r : R.retired)
      if (r.ticket == ticket) {
        if (int rc = ring_wait(ctx, r.slot, r.seq)) return rc;
        *out_pixels = reinterpret_cast<const uint8_t*>(r.img);
        if (out_bytes) *out_bytes = r.bytes;
        return FRM_OK;
      }
  }
  for (uint32_t i = 0; i < ctx->nslots && ticket; ++i) {
    Slot& sl = ctx->slots[i];
    if (sl.copy_ticket != ticket) continue;
    FRM_HIP(ctx, hipSetDevice(ctx->device));
    FRM_HIP(ctx, hipEventSynchronize(sl.copied));
    *out_pixels = sl.host_img;
    if (out_bytes) *out_bytes = sl.copy_bytes;
    return FRM_OK;
  }
  return fail(ctx, FRM_ERR_INVALID_ARGUMENT,
              "ticket %llu is not held (expired: its slot has been read back again since, or never issued)",
              (unsigned long long)ticket);
}

int frm_reload(frm_ctx* ctx, const char* source_dir) {
  if (!ctx) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx is NULL");
  // a group reloads every member: all compile, or every member keeps its kernels
  const uint32_t n = ctx->group ? ctx->group->n : 1u;
  ReloadedKernels* rk[FRM_MAX_DEVICES] = {};
  if (source_dir)
    for (uint32_t r = 0; r < n; ++r) {
      std::string log;
      const int rc = compile_reloaded(source_dir, member(ctx, r)->device, &rk[r], &log);
      if (rc != FRM_OK) {
        for (uint32_t q = 0; q < r; ++q) unload_reloaded(rk[q]);
        return fail(ctx, rc, "reload failed, previous kernels kept: %s", log.c_str());
      }
    }
  if (int rc = ring_leave(ctx)) {
    for (uint32_t r = 0; r < n; ++r) unload_reloaded(rk[r]);
    return rc;
  }
  for (uint32_t r = 0; r < n; ++r) {
    frm_ctx* c = member(ctx, r);
    // the old module may still run, on this context's stream or a caller's (frm_render_bands)
    FRM_HIP(ctx, hipSetDevice(c->device));
    FRM_HIP(ctx, hipDeviceSynchronize());
    unload_reloaded(c->reloaded);
    c->reloaded = rk[r];
  }
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  return FRM_OK;
}

int frm_synchronize(frm_ctx* ctx) {
  if (!ctx) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx is NULL");
  if (ctx->group) return group_synchronize(ctx);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = ring_quiesce(ctx)) return rc;
  return synchronize_all(ctx);
}

int frm_kernel_for_pixels(const frm_ctx* ctx, uint64_t pixels, uint32_t* out_kernel) {
  if (!ctx || !out_kernel) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx/out_kernel is NULL");
  *out_kernel = kernel_for(ctx, pixels) == kKernelSimple ? FRM_KERNEL_SIMPLE : FRM_KERNEL_PERSISTENT;
  return FRM_OK;
}

int frm_group_band_rows(uint32_t height, uint32_t devices, uint32_t* out_band_rows) {
  if (!out_band_rows || height == 0 || devices == 0 || devices > FRM_MAX_DEVICES)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "invalid height %u or device count %u", height, devices);
  *out_band_rows = group_band_rows(height, devices);
  return FRM_OK;
}

int frm_band_rows_for(uint32_t height, uint32_t band_rows, uint32_t first_band, uint32_t band_stride,
                      uint32_t* out_rows) {
  if (!out_rows || height == 0 || band_rows == 0 || band_stride == 0)
    return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "invalid band geometry");
  *out_rows = band_local_rows(height, band_rows, first_band, band_stride);
  return FRM_OK;
}

int frm_render_bands(frm_ctx* ctx, uint8_t* dev_dst, size_t dst_bytes, uint32_t band_rows,
                     uint32_t first_band, uint32_t band_stride, void* stream, uint64_t* dev_counters) {
  int rc = ensure_ready(ctx);
  if (rc) return rc;
  if (ctx->group) return not_on_group(ctx, "frm_render_bands");
  if (!dev_dst || band_rows == 0 || band_stride == 0)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "invalid dst or band geometry");
  uint32_t rows = band_local_rows(ctx->height, band_rows, first_band, band_stride);
  size_t need = (size_t)rows * ctx->width * 4u;
  if (dst_bytes < need)
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "dst holds %zu bytes, bands need %zu", dst_bytes, need);
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if ((rc = ring_leave(ctx))) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  unsigned long long* counters = dev_counters ? (unsigned long long*)dev_counters : ctx->counters;
  KernelArgs a = make_args(ctx, dev_dst, counters, band_rows, first_band, band_stride, rows);
  return launch(ctx, a, s);
}

int frm_render_bands_batch(frm_ctx* ctx, uint32_t count, const frm_parameters* params, uint8_t* dev_dst,
                           size_t dst_bytes, size_t frame_stride_bytes, uint32_t band_rows, uint32_t first_band,
                           uint32_t band_stride,
                           void* stream, uint64_t* dev_counters) {
  if (!ctx) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "ctx is NULL");
  if (ctx->group) return not_on_group(ctx, "frm_render_bands_batch");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  if (!params || !dev_dst || count == 0 || count > FRM_MAX_BATCH || band_rows == 0 || band_stride == 0)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "invalid batch (count %u, at most %u) or band geometry", count,
                FRM_MAX_BATCH);
  const uint32_t rows = band_local_rows(ctx->height, band_rows, first_band, band_stride);
  const size_t need = (size_t)rows * ctx->width * 4u;
  if (frame_stride_bytes < need || frame_stride_bytes % 4u || frame_stride_bytes / 4u > 0xFFFFFFFFull)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT,
                "frame stride %zu: below a frame's %zu bytes, not a multiple of 4 or not below 16 GiB",
                frame_stride_bytes, need);
  // a stride of 0 passes the check above only for a rank without bands (need == 0): its frames
  // occupy no bytes
  if (dst_bytes < need || (frame_stride_bytes != 0 && (dst_bytes - need) / frame_stride_bytes < count - 1u))
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "dst holds %zu bytes, %u frames %zu bytes apart need %zu", dst_bytes,
                count, frame_stride_bytes, (size_t)(count - 1u) * frame_stride_bytes + need);
  // fetch positions are u32 and every wave's last queue claims run up to two chunks past the
  // end (kQueueHeadroom covers any persistent grid): keep them from wrapping
  if ((uint64_t)rows * ctx->width * count >= 0xFFFFFFFFull - kQueueHeadroom)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "batch of %u frames of %u x %u local pixels too large", count,
                ctx->width, rows);
  // frames of one launch may differ in camera, and for the Mandelbulb in time (its power,
  // fragment.wgsl:75, is the only time-derived constant): otherwise the same scene uniforms
  // (scene, iterations, time-derived constants) and aspect
  SceneUniforms s0;
  compute_scene_uniforms(params[0], ctx->flags, &s0);
  if (int rc = check_parameters(ctx, s0, params[0])) return rc;
  bool anim = false;
  float powers[FRM_MAX_BATCH];
  powers[0] = s0.mb_power;
  for (uint32_t k = 1; k < count; ++k) {
    SceneUniforms sk;
    compute_scene_uniforms(params[k], ctx->flags, &sk);
    powers[k] = sk.mb_power;
    if (is_mandelbulb(s0.family) && sk.family == s0.family && sk.mb_power != s0.mb_power) {
      anim = true;
      sk.mb_power = s0.mb_power;
      sk.mb_power_m1 = s0.mb_power_m1;
    }
    if (memcmp(&s0, &sk, sizeof(s0)) != 0 || params[k].aspect_scale[0] != params[0].aspect_scale[0] ||
        params[k].aspect_scale[1] != params[0].aspect_scale[1])
      return fail(ctx, FRM_ERR_INVALID_ARGUMENT,
                  "batch frame %u differs from frame 0 in more than the camera and the Mandelbulb's time "
                  "(scene, iterations, time-derived constants, aspect)",
                  k);
  }
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = ring_leave(ctx)) return rc;
  ctx->params = params[count - 1];  // the context's parameters: the batch's last frame
  compute_scene_uniforms(params[count - 1], ctx->flags, &ctx->scene);
  ctx->has_params = true;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  unsigned long long* counters = dev_counters ? (unsigned long long*)dev_counters : ctx->counters;
  KernelArgs a = make_args(ctx, dev_dst, counters, band_rows, first_band, band_stride, rows);
  FrameUniforms fk;
  // one launch per frame: the simple kernel has no queue to share; runtime-reloaded modules carry
  // the single-frame kernels only; per-frame powers need the Mandelbulb's N >= 1 kernels
  if (count == 1 || kernel_for(ctx, a.npix) == kKernelSimple || ctx->reloaded || (anim && s0.n == 0)) {
    for (uint32_t k = 0; k < count; ++k) {
      compute_scene_uniforms(params[k], ctx->flags, &a.s);
      compute_frame_uniforms(params[k], ctx->width, ctx->height, ctx->max_steps, &a.f);
      memcpy(a.cams[0].row, a.f.row, sizeof(a.f.row));
      a.cams[0].origin = a.f.origin;
      a.out = (uint32_t*)(dev_dst + (size_t)k * frame_stride_bytes);
      int rc = launch(ctx, a, s);
      if (rc) return rc;
    }
    return FRM_OK;
  }
  a.batch = count;
  a.out_stride = (uint32_t)(frame_stride_bytes / 4u);
  a.anim = anim ? 1u : 0u;
  memcpy(a.mb_powers, powers, sizeof(float) * count);
  for (uint32_t k = 0; k < count; ++k) {
    compute_frame_uniforms(params[k], ctx->width, ctx->height, ctx->max_steps, &fk);
    memcpy(a.cams[k].row, fk.row, sizeof(fk.row));
    a.cams[k].origin = fk.origin;
  }
  return launch(ctx, a, s);
}

int frm_unshuffle_bands(frm_ctx* ctx, const uint8_t* dev_src, size_t rank_stride_bytes, uint8_t* dev_dst,
                        size_t dst_bytes, uint32_t band_rows, uint32_t ranks, void* stream) {
  if (!ctx || !dev_src || !dev_dst || band_rows == 0 || ranks == 0)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "invalid unshuffle arguments");
  if (!ctx->width) return fail(ctx, FRM_ERR_NOT_READY, "frm_resize has not been called");
  size_t need = (size_t)ctx->width * ctx->height * 4u;
  if (dst_bytes < need)
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "dst holds %zu bytes, frame needs %zu", dst_bytes, need);
  uint32_t rows = band_local_rows(ctx->height, band_rows, 0, ranks);
  if (rank_stride_bytes < (size_t)rows * ctx->width * 4u)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "rank stride %zu below one rank's bands", rank_stride_bytes);
  if (rank_stride_bytes % 4u)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "rank stride must be a multiple of 4");
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FRM_HIP(ctx, launch_unshuffle(dev_src, rank_stride_bytes, dev_dst, ctx->width, ctx->height, band_rows,
                                ranks, s));
  return FRM_OK;
}

#ifdef FRM_STAMPS
extern "C" int frm_debug_read(frm_ctx* ctx, uint64_t* out5) {
  const Slot& sl = ctx->slots[(ctx->next_slot + ctx->nslots - 1u) % ctx->nslots];  // last launch
  return hipMemcpy(out5, sl.queue + kQueueDebugWord, 40, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

// per-pixel cost keys recorded by the last persistent launch (local pixel order; before
// the next launch overwrites them)
int frm_debug_pixel_keys(frm_ctx* ctx, uint8_t* out, size_t n) {
  if (!ctx || !out) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "NULL argument");
  if (ctx->group) return not_on_group(ctx, "frm_debug_pixel_keys");
  if (int rc = ring_leave(ctx)) return rc;
  const Slot& sl = ctx->slots[(ctx->next_slot + ctx->nslots - 1u) % ctx->nslots];  // last launch
  if (!sl.sched_keys) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "no persistent launch yet");
  if (n > sl.sched_cap) n = sl.sched_cap;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  FRM_HIP(ctx, hipDeviceSynchronize());
  FRM_HIP(ctx, hipMemcpy(out, sl.sched_keys, n, hipMemcpyDeviceToHost));
  return (int)n;
}

// replaces the cost keys the next launch sorts its pixels by (scheduling experiments): the
// slot of the next launch must hold the history of a whole frame of the current size
int frm_debug_set_pixel_keys(frm_ctx* ctx, const uint8_t* keys, size_t n) {
  if (!ctx || !keys) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "NULL argument");
  if (ctx->group) return not_on_group(ctx, "frm_debug_set_pixel_keys");
  if (int rc = ring_leave(ctx)) return rc;
  Slot& sl = ctx->slots[ctx->next_slot];
  if (!sl.sched_history || !sl.sched_whole || sl.sched_w != ctx->width || sl.sched_h != ctx->height ||
      n != (size_t)ctx->width * ctx->height || n > sl.sched_cap)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "no whole-frame history of this size in the next slot");
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  int rc = wait_slot(ctx, sl);
  if (rc) return rc;
  if (sl.keys_reader) FRM_HIP(ctx, hipEventSynchronize(sl.keys_read));
  FRM_HIP(ctx, hipMemcpy(sl.sched_keys, keys, n, hipMemcpyHostToDevice));
  sl.order_ready = false;  // the next launch sorts by these keys
  return FRM_OK;
}

// per-pixel shading inputs of the last frm_render (a whole persistent frame of the current size
// and parameters): 10 floats per pixel, row-major, as the oracle's om_render_trace
int frm_debug_trace(frm_ctx* ctx, float* out, size_t n_floats) {
  int rc = ensure_ready(ctx);
  if (rc) return rc;
  if (ctx->group) return not_on_group(ctx, "frm_debug_trace");
  if ((rc = ring_leave(ctx))) return rc;
  if (!out) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "out is NULL");
  const size_t npix = (size_t)ctx->width * ctx->height;
  if (n_floats < npix * 10u)
    return fail(ctx, FRM_ERR_BUFFER_TOO_SMALL, "out holds %zu floats, the trace needs %zu", n_floats, npix * 10u);
  const Slot& sl = ctx->slots[ctx->last_slot];
  if (!ctx->render_seq || sl.seq != ctx->render_seq)
    return fail(ctx, FRM_ERR_NOT_READY, "no frm_render, or a later launch reused its slot's records");
  if (!sl.records || sl.records_cap < npix || !sl.sched_whole || sl.sched_w != ctx->width || sl.sched_h != ctx->height)
    return fail(ctx, FRM_ERR_NOT_READY, "the last frm_render was not a persistent launch of this frame size");
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  // the rays and colours of that render: its own parameters, not those set since
  const frm_parameters cur_params = ctx->params;
  const SceneUniforms cur_scene = ctx->scene;
  ctx->params = ctx->render_params;
  ctx->scene = ctx->render_scene;
  KernelArgs a = make_args(ctx, sl.fb, ctx->counters, ctx->height, 0, 1, ctx->height);
  ctx->params = cur_params;
  ctx->scene = cur_scene;
  a.geom = reinterpret_cast<ShadeGeom*>(sl.records);
  a.tails = reinterpret_cast<ShadeTail*>(sl.records + sl.records_cap * sizeof(ShadeGeom));
  float* d = nullptr;
  FRM_HIP(ctx, hipMalloc(&d, npix * 10u * sizeof(float)));
  hipError_t e = launch_trace(a, d, sl.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, npix * 10u * sizeof(float), hipMemcpyDeviceToHost, sl.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sl.stream);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "frm_debug_trace");
  return FRM_OK;
}

int frm_stats_from_counters(const frm_ctx* ctx, const uint64_t* c, frm_stats* out) {
  if (!ctx || !c || !out) return fail(nullptr, FRM_ERR_INVALID_ARGUMENT, "NULL argument");
  memset(out, 0, sizeof(*out));
  out->pixels = c[kCntPixels];
  out->hit_pixels = c[kCntHits];
  out->primary_steps = c[kCntPrimary];
  out->shadow_steps = c[kCntShadow];
  out->normal_evals = c[kCntNormal];
  out->fractal_bodies = c[kCntBodies];
  out->fractal_bailouts = c[kCntBailouts];
  out->march_steps = c[kCntPrimary] + c[kCntShadow];
  out->wom_ops = wom_ops(ctx->scene, c);
  return FRM_OK;
}

int frm_eval_scene(frm_ctx* ctx, const float* points, uint32_t n, float* out_distance, float* out_color) {
  if (!ctx || !points || !out_distance || !out_color)
    return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "NULL argument");
  if (!ctx->has_params) return fail(ctx, FRM_ERR_NOT_READY, "frm_set_parameters has not been called");
  if (n == 0) return FRM_OK;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  float* d = nullptr;
  FRM_HIP(ctx, hipMalloc(&d, (size_t)n * 7 * sizeof(float)));
  float *pts = d, *dist = d + 3 * (size_t)n, *col = d + 4 * (size_t)n;
  hipError_t e = hipMemcpyAsync(pts, points, (size_t)n * 12, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = launch_eval_scene(ctx->scene, pts, n, dist, col, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_distance, dist, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_color, col, (size_t)n * 12, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "frm_eval_scene");
  return FRM_OK;
}

int frm_eval_math(frm_ctx* ctx, int32_t fn, const float* a, const float* b, uint32_t n, float* out) {
  if (!ctx || !a || !out || fn < 0 || fn > FRM_MATH_SRGB_ENCODE) return fail(ctx, FRM_ERR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return FRM_OK;
  FRM_HIP(ctx, hipSetDevice(ctx->device));
  float* d = nullptr;
  FRM_HIP(ctx, hipMalloc(&d, (size_t)n * 3 * sizeof(float)));
  float *da = d, *db = b ? d + n : nullptr, *dout = d + 2 * (size_t)n;
  hipError_t e = hipMemcpyAsync(da, a, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess && b) e = hipMemcpyAsync(db, b, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = launch_eval_math(fn, da, db, n, dout, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "frm_eval_math");
  return FRM_OK;
}

}  // extern "C"
