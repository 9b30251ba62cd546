// frm_internal.h — declarations shared by libfrm's translation units (not installed).
#pragma once
#if !defined(__HIPCC_RTC__)  // hiprtc (frm_reload) provides the HIP runtime itself
#include <hip/hip_runtime.h>

#include <string>
#endif

#include "frm_uniforms.h"

namespace frm {
constexpr uint32_t kMaxBatch = FRM_MAX_BATCH;  // frames per multi-frame launch

// Row-band geometry of one launch: local row lr lives in band (lr / band_rows) of this
// launch; that band is global band first_band + (lr / band_rows) * band_stride.
struct BandGeometry {
  uint32_t band_rows, first_band, band_stride, local_rows;
};

// Per-pixel results of the persistent march kernel, consumed by the shading pass: two arrays
// indexed by local pixel.
//  * ShadeTail (8 B, every pixel, one store when its march ends): the shadow march's
//    closeness and one word packing the primary steps (bits 0-21), kRecHit, kRecSunMiss and
//    the scheduling cost key (bits 24-31, frm_sched.hip; shade_pass copies it out).
//  * ShadeGeom (16 B, hit pixels only, one store at the last normal tap): primary hit
//    distance and surface normal. Misses never touch it.
struct ShadeTail {
  float closeness;
  uint32_t word;
};
struct ShadeGeom {
  float t, nx, ny, nz;
};
constexpr uint32_t kRecStepsMask = (1u << 22) - 1u;  // primary steps < 2^22 (FRM_MAX_STEPS_LIMIT)
constexpr uint32_t kRecHit = 1u << 22, kRecSunMiss = 1u << 23;
constexpr uint32_t kRecKeyShift = 24;
constexpr size_t kRecordBytes = sizeof(ShadeTail) + sizeof(ShadeGeom);  // scratch per local pixel

// One wave per workgroup: a persistent wave frees its CU slot the moment its last pixel ends, not
// when the slowest of a 4-wave workgroup's does, so the next frame in flight fills the slots of a
// draining frame sooner (round 4, profiles/round4/ab_wg: moving-camera drop-in loop 12.62 -> 12.33
// ms/frame, HEADLINE_FLY 11.96 -> 11.75; headline, C2, C3 and the 8-way share unchanged)
#ifndef FRM_MARCH_BLOCK
#define FRM_MARCH_BLOCK 64
#endif
constexpr uint32_t kMarchBlock = FRM_MARCH_BLOCK;  // march_persistent threads per workgroup
// The persistent kernel's work queue (its chunks of 64 fetch positions, most expensive first),
// XCD-aware. One claim counter for the whole GPU serialised every claim at one address: C3 waves
// parked 57 % of their cycles in the claim's wait (PMC SQ_WAIT_ANY; tools/diag_waves.py: the refill
// block took 62 % of wave time). Now the head of the order (its first 1/kQueueHeadDiv chunks, the
// most expensive) is claimed from one shared counter, so waves of every XCD start the frame's
// longest pixels first; the rest is dealt round-robin over kQueueParts partitions (chunk c to
// partition c % kQueueParts, keeping the order's slope in each), one per XCD, each claimed through
// its own counter in its own 256-B line by the waves of that XCD (HW_REG_XCC_ID); a wave whose
// partition is drained moves on to the next. C3 1.75 -> 1.11 ms, headline 10.40 -> 10.25 ms, the
// moving-camera loops within noise (profiles/round4/ab_xq; 32 partitions or a head of 1/32: no
// better, profiles/round4/ab_qs). Placement only ever changes which lane computes a pixel, never
// its bytes.
#ifndef FRM_QUEUE_PARTS
#define FRM_QUEUE_PARTS 8
#endif
#ifndef FRM_QUEUE_HEAD_DIV
#define FRM_QUEUE_HEAD_DIV 8
#endif
constexpr uint32_t kXcds = 8;                           // MI355X
constexpr uint32_t kQueueParts = FRM_QUEUE_PARTS;       // a multiple of kXcds: kQueueParts / 8 per XCD
constexpr uint32_t kQueueHeadDiv = FRM_QUEUE_HEAD_DIV;  // the shared head: nchunks / kQueueHeadDiv chunks
static_assert(kQueueParts % kXcds == 0 && kQueueParts <= 32, "queue partitions: a multiple of the XCDs, <= 32");
constexpr uint32_t kQueuePartWords = 64;    // u32 words between two counters (256 B); the head's is
                                            // counter kQueueParts
constexpr uint32_t kQueueDebugWord = (kQueueParts + 1u) * kQueuePartWords;  // FRM_STAMPS words after the counters
constexpr size_t kQueueBytes = (kQueueDebugWord + 64u) * 4u;
constexpr uint32_t kMarchWaves = kMarchBlock / 64u;
// KernelArgs::first_info bits: the frame skips step 0 / the step exited by bailout / its cost
constexpr uint32_t kFirstSkip = 1u << 31, kFirstBail = 1u << 30, kFirstCostMask = (1u << 30) - 1u;
constexpr uint32_t kRankWords = 512;  // one launch's key_hist: 256 counts + 256 cursors
constexpr uint32_t kShadeBlockPixels = 4096;  // shade_pass / rank_pass: local pixels per 256-thread block

// ---- resident frame ring (frm_api.hip resident_render; march_persistent<..., RES>) ----------
// Single-frame frm_render calls on a context with frames in flight post their frames to a ring
// of kRingSlots-or-fewer slots instead of launching a grid per frame. One persistent grid serves
// the ring for as long as frames keep arriving: its march waves claim the oldest posted frame's
// chunks and move on to the next frame when that one's queue drains (as a multi-frame launch
// interleaves its frames), and a few service waves of the same grid shade, rank and publish each
// frame once its last pixel has marched. Frames are numbered 1, 2, ... (seq); frame g uses slot
// (g - 1) % slots. The host posts frame g only after frame g - slots is done (its slot is free).
constexpr uint32_t kRingSlots = 4;
constexpr uint32_t kRingGridIds = 8;  // RingHost::grid_stop entries (grid id % 8)
constexpr uint32_t kRingTaskPixels = 16384;  // local pixels per shade or rank task (256 per lane)

// One posted frame (pinned host memory; the host writes it before it posts the frame, the
// device reads it with system-scope loads).
struct RingFrame {
  float row[3][4];     // camera_matrix rows (FrameCamera)
  float ox, oy, oz;    // camera origin
  float mb_power;      // the Mandelbulb's power at the frame's time (fragment.wgsl:75)
  uint32_t seq;
  uint32_t pad0;
  uint32_t* host_img;  // zero-copy readback: the shading also stores the frame here (or nullptr)
  uint32_t pad[12];
};
static_assert(sizeof(RingFrame) == 128, "RingFrame: 128 bytes");

// Host <-> device words (pinned, fine-grained host memory), each in its own 128-byte line.
struct RingHost {
  uint32_t posted;               // host: the last posted seq (release store after the frame's data)
  uint32_t pad0[31];
  uint32_t closed;               // device: id of the last grid that closed (stopped taking frames)
  uint32_t pad1[31];
  uint32_t grid_stop[kRingGridIds][32];  // host: grid id i serves no frame >= grid_stop[i % 8][0]
  uint32_t done[kRingSlots][32];         // device: seq of the slot's last completed frame
  RingFrame frames[kRingSlots];
};

// Per-frame device state: the claim and completion counters of one frame, in one of 2 x slots
// sets (frame g: set (g - 1) % (2 R)). Each counter is a 64-bit word whose high half is the seq of
// the frame it counts (an "epoch"). The frame that completes writes the set of frame g + R (last used
// by frame g - R, done before g was posted) with that frame's epoch and zero counts, so an atomic
// that arrives late for a finished frame lands on a set nobody reuses for another frame's length,
// and one that meets a foreign epoch is recognised. Each word sits in its own 256-byte line.
struct RingFrameCtl {
  unsigned long long queue[(kQueueParts + 1u) * (kQueuePartWords / 2u)];  // claim counters: partition x at
                                                                          // x * 32, the head at kQueueParts * 32
  unsigned long long pix_done[32];    // local pixels whose march has ended
  unsigned long long shade_next[32];  // shade tasks claimed
  unsigned long long shade_done[32];  // shade tasks done
  unsigned long long rank_next[32];   // rank tasks claimed
  unsigned long long rank_done[32];   // rank tasks done
  uint32_t hist[kRankWords];          // cost-key histogram (256) + rank cursors (256)
};
constexpr uint32_t kRingSets = 2u * kRingSlots;

struct RingGridCtl {  // per grid launch (zeroed before it)
  uint32_t closed, limit, limit_valid, pad[61];
};

struct RingDev {  // device memory, per context
  uint32_t base;  // the first seq the next grid serves (its predecessor's last + 1)
  uint32_t pad[63];
  RingGridCtl grid;
  uint32_t done_seq[kRingSlots][64];  // per slot: its last completed frame (device copy of RingHost::done)
  RingFrameCtl set[kRingSets];
  // FRM_RING_TRACE builds: per frame (seq % 64) the 100 MHz device time of its first posting seen,
  // first claim, last claim, march end, shading end, completion; per grid (id % 64) start and close
  unsigned long long trace[64][8];
  unsigned long long grid_trace[64][4];
};

// A grid's view of the ring (KernelArgs::ring).
struct RingArgs {
  RingHost* host;
  RingDev* dev;
  uint32_t slots;          // ring size R: 2 or 4 (slot = (seq - 1) & (R - 1))
  uint32_t grid_id;
  uint32_t first_seq;      // the frame this grid was launched for
  uint32_t service_waves;  // workgroups 0..service_waves-1 shade, rank and publish
  uint32_t* out;           // device framebuffers: slot s at out + s * rec_stride words
  uint32_t* order;         // fetch orders: slot s at order + s * rec_stride
  uint8_t* keys;           // cost keys: slot s at keys + s * rec_stride
};

struct KernelArgs {
  FrameUniforms f;
  SceneUniforms s;
  BandGeometry g;
  uint32_t* out;                  // packed RGBA8 words, local row-major, pitch = width
  unsigned long long* counters;   // FRM_NUM_COUNTERS, accumulated
  unsigned int* queue;            // persistent kernel: work-queue head (zeroed per launch)
  ShadeGeom* geom;                // persistent kernel: local_rows * width hit records
  ShadeTail* tails;               // persistent kernel: local_rows * width march-end records
  uint32_t npix;                  // persistent kernel: pixels of the launch (= fetch positions)
  uint32_t service_min;           // persistent kernel: lanes waiting before a service pass
  unsigned long long* debug;      // diagnostic builds only (FRM_STAMPS): 5 x u64
  const uint32_t* pixel_order;    // persistent kernel: local pixel index at each fetch position
  uint8_t* pixel_key;             // persistent kernel: cost key per local pixel (out)
  // Multi-frame launch (frm_render_bands_batch): `batch` frames of the same scene share one
  // work queue; queue chunk c (64 positions) holds pixel_order[(c / batch) * 64 + 0..63] of
  // frame c % batch (each frame's pixels heaviest first, frames interleaved chunk by chunk).
  // Frame k's records start at k * rec_stride, its output at out + k * out_stride, its
  // camera is cams[k]. batch = 1: cams[0] = f.row / f.origin (the built-in persistent kernel
  // reads cams[] for every launch; frm_reload's single-frame kernels read f).
  uint32_t batch;
  uint32_t rec_stride;            // records per frame
  uint32_t out_stride;            // packed RGBA8 words per frame
  // Fused scheduling (frm_api.hip launch; nullptr: off). The shading pass counts the cost keys
  // of the launch's last frame into key_hist[0..255]; rank_pass then ranks the local pixels by
  // descending key into order_out (the 8-bit counting sort the hipcub path does: bucket bases from
  // that histogram, per-block ranges reserved through the cursors key_hist[256..511]), the fetch
  // order of the slot's next launch; the shading pass also zeroes that launch's histogram and
  // cursors (key_hist_next[0..511]) and its work-queue counters. A steady-state frame then has two
  // short dispatches (shade, rank) between its march and the slot's next march, instead of the
  // queue memset and the hipcub sort's dispatches.
  uint32_t* key_hist;
  uint32_t* key_hist_next;
  uint32_t* order_out;
  FrameCamera cams[kMaxBatch];
  // Multi-frame launch of an animated Mandelbulb (frames that differ in time, hence in the power
  // only: fragment.wgsl:75): frame k's power. Used by the ANIM instantiation of march_persistent,
  // which carries a per-lane power; s.mb_power otherwise.
  float mb_powers[kMaxBatch];
  // Step 0 of frame k's primary rays (launch_persistent, built-in kernels; 0 = none): every one
  // samples ray_at(origin, 0, dir) = origin, the same point for all the frame's pixels, so its DE
  // is evaluated once on the host with the kernels' own source (frm_scene.h, bit-identical to the
  // device: tests/native) and each fetched pixel starts at step 1 with t = first_t[k].
  // first_info[k]: the step's cost (Mandelbulb bodies, else 1 DE) | kFirstBail | kFirstSkip.
  float first_t[kMaxBatch];
  uint32_t first_info[kMaxBatch];
  // the skipped steps' counts over the launch (primary DEs, Mandelbulb bodies, bailouts), added to
  // the counters once by the first wave
  unsigned long long first_counts[3];
  uint32_t anim;
  RingArgs ring;  // march_persistent<..., RES = true>: the resident frame ring
};


#if !defined(__HIPCC_RTC__)  // host-side launchers; hiprtc only needs the types above
// Render kernels compiled at run time from edited sources (frm_reload.hip), per DE family
// (Family in frm_scene.h) and ITERS.
constexpr uint32_t kNumFamilies = 6;
struct ReloadedKernels {
  hipModule_t module = nullptr;
  hipFunction_t simple[kNumFamilies][2] = {};
  hipFunction_t persistent[kNumFamilies][2] = {};
  hipFunction_t shade[kNumFamilies] = {};
  int persistent_blocks_per_cu[kNumFamilies][2] = {};
};
// frm_reload.hip: FRM_OK and *out, or an FRM_ERR_* code and the compiler log in *log.
int compile_reloaded(const char* dir, int device, ReloadedKernels** out, std::string* log);
void unload_reloaded(ReloadedKernels* rk);

// frm_kernels.hip (rk: a reloaded module's kernels, or nullptr for the built-in ones)
enum KernelKind : uint32_t { kKernelPersistent = 0, kKernelSimple = 1 };
// blocks_cap: at most this many persistent workgroups (one wave each) per CU; 0 = the occupancy limit
hipError_t launch_render(const KernelArgs& args, KernelKind kind, int cu_count, hipStream_t stream,
                         const ReloadedKernels* rk, int blocks_cap = 0);
// A resident ring grid (RingArgs in args.ring) on `stream`; *out_blocks: its workgroups.
hipError_t launch_ring(const KernelArgs& args, int cu_count, hipStream_t stream, int* out_blocks);
hipError_t launch_blit(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh,
                       uint32_t flags, hipStream_t stream);
hipError_t launch_unshuffle(const uint8_t* src, size_t rank_stride, uint8_t* dst, uint32_t width,
                            uint32_t height, uint32_t band_rows, uint32_t ranks,
                            hipStream_t stream);
// Pixel scheduling (frm_sched.hip). With history, order = the local pixels 0..npix-1
// (iota) by descending key[p], the cost key the last launch recorded for pixel p (stable,
// one 8-bit radix pass); without, order = iota (row-major).
hipError_t schedule_pixels(uint32_t npix, bool has_history, const uint8_t* key, uint8_t* key_sorted,
                           const uint32_t* iota, uint32_t* order, void* temp, size_t temp_bytes,
                           hipStream_t stream);
hipError_t fill_iota(uint32_t* out, uint32_t n, hipStream_t stream);
// Whole-frame key map sw x sh -> dw x dh, nearest neighbour (history across a resize).
hipError_t rescale_keys(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh,
                        hipStream_t stream);
size_t schedule_temp_bytes(uint32_t npix);
hipError_t launch_eval_scene(const SceneUniforms& s, const float* pts, uint32_t n, float* dist, float* color,
                             hipStream_t stream);
hipError_t launch_eval_math(int fn, const float* a, const float* b, uint32_t n, float* out, hipStream_t stream);
// 10 floats per local pixel from a persistent launch's records (frm_debug_trace)
hipError_t launch_trace(const KernelArgs& a, float* out, hipStream_t stream);

#endif  // !__HIPCC_RTC__

}  // namespace frm
