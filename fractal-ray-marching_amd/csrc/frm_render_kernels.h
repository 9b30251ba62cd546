// frm_render_kernels.h — the render kernels of the fractal ray-marcher (gfx950):
// render_simple<FAM, ITERS>, march_persistent<FAM, ITERS> and shade_pass<FAM>, with their
// device helpers. Included by frm_kernels.hip (compiled ahead of time by hipcc) and by the
// source frm_reload compiles at run time with hiprtc (frm_reload.hip), so an edited copy of
// these headers can replace the running kernels without rebuilding the library.
//
// render_simple<FAM>: one thread per pixel, one wave64 per 8x8 pixel tile (so the 64
//   lanes of a wave march spatially coherent rays), 256-thread blocks = 16x16 pixels.
//   Literal restatement of fragment_main (fragment.wgsl:327-349): primary march, on hit
//   the four normal taps, the shadow march toward the sun and the shading; sRGB encode
//   and a packed 32-bit RGBA8 store. Work counters are reduced per wave in registers and
//   added with one 64-bit atomic per wave and counter.
#pragma once
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

// ---- persistent ray-regeneration kernel + deferred shading pass -------------------
// march_persistent<FAM>: one lane = one pixel at a time, driven by a per-lane state machine
// over the phases of fragment_main (primary march -> 4 normal taps -> shadow march).
// Every loop iteration advances every live lane by exactly one unit of DE work: one
// Mandelbulb loop body (the DE is resumable: z, dr, magnitude and body index live in
// registers), or one whole DE for the fixed-trip-count families. A lane whose pixel is
// done takes the next pixel of its wave's current chunk; a wave fetches chunks of 64
// pixels from a global queue (one atomic per chunk) in the order frm_sched.hip chose
// (most expensive pixels first), and computes the chunk's 64 camera rays in one coherent
// pass into LDS. Instead of shading at low lane occupancy, a finished
// pixel stores an 8-byte ShadeTail (+ a 16-byte ShadeGeom for a hit, at its last normal
// tap); shade_pass then shades and sRGB-packs all pixels
// coherently. Per-pixel arithmetic is the same operation sequence as shade_pixel<>, so
// the bytes are identical to render_simple and the oracle.
constexpr uint32_t kIdle = 0xFFFFFFFFu;
constexpr uint32_t kChunk = 64u;  // pixels per queue fetch (one per lane of the fetching wave)


enum Phase : uint32_t { kPrimary = 0, kTap0 = 1, kTap3 = 4, kShadow = 5 };

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// The work-queue partition a wave claims from first (frm_internal.h kQueueParts): one of the
// kQueueParts / 8 partitions of the XCD (XCC) it runs on (s_getreg HW_REG_XCC_ID, 0..7), picked by
// its workgroup index (workgroups b and b + 8 share an XCD). Placement only, never a pixel's bytes.
__device__ __forceinline__ uint32_t queue_part() {
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & (kXcds - 1u);
  constexpr uint32_t per = kQueueParts / kXcds;
  return xcc * per + (per > 1u ? (blockIdx.x / kXcds) % per : 0u);
}
__device__ __forceinline__ uint64_t count(bool c) { return (uint64_t)__popcll(ballot(c)); }

// Scheduling key of a finished pixel: 16 x log2(cost + 1), 0..255 (~4.4 % steps); cost =
// Mandelbulb bodies, or DE evaluations for the fixed-trip families. Only orders the next
// frame's fetches; never touches a pixel's bytes.
__device__ __forceinline__ uint8_t cost_key(uint32_t bodies) {
  return (uint8_t)min(255.0f, 16.0f * __log2f((float)bodies + 1.0f));
}

// ---- resident frame ring: device side (frm_internal.h RingArgs) ----------------------------
// The ring's memory is shared by waves on different XCDs, whose L2s are not coherent with each
// other, and with the host. The rules the code below follows:
//  * counters and flags are only touched by atomics, which are performed at the coherence point;
//    a poll is an atomic fetch (never a load that an acquire would have to make fresh: an acquire
//    invalidates the wave's whole L2, and polling with acquire loads ran the ring 3.5x slower);
//  * data one wave writes for another (records, cost keys, fetch orders) is stored with agent-scope
//    stores, which write through the L2, and the writer waits for its stores (ring_wait_mem) before
//    the atomic that publishes them;
//  * such data is read with agent-scope loads, which never return a stale line of the reader's
//    XCD L2 (an acquire fence instead invalidates that whole L2: one per shade/rank task and per
//    frame a march wave entered, ~10^4 per frame, slowed every wave on the XCD);
//  * host memory (RingHost: posted, descriptors; zero-copy images) is uncached: system-scope loads
//    and stores, ordered by waiting.
__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T dev_poll(T* p) {
  return __hip_atomic_fetch_add(p, (T)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T dev_load(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void dev_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits until this wave's memory accesses so far have completed.
__device__ __forceinline__ void ring_wait_mem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz
constexpr uint64_t kRingWatchdogTicks = 200000000ull;  // 2 s of the 100 MHz clock without progress
constexpr unsigned long long kEpochMask = 0xFFFFFFFF00000000ull;
__device__ __forceinline__ unsigned long long epoch_of(uint32_t seq) { return (unsigned long long)seq << 32; }
#ifdef FRM_RING_TRACE
#define RING_TRACE_MIN(r, seq, k) atomicMin(&(r).dev->trace[(seq) & 63u][k], (unsigned long long)realtime())
#define RING_TRACE_MAX(r, seq, k) atomicMax(&(r).dev->trace[(seq) & 63u][k], (unsigned long long)realtime())
#define RING_GRID_TRACE(r, k) atomicMin(&(r).dev->grid_trace[(r).grid_id & 63u][k], (unsigned long long)realtime())
#else
#define RING_TRACE_MIN(r, seq, k)
#define RING_TRACE_MAX(r, seq, k)
#define RING_GRID_TRACE(r, k)
#endif
__device__ __forceinline__ RingFrameCtl& ring_ctl(const RingArgs& r, uint32_t seq) {
  return r.dev->set[(seq - 1u) & (2u * r.slots - 1u)];
}
// The ring arguments a march wave needs, kept in LDS and read (volatile) where they are used: held
// in kernel-argument SGPRs for the whole march loop they pushed its SGPRs into VGPR lanes and those
// into scratch, reloaded on every service pass (the ring ran at 60 % of the batched march's rate).
struct RingLds {
  RingHost* host;
  RingDev* dev;
  uint32_t* order;
  uint32_t slots, grid_id, rec_stride, npix;
};
__device__ __forceinline__ uint32_t rl_u32(const volatile uint32_t& v) { return uniform(v); }
template <class T>
__device__ __forceinline__ T* rl_ptr(T* const volatile& v) {
  const uint64_t x = reinterpret_cast<uint64_t>(v);
  return reinterpret_cast<T*>((uint64_t)uniform((uint32_t)x) | ((uint64_t)uniform((uint32_t)(x >> 32)) << 32));
}
// The march-path view of the ring arguments (see RingLds), fields read at this point.
__device__ __forceinline__ RingArgs ring_view(const volatile RingLds* rl) {
  RingArgs r;
  r.host = rl_ptr(rl->host);
  r.dev = rl_ptr(rl->dev);
  r.order = rl_ptr(rl->order);
  r.slots = rl_u32(rl->slots);
  r.grid_id = rl_u32(rl->grid_id);
  r.first_seq = 0;
  r.service_waves = 0;
  r.out = nullptr;
  r.keys = nullptr;
  return r;
}

// Lane 0 adds v to an epoch-tagged counter of frame `seq` (frm_internal.h RingFrameCtl); broadcast:
// the count before the add, or ~0u when the word counts another frame.
__device__ __forceinline__ uint32_t epoch_add(unsigned long long* w, uint32_t seq, uint32_t v) {
  unsigned long long old = 0;
  if ((threadIdx.x & 63u) == 0) old = atomicAdd(w, (unsigned long long)v);
  old = __shfl(old, 0, 64);
  return (old & kEpochMask) == epoch_of(seq) ? (uint32_t)old : 0xFFFFFFFFu;
}
// A claim of one of n items: its index, or ~0u (all claimed, or another frame's counter).
__device__ __forceinline__ uint32_t epoch_claim(unsigned long long* w, uint32_t seq, uint32_t n) {
  const uint32_t t = epoch_add(w, seq, 1u);
  return t < n ? t : 0xFFFFFFFFu;
}

// The frames a grid may serve: those up to min(posted, grid_stop - 1), and after the grid has
// closed (a march wave found nothing left to claim), those up to the limit its closer fixed.
struct RingView {
  uint32_t limit;  // the last seq this wave knows it may serve
  bool closed;     // `limit` is the grid's final limit
};
__device__ __forceinline__ void ring_refresh(const RingArgs& r, RingView& v) {
  if (v.closed) return;
  uint32_t lim = 0, closed = 0;
  if ((threadIdx.x & 63u) == 0) {
    closed = dev_poll(&r.dev->grid.limit_valid);
    if (closed) {
      lim = dev_poll(&r.dev->grid.limit);
    } else {
      const uint32_t posted = sys_load(&r.host->posted);
      const uint32_t stop = sys_load(&r.host->grid_stop[r.grid_id % kRingGridIds][0]);
      lim = min(posted, stop - 1u);
#ifdef FRM_RING_TRACE
      if (lim >= 1u) RING_TRACE_MIN(r, lim, 0);
#endif
    }
  }
  v.closed = uniform(__shfl(closed, 0, 64)) != 0;
  v.limit = uniform(__shfl(lim, 0, 64));
}
// A march wave with nothing left to claim up to v.limit closes the grid: the first to get there
// publishes `closed` to the host, waits for that store, reads `posted` once more and fixes the last
// frame the grid serves; every other wave waits for that limit. Frames posted later belong to the
// next grid, which the host launches when it sees `closed` after its own post (frm_api.hip
// ring_render: each side stores, then loads the other's word, so one of them sees the other's store).
__device__ __forceinline__ void ring_close(const RingArgs& r, RingView& v) {
  uint32_t lim = 0, ok = 1;
  if ((threadIdx.x & 63u) == 0) {
    if (atomicCAS(&r.dev->grid.closed, 0u, 1u) == 0u) {
      sys_store(&r.host->closed, r.grid_id);
      RING_GRID_TRACE(r, 1);
      ring_wait_mem();
      const uint32_t posted = sys_load(&r.host->posted);
      const uint32_t stop = sys_load(&r.host->grid_stop[r.grid_id % kRingGridIds][0]);
      lim = min(posted, stop - 1u);
      atomicExch(&r.dev->grid.limit, lim);
      atomicExch(&r.dev->base, lim + 1u);
      ring_wait_mem();
      atomicExch(&r.dev->grid.limit_valid, 1u);
    } else {
      const uint64_t t0 = realtime();
      while (!dev_poll(&r.dev->grid.limit_valid)) {
        if (realtime() - t0 > 1000000ull) { ok = 0; break; }  // 10 ms: the closer stalled; stop here
        __builtin_amdgcn_s_sleep(2);
      }
      lim = dev_poll(&r.dev->grid.limit);
    }
  }
  v.closed = true;
  v.limit = uniform(__shfl(ok ? lim : 0u, 0, 64));
}

// The camera (and zero-copy image) of ring frame slot `slot`, from its RingFrame in host memory.
struct RingCam {
  float row[3][4];
  v3 origin;
  float power;
  uint32_t* host_img;
};
// The first 16 words of the RingFrame (camera rows, origin, power) into LDS (march waves).
__device__ __forceinline__ void ring_camera_lds(const RingArgs& r, uint32_t slot, float* lds) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&r.host->frames[slot]);
  const uint32_t lane = threadIdx.x & 63u;
  if (lane < 16u) lds[lane] = __uint_as_float(sys_load(w + lane));
  __syncthreads();  // one-wave workgroup: orders the LDS accesses
}
__device__ __forceinline__ RingCam ring_camera(const RingArgs& r, uint32_t slot) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&r.host->frames[slot]);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t mine = lane < 20u ? sys_load(w + lane) : 0u;  // row[12], origin[3], power, seq, pad, host_img
  RingCam c;
#pragma unroll
  for (int i = 0; i < 12; ++i) c.row[i / 4][i % 4] = __uint_as_float(uniform(__shfl(mine, i, 64)));
  c.origin = mk(__uint_as_float(uniform(__shfl(mine, 12, 64))), __uint_as_float(uniform(__shfl(mine, 13, 64))),
                __uint_as_float(uniform(__shfl(mine, 14, 64))));
  c.power = __uint_as_float(uniform(__shfl(mine, 15, 64)));
  const uint64_t lo = uniform(__shfl(mine, 18, 64)), hi = uniform(__shfl(mine, 19, 64));
  c.host_img = reinterpret_cast<uint32_t*>(lo | (hi << 32));
  return c;
}

// A ring march wave's claim state, all of it in LDS (SGPRs and VGPRs are the march's): the oldest
// frame it has not drained, the grid's frames as it last saw them, and per slot the frame the slot's
// state belongs to, its camera, its queue drain state and the pixels of that frame whose march
// ended in this wave and that the frame's pix_done does not count yet; and the slots whose frames
// the wave has drained. A slot's count goes out once the wave has drained the frame (it never
// claims from it again) and none of its lanes holds a pixel of it (ring_settle), so a frame's count
// completes only after every wave is done with it.
enum RingWaveWord : uint32_t {
  kRwLo = 0,       // the oldest frame the wave has not drained
  kRwLimit,        // the grid's frames as this wave last saw them (RingView)
  kRwClosed,
  kRwSeqOf,        // + slot: the frame the slot's state (camera, drain state) belongs to
  kRwPart = kRwSeqOf + kRingSlots,       // + slot: the queue partition the wave claims from
  kRwDrainLo = kRwPart + kRingSlots,     // + slot: drained partitions (bits 0..31; bit kQueueParts: the head)
  kRwDrainHi = kRwDrainLo + kRingSlots,  // + slot: high half
  kRwPend = kRwDrainHi + kRingSlots,     // + slot: finished pixels not yet added to pix_done
  kRwGone = kRwPend + kRingSlots,        // bit s: the wave has drained slot s's frame
  kRwWords
};
__device__ __forceinline__ uint32_t rw_get(const uint32_t* rw, uint32_t i) { return uniform(rw[i]); }
__device__ __forceinline__ void rw_set(uint32_t* rw, uint32_t i, uint32_t v) {
  if ((threadIdx.x & 63u) == 0) rw[i] = v;
}
// Records of a ring frame are read by the service waves' shading, maybe on another XCD: written
// through (agent-scope stores) and waited for (ring_add_done) before their pixels are counted, and
// read with agent-scope loads (never from a stale line of the reader's L2).
__device__ __forceinline__ void coherent_store(ShadeTail* p, uint2 v) {
  dev_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v.x | ((unsigned long long)v.y << 32));
}
__device__ __forceinline__ void coherent_store(ShadeGeom* p, float4 v) {
  unsigned long long* w = reinterpret_cast<unsigned long long*>(p);
  dev_store(w, (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32));
  dev_store(w + 1, (unsigned long long)__float_as_uint(v.z) | ((unsigned long long)__float_as_uint(v.w) << 32));
}
__device__ __forceinline__ uint2 coherent_load(const ShadeTail* p) {
  const unsigned long long v = dev_load(reinterpret_cast<const unsigned long long*>(p));
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ float4 coherent_load(const ShadeGeom* p) {
  const unsigned long long* w = reinterpret_cast<const unsigned long long*>(p);
  const unsigned long long lo = dev_load(w), hi = dev_load(w + 1);
  return make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)), __uint_as_float((uint32_t)hi),
                     __uint_as_float((uint32_t)(hi >> 32)));
}
// Adds n finished pixels to frame seq's pix_done, after the wave's record stores have completed.
__device__ __forceinline__ void ring_add_done(const volatile RingLds* rl, uint32_t seq, uint32_t n) {
  ring_wait_mem();
  const RingArgs r = ring_view(rl);
  const uint32_t before = epoch_add(&ring_ctl(r, seq).pix_done[0], seq, n);
#ifdef FRM_RING_TRACE
  if (before + n == rl_u32(rl->npix) && (threadIdx.x & 63u) == 0) RING_TRACE_MIN(r, seq, 3);
#else
  (void)before;
#endif
}
// Slot s's finished pixels into its frame's pix_done (see ring_settle).
__device__ __forceinline__ void ring_flush(const volatile RingLds* rl, uint32_t* rw, uint32_t s) {
  const uint32_t n = rw_get(rw, kRwPend + s);
  if (n) {
    ring_add_done(rl, rw_get(rw, kRwSeqOf + s), n);
    rw_set(rw, kRwPend + s, 0u);
  }
}
// A slot the wave has drained (bit s of kRwGone) whose pixels have all left its lanes (pix: the
// lanes' pixels now) is settled: its count goes out and the bit clears, once per wave and frame.
// (Counts added at every claim and every finished pixel of a drained frame were an atomic on one
// word per service pass of every wave, each behind a wait for the wave's stores: the ring marched
// at 60 % of the batched rate.)
__device__ __forceinline__ void ring_settle(const volatile RingLds* rl, uint32_t* rw, uint32_t gone, uint32_t pix) {
  const uint32_t rs = rl_u32(rl->rec_stride);
#pragma unroll
  for (uint32_t sl = 0; sl < kRingSlots; ++sl) {
    if (!((gone >> sl) & 1u) || ballot(pix - sl * rs < rs) != 0) continue;
    ring_flush(rl, rw, sl);
    rw_set(rw, kRwGone, rw_get(rw, kRwGone) & ~(1u << sl));
  }
}
// The slot of a record index (slot * rec_stride + local pixel; at most kRingSlots slots).
__device__ __forceinline__ uint32_t ring_slot_of(uint32_t pix, uint32_t rs) {
  return (uint32_t)(pix >= rs) + (uint32_t)(pix >= 2u * rs) + (uint32_t)(pix >= 3u * rs);
}
// One claim from frame seq's queue (slot s): the head of its order first, then the partitions, as
// the single-frame claim. Returns the chunk's first fetch position or kIdle (drained for this wave).
__device__ __forceinline__ uint32_t ring_claim_frame(const RingArgs& r, uint32_t* rw, uint32_t seq, uint32_t s,
                                                     uint32_t nchunks, uint32_t nhead) {
  unsigned long long* q = ring_ctl(r, seq).queue;
  constexpr uint32_t kW = kQueuePartWords / 2u;
  uint64_t drained = (uint64_t)rw_get(rw, kRwDrainLo + s) | ((uint64_t)rw_get(rw, kRwDrainHi + s) << 32);
  uint32_t part = rw_get(rw, kRwPart + s);
  uint32_t base = kIdle;
  if (!(drained >> kQueueParts)) {
    const uint32_t j = epoch_claim(q + kQueueParts * kW, seq, nhead);
    if (j != kIdle)
      base = j * kChunk;
    else
      drained |= 1ull << kQueueParts;
  }
  while (base == kIdle) {
    // partition `part` holds chunks nhead + j * kQueueParts + part below nchunks
    const uint32_t jmax = nchunks > nhead + part ? (nchunks - nhead - part + kQueueParts - 1u) / kQueueParts : 0u;
    const uint32_t j = jmax ? epoch_claim(q + part * kW, seq, jmax) : kIdle;
    if (j != kIdle) {
      base = (nhead + j * kQueueParts + part) * kChunk;
      break;
    }
    drained |= 1ull << part;
    if ((drained & ((1ull << kQueueParts) - 1ull)) == (1ull << kQueueParts) - 1ull) break;
    do part = (part + 1u) % kQueueParts;
    while ((drained >> part) & 1u);
  }
  rw_set(rw, kRwDrainLo + s, (uint32_t)drained);
  rw_set(rw, kRwDrainHi + s, (uint32_t)(drained >> 32));
  rw_set(rw, kRwPart + s, part);
  return base;
}
// The claim's rare steps, as calls (inlined, their registers pushed the march state into scratch):
// a new look at the grid's frames (and closing it), and the wave's first claim from a frame.
__device__ __noinline__ void ring_update_view(const volatile RingLds* rl, uint32_t* rw, uint32_t lo) {
  const RingArgs r = ring_view(rl);
  RingView v = {rw_get(rw, kRwLimit), rw_get(rw, kRwClosed) != 0};
  ring_refresh(r, v);
  if (lo > v.limit && !v.closed) ring_close(r, v);
  rw_set(rw, kRwLimit, v.limit);
  rw_set(rw, kRwClosed, v.closed ? 1u : 0u);
  __builtin_amdgcn_wave_barrier();
}
__device__ __noinline__ void ring_enter_frame(const volatile RingLds* rl, uint32_t* rw, float* cam, uint32_t s,
                                              uint32_t f) {
  const RingArgs r = ring_view(rl);
  ring_camera_lds(r, s, cam);
  rw_set(rw, kRwSeqOf + s, f);
  rw_set(rw, kRwDrainLo + s, 0u);
  rw_set(rw, kRwDrainHi + s, 0u);
  rw_set(rw, kRwPart + s, queue_part());
  __builtin_amdgcn_wave_barrier();
}
// The next chunk for a ring march wave. Returns the chunk's first fetch position (kIdle: nothing
// left for this grid) and its slot (*out_slot); the slot's camera is in cam_lds[slot].
// Frames in posting order: the wave claims from the oldest frame it has not drained and moves on
// when that frame's queue is empty for it. Each frame's claims thus end while the next frame still
// has most of its chunks, so the frame completes (is shaded and published, its slot freed) while
// the grid marches the next one, and the host posts the frame after that before the grid runs
// dry: with two slots the grid never closes in a steady loop. (Round-robin claims over the posted
// frames drained two frames together, as a 2-frame multi-frame launch: the grid then closed after
// every pair and paid a drain per pair; measured no faster.)
__device__ __forceinline__ uint32_t ring_claim(const volatile RingLds* rl, uint32_t* rw, float (*cam_lds)[16],
                                               uint32_t nchunks, uint32_t nhead, uint32_t pix, uint32_t* out_slot) {
  const uint32_t R = rl_u32(rl->slots);
  for (;;) {
    const uint32_t f = rw_get(rw, kRwLo);
    if (f > rw_get(rw, kRwLimit)) {
      ring_update_view(rl, rw, f);
      if (f > rw_get(rw, kRwLimit)) return kIdle;  // nothing left for this grid
    }
    const uint32_t s = (f - 1u) & (R - 1u);
    if (rw_get(rw, kRwSeqOf + s) != f) {  // the wave's first claim from frame f
      ring_enter_frame(rl, rw, cam_lds[s], s, f);
      rw_set(rw, kRwGone, rw_get(rw, kRwGone) & ~(1u << s));
    }
    const RingArgs r = ring_view(rl);
    const uint32_t base = ring_claim_frame(r, rw, f, s, nchunks, nhead);
    if (base != kIdle) {
#ifdef FRM_RING_TRACE
      if ((threadIdx.x & 63u) == 0) {
        RING_TRACE_MIN(r, f, 1);
        RING_TRACE_MAX(r, f, 2);
      }
#endif
      *out_slot = s;
      return base;
    }
    rw_set(rw, kRwGone, rw_get(rw, kRwGone) | (1u << s));  // drained for this wave: it never claims from frame f again
    ring_settle(rl, rw, 1u << s, pix);
    rw_set(rw, kRwLo, f + 1u);
  }
}

// Wave-wide exclusive prefix sum of one value per lane.
__device__ __forceinline__ uint32_t wave_exclusive_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(inc, off, 64);
    if (lane >= (uint32_t)off) inc += u;
  }
  return inc - v;
}

// Shade task t of ring frame `seq` (slot s): kRingTaskPixels local pixels, 64 at a time, as
// shade_pass (fragment.wgsl:333-348 + the Rgba8UnormSrgb store) with the frame's ring camera; the
// cost keys go out for the slot's next fetch order and into the frame's key histogram.
template <uint32_t FAM>
__device__ void ring_shade_task(const KernelArgs& a, const RingCam& cam, uint32_t seq, uint32_t s, uint32_t t,
                                const float* table, uint32_t* cnt) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t width = a.f.width, npix = a.npix, rs = a.rec_stride;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) cnt[lane * 4u + k] = 0u;
  __syncthreads();  // one-wave workgroup: orders the LDS accesses
  for (uint32_t j = 0; j < kRingTaskPixels / 64u; ++j) {
    const uint32_t idx = t * kRingTaskPixels + j * 64u + lane;
    if (idx >= npix) break;
    const uint32_t lr = idx / width, x = idx - lr * width;
    const uint32_t y = band_row_to_global(a.g, lr);
    const uint32_t rec = s * rs + idx;
    const uint2 r1 = coherent_load(&a.tails[rec]);
    const uint32_t key = r1.y >> kRecKeyShift;
    dev_store(&a.ring.keys[rec], (uint8_t)key);
    atomicAdd(&cnt[key], 1u);
    uint32_t word = 255u << 24;  // miss: BACKGROUND_COLOR
    if (r1.y & kRecHit) {
      const float4 r0 = coherent_load(&a.geom[rec]);
      const v3 dir = camera_ray_rows(a.f, cam.row, x, y);
      const v3 hp = ray_at(cam.origin, r0.x, dir);
      const v3 n = mk(r0.y, r0.z, r0.w);
      float spec;
      v3 color = shade_hit_pre(a.f, scene_color<FAM>(hp), dir, n, r1.y & kRecStepsMask, &spec);
      color = shade_hit_post(color, spec, (r1.y & kRecSunMiss) ? -kInfinity : 0.0f, __uint_as_float(r1.x));
      word = pack_rgba(color, table);
    }
    a.ring.out[rec] = word;
    if (cam.host_img) cam.host_img[idx] = word;  // zero-copy readback (pinned host image)
  }
  __syncthreads();
  uint32_t* hist = ring_ctl(a.ring, seq).hist;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (const uint32_t c = cnt[lane * 4u + k]) atomicAdd(&hist[lane * 4u + k], c);
}

// Rank task t of ring frame `seq` (slot s): kRingTaskPixels local pixels into the slot's next fetch
// order, by descending cost key (rank_pass's counting sort: bucket bases from the frame's complete
// histogram, a range per task and key reserved through the cursors hist[256..511]; a pixel's place in
// its range from an LDS atomic on a second pass over the keys). Placement only: never a pixel's bytes.
__device__ __forceinline__ void ring_rank_task(const KernelArgs& a, uint32_t seq, uint32_t s, uint32_t t,
                                               uint32_t* cnt) {
  const uint32_t lane = threadIdx.x & 63u, npix = a.npix, rs = a.rec_stride;
  const uint8_t* keys = a.ring.keys + (size_t)s * rs;
  uint32_t* order = a.ring.order + (size_t)s * rs;
  uint32_t* hist = ring_ctl(a.ring, seq).hist;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) cnt[lane * 4u + k] = 0u;
  __syncthreads();
  for (uint32_t j = 0; j < kRingTaskPixels / 64u; ++j) {
    const uint32_t idx = t * kRingTaskPixels + j * 64u + lane;
    if (idx >= npix) break;
    atomicAdd(&cnt[dev_load(&keys[idx])], 1u);
  }
  __syncthreads();
  // descending key order: lane l holds keys 255 - 4l .. 252 - 4l; base[k] = pixels with a key above
  // k plus this task's reserved offset in bucket k
  uint32_t h[4], sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    h[i] = dev_load(&hist[255u - (lane * 4u + i)]);
    sum += h[i];
  }
  uint32_t before = wave_exclusive_scan(sum);
  uint32_t b[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t k = 255u - (lane * 4u + i);
    const uint32_t c = cnt[k];
    b[i] = before + (c ? atomicAdd(&hist[256u + k], c) : 0u);
    before += h[i];
  }
  __syncthreads();  // every lane has read its counts: the array now takes the bases
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) cnt[255u - (lane * 4u + i)] = b[i];
  __syncthreads();
  for (uint32_t j = 0; j < kRingTaskPixels / 64u; ++j) {
    const uint32_t idx = t * kRingTaskPixels + j * 64u + lane;
    if (idx >= npix) break;
    const uint32_t pos = atomicAdd(&cnt[dev_load(&keys[idx])], 1u);
    if (pos < npix) dev_store(&order[pos], idx);  // always, for a histogram of these keys
  }
}

// Every task of ring frame `seq` (slot s) is done: set up the counters of frame seq + slots (its
// epoch, zero counts, histogram and cursors), then publish the frame.
__device__ __forceinline__ void ring_finish(const KernelArgs& a, uint32_t seq, uint32_t s) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t next_seq = seq + a.ring.slots;
  RingFrameCtl& c = ring_ctl(a.ring, next_seq);
  const unsigned long long next = epoch_of(next_seq);
  if (lane <= kQueueParts) dev_store(&c.queue[lane * (kQueuePartWords / 2u)], next);
  if (lane == 16u) dev_store(&c.pix_done[0], next);
  if (lane == 17u) dev_store(&c.shade_next[0], next);
  if (lane == 18u) dev_store(&c.shade_done[0], next);
  if (lane == 19u) dev_store(&c.rank_next[0], next);
  if (lane == 20u) dev_store(&c.rank_done[0], next);
#pragma unroll
  for (uint32_t k = 0; k < kRankWords / 64u; ++k) dev_store(&c.hist[k * 64u + lane], 0u);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: before the host sees the frame done
  if (lane == 0) {
    RING_TRACE_MIN(a.ring, seq, 5);
    atomicExch(&a.ring.dev->done_seq[s][0], seq);
    sys_store(&a.ring.host->done[s][0], seq);
  }
}

// An idle service wave's pause between polls, ~13 us (4 x 127 x 64 clocks): its polls are atomics at
// the coherence point, which the march's claims and counts also go through; polling every half
// microsecond from 128 waves slowed the march to about half its rate (128 -> 512 waves: 4x worse).
__device__ __forceinline__ void ring_idle() {
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_amdgcn_s_sleep(127);
}

// A ring grid's service wave: shades, ranks and publishes the grid's frames as their marches
// complete (oldest first, any of the `slots` frames in flight), until the grid has closed and
// every frame up to its limit is done. Sleeps between polls; gives up after kRingWatchdogTicks
// without progress (the host then reports the frame as never completed, frm_api.hip).
template <uint32_t FAM>
__device__ __noinline__ void ring_service(const KernelArgs& a, uint32_t* cnt) {
  const RingArgs& R = a.ring;
  const uint32_t lane = threadIdx.x & 63u;
  const float* table = kSrgbThresholds;  // (global: the service waves share the march waves' LDS budget)
  const uint32_t npix = a.npix;
  const uint32_t ntask = (npix + kRingTaskPixels - 1u) / kRingTaskPixels;
  uint32_t seq0 = 0;
  if (lane == 0) seq0 = max(R.first_seq, dev_poll(&R.dev->base));
  seq0 = uniform(__shfl(seq0, 0, 64));
  RingView rv = {0u, false};
  uint64_t last_progress = realtime();
  unsigned long long last_pd = 0;
  for (;;) {
    if (seq0 > rv.limit) ring_refresh(R, rv);
    // skip the frames already done (another service wave finished them)
    for (;;) {
      if (seq0 > rv.limit) break;
      uint32_t d = 0;
      if (lane == 0) d = dev_poll(&R.dev->done_seq[(seq0 - 1u) & (R.slots - 1u)][0]);
      if (uniform(__shfl(d, 0, 64)) < seq0) break;
      ++seq0;
    }
    if (seq0 > rv.limit) {
      if (rv.closed) return;  // every frame of this grid is done
      if (realtime() - last_progress > kRingWatchdogTicks) return;
      ring_idle();
      continue;
    }
    bool worked = false;
    for (uint32_t g = seq0; g <= rv.limit && g < seq0 + R.slots && !worked; ++g) {
      const uint32_t s = (g - 1u) & (R.slots - 1u);
      RingFrameCtl& c = ring_ctl(R, g);
      unsigned long long pd = 0, sd = 0;
      if (lane == 0) {
        pd = dev_poll(&c.pix_done[0]);
        sd = dev_poll(&c.shade_done[0]);
      }
      pd = __shfl(pd, 0, 64);
      sd = __shfl(sd, 0, 64);
      if (g == seq0 && pd != last_pd) {  // the oldest frame's march moves: progress
        last_pd = pd;
        last_progress = realtime();
      }
      if (pd != (epoch_of(g) | npix)) continue;  // its march has not ended yet
      if (sd == (epoch_of(g) | ntask)) {
        const uint32_t t = epoch_claim(&c.rank_next[0], g, ntask);
        if (t == kIdle) continue;
        ring_rank_task(a, g, s, t, cnt);
        ring_wait_mem();  // its order entries and cursors, before it counts as done
        if (epoch_add(&c.rank_done[0], g, 1u) == ntask - 1u) ring_finish(a, g, s);
        worked = true;
      } else {
        const uint32_t t = epoch_claim(&c.shade_next[0], g, ntask);
        if (t == kIdle) continue;
        const RingCam cam = ring_camera(R, s);
        ring_shade_task<FAM>(a, cam, g, s, t, table, cnt);
        // its pixels, keys and histogram counts first; the zero-copy image's stores reach the host
        // before the frame is published (a system-scope release: the image is read by the host)
        if (cam.host_img)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        else
          ring_wait_mem();
        if (epoch_add(&c.shade_done[0], g, 1u) == ntask - 1u && lane == 0) RING_TRACE_MIN(R, g, 4);
        worked = true;
      }
    }
    if (worked) {
      last_progress = realtime();
    } else {
      if (realtime() - last_progress > kRingWatchdogTicks) return;
      ring_idle();
    }
  }
}

#ifdef FRM_STAMPS
// diagnostic build: one 16 x u64 record per wave of the last persistent launch
constexpr uint32_t kWaveDebugSlots = 16384u;
__device__ unsigned long long g_wave_debug[16u * kWaveDebugSlots];
#endif

// MULTI: a multi-frame launch (frm_render_bands_batch, a.batch > 1), a separate instantiation.
// Queue chunk c (64 fetch positions) is chunk c / batch of frame c % batch: the frames'
// pixels interleave chunk by chunk, each frame's longest first, and a chunk's frame (camera)
// is wave-uniform.
// ANIM (MULTI, Mandelbulb): the frames of the launch differ in time, so in the power; each lane
// carries its pixel's frame's power (a.mb_powers) instead of the uniform one.
// RES: a resident ring grid (frm_internal.h RingArgs): workgroups below a.ring.service_waves run
// ring_service; the others march the ring's frames in posting order, each frame's chunks as a
// single-frame launch's, moving on to the next frame when one's queue drains. A lane's record index
// is slot * rec_stride + its local pixel (as a multi-frame launch's frame * rec_stride + ...).
template <uint32_t FAM, bool ITERS, bool MULTI = false, bool ANIM = false, bool RES = false>
#ifndef FRM_MARCH_WAVES_PER_SIMD
#define FRM_MARCH_WAVES_PER_SIMD 1
#endif
#ifndef FRM_RING_WAVES_PER_SIMD
#define FRM_RING_WAVES_PER_SIMD FRM_MARCH_WAVES_PER_SIMD
#endif
__global__ __launch_bounds__(kMarchBlock, RES ? FRM_RING_WAVES_PER_SIMD : FRM_MARCH_WAVES_PER_SIMD) void march_persistent(
    KernelArgs a) {
  __shared__ float4 chunk_rays[kMarchWaves][kChunk];  // per wave: camera ray xyz + record index bits
  static_assert(!RES || (!MULTI && kMarchWaves == 1u), "ring grids: one-wave workgroups, one frame per chunk");
  __shared__ float cam_lds[RES ? kRingSlots : 1][16];  // RES: per slot the camera of its frame (rows, origin, power)
  __shared__ uint32_t rw[RES ? (uint32_t)kRwWords : 1u];  // RES: the wave's claim state (RingWaveWord)
  __shared__ RingLds ring_lds[RES ? 1 : 0 + 1];           // RES: the ring arguments of the march (RingLds)
  if constexpr (RES) {
    // service waves: key counts / bucket bases in the LDS the march waves use for chunk rays (one
    // workgroup is one wave: either kind)
    if (blockIdx.x < a.ring.service_waves) {
      // a call (inlined, the service's registers pushed the march state into scratch), on the
      // kernel arguments where they lie (a reference to the parameter copies it to scratch)
      ring_service<FAM>(*(const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr(),
                        reinterpret_cast<uint32_t*>(&chunk_rays[0][0]));
      return;
    }
  }

  const FrameUniforms& f = a.f;
  const SceneUniforms& su = a.s;
  constexpr bool kMb = is_mandelbulb(FAM);     // resumable body loop
  constexpr bool kHw = FAM == kMandelbulbHw;   // FRM_FLAG_HW_MATH
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t lane_bit = 1ull << lane;
  constexpr bool multi = MULTI;
  // fetch positions (host: < 2^32 - 1); a multi-frame launch pads each frame to whole chunks
  const uint32_t total = multi ? a.batch * ((a.npix + kChunk - 1u) / kChunk) * kChunk : a.npix;
  uint32_t chunk_frame = 0;  // wave-uniform: the frame of the wave's current chunk
  const uint32_t n_iter = iterations<ITERS>(su.n);
  static_assert(!ANIM || ((MULTI || RES) && is_mandelbulb(FAM)), "per-lane powers: multi-frame or ring Mandelbulb launches");
  float lane_power = su.mb_power;  // ANIM: the power of the lane's pixel's frame
  ShadeGeom* __restrict__ geom = a.geom;
  ShadeTail* __restrict__ tails = a.tails;

  // wave-uniform state: current chunk of 64 fetched pixels, how many were handed out
  uint32_t slots_used = kChunk;
  bool exhausted = false;
  // the work-queue partition the wave claims from (its XCD's first, kQueueParts in frm_internal.h)
  // and the partitions it has found drained
  const uint32_t nchunks = (total + kChunk - 1u) / kChunk;
  uint32_t part = queue_part();
  uint64_t drained = 0;  // bit x: partition x drained; bit kQueueParts: the head
  const uint32_t nhead = nchunks / kQueueHeadDiv;
  uint64_t n_pix = 0, n_hit = 0, n_prim = 0, n_shadow = 0, n_body = 0, n_bail = 0;
#ifdef FRM_COUNT_EXACT
  uint64_t n_dbg_total = 0, n_dbg_exact = 0;
#endif
  uint32_t r_slot = 0;                    // RES: the slot of the wave's current chunk
  if constexpr (RES) {
    uint32_t b = 0;
    if (lane == 0) {
      RING_GRID_TRACE(a.ring, 0);
      b = max(a.ring.first_seq, dev_poll(&a.ring.dev->base));
      ring_lds->host = a.ring.host;
      ring_lds->dev = a.ring.dev;
      ring_lds->order = a.ring.order;
      ring_lds->slots = a.ring.slots;
      ring_lds->grid_id = a.ring.grid_id;
      ring_lds->rec_stride = a.rec_stride;
      ring_lds->npix = a.npix;
    }
    __syncthreads();
    if (lane < (uint32_t)kRwWords) rw[lane] = 0u;
    rw_set(rw, kRwLo, uniform(__shfl(b, 0, 64)));
  }

  // per-lane state
  uint32_t pix = kIdle;      // local pixel index (lr * width + x) being marched
  uint32_t phase = kPrimary;
  bool done = false;         // the current DE has its result
  v3 o = mk(0.f, 0.f, 0.f), d = o, nsum = o, q = o, z = o;
  float t = 0.f, closeness = 0.f, dr = 1.f, mag = 0.f, de = 0.f;
  uint32_t it = 0, psteps = 0, body = 0;
  uint32_t pix_cost = 0;  // the lane's pixel's Mandelbulb bodies (other families: DEs) so far, for
                          // its scheduling key; the wave's body total is counted in SGPRs
#ifdef FRM_STAMPS
  uint64_t stamp_service = 0, n_service = 0, n_loop = 0, real_exhaust = 0;
  uint64_t stamp_consume = 0, stamp_refill = 0, n_fetch = 0;
  uint64_t stamp_sub[4] = {0, 0, 0, 0};  // consume: distance, primary, taps, shadow
  const uint64_t stamp_begin = __builtin_amdgcn_s_memtime();
  const uint64_t stamp_real0 = __builtin_amdgcn_s_memrealtime();
#define FRM_SUB_BEGIN() const uint64_t sub0 = __builtin_amdgcn_s_memtime()
#define FRM_SUB_END(k) stamp_sub[k] += __builtin_amdgcn_s_memtime() - sub0
#else
#define FRM_SUB_BEGIN()
#define FRM_SUB_END(k)
#endif

  for (;;) {
    // Body phase (Mandelbulb): one loop body per computing lane per iteration, until
    // a.service_min lanes wait for a service pass (finished DE, or idle with work left)
    // or no lane computes. The service pass costs the same however many lanes take part.
    if constexpr (kMb) {
      // The loop keeps its lane sets as wave-uniform masks (SGPRs): `pending` predicates the
      // body directly (inverse ballot -> exec) and one ballot per iteration retires lanes,
      // instead of a per-lane flag merged under exec masks every iteration.
      const uint64_t live = ballot(pix != kIdle);
      uint64_t pending = live & ~ballot(done);
      // lanes that count as waiting when not pending: finished DEs, and idle lanes while
      // the queue still has pixels
      const uint64_t waitable = exhausted ? live : ~0ull;
      for (;;) {
        if (pending == 0 || (uint32_t)__popcll(waitable & ~pending) >= a.service_min) break;
        // one body per computing lane this iteration (a DE that bails out at entry never
        // becomes pending, so this counts bodies exactly: fragment.wgsl:245-249)
        if constexpr (!RES) n_body += (uint64_t)__popcll(pending);
#ifdef FRM_STAMPS
        n_loop++;
#endif
        if (lane_in(pending)) {
#if defined(FRM_COUNT_EXACT) && defined(__HIP_DEVICE_COMPILE__)  // diagnostic: body-loop iterations, and those that ran the exact body
          n_dbg_total++;
          if (ballot(!mb_tame(z, mag)) != 0) n_dbg_exact++;
#endif
          if constexpr (ANIM)
            mb_step<kHw>(lane_power, lane_power - 1.0f, q, mag, z, dr);  // = the host's mb_power_m1
          else
            mb_step<kHw>(su, q, mag, z, dr);
          body++;
          // N+1 bodies: the distance uses the last loop-top magnitude
          if (body <= n_iter) mag = mb_length<kHw>(z);
        }
        // the lanes whose DE ends, tested by every lane outside the body's branch (other lanes'
        // bits fall outside `pending`): a flag set inside it reached the mask through a VGPR
        pending &= ~(ballot(body > n_iter) | ballot(mag > su.mb_bailout));
      }
      done = !lane_in(pending);  // idle lanes: masked by cons
    }

    // Service pass.
#ifdef FRM_STAMPS  // diagnostic build: wave cycles spent in service passes -> counters[7]
    const uint64_t stamp0 = __builtin_amdgcn_s_memtime();
#endif
    // 1. consume finished DEs. Branch-light: the bookkeeping of every phase is computed for
    //    every lane with selects; only the distance, the last-tap transition (normal, record,
    //    shadow ray) and the record store of a finished pixel are branches.
    const bool cons = pix != kIdle && done;
    bool ev_bail = false;
    // the distance's log without its special-value selects (and with the integer exponent
    // split) when every consuming lane's magnitude is positive, normal and finite
    // (wave-uniform test; same bits)
    bool plain_log = true;
    if constexpr (kMb && !kHw)
      plain_log = ballot(cons && !__builtin_amdgcn_classf(mag, 0x100 /* +normal */)) == 0;
    if (cons) {
      done = false;
      if constexpr (kMb) {
        FRM_SUB_BEGIN();
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (kHw)
          de = mb_distance_hw(mag, dr);
        else
          de = plain_log ? mb_distance_posnormal(mag, dr) : mb_distance(mag, dr);
#else
        (void)plain_log;
        de = mb_distance(mag, dr);
#endif
        pix_cost += body;          // bodies this DE ran (N+1 on a count exit)
        ev_bail = body <= n_iter;  // exit by bailout (incl. before the first body)
        FRM_SUB_END(0);
      }
    }
    const bool ev_prim = cons && phase == kPrimary, ev_shadow = cons && phase == kShadow;
    const bool tap = cons && !ev_prim && !ev_shadow;  // normal taps k.xyy, k.yyx, k.yxy, k.xxx
    const bool hit = de <= kMinDistance;              // object_result.distance >= 0
    const bool ev_hit = ev_prim && hit;
    // shadow closeness = min(closeness, d / t) before t moves (d / 0 on step 0, as in
    // fragment.wgsl:292); computed by every lane, kept by shadow lanes
    const float cl = min_(closeness, de / t);
    closeness = ev_shadow ? cl : closeness;
    const bool step = (ev_prim || ev_shadow) && !hit;  // march on: t += d, it++
    const float t_next = t + de;
    const uint32_t it_next = it + 1u;
    const bool more = it_next < f.max_steps && t_next < kMaxTotalDistance;
    t = step ? t_next : t;
    it = step ? it_next : it;
    psteps = ev_hit ? it : psteps;
    const bool fin = (step && !more) || (ev_shadow && hit);  // primary miss, or shadow march ends
    const bool sun_miss = ev_shadow && step && !more;
    bool need_point = ev_hit || (step && more) || tap;  // start a DE at the phase's next sample point
    // tap k adds s_k * d to the sum (k = 0 sets it); s_0..s_3 = (+--), (--+), (-+-), (+++)
    const uint32_t k = phase - kTap0;
    const float dx = (k == 0u || k == 3u) ? de : -de, dy = (k >= 2u) ? de : -de,
                dz = (k == 1u || k == 3u) ? de : -de;
    // (component-wise: a select of whole structs compiles to a select of stack addresses)
    const float sx = (k == 0u) ? dx : nsum.x + dx, sy = (k == 0u) ? dy : nsum.y + dy,
                sz = (k == 0u) ? dz : nsum.z + dz;
    nsum = mk(tap ? sx : nsum.x, tap ? sy : nsum.y, tap ? sz : nsum.z);
    phase = ev_hit ? kTap0 : (tap ? phase + 1u : phase);  // after the last tap: kShadow
    if (tap && k == kTap3 - kTap0) {  // normal, then the shadow ray toward the sun
      FRM_SUB_BEGIN();
      const v3 n = normalize(nsum);
      const v3 hp = ray_at(o, t, d);
      if constexpr (RES) {  // read by another wave's shading, maybe on another XCD (ring_flush)
        coherent_store(&geom[pix], make_float4(t, n.x, n.y, n.z));
      } else {
        *reinterpret_cast<float4*>(&geom[pix]) = make_float4(t, n.x, n.y, n.z);
      }
      o = shadow_origin(hp, n);
      d = to_sun();
      t = 0.f;
      it = 0;
      closeness = kInfinity;
      FRM_SUB_END(2);
    }
    if (fin) {  // primary miss (flags 0: BACKGROUND_COLOR) or end of the shadow march
      FRM_SUB_BEGIN();
      const uint32_t flags = ev_shadow ? (kRecHit | (sun_miss ? kRecSunMiss : 0u)) : 0u;
      const uint32_t ck = cost_key(pix_cost);
      const uint2 tail = make_uint2(__float_as_uint(closeness), psteps | flags | (ck << kRecKeyShift));
      if constexpr (RES)
        coherent_store(&tails[pix], tail);
      else
        *reinterpret_cast<uint2*>(&tails[pix]) = tail;
      if constexpr (RES)  // the finished pixel into its slot's count (published by ring_settle)
        atomicAdd(&rw[kRwPend + ring_slot_of(pix, rl_u32(ring_lds->rec_stride))], 1u);
      pix = kIdle;
      FRM_SUB_END(3);
    }
    if constexpr (RES) {  // drained slots whose last pixels left the lanes
      const uint32_t gone = rw_get(rw, kRwGone);
      if (gone) ring_settle(ring_lds, rw, gone, pix);
    }
    // 2. refill idle lanes from the wave's current chunk; fetch + ray-gen a new chunk
#ifdef FRM_STAMPS
    const uint64_t stamp1 = __builtin_amdgcn_s_memtime();
    stamp_consume += stamp1 - stamp0;
#endif
    const uint64_t want = ballot(pix == kIdle);
    if (want != 0 && !exhausted) {
      if (slots_used == kChunk) {
        uint32_t base = kIdle;
        if constexpr (RES) {
          base = ring_claim(ring_lds, rw, cam_lds, nchunks, nhead, pix, &r_slot);
        } else {
        // the head of the order (its most expensive chunks) from the shared counter
        if (!(drained >> kQueueParts)) {
          uint32_t j = 0;
          if (lane == 0) j = atomicAdd(a.queue + kQueueParts * kQueuePartWords, 1u);
          j = uniform(__shfl(j, 0, 64));
          if (j < nhead)
            base = j * kChunk;
          else
            drained |= 1ull << kQueueParts;
        }
        // then chunk j of the XCD's partition x is queue chunk nhead + j * kQueueParts + x; a
        // drained partition passes the wave on to the next one
        while (base == kIdle) {
          uint32_t j = 0;
          if (lane == 0) j = atomicAdd(a.queue + part * kQueuePartWords, 1u);
          j = uniform(__shfl(j, 0, 64));
          const uint32_t c = nhead + j * kQueueParts + part;
          if (c < nchunks) {
            base = c * kChunk;
            break;
          }
          drained |= 1ull << part;
          if ((drained & ((1ull << kQueueParts) - 1ull)) == (1ull << kQueueParts) - 1ull) break;
          do part = (part + 1u) % kQueueParts;
          while ((drained >> part) & 1u);
        }
        }  // !RES
#ifdef FRM_STAMPS
        n_fetch++;
#endif
        if (base == kIdle) {
          exhausted = true;
#ifdef FRM_STAMPS
          real_exhaust = __builtin_amdgcn_s_memrealtime();
          if (lane == 0) atomicMin(a.debug + 2, (unsigned long long)real_exhaust);
#endif
        } else {
          // the i-th pixel fetched is pixel_order[i]: most expensive first (the previous
          // frame's cost keys, frm_sched.hip), row-major without history
          uint32_t p = kIdle;
          v3 ray = mk(0.f, 0.f, 0.f);
          uint32_t pos0 = base, lim = total;
          // RES: the chunk's frame's camera rows (wave-uniform, SGPRs): one LDS word per lane, then
          // lane reads (twelve loads into VGPRs before their readfirstlanes pushed the march state
          // into scratch). The load is pinned here, where every lane runs: the compiler would
          // otherwise sink it into the branch below, and a lane read of a lane outside that
          // branch's mask returns garbage.
          [[maybe_unused]] float row[3][4];
          if constexpr (RES) {
            uint32_t mine = __float_as_uint(cam_lds[r_slot][lane & 15u]);
            asm volatile("" : "+v"(mine));
#pragma unroll
            for (int i = 0; i < 12; ++i) row[i / 4][i % 4] = __uint_as_float(__builtin_amdgcn_readlane(mine, i));
          }
          if constexpr (multi) {
            const uint32_t c = base / kChunk;
            chunk_frame = uniform(c % a.batch);
            pos0 = (c / a.batch) * kChunk;
            lim = a.npix;
          }
          if (pos0 + lane < lim) {
            const uint32_t lp =
                RES ? dev_load(&rl_ptr(((const volatile RingLds*)ring_lds)->order)[r_slot * a.rec_stride + pos0 + lane])
                    : a.pixel_order[pos0 + lane];
            const uint32_t lr = lp / f.width, x = lp - lr * f.width, y = band_row_to_global(a.g, lr);
            if constexpr (RES)
              ray = camera_ray_rows(f, row, x, y);
            else if constexpr (multi)
              ray = camera_ray_rows(f, a.cams[chunk_frame].row, x, y);
            else
              ray = camera_ray(f, x, y);
            p = (RES ? r_slot * a.rec_stride : chunk_frame * a.rec_stride) + lp;  // the pixel's record index
          }
          if constexpr (!RES) n_pix += count(p != kIdle);
          chunk_rays[wave][lane] = make_float4(ray.x, ray.y, ray.z, __uint_as_float(p));
          __builtin_amdgcn_wave_barrier();
          slots_used = 0;
        }
      }
      if (slots_used < kChunk) {
        const uint32_t slot = slots_used + __popcll(want & (lane_bit - 1ull));
        // RES: the chunk's frame's origin and power, read as the camera rows above
        [[maybe_unused]] float cam_o[4];
        if constexpr (RES) {
          uint32_t mine = __float_as_uint(cam_lds[r_slot][12u + (lane & 3u)]);
          asm volatile("" : "+v"(mine));
#pragma unroll
          for (int i = 0; i < 4; ++i) cam_o[i] = __uint_as_float(__builtin_amdgcn_readlane(mine, i));
        }
        if ((want & lane_bit) && slot < kChunk) {
          const float4 r = chunk_rays[wave][slot];
          pix = __float_as_uint(r.w);
          if (pix != kIdle) {
            // the frame's step 0 done once (KernelArgs::first_info; ring frames run it per pixel):
            // start at step 1 where consuming it would leave the pixel
            const uint32_t fy = RES ? 0u : a.first_info[chunk_frame];
            const bool first_skip = (fy & kFirstSkip) != 0u;
            pix_cost = first_skip ? (fy & kFirstCostMask) : 0u;
            d = mk(r.x, r.y, r.z);
            if constexpr (RES)
              o = mk(cam_o[0], cam_o[1], cam_o[2]);
            else
              o = multi ? a.cams[chunk_frame].origin : f.origin;
            if constexpr (RES && ANIM)
              lane_power = cam_o[3];
            else if constexpr (ANIM)
              lane_power = a.mb_powers[chunk_frame];
            t = first_skip ? a.first_t[chunk_frame] : 0.f;
            it = first_skip ? 1u : 0u;
            phase = kPrimary;
            need_point = true;
          }
        }
        slots_used = min(kChunk, slots_used + (uint32_t)__popcll(want));
      }
    }

#ifdef FRM_STAMPS
    stamp_refill += __builtin_amdgcn_s_memtime() - stamp1;
#endif
    // 3. start the next DE of every lane that needs one (the hit point of the normal
    //    taps is recomputed from the unchanged primary ray: ray_at(o, t_hit, d))
    if (need_point) {
      const v3 r = ray_at(o, t, d);
      // normal tap k samples r + s_k * MIN_DISTANCE (normal_tap_pos), with selects
      const uint32_t kq = phase - kTap0;
      const bool is_tap = kq <= kTap3 - kTap0;
      const float e = kMinDistance;
      const float ex = (kq == 0u || kq == 3u) ? e : -e, ey = (kq >= 2u) ? e : -e, ez = (kq == 1u || kq == 3u) ? e : -e;
      q = mk(is_tap ? r.x + ex : r.x, is_tap ? r.y + ey : r.y, is_tap ? r.z + ez : r.z);
      if constexpr (kMb) {
        z = q;
        dr = 1.f;
        body = 0;
        mag = mb_length<kHw>(q);
        done = mag > su.mb_bailout;
      } else {
        DeCount unused = {0u, 0u};
        de = scene_de<FAM, ITERS>(su, q, unused);
        done = true;
        pix_cost++;  // fixed-trip families: the scheduling cost unit is one DE
      }
    }

    // work counters (frm_stats); a ring grid's frames report none (frm_render with stats renders
    // outside the ring), so it keeps no counters
    if constexpr (!RES) {
      n_prim += count(ev_prim);
      n_hit += count(ev_hit);
      n_shadow += count(ev_shadow);
      n_bail += count(ev_bail);
    }
#ifdef FRM_STAMPS
    stamp_service += __builtin_amdgcn_s_memtime() - stamp0;
    n_service++;
#endif

    if (exhausted && ballot(pix != kIdle) == 0) break;
  }
  if constexpr (RES) {
#pragma unroll
    for (uint32_t sl = 0; sl < kRingSlots; ++sl)
      if (sl < a.ring.slots) ring_flush(ring_lds, rw, sl);
  }

#ifdef FRM_STAMPS
  if (lane == 0) {
    atomicAdd(&a.counters[7], (unsigned long long)stamp_service);
    atomicAdd(a.debug, (unsigned long long)(__builtin_amdgcn_s_memtime() - stamp_begin));
    atomicAdd(a.debug + 1, (unsigned long long)n_service);
    atomicMin(a.debug + 3, (unsigned long long)stamp_real0);  // first wave start (100 MHz)
    atomicMax(a.debug + 4, (unsigned long long)__builtin_amdgcn_s_memrealtime());  // last wave end
  }
  {
    const uint32_t w = blockIdx.x * kMarchWaves + wave;
    uint32_t hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (lane == 0 && w < kWaveDebugSlots) {
      unsigned long long* r = g_wave_debug + 16u * w;
      r[8] = stamp_consume;
      r[9] = stamp_refill;
      r[10] = n_fetch;
      for (int k = 0; k < 4; ++k) r[11 + k] = stamp_sub[k];
      r[0] = n_loop;
      r[1] = n_body;
      r[2] = n_service;
      r[3] = stamp_service;
      r[4] = __builtin_amdgcn_s_memtime() - stamp_begin;
      r[5] = stamp_real0;
      r[6] = real_exhaust;
      r[7] = ((unsigned long long)hw << 32) | (uint32_t)(__builtin_amdgcn_s_memrealtime() - stamp_real0);
    }
  }
#endif
  if (lane == 0 && !RES) {
#ifdef FRM_COUNT_EXACT
    atomicAdd(&a.counters[7], (unsigned long long)((n_dbg_total << 32) | n_dbg_exact));
#endif
    if (blockIdx.x == 0 && wave == 0) {  // the launch's skipped steps 0 (KernelArgs::first_counts)
      n_prim += a.first_counts[0];
      n_body += a.first_counts[1];
      n_bail += a.first_counts[2];
    }
    unsigned long long v[7] = {n_pix, n_hit, n_prim, n_shadow, 4ull * n_hit, n_body, n_bail};
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (v[k]) atomicAdd(&a.counters[k], v[k]);
  }
}

// Exclusive prefix sum over the 256 threads of a block (4 waves), one value per thread.
__device__ __forceinline__ uint32_t block_exclusive_scan256(uint32_t v, uint32_t* wave_tot) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(inc, off, 64);
    if (lane >= (uint32_t)off) inc += u;
  }
  if (lane == 63u) wave_tot[wave] = inc;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += wave_tot[w];
  return before + inc - v;
}

// The shading of one pixel's records (fragment.wgsl:333-348 + the Rgba8UnormSrgb store).
template <uint32_t FAM>
__device__ __forceinline__ void shade_record(const KernelArgs& a, uint2 r1, uint32_t rec, uint32_t fr, uint32_t idx,
                                             uint32_t x, uint32_t y, const float* table) {
  uint32_t word = 255u << 24;  // miss: BACKGROUND_COLOR
  if (r1.y & kRecHit) {
    const float4 r0 = *reinterpret_cast<const float4*>(&a.geom[rec]);
    const bool multi = a.batch > 1u;
    const v3 dir = multi ? camera_ray_rows(a.f, a.cams[fr].row, x, y) : camera_ray(a.f, x, y);
    const v3 hp = ray_at(multi ? a.cams[fr].origin : a.f.origin, r0.x, dir);
    const v3 n = mk(r0.y, r0.z, r0.w);
    float spec;
    v3 color = shade_hit_pre(a.f, scene_color<FAM>(hp), dir, n, r1.y & kRecStepsMask, &spec);
    color = shade_hit_post(color, spec, (r1.y & kRecSunMiss) ? -kInfinity : 0.0f, __uint_as_float(r1.x));
    word = pack_rgba(color, table);
  }
  a.out[(size_t)fr * a.out_stride + idx] = word;
}

// Coherent shading of the records written by march_persistent: fragment.wgsl:333-348
// (+ the Rgba8UnormSrgb store). A block shades kShadeBlockPixels local pixels, row-major, 256
// at a time (coalesced). With fused scheduling (KernelArgs::key_hist) it also counts the cost
// keys of the launch's last frame (an LDS histogram per block, one global add per key present:
// few blocks, so few adds on the hot keys' counters) and resets the slot's next launch.
template <uint32_t FAM>
__global__ __launch_bounds__(256) void shade_pass(KernelArgs a) {
  __shared__ float table[256];
  __shared__ uint32_t s_count[256];
  const uint32_t t = threadIdx.x;
  const uint32_t fr = blockIdx.y;  // frame of a multi-frame launch (0 otherwise)
  // fused scheduling: the key histogram of the launch's last frame (block-uniform)
  const bool hist = a.key_hist != nullptr && fr + 1u == a.batch;
  table[t] = kSrgbThresholds[t];
  if (hist) s_count[t] = 0u;
  __syncthreads();
  const uint32_t width = a.f.width, local = a.g.local_rows * width;
  for (uint32_t j = 0; j < kShadeBlockPixels / 256u; ++j) {
    const uint32_t idx = (blockIdx.x * (kShadeBlockPixels / 256u) + j) * 256u + t;
    if (idx >= local) break;
    const uint32_t lr = idx / width, x = idx - lr * width;
    const uint32_t y = band_row_to_global(a.g, lr);
    if (y >= a.f.height) break;  // the short last band's missing rows: the launch's last local rows
    const uint32_t rec = fr * a.rec_stride + idx;
    const uint2 r1 = *reinterpret_cast<const uint2*>(&a.tails[rec]);
    const uint32_t key = r1.y >> kRecKeyShift;
    // coalesced, for the next launch's order (a multi-frame launch: its last frame's costs)
    if (a.pixel_key && fr + 1u == a.batch) a.pixel_key[idx] = (uint8_t)key;
    if (hist) atomicAdd(&s_count[key], 1u);
    shade_record<FAM>(a, r1, rec, fr, idx, x, y, table);
  }
  if (!hist) return;
  __syncthreads();
  if (const uint32_t c = s_count[t]) atomicAdd(a.key_hist + t, c);
  if (blockIdx.x == 0) {  // the slot's next launch starts from zeroed counts, cursors and queue
    a.key_hist_next[t] = 0u;
    a.key_hist_next[256u + t] = 0u;
    for (uint32_t w = t; w < kQueueDebugWord; w += 256u) a.queue[w] = 0u;
  }
}

// Fused scheduling, after shade_pass: the next launch's fetch order, the local pixels by descending
// cost key (an 8-bit counting sort: bucket bases from the shading pass's histogram, one range per
// block and bucket reserved through the cursors key_hist[256..511], the block's kShadeBlockPixels
// pixels ranked in LDS). Ties are ordered by block, then as the LDS atomics happen to run: the
// order places pixels on lanes, it never changes a pixel's bytes.
__global__ __launch_bounds__(256) void rank_pass(const uint8_t* __restrict__ keys, uint32_t npix,
                                                 uint32_t* __restrict__ hist, uint32_t* __restrict__ order) {
  constexpr uint32_t kPer = kShadeBlockPixels / 256u;
  __shared__ uint32_t s_base[256], s_count[256], s_res[256], s_wave[4];
  const uint32_t t = threadIdx.x;
  s_count[t] = 0u;
  __syncthreads();
  uint32_t key[kPer], rank[kPer];
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t idx = (blockIdx.x * kPer + j) * 256u + t;
    key[j] = idx < npix ? keys[idx] : 0u;
    rank[j] = idx < npix ? atomicAdd(&s_count[key[j]], 1u) : 0u;
  }
  // bucket bases in descending key order: base[k] = pixels with a key above k
  const uint32_t k_desc = 255u - t;
  s_base[k_desc] = block_exclusive_scan256(hist[k_desc], s_wave);  // its barrier completes s_count
  const uint32_t c = s_count[t];
  s_res[t] = c ? atomicAdd(hist + 256u + t, c) : 0u;
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t idx = (blockIdx.x * kPer + j) * 256u + t;
    const uint32_t pos = s_base[key[j]] + s_res[key[j]] + rank[j];
    if (idx < npix && pos < npix) order[pos] = idx;  // pos < npix always, for a histogram of these keys
  }
}

// dst row y <- band b = y / band_rows, held by rank b % ranks as its (b / ranks)-th band.
// T = uint4 when rows and rank strides are 16-byte multiples, else uint32_t.
}  // namespace frm
