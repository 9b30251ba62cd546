// frm_pool_kernel.h — march_pool<MULTI>: the persistent Mandelbulb march with its pixel
// bookkeeping decoupled from the lanes that run the distance estimator (gfx950).
//
// march_persistent keeps one pixel per lane: a lane whose DE finished waits until a.service_min
// lanes of its wave wait, then the whole wave runs one service pass (distance, march step,
// normal taps, records, refill, next DE start) for the ~25 lanes that take part, and the pass
// costs the same instructions however few lanes do. Here a wave owns 128 pixels: their march
// state lives in LDS (the pool), 64 of them have a DE running in the wave's lanes and the other
// 64 sit in a per-wave exchange of 64 entries. A lane whose DE finished swaps: it deposits
// (slot, magnitude, dr, bodies) into the next exchange entry and takes the DE start stored
// there (slot, sample point, its magnitude), which costs a few instructions and two LDS
// accesses, so the lanes stay busy. When all 64 entries hold results the wave services them
// in one pass with every lane working on one entry: it loads the pixel's state from the pool,
// runs the same consume / refill / next-DE code as march_persistent's service pass (same
// operation sequence per pixel, so the same bytes and counters), stores the state back and
// leaves the next DE start in the entry.
//
// Exchange layout (wave-uniform bounds): positions [0, head) hold results (or empty slots an
// idle lane deposited), [head, n_live) DE starts not yet taken, [n_live, 64) empty slots (no
// pixel left in the queue). The service pass handles positions < head and then compacts the
// 64 entries so the DE starts come first. Slots are conserved: every swap exchanges one.
//
// Pool state of a slot (44 B in four LDS arrays):
//   P0 = (od.xyz, t): primary ray direction | the hit point during the four normal taps |
//        the shadow ray origin; the march distance (the hit distance during the taps)
//   P1 = (nsum.xyz | closeness in .x, pix): tap sum | shadow closeness; record index (kIdle:
//        empty slot)
//   P2 = (it | phase << 22 | frame << 25, psteps), P3 = cost (bodies so far, scheduling key)
#pragma once
#include "frm_render_kernels.h"

namespace frm {

constexpr uint32_t kPoolSlots = 128u;
#ifdef FRM_POOL_STAMPS
__device__ unsigned long long g_pool_debug[8];
#endif

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {  // popcount of mask's bits below this lane
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
#else
  return (uint32_t)__builtin_popcountll(mask & ((1ull << (threadIdx.x & 63u)) - 1ull));
#endif
}

template <bool MULTI>
__global__ __launch_bounds__(kMarchBlock, 5) void march_pool(KernelArgs a) {
  __shared__ float4 P0[kMarchWaves][kPoolSlots];
  __shared__ float4 P1[kMarchWaves][kPoolSlots];
  __shared__ uint2 P2[kMarchWaves][kPoolSlots];
  __shared__ uint32_t P3[kMarchWaves][kPoolSlots];
  __shared__ float4 X0[kMarchWaves][kChunk];  // result (slot, mag, dr, bodies) | DE start (slot, q)
  __shared__ float X1[kMarchWaves][kChunk];   // DE start: magnitude of q
  __shared__ float4 chunk_rays[kMarchWaves][kChunk];
  __shared__ float4 cam_origin[kMaxBatch];

  const FrameUniforms& f = a.f;
  const SceneUniforms& su = a.s;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t lane_bit = 1ull << lane;
  constexpr bool multi = MULTI;
  const uint32_t total = multi ? a.batch * ((a.npix + kChunk - 1u) / kChunk) * kChunk : a.npix;
  const uint32_t n_iter = iterations<true>(su.n);
  ShadeGeom* __restrict__ geom = a.geom;
  ShadeTail* __restrict__ tails = a.tails;

  if (threadIdx.x < kMaxBatch) {
    const v3 o = multi ? a.cams[threadIdx.x].origin : f.origin;
    cam_origin[threadIdx.x] = make_float4(o.x, o.y, o.z, 0.0f);
  }
  // every slot starts empty; lane i holds slot i, exchange entry j holds slot 64 + j
  P1[wave][lane] = make_float4(0.f, 0.f, 0.f, __uint_as_float(kIdle));
  P1[wave][lane + kChunk] = make_float4(0.f, 0.f, 0.f, __uint_as_float(kIdle));
  X0[wave][lane] = make_float4(__uint_as_float(lane + kChunk), 0.f, 0.f, 0.f);
  __syncthreads();

  // wave-uniform state
  uint32_t slots_used = kChunk, chunk_frame = 0;
  bool exhausted = false;
  uint32_t head = kChunk, n_live = 0;
  // per-wave event counts (a wave's share of one launch stays far below 2^32 events; the
  // body count is 64-bit)
  uint32_t n_pix = 0, n_hit = 0, n_prim = 0, n_shadow = 0, n_bail = 0;
  uint64_t n_body = 0;
  const uint64_t t_begin = __builtin_amdgcn_s_memrealtime();
  uint32_t n_outer = 0;
  const uint32_t swap_min = a.service_min;
#ifdef FRM_POOL_STAMPS  // diagnostic build: cycles in the service passes, swaps and body loops
  uint64_t st_service = 0, st_swap = 0, st_body = 0, n_service = 0, n_full = 0, n_swap = 0, n_loop = 0;
  const uint64_t st_begin = __builtin_amdgcn_s_memtime();
#define POOL_T0() const uint64_t pt0 = __builtin_amdgcn_s_memtime()
#define POOL_T1(acc) acc += __builtin_amdgcn_s_memtime() - pt0
#else
#define POOL_T0()
#define POOL_T1(acc)
#endif

  // lane state: the DE this lane runs (if any) and the pool slot it belongs to
  uint32_t slot = lane;
  bool has_de = false, done = false;
  v3 q = mk(0.f, 0.f, 0.f), z = q;
  float dr = 1.f, mag = 0.f;
  uint32_t body = 0;

  for (;;) {
    // ---- 1. service pass over the exchange's results: full wave when the exchange is full
    const uint64_t computing = ballot(has_de && !done);
    if (head == kChunk || (computing == 0 && head > 0)) {
      POOL_T0();
#ifdef FRM_POOL_STAMPS
      n_service++;
      n_full += head == kChunk;
#endif
      const bool mine = lane < head;  // this lane services exchange entry `lane`
      float4 e = X0[wave][lane];
      float e_mag = X1[wave][lane];
      const uint32_t s_slot = __float_as_uint(e.x) & (kPoolSlots - 1u);
      // the slot's march state
      float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = make_float4(0.f, 0.f, 0.f, __uint_as_float(kIdle));
      uint2 s2 = make_uint2(0u, 0u);
      uint32_t cost = 0;
      if (mine) {
        s0 = P0[wave][s_slot];
        s1 = P1[wave][s_slot];
        s2 = P2[wave][s_slot];
        cost = P3[wave][s_slot];
      }
      v3 od = mk(s0.x, s0.y, s0.z), nsum = mk(s1.x, s1.y, s1.z);
      float t = s0.w, closeness = s1.x;
      uint32_t pix = __float_as_uint(s1.w);
      uint32_t it = s2.x & kRecStepsMask, phase = (s2.x >> 22) & 7u, frame = s2.x >> 25, psteps = s2.y;
      const float r_mag = e.y, r_dr = e.z;
      const uint32_t r_body = __float_as_uint(e.w);

      // consume the finished DE (march_persistent's consume block on the pool state)
      const bool cons = mine && pix != kIdle;
      const bool plain_log = ballot(cons && !__builtin_amdgcn_classf(r_mag, 0x100 /* +normal */)) == 0;
      float de = 0.f;
      bool ev_bail = false;
      if (cons) {
#if defined(__HIP_DEVICE_COMPILE__)
        de = plain_log ? mb_distance_posnormal(r_mag, r_dr) : mb_distance(r_mag, r_dr);
#else
        (void)plain_log;
        de = mb_distance(r_mag, r_dr);
#endif
        cost += r_body;
        ev_bail = r_body <= n_iter;
      }
      const bool ev_prim = cons && phase == kPrimary, ev_shadow = cons && phase == kShadow;
      const bool tap = cons && !ev_prim && !ev_shadow;
      const bool hit = de <= kMinDistance;
      const bool ev_hit = ev_prim && hit;
      const float cl = min_(closeness, de / t);
      closeness = ev_shadow ? cl : closeness;
      const bool step = (ev_prim || ev_shadow) && !hit;
      const float t_next = t + de;
      const uint32_t it_next = it + 1u;
      const bool more = it_next < f.max_steps && t_next < kMaxTotalDistance;
      t = step ? t_next : t;
      it = step ? it_next : it;
      psteps = ev_hit ? it : psteps;
      const bool fin = (step && !more) || (ev_shadow && hit);
      const bool sun_miss = ev_shadow && step && !more;
      bool need_point = ev_hit || (step && more) || tap;
      const uint32_t k = phase - kTap0;
      const float dx = (k == 0u || k == 3u) ? de : -de, dy = (k >= 2u) ? de : -de,
                  dz = (k == 1u || k == 3u) ? de : -de;
      const float sx = (k == 0u) ? dx : nsum.x + dx, sy = (k == 0u) ? dy : nsum.y + dy,
                  sz = (k == 0u) ? dz : nsum.z + dz;
      nsum = mk(tap ? sx : nsum.x, tap ? sy : nsum.y, tap ? sz : nsum.z);
      if (ev_hit) {  // the taps sample around the hit point ray_at(o, t, d)
        const float4 oc = cam_origin[frame];
        od = ray_at(mk(oc.x, oc.y, oc.z), t, od);
      }
      phase = ev_hit ? kTap0 : (tap ? phase + 1u : phase);
      if (tap && k == kTap3 - kTap0) {  // normal, then the shadow ray toward the sun
        const v3 n = normalize(nsum);
        *reinterpret_cast<float4*>(&geom[pix]) = make_float4(t, n.x, n.y, n.z);
        od = shadow_origin(od, n);
        t = 0.f;
        it = 0;
        closeness = kInfinity;
      }
      if (fin) {
        const uint32_t flags = ev_shadow ? (kRecHit | (sun_miss ? kRecSunMiss : 0u)) : 0u;
        *reinterpret_cast<uint2*>(&tails[pix]) =
            make_uint2(__float_as_uint(closeness), psteps | flags | ((uint32_t)cost_key(cost) << kRecKeyShift));
        pix = kIdle;
      }
      n_prim += (uint32_t)__popcll(ballot(ev_prim));
      n_hit += (uint32_t)__popcll(ballot(ev_hit));
      n_shadow += (uint32_t)__popcll(ballot(ev_shadow));
      n_bail += (uint32_t)__popcll(ballot(ev_bail));

      // refill empty slots from the wave's chunk (fetch + ray-gen a new chunk as needed)
      for (int round = 0; round < 2; ++round) {
        const uint64_t want = ballot(mine && pix == kIdle);
        if (want == 0 || exhausted) break;
        if (slots_used == kChunk) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(a.queue, kChunk);
          base = uniform(__shfl(base, 0, 64));
          if (base >= total) {
            exhausted = true;
            break;
          }
          uint32_t p = kIdle;
          v3 ray = mk(0.f, 0.f, 0.f);
          uint32_t pos0 = base, lim = total;
          if constexpr (multi) {
            const uint32_t c = base / kChunk;
            chunk_frame = uniform(c % a.batch);
            pos0 = (c / a.batch) * kChunk;
            lim = a.npix;
          }
          if (pos0 + lane < lim) {
            const uint32_t lp = a.pixel_order[pos0 + lane];
            const uint32_t lr = lp / f.width, x = lp - lr * f.width, y = band_row_to_global(a.g, lr);
            if constexpr (multi)
              ray = camera_ray_rows(f, a.cams[chunk_frame].row, x, y);
            else
              ray = camera_ray(f, x, y);
            p = chunk_frame * a.rec_stride + lp;
          }
          n_pix += (uint32_t)__popcll(ballot(p != kIdle));
          chunk_rays[wave][lane] = make_float4(ray.x, ray.y, ray.z, __uint_as_float(p));
          __builtin_amdgcn_wave_barrier();
          slots_used = 0;
        }
        const uint32_t sl = slots_used + lanes_below(want);
        if ((want & lane_bit) && sl < kChunk) {
          const float4 r = chunk_rays[wave][sl];
          pix = __float_as_uint(r.w);
          if (pix != kIdle) {
            cost = 0;
            od = mk(r.x, r.y, r.z);
            t = 0.f;
            it = 0;
            phase = kPrimary;
            frame = chunk_frame;
            need_point = true;
          }
        }
        slots_used = min(kChunk, slots_used + (uint32_t)__popcll(want));
      }

      // next DE start: primary ray_at(o, t, d), taps hit point + s_k * MIN_DISTANCE, shadow
      // ray_at(origin, t, to_sun)
      float new_mag = 0.f;
      v3 sq = mk(0.f, 0.f, 0.f);
      if (need_point) {
        const uint32_t kq = phase - kTap0;
        const bool is_tap = kq <= kTap3 - kTap0;
        const bool sh = phase == kShadow;
        const float4 oc = cam_origin[frame];
        const v3 ro = sh ? od : mk(oc.x, oc.y, oc.z);
        const v3 rd = sh ? to_sun() : od;
        const v3 r = ray_at(ro, t, rd);
        const float eps = kMinDistance;
        const float ex = (kq == 0u || kq == 3u) ? eps : -eps, ey = (kq >= 2u) ? eps : -eps,
                    ez = (kq == 1u || kq == 3u) ? eps : -eps;
        sq = mk(is_tap ? od.x + ex : r.x, is_tap ? od.y + ey : r.y, is_tap ? od.z + ez : r.z);
        new_mag = mb_length(sq);
      }
      if (mine) {
        P0[wave][s_slot] = make_float4(od.x, od.y, od.z, t);
        P1[wave][s_slot] = make_float4(phase == kShadow ? closeness : nsum.x, nsum.y, nsum.z, __uint_as_float(pix));
        P2[wave][s_slot] = make_uint2(it | (phase << 22) | (frame << 25), psteps);
        P3[wave][s_slot] = cost;
        e = make_float4(e.x, sq.x, sq.y, sq.z);
        e_mag = new_mag;
      }
      // compact: DE starts first (new ones from this pass, then the untaken ones)
      const bool live = mine ? pix != kIdle : lane < n_live;
      const uint64_t live_mask = ballot(live);
      const uint32_t nl = (uint32_t)__popcll(live_mask);
      const uint32_t dst = live ? lanes_below(live_mask) : nl + lanes_below(~live_mask);
      __builtin_amdgcn_wave_barrier();
      X0[wave][dst] = e;
      X1[wave][dst] = e_mag;
      __builtin_amdgcn_wave_barrier();
      head = 0;
      n_live = nl;
      POOL_T1(st_service);
    }

    if (exhausted && head == 0 && n_live == 0 && ballot(has_de) == 0) break;
    if ((++n_outer & 63u) == 0 && __builtin_amdgcn_s_memrealtime() - t_begin > 400000000ull) {  // 4 s watchdog
      if (lane == 0) atomicOr((unsigned int*)a.queue + 1, 1u);
      break;
    }

    // ---- 2. swap: finished lanes deposit their result and take the next entry; idle lanes
    //         take DE starts while untaken ones remain
    {
      POOL_T0();
      const uint64_t dmask = ballot(has_de && done);
      const uint64_t imask = ballot(!has_de);
      const uint32_t nd = min((uint32_t)__popcll(dmask), kChunk - head);
      const uint32_t room = n_live > head + nd ? n_live - head - nd : 0u;
      const uint32_t ni = min((uint32_t)__popcll(imask), room);
      if (nd + ni > 0) {
        uint32_t rank;
        bool take;
        if (imask == 0) {  // steady state: every lane holds a DE
          rank = lanes_below(dmask);
          take = (dmask & lane_bit) != 0 && rank < nd;
        } else {
          const bool is_d = (dmask & lane_bit) != 0;
          rank = is_d ? lanes_below(dmask) : nd + lanes_below(imask);
          take = is_d ? rank < nd : ((imask & lane_bit) != 0 && rank < nd + ni);
        }
        if (take) {
          const uint32_t p = head + rank;
          const float4 e = X0[wave][p];
          const float m = X1[wave][p];
          X0[wave][p] = make_float4(__uint_as_float(slot), mag, dr, __uint_as_float(body));
          slot = __float_as_uint(e.x) & (kPoolSlots - 1u);
          has_de = p < n_live;
          q = mk(e.y, e.z, e.w);
          z = q;
          dr = 1.f;
          body = 0;
          mag = m;
          done = m > su.mb_bailout;  // bailout before the first body
        }
        head += nd + ni;
#ifdef FRM_POOL_STAMPS
        n_swap++;
#endif
      }
      POOL_T1(st_swap);
    }

    // ---- 3. bodies: one per computing lane per iteration, until a.service_min lanes can swap
    {
      POOL_T0();
      uint64_t pending = ballot(has_de && !done);
      const uint64_t waitable = ballot(has_de) | (n_live > head ? ~0ull : 0ull);
      for (;;) {
        if (pending == 0 || (uint32_t)__popcll(waitable & ~pending) >= swap_min) break;
        n_body += (uint64_t)__popcll(pending);
#ifdef FRM_POOL_STAMPS
        n_loop++;
#endif
        uint32_t fin = 0;
        if (lane_in(pending)) {
          mb_step(su, q, mag, z, dr);
          body++;
          if (body > n_iter) {
            fin = 1;
          } else {
            mag = mb_length(z);
            fin = mag > su.mb_bailout;
          }
        }
        pending &= ~ballot(fin != 0);
      }
      done = has_de && !lane_in(pending);
      POOL_T1(st_body);
    }
  }
#ifdef FRM_POOL_STAMPS
  if (lane == 0) {
    const uint64_t v[8] = {__builtin_amdgcn_s_memtime() - st_begin, st_service, st_swap, st_body,
                           n_service, n_full, n_swap, n_loop};
    for (int k = 0; k < 8; ++k) atomicAdd(&g_pool_debug[k], (unsigned long long)v[k]);
  }
#endif

  if (lane == 0) {
    unsigned long long v[7] = {n_pix, n_hit, n_prim, n_shadow, 4ull * n_hit, n_body, n_bail};  // widened
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (v[k]) atomicAdd(&a.counters[k], v[k]);
  }
}

}  // namespace frm
