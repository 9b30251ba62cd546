// Round 6: mechanisms a resident frame pipeline would rest on, measured on the MI355X before any
// libfrm code depends on them (C host, /opt/rocm runtime, no torch). Every device spin loop is
// bounded by a deadline on the 100 MHz s_memrealtime clock, so no wave outlives its test.
//  A. hipStreamWaitValue32 on hipMallocSignalMemory / hipMalloc / pinned host memory, released by
//     a kernel's system-scope store on another stream: does the wait hold, and how late does the
//     waiting stream's next kernel start after the store?
//  B. host -> device -> host round trip through fine-grained pinned memory: a one-wave kernel polls
//     a word the host writes and acknowledges it in another word.
//  C. zero-copy: a kernel writing a 33 MB frame straight into pinned host memory (GB/s).
//  D. a full-occupancy grid whose waves sleep-poll a pinned word while a D2H hipMemcpyAsync runs on
//     another stream: does the copy finish before the grid is released?
//   resident_probe  -> one JSON object per test on stdout
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

using Clock = std::chrono::steady_clock;
static double us_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
}

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// waits `ticks` of the 100 MHz clock, then stores v at p (system scope) and the store time at stamp[0]
__global__ void delayed_store(uint32_t* p, uint32_t v, uint64_t ticks, uint64_t* stamp) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = rt();
  while (rt() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  stamp[0] = rt();
  sys_store(p, v);
}
// records its start time and the value it sees at p
__global__ void mark(uint64_t* stamp, const uint32_t* p, uint32_t* seen) {
  if (threadIdx.x != 0) return;
  stamp[1] = rt();
  seen[0] = sys_load(p);
}

// B: polls *in until it equals the expected round, echoes it to *out; rounds times; deadline
__global__ void echo(const uint32_t* in, uint32_t* out, uint32_t rounds, uint64_t deadline_ticks, uint32_t* status) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = rt();
  for (uint32_t r = 1; r <= rounds; ++r) {
    while (sys_load(in) != r) {
      if (rt() - t0 > deadline_ticks) { sys_store(status, 0xDEAD0000u | r); return; }
    }
    sys_store(out, r);
  }
  sys_store(status, 1u);
}

// C: zero-copy frame store (16-byte vector stores, coalesced)
__global__ void fill_host(uint4* dst, size_t n16, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4((uint32_t)i ^ seed, (uint32_t)(i >> 32), seed, 0xFF000000u);
}

// D: every wave sleep-polls *flag until it is nonzero or the deadline passes; lane 0 of block 0
// records when it saw the release
__global__ void hold_slots(const uint32_t* flag, uint64_t deadline_ticks, uint64_t* stamp) {
  const uint64_t t0 = rt();
  bool timed_out = false;
  while (true) {
    uint32_t v = 0;
    if ((threadIdx.x & 63u) == 0) v = sys_load(flag);
    v = __shfl(v, 0, 64);
    if (v) break;
    if (rt() - t0 > deadline_ticks) { timed_out = true; break; }
    __builtin_amdgcn_s_sleep(32);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) { stamp[0] = rt(); stamp[1] = timed_out ? 1 : 0; }
}

static int test_wait_value(const char* kind, void* word, hipStream_t sa, hipStream_t sb, uint64_t* stamps,
                           uint32_t* seen) {
  // the watched word starts at 0; stream A waits for >= 1, then marks; stream B stores 1 after 2 ms
  CK(hipMemsetAsync(word, 0, 8, sb));
  CK(hipStreamSynchronize(sb));
  const hipError_t ew = hipStreamWaitValue32(sa, word, 1, hipStreamWaitValueGte, 0xFFFFFFFFu);
  if (ew != hipSuccess) {
    printf("{\"test\": \"A_wait_value\", \"memory\": \"%s\", \"error\": \"%s\"}\n", kind, hipGetErrorString(ew));
    (void)hipGetLastError();
    return 0;
  }
  hipLaunchKernelGGL(mark, dim3(1), dim3(64), 0, sa, stamps, (const uint32_t*)word, seen);
  hipLaunchKernelGGL(delayed_store, dim3(1), dim3(64), 0, sb, (uint32_t*)word, 1u, (uint64_t)200000, stamps);
  // host deadline: 2 s (the store comes after 2 ms)
  const auto t0 = Clock::now();
  hipError_t q = hipErrorNotReady;
  while ((q = hipStreamQuery(sa)) == hipErrorNotReady && us_since(t0) < 2e6) std::this_thread::sleep_for(std::chrono::microseconds(50));
  if (q == hipErrorNotReady) {
    // release it from the host side in case the device store is not seen by the wait
    printf("{\"test\": \"A_wait_value\", \"memory\": \"%s\", \"hang\": true}\n", kind);
    fflush(stdout);
    uint32_t one = 1;
    CK(hipMemcpy(word, &one, 4, hipMemcpyHostToDevice));
    CK(hipStreamSynchronize(sa));
    return 0;
  }
  CK(hipStreamSynchronize(sb));
  uint64_t h[2];
  uint32_t s = 0;
  CK(hipMemcpy(h, stamps, 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&s, seen, 4, hipMemcpyDeviceToHost));
  printf("{\"test\": \"A_wait_value\", \"memory\": \"%s\", \"mark_after_store_us\": %.2f, \"seen\": %u}\n", kind,
         ((double)(int64_t)(h[1] - h[0])) / 100.0, s);
  return 0;
}

int main() {
  CK(hipSetDevice(0));
  int can_wait = 0;
  CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("{\"test\": \"attr\", \"can_use_stream_wait_value\": %d}\n", can_wait);
  hipStream_t sa, sb, sc;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  uint64_t* stamps = nullptr;
  uint32_t* seen = nullptr;
  CK(hipMalloc(&stamps, 64));
  CK(hipMalloc(&seen, 64));

  // A
  void* sig = nullptr;
  if (hipExtMallocWithFlags(&sig, 8, hipMallocSignalMemory) == hipSuccess) {
    if (test_wait_value("signal", sig, sa, sb, stamps, seen)) return 1;
  } else {
    printf("{\"test\": \"A_wait_value\", \"memory\": \"signal\", \"error\": \"alloc\"}\n");
    (void)hipGetLastError();
  }
  void* dmem = nullptr;
  CK(hipMalloc(&dmem, 64));
  if (test_wait_value("device", dmem, sa, sb, stamps, seen)) return 1;
  void* hmem = nullptr;
  CK(hipHostMalloc(&hmem, 64, hipHostMallocCoherent));
  if (test_wait_value("host_coherent", hmem, sa, sb, stamps, seen)) return 1;
  fflush(stdout);

  // B: round trips
  {
    uint32_t* in = nullptr;
    uint32_t* out = nullptr;
    uint32_t* status = nullptr;
    CK(hipHostMalloc(&in, 64, hipHostMallocCoherent));
    CK(hipHostMalloc(&out, 64, hipHostMallocCoherent));
    CK(hipHostMalloc(&status, 64, hipHostMallocCoherent));
    auto* ain = reinterpret_cast<std::atomic<uint32_t>*>(in);
    auto* aout = reinterpret_cast<std::atomic<uint32_t>*>(out);
    auto* ast = reinterpret_cast<std::atomic<uint32_t>*>(status);
    ain->store(0);
    aout->store(0);
    ast->store(0);
    const uint32_t rounds = 2000;
    hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, sa, in, out, rounds, (uint64_t)100000000 /* 1 s */, status);
    std::vector<double> lat;
    bool ok = true;
    const auto tstart = Clock::now();
    for (uint32_t r = 1; r <= rounds && ok; ++r) {
      const auto t0 = Clock::now();
      ain->store(r, std::memory_order_seq_cst);
      while (aout->load(std::memory_order_acquire) != r) {
        if (us_since(tstart) > 2e6) { ok = false; break; }
      }
      lat.push_back(us_since(t0));
    }
    CK(hipStreamSynchronize(sa));
    std::sort(lat.begin(), lat.end());
    printf("{\"test\": \"B_round_trip\", \"ok\": %s, \"status\": %u, \"rounds\": %zu, \"median_us\": %.2f, "
           "\"p99_us\": %.2f}\n",
           ok ? "true" : "false", ast->load(), lat.size(), lat.empty() ? -1.0 : lat[lat.size() / 2],
           lat.empty() ? -1.0 : lat[lat.size() * 99 / 100]);
    fflush(stdout);
  }

  // C: zero-copy 33 MB (the 4K frame)
  {
    const size_t bytes = 3840ull * 2160ull * 4ull;
    uint4* hdst = nullptr;
    uint4* ddst = nullptr;
    CK(hipHostMalloc(&hdst, bytes, hipHostMallocDefault));
    CK(hipMalloc(&ddst, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int pass = 0; pass < 2; ++pass) {
      for (int dev = 0; dev < 2; ++dev) {
        uint4* dst = dev ? ddst : hdst;
        for (int grid : {256, 1024, 4096}) {
          CK(hipEventRecord(e0, sa));
          for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(fill_host, dim3(grid), dim3(256), 0, sa, dst, bytes / 16, (uint32_t)k);
          CK(hipEventRecord(e1, sa));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (pass == 1)
            printf("{\"test\": \"C_zero_copy\", \"dst\": \"%s\", \"grid\": %d, \"ms_per_frame\": %.4f, \"GBps\": %.1f}\n",
                   dev ? "device" : "pinned_host", grid, ms / 5, bytes * 5 / (ms * 1e6));
        }
      }
    }
    uint32_t first[4];
    memcpy(first, hdst, 16);
    printf("{\"test\": \"C_check\", \"first_word\": %u}\n", first[2]);
    // D: copy behind a slot-holding grid
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent));
    auto* af = reinterpret_cast<std::atomic<uint32_t>*>(flag);
    af->store(0);
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, hold_slots, 64, 0));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipLaunchKernelGGL(hold_slots, dim3(bpc * cus), dim3(64), 0, sa, flag, (uint64_t)50000000 /* 0.5 s */, stamps);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    const auto t0 = Clock::now();
    CK(hipMemcpyAsync(hdst, ddst, bytes, hipMemcpyDeviceToHost, sb));
    hipError_t q = hipErrorNotReady;
    while ((q = hipStreamQuery(sb)) == hipErrorNotReady && us_since(t0) < 200000) std::this_thread::sleep_for(std::chrono::microseconds(20));
    const double copy_us = us_since(t0);
    af->store(1);
    CK(hipStreamSynchronize(sa));
    CK(hipStreamSynchronize(sb));
    uint64_t h[2];
    CK(hipMemcpy(h, stamps, 16, hipMemcpyDeviceToHost));
    printf("{\"test\": \"D_copy_behind_full_grid\", \"blocks_per_cu\": %d, \"copy_done_while_held\": %s, "
           "\"copy_us\": %.1f, \"grid_timed_out\": %llu}\n",
           bpc, q == hipSuccess ? "true" : "false", copy_us, (unsigned long long)h[1]);
  }
  printf("{\"test\": \"done\"}\n");
  return 0;
}
