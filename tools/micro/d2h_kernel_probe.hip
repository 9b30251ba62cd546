// Device -> pinned host copy by a kernel with a small grid: which grid reaches the link's write
// bandwidth (so a frame's readback can run beside a persistent render grid on a few CUs)?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy_to_host(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256u;
  size_t i = blockIdx.x * 256u + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {  // 4 independent 16-B loads in flight per lane
    u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(src[i], dst + i);
}

int main() {
  const size_t n = 3840ull * 2160 * 4;
  uint4* d = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  void* h = nullptr;
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int grid : {8, 16, 32, 64, 128, 256, 1024}) {
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      copy_to_host<<<grid, 256, 0, s>>>((const u32x4*)d, (u32x4*)h, n / 16);
      CK(hipStreamSynchronize(s));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("grid %5d: %.3f ms  %.1f GB/s\n", grid, best, n / best / 1e6);
  }
  const uint32_t* hw = (const uint32_t*)h;
  printf("check %08x %08x\n", hw[0], hw[n / 4 - 1]);
  return 0;
}
