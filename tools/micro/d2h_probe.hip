// D2H copy engine probe: when does hipMemcpyAsync device->host (pinned host memory) run on a DMA
// engine and when as a blit kernel (which occupies CUs)? Run under rocprofv3 --kernel-trace
// --memory-copy-trace. Cases: plain stream, a kernel right before the copy on the same stream,
// a CU-masked stream (libfrm's render slots > 0).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void touch(uint32_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1u;
}

int main() {
  const size_t n = 3840ull * 2160 * 4;
  uint32_t* d = nullptr;
  CK(hipMalloc(&d, n));
  void* h = nullptr;
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  hipStream_t plain, masked;
  CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  uint32_t mask[8] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
  CK(hipExtStreamCreateWithCUMask(&masked, (prop.multiProcessorCount + 31) / 32, mask));
  struct Case { const char* name; hipStream_t s; bool kernel_first; } cases[] = {
      {"plain stream", plain, false}, {"plain, kernel before", plain, true},
      {"cu-masked stream", masked, false}, {"cu-masked, kernel before", masked, true}};
  for (const Case& c : cases) {
    double best = 1e9;
    for (int r = 0; r < 4; ++r) {
      if (c.kernel_first) touch<<<(n / 4 + 255) / 256, 256, 0, c.s>>>(d, n / 4);
      CK(hipStreamSynchronize(c.s));
      auto t0 = std::chrono::steady_clock::now();
      if (c.kernel_first) touch<<<1, 64, 0, c.s>>>(d, 64);
      CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, c.s));
      CK(hipStreamSynchronize(c.s));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("%-28s %.3f ms  %.1f GB/s\n", c.name, best, n / best / 1e6);
  }
  return 0;
}
