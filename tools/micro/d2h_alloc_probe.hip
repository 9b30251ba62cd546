// Which host allocation lets hipMemcpyAsync device->host run on a DMA engine (rocprofv3
// --memory-copy-trace) instead of a blit kernel, under a given HIP runtime (LD_LIBRARY_PATH).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const size_t n = 3840ull * 2160 * 4;
  void* d = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Mode { const char* name; unsigned flags; int kind; } modes[] = {
      {"hipHostMalloc default", hipHostMallocDefault, 0},
      {"hipHostMalloc noncoherent", hipHostMallocNonCoherent, 0},
      {"hipHostMalloc writecombined", hipHostMallocWriteCombined, 0},
      {"hipHostMalloc numa", hipHostMallocNumaUser, 0},
      {"malloc + hipHostRegister", 0, 1},
      {"pageable malloc", 0, 2},
  };
  for (const Mode& m : modes) {
    void* h = nullptr;
    if (m.kind == 0) CK(hipHostMalloc(&h, n, m.flags));
    else h = aligned_alloc(4096, n);
    if (m.kind == 1) CK(hipHostRegister(h, n, hipHostRegisterDefault));
    memset(h, 0, n);
    CK(hipDeviceSynchronize());
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("%-32s %.3f ms  %.1f GB/s\n", m.name, best, n / best / 1e6);
    fflush(stdout);
    if (m.kind == 0) CK(hipHostFree(h));
    else { if (m.kind == 1) CK(hipHostUnregister(h)); free(h); }
  }
  return 0;
}
