// Device -> pinned-host copy paths, one per run (argv[1]), to be counted under rocprofv3
// --kernel-trace --memory-copy-trace (a blit kernel needs CU slots; a DMA copy does not):
//   plain      hipMemcpyAsync D2H on an idle stream
//   after      the same right after a kernel that writes the source, on the same stream
//   evwait     the kernel on stream A, an event, stream B waits for it and copies (libfrm's readback)
//   nocu       hipMemcpyDeviceToDeviceNoCU into the pinned (device-mapped) host buffer
// Prints the copy time and whether the host bytes are right.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + (uint32_t)i;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "plain";
  const size_t words = 3840ull * 2160, n = words * 4;
  uint32_t* d = nullptr;
  CK(hipMalloc(&d, n));
  uint32_t* h = nullptr;
  CK(hipHostMalloc((void**)&h, n, hipHostMallocDefault));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  double best = 1e9;
  bool ok = true;
  for (int r = 0; r < 3; ++r) {
    const uint32_t v = 7u * (r + 1);
    memset(h, 0, n);
    hipLaunchKernelGGL(fill, dim3((words + 255) / 256), dim3(256), 0, a, d, words, v);
    if (!strcmp(mode, "plain")) CK(hipStreamSynchronize(a));
    auto t0 = std::chrono::steady_clock::now();
    if (!strcmp(mode, "evwait")) {
      CK(hipEventRecord(ev, a));
      CK(hipStreamWaitEvent(b, ev, 0));
      CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, b));
      CK(hipStreamSynchronize(b));
    } else if (!strcmp(mode, "nocu")) {
      CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToDeviceNoCU, a));
      CK(hipStreamSynchronize(a));
    } else {
      CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, a));
      CK(hipStreamSynchronize(a));
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms < best) best = ms;
    for (size_t i = 0; i < words; i += 4099) ok = ok && h[i] == v + (uint32_t)i;
    ok = ok && h[words - 1] == v + (uint32_t)(words - 1);
  }
  printf("%-8s %.3f ms  bytes %s\n", mode, best, ok ? "ok" : "WRONG");
  return ok ? 0 : 1;
}
