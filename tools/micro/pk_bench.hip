// Microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 (8 independent f32 FMA chains
// per lane either way, same FLOPs) at 1, 2, 4, 8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/pk_bench.hip -o tools/micro/pk_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void scalar_fma(int iters, float* out) {
  float a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  const float m = 0.999f, c = 1e-4f;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], m, c);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void packed_fma(int iters, float* out) {
  float2v a[4];
  for (int k = 0; k < 4; ++k) a[k] = (float2v){threadIdx.x * 1e-3f + k, threadIdx.x * 1e-3f + k + 4};
  const float2v m = {0.999f, 0.999f}, c = {1e-4f, 1e-4f};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = __builtin_elementwise_fma(a[k], m, c);
  float s = 0;
  for (int k = 0; k < 4; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int cu;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, 64 << 20);
  const int iters = 20000;
  for (int occ : {1, 2, 4, 8}) {
    for (int packed = 0; packed < 2; ++packed) {
      int blocks = cu * occ;
      auto k = packed ? packed_fma : scalar_fma;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, 10, out);
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, iters, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double fmas = (double)blocks * 256 * iters * 8;
      printf("%s waves/SIMD %d: %.1f TFLOP/s (f32 FMA = 2)\n", packed ? "v_pk_fma_f32" : "v_fma_f32   ", occ,
             2 * fmas / ms / 1e9);
    }
  }
  return 0;
}
