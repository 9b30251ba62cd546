// Microbenchmark: Mandelbulb bodies in a tight loop (no march/state machine) to measure
// the attainable issue rate of the body's instruction mix on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "frm_scene.h"
using namespace frm;

__global__ __launch_bounds__(256) void bodies(SceneUniforms su, int iters, float* out) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  v3 c = mk(0.3f + 1e-6f * (i & 1023), -0.2f + 1e-6f * (i >> 10), 0.5f);
  v3 z = c;
  float dr = 1.f, acc = 0.f;
  for (int k = 0; k < iters; ++k) {
    float r = length(z);
    mb_body(su, c, r, z, dr);
    if (r > 100.f) { z = c; dr = 1.f; acc += r; }  // keep values bounded
  }
  out[i] = z.x + z.y + z.z + dr + acc;
}

int main() {
  SceneUniforms su = {};
  su.family = kMandelbulb; su.n = 12; su.mb_power = 8.f; su.mb_power_m1 = 7.f; su.mb_bailout = 100.f;
  int cu; hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out; hipMalloc(&out, 64 << 20);
  for (int occ = 1; occ <= 8; occ *= 2) {
    int blocks = cu * occ * 1;  // 4 waves per block -> occ waves/SIMD
    int iters = 2000;
    hipLaunchKernelGGL(bodies, dim3(blocks), dim3(256), 0, 0, su, 10, out);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(bodies, dim3(blocks), dim3(256), 0, 0, su, iters, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double bodies_total = (double)blocks * 256 * iters;
    printf("waves/SIMD %d: %.3f ms, %.2f G bodies/s, %.1f ns per wave-body\n", occ, ms, bodies_total / ms / 1e6,
           ms * 1e6 / (bodies_total / 64 / (cu * 4)));
  }
  return 0;
}
