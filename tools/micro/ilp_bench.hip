// Microbenchmark: is the tame Mandelbulb body latency-bound? Runs K independent body
// chains per lane (K = 1, 2) at 1..8 waves per SIMD and reports bodies/s. If K = 2 at
// W waves beats K = 1 at 2W waves, the VALU idles on dependency latency, not on issue.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I fractal-ray-marching_amd/csrc
//        tools/micro/ilp_bench.hip -o tools/micro/ilp_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "frm_scene.h"
#include "frm_fast.h"
using namespace frm;

template <int K>
__global__ __launch_bounds__(256) void chains(SceneUniforms su, int iters, float* out) {
#if defined(__HIP_DEVICE_COMPILE__)  // the tame primitives are device-only
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  v3 c[K], z[K];
  float dr[K], r[K], acc = 0.f;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    c[j] = mk(0.3f + 1e-6f * (i & 1023) + 0.01f * j, -0.2f + 1e-6f * (i >> 10), 0.5f);
    z[j] = c[j];
    dr[j] = 1.f;
    r[j] = length_nosmall(z[j]);
  }
  for (int k = 0; k < iters; ++k) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      mb_body_tame(su, c[j], r[j], z[j], dr[j]);
      r[j] = length_nosmall(z[j]);
      if (r[j] > 100.f) { z[j] = c[j]; dr[j] = 1.f; acc += r[j]; r[j] = length_nosmall(c[j]); }
    }
  }
  float s = acc;
#pragma unroll
  for (int j = 0; j < K; ++j) s += z[j].x + z[j].y + z[j].z + dr[j];
  out[i] = s;
#endif
}

template <int K>
void run(const SceneUniforms& su, int cu, float* out) {
  const int occs[] = {1, 2, 3, 4, 5, 6, 8};
  for (int occ : occs) {
    int blocks = cu * occ;
    int iters = 1000;
    hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(256), 0, 0, su, 10, out);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(256), 0, 0, su, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double bodies_total = (double)blocks * 256 * iters * K;
    printf("K=%d waves/SIMD %d: %.3f ms, %.1f G bodies/s\n", K, occ, ms, bodies_total / ms / 1e6);
  }
}

int main() {
  SceneUniforms su = {};
  su.family = kMandelbulb;
  su.n = 12;
  su.mb_power = 8.f;
  su.mb_power_m1 = 7.f;
  su.mb_bailout = 100.f;
  int cu;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, 64 << 20);
  run<1>(su, cu, out);
  run<2>(su, cu, out);
  return 0;
}
