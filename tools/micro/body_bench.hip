// Microbenchmark: Mandelbulb bodies in a tight loop (no march/state machine) to measure
// the attainable issue rate of the body's instruction mix on gfx950: the exact body
// (mb_body) and the production step (mb_step: wave-uniform tame/exact dispatch +
// mb_length), at 1..8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I fractal-ray-marching_amd/csrc
//        tools/micro/body_bench.hip -o tools/micro/body_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "frm_scene.h"
using namespace frm;

template <bool STEP>
__global__ __launch_bounds__(256) void bodies(SceneUniforms su, int iters, float* out) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  v3 c = mk(0.3f + 1e-6f * (i & 1023), -0.2f + 1e-6f * (i >> 10), 0.5f);
  v3 z = c;
  float dr = 1.f, acc = 0.f;
  float r = length(z);
  for (int k = 0; k < iters; ++k) {
    if constexpr (STEP) {
      mb_step(su, c, r, z, dr);
      r = mb_length(z);
    } else {
      mb_body(su, c, r, z, dr);
      r = length(z);
    }
    if (r > 100.f) { z = c; dr = 1.f; acc += r; r = length(c); }  // keep values bounded
  }
  out[i] = z.x + z.y + z.z + dr + acc;
}

template <bool STEP>
void run(const SceneUniforms& su, int cu, float* out, const char* name) {
  const int occs[] = {1, 2, 3, 4, 5, 8};
  for (int occ : occs) {
    int blocks = cu * occ;  // 4 waves per block -> occ waves/SIMD
    int iters = 2000;
    hipLaunchKernelGGL(bodies<STEP>, dim3(blocks), dim3(256), 0, 0, su, 10, out);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(bodies<STEP>, dim3(blocks), dim3(256), 0, 0, su, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double bodies_total = (double)blocks * 256 * iters;
    double ns_simd = ms * 1e6 / (bodies_total / 64 / (cu * 4));  // per wave-body, per SIMD
    printf("%s waves/SIMD %d: %.3f ms, %.1f G bodies/s, %.1f ns per wave-body per SIMD, "
           "%.0f cycles per wave-iteration at 2.4 GHz\n",
           name, occ, ms, bodies_total / ms / 1e6, ns_simd, ns_simd * occ * 2.4);
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
  run<false>(su, cu, out, "exact");
  run<true>(su, cu, out, "step ");
  return 0;
}
