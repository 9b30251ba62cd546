// A/B of two code objects of tools/micro/ilp_bench.hip (e.g. compiler asm vs a peephole-
// rewritten copy): loads each .hsaco with hipModuleLoad and times chains<1>/<2> at 1..8
// waves per SIMD, interleaved. Usage: hsaco_ab a.hsaco b.hsaco
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "frm_scene.h"
using namespace frm;

int main(int argc, char** argv) {
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
  hipModule_t mod[8];
  for (int i = 1; i < argc; ++i)
    if (hipModuleLoad(&mod[i], argv[i]) != hipSuccess) { printf("load %s failed\n", argv[i]); return 1; }
  const char* names[2] = {"_Z6chainsILi1EEvN3frm13SceneUniformsEiPf", "_Z6chainsILi2EEvN3frm13SceneUniformsEiPf"};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int round = 0; round < 2; ++round)
    for (int k = 0; k < 2; ++k)
      for (int occ : {4, 5, 6, 8})
        for (int i = 1; i < argc; ++i) {
          hipFunction_t fn;
          hipModuleGetFunction(&fn, mod[i], names[k]);
          int iters = 10;
          void* params[] = {&su, &iters, &out};
          hipModuleLaunchKernel(fn, cu * occ, 1, 1, 256, 1, 1, 0, 0, params, nullptr);
          iters = 1000;
          hipEventRecord(a);
          hipModuleLaunchKernel(fn, cu * occ, 1, 1, 256, 1, 1, 0, 0, params, nullptr);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          printf("round %d K=%d waves/SIMD %d %-28s %.3f ms %.1f G bodies/s\n", round, k + 1, occ, argv[i], ms,
                 (double)cu * occ * 256 * iters * (k + 1) / ms / 1e6);
        }
  return 0;
}
