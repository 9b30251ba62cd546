// Microbenchmark: issue cost of the VALU instruction kinds the Mandelbulb body is made of,
// on gfx950. Every variant runs 8 independent instruction streams per lane (no dependency
// stalls) in an inline-asm loop; waves per SIMD = 1, 2, 4, 8. Prints shader cycles per
// wave-instruction per SIMD (s_memtime span of the loop x waves/SIMD / instructions).
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/isa_rate.hip -o /tmp/isa_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ __launch_bounds__(256) void kern(int iters, float* out, unsigned long long* cyc) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  float b = 1.0001f + threadIdx.x * 1e-7f, c = 0.5f;
  if constexpr (KIND == 22) asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(a0), "v"(b) : "vcc");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < iters; ++k) {
#define OPS(I)                                                                                               \
    if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c));         \
    if constexpr (KIND == 1) asm volatile("v_fmaak_f32 %0, %0, %1, 0x3d2cb352" : "+v"(a##I) : "v"(b));      \
    if constexpr (KIND == 2) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b));            \
    if constexpr (KIND == 3) asm volatile("v_cmp_gt_f32 s[20:21], %0, %1" : : "v"(a##I), "v"(b) : "s20", "s21"); \
    if constexpr (KIND == 4) asm volatile("v_rndne_f32 %0, %0" : "+v"(a##I));                                \
    if constexpr (KIND == 5) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a##I));                              \
    if constexpr (KIND == 6) asm volatile("v_ldexp_f32 %0, %0, 1" : "+v"(a##I));                             \
    if constexpr (KIND == 7) asm volatile("v_frexp_mant_f32 %0, %0" : "+v"(a##I));                           \
    if constexpr (KIND == 8) asm volatile("v_rcp_f32 %0, %0" : "+v"(a##I));                                  \
    if constexpr (KIND == 9) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a##I));                                 \
    if constexpr (KIND == 10) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c));       \
    if constexpr (KIND == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##I) : "v"(b));                    \
    if constexpr (KIND == 12) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a##I) : "v"(b));                    \
    if constexpr (KIND == 13) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(a##I) : "v"(b));               \
    if constexpr (KIND == 14) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a##I) : "v"(b) : "s20", "s21"); \
    if constexpr (KIND == 15) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a##I));                             \
    if constexpr (KIND == 16) asm volatile("v_max3_f32 %0, |%0|, |%1|, %2" : "+v"(a##I) : "v"(b), "v"(c));   \
    if constexpr (KIND == 17) asm volatile("v_frexp_exp_i32_f32 %0, %0" : "+v"(a##I));                       \
    if constexpr (KIND == 18) asm volatile("v_sub_f32 %0, 0x40490fdb, %0" : "+v"(a##I));                     \
    if constexpr (KIND == 19) asm volatile("v_cmp_class_f32 vcc, %0, %1" : : "v"(a##I), "v"(b) : "vcc");     \
    if constexpr (KIND == 20) asm volatile("v_mov_b32 %0, %1" : "=v"(a##I) : "v"(b));                       \
    if constexpr (KIND == 21) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b));       \
    if constexpr (KIND == 22) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b));          \
    if constexpr (KIND == 23) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if constexpr (KIND == 24) asm volatile("v_cmp_gt_f32_e64 s[20:21], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a##I) : "v"(b) : "s20", "s21"); \
    if constexpr (KIND == 25) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if constexpr (KIND == 26) asm volatile("v_subbrev_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a##I) : : "vcc");   \
    if constexpr (KIND == 27) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a##I) : "v"(b));          \
    if constexpr (KIND == 28) asm volatile("v_cndmask_b32 %0, 0, %0, vcc" : "+v"(a##I));                    \
    if constexpr (KIND == 29) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if constexpr (KIND == 30) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32_e64 %0, %0, %1, vcc\n v_cndmask_b32_e64 %0, %1, %0, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if constexpr (KIND == 31) asm volatile("v_fma_f32 %0, %0, %1, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b)); \
    if constexpr (KIND == 32) asm volatile("v_fma_f32 %0, %0, %1, %1\n v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b));
    R8(OPS)
    R8(OPS)
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}

static const char* kNames[] = {"v_fma_f32", "v_fmaak_f32 (literal)", "v_cndmask_b32 vcc", "v_cmp_gt_f32 -> sgpr",
                               "v_rndne_f32", "v_cvt_i32_f32", "v_ldexp_f32", "v_frexp_mant_f32", "v_rcp_f32",
                               "v_sqrt_f32", "v_bfi_b32", "v_add_u32", "v_mul_f32", "v_fma_f32 inline 1.0",
                               "v_cndmask_b32_e64 sgpr", "v_cvt_f32_i32", "v_max3_f32 |.|", "v_frexp_exp_i32_f32",
                               "v_sub_f32 literal", "v_cmp_class_f32 vcc", "v_mov_b32", "v_cndmask_b32_e64 vcc", "v_cndmask_b32 vcc (set)",
                               "cmp vcc + cndmask e32 (2)", "cmp_e64 + cndmask_e64 (2)", "cmp vcc + cndmask_e64 (2)",
                               "v_subbrev_co_u32 vcc", "v_cndmask_b32 src swap", "v_cndmask_b32 0,v",
                               "cmp + 2 cndmask e32 (3)", "cmp + 2 cndmask e64 (3)", "fma + cndmask e32 (2)",
                               "fma + cndmask e64 (2)"};

template <int KIND>
void run(int cu, float* out, unsigned long long* cyc) {
  const int iters = 2000, per_iter = 16;
  printf("%-24s", kNames[KIND]);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w : {1, 2, 4, 8}) {
    hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL(kern<KIND>, dim3(cu * w), dim3(256), 0, 0, 10, out, cyc);
    hipMemset(cyc, 0, 8);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<KIND>, dim3(cu * w), dim3(256), 0, 0, iters, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = (double)cu * w * 4;
    const double per_wave = c / (double)(cu * w);  // s_memtime ticks per wave (one stamp per block)
    // wall: ns per wave-instruction per SIMD (x 2.4 = cycles at 2.4 GHz)
    printf("  w%d %5.2f|%5.2f", w, per_wave / w / (iters * per_iter), ms * 1e6 / ((double)w * iters * per_iter) * 2.4);
    (void)waves;
  }
  printf("  stamp|wall cyc per wave-instr per SIMD\n");
}

template <int... K>
void run_all(int cu, float* out, unsigned long long* cyc, std::integer_sequence<int, K...>) {
  (run<K>(cu, out, cyc), ...);
}

int main() {
  int cu;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 << 20);
  hipMalloc(&cyc, 8);
  run_all(cu, out, cyc, std::make_integer_sequence<int, 33>{});
  return 0;
}
