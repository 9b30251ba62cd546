// omod_probe.hip — does the VOP3 output modifier `div:2` on the residual fma keep the correctly
// rounded sqrt of frm_fast.h exact on gfx950 (f32 denormals enabled, as in the render kernels)?
// sqrt_rsq computes fma(fma(-s, s, x), 0.5 * y, s); the candidate computes fma(e2, y, s) with
// e2 = fma(-s, s, x) * 0.5 by the output modifier (the residual is exact, so halving it is exact
// while it stays normal), one VALU fewer. Exhaustive over every f32 x in [2^-96, 2^128) and over
// x + 2^-126 for x in {+0} U [2^-96, 1] (sqrt_nosmall, the acos argument), against sqrtf.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o omod_probe omod_probe.hip && ./omod_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ float sqrt_omod(float x, float bias) {
  const float y = __builtin_amdgcn_rsqf(x + bias);
  const float s = x * y;
  float e2;
  asm("v_fma_f32 %0, -%1, %1, %2 div:2" : "=v"(e2) : "v"(s), "v"(x));
  return fmaf(e2, y, s);
}

__global__ void probe(unsigned long long* bad, uint32_t* first, uint32_t lo, uint32_t hi, float bias) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    const float got = sqrt_omod(x, bias), ref = sqrtf(x);
    if (__float_as_uint(got) != __float_as_uint(ref)) {
      if (atomicAdd(bad, 1ull) == 0ull) {
        first[0] = (uint32_t)i;
        first[1] = __float_as_uint(got);
        first[2] = __float_as_uint(ref);
      }
    }
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  CHECK(hipMalloc(&bad, sizeof(unsigned long long)));
  CHECK(hipMalloc(&first, 3 * sizeof(uint32_t)));
  struct Range { const char* name; uint32_t lo, hi; float bias; } ranges[] = {
      {"sqrt_rsq  x in [2^-96, 2^128)", 0x0f800000u, 0x7f800000u, 0.0f},
      {"sqrt_nosmall x in [2^-96, 1]", 0x0f800000u, 0x3f800001u, 0x1p-126f},
      {"sqrt_nosmall x = +0", 0x00000000u, 0x00000001u, 0x1p-126f},
  };
  int rc = 0;
  for (const Range& r : ranges) {
    CHECK(hipMemset(bad, 0, sizeof(unsigned long long)));
    CHECK(hipMemset(first, 0, 3 * sizeof(uint32_t)));
    hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, bad, first, r.lo, r.hi, r.bias);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long nb = 0;
    uint32_t f[3];
    CHECK(hipMemcpy(&nb, bad, sizeof(nb), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost));
    printf("%-32s %llu mismatches", r.name, nb);
    if (nb) printf(" (first x=%08x got %08x ref %08x)", f[0], f[1], f[2]);
    printf("\n");
    if (nb) rc = 2;
  }
  return rc;
}
