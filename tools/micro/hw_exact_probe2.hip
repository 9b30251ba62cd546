// hw_exact_probe2.hip — candidate seed-independent sequences for correctly rounded sqrt and
// division on gfx950, checked against hipcc's correctly rounded sqrtf / operator/.
//  * sqrt: every f32 x in [2^-96, 2^128) (exhaustive), three candidate corrections of a
//    hardware seed (v_rsq_f32 or v_sqrt_f32) by one fma residual.
//  * division: q = RN(a * RN(1/b)) with RN(1/b) from v_rcp_f32 + one Newton step (exact on
//    [2^-125, 2^125], hw_exact_probe.hip), then one Markstein correction; random pairs
//    (2^36 of them, exponents spread over the tame domain) plus every a for a few b.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

enum { kTests = 6, kEx = 8 };
static const char* kNames[kTests] = {
    "sqrt A: y=rsq(x); s=x*y; h=0.5*y; s+=fma(-s,s,x)*h",
    "sqrt B: s=sqrt(x); h=0.5*rcp(s); s+=fma(-s,s,x)*h",
    "sqrt C: y=rsq(x); s=x*y; h=0.5*y; e=fma(-s,h,0.5); s=fma(s,e,s); h=fma(h,e,h); s+=fma(-s,s,x)*h",
    "div   q=a*rcpN(b); q+=fma(-b,q,a)*rcpN(b)   (random pairs)",
    "div   same, every a in [1,2) x 64 b",
    "div   q=a*rcpN(b) equals RN(a*RN(1/b)) (random pairs)",
};

__device__ __forceinline__ float rcpN(float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  return fmaf(fmaf(-b, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_m(float a, float b) {
  const float r = rcpN(b);
  const float q = a * r;
  return fmaf(fmaf(-b, q, a), r, q);
}
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ void note(unsigned long long* bad, uint32_t* ex, int t, uint32_t a, uint32_t b, float got, float ref) {
  const unsigned long long k = atomicAdd(&bad[t], 1ull);
  if (k < kEx) {
    ex[(t * kEx + k) * 4 + 0] = a;
    ex[(t * kEx + k) * 4 + 1] = b;
    ex[(t * kEx + k) * 4 + 2] = __float_as_uint(got);
    ex[(t * kEx + k) * 4 + 3] = __float_as_uint(ref);
  }
}

__global__ void sqrt_probe(unsigned long long* bad, uint32_t* ex, uint64_t lo, uint64_t hi) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    const float ref = sqrtf(x);
    {
      const float y = __builtin_amdgcn_rsqf(x);
      const float s = x * y, h = 0.5f * y;
      const float r = fmaf(fmaf(-s, s, x), h, s);
      if (__float_as_uint(r) != __float_as_uint(ref)) note(bad, ex, 0, (uint32_t)i, 0, r, ref);
    }
    {
      const float s = __builtin_amdgcn_sqrtf(x);
      const float h = 0.5f * __builtin_amdgcn_rcpf(s);
      const float r = fmaf(fmaf(-s, s, x), h, s);
      if (__float_as_uint(r) != __float_as_uint(ref)) note(bad, ex, 1, (uint32_t)i, 0, r, ref);
    }
    {
      const float y = __builtin_amdgcn_rsqf(x);
      float s = x * y, h = 0.5f * y;
      const float e = fmaf(-s, h, 0.5f);
      s = fmaf(s, e, s);
      h = fmaf(h, e, h);
      const float r = fmaf(fmaf(-s, s, x), h, s);
      if (__float_as_uint(r) != __float_as_uint(ref)) note(bad, ex, 2, (uint32_t)i, 0, r, ref);
    }
  }
}

// a, b with random mantissas and exponents: |a| in [2^-60, 2^40] or 0, |b| in [2^-60, 2^40]
__global__ void div_probe(unsigned long long* bad, uint32_t* ex, uint64_t seed, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t z = mix64(seed + i);
    const uint32_t ea = 67u + (uint32_t)((z >> 0) % 101u), eb = 67u + (uint32_t)((z >> 8) % 101u);
    const uint32_t ab = (ea << 23) | (uint32_t)((z >> 16) & 0x7fffffu) | ((uint32_t)(z >> 62) << 31);
    const uint32_t bb = (eb << 23) | (uint32_t)((z >> 39) & 0x7fffffu) | ((uint32_t)(z >> 63) << 31);
    const float a = __uint_as_float(ab), b = __uint_as_float(bb);
    const float q = div_m(a, b), ref = a / b;
    if (__float_as_uint(q) != __float_as_uint(ref)) note(bad, ex, 3, ab, bb, q, ref);
    const float q0 = a * rcpN(b), ref0 = a * (1.0f / b);
    if (__float_as_uint(q0) != __float_as_uint(ref0)) note(bad, ex, 5, ab, bb, q0, ref0);
  }
}

__global__ void div_sweep(unsigned long long* bad, uint32_t* ex, uint64_t seed) {
  // every mantissa of a in [1, 2) against 64 random b (blockIdx.y)
  const uint64_t z = mix64(seed + blockIdx.y);
  const uint32_t bb = (uint32_t)(120u + (z % 16u)) << 23 | (uint32_t)((z >> 8) & 0x7fffffu);
  const float b = __uint_as_float(bb);
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < (1u << 23); m += gridDim.x * blockDim.x) {
    const uint32_t ab = 0x3f800000u | m;
    const float a = __uint_as_float(ab);
    const float q = div_m(a, b), ref = a / b;
    if (__float_as_uint(q) != __float_as_uint(ref)) note(bad, ex, 4, ab, bb, q, ref);
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* ex;
  CHECK(hipMalloc(&bad, sizeof(unsigned long long) * kTests));
  CHECK(hipMalloc(&ex, sizeof(uint32_t) * kTests * kEx * 4));
  CHECK(hipMemset(bad, 0, sizeof(unsigned long long) * kTests));
  CHECK(hipMemset(ex, 0, sizeof(uint32_t) * kTests * kEx * 4));
  const uint64_t lo = 0x0f800000ull, hi = 0x7f800000ull;  // [2^-96, inf)
  for (uint64_t c = lo; c < hi; c += 1ull << 28) {
    hipLaunchKernelGGL(sqrt_probe, dim3(4096), dim3(256), 0, 0, bad, ex, c, c + (1ull << 28) < hi ? c + (1ull << 28) : hi);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  for (int k = 0; k < 64; ++k) {
    hipLaunchKernelGGL(div_probe, dim3(8192), dim3(256), 0, 0, bad, ex, (uint64_t)k << 40, 1ull << 30);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  hipLaunchKernelGGL(div_sweep, dim3(1024, 64), dim3(256), 0, 0, bad, ex, 12345ull);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned long long h[kTests];
  uint32_t e[kTests * kEx * 4];
  CHECK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(e, ex, sizeof(e), hipMemcpyDeviceToHost));
  printf("{\"tests\": [\n");
  for (int t = 0; t < kTests; ++t) {
    printf("  {\"name\": \"%s\", \"mismatches\": %llu, \"examples\": [", kNames[t], h[t]);
    const unsigned long long n = h[t] < kEx ? h[t] : kEx;
    for (unsigned long long k = 0; k < n; ++k)
      printf("%s[\"0x%08x\", \"0x%08x\", \"0x%08x\", \"0x%08x\"]", k ? ", " : "", e[(t * kEx + k) * 4],
             e[(t * kEx + k) * 4 + 1], e[(t * kEx + k) * 4 + 2], e[(t * kEx + k) * 4 + 3]);
    printf("]}%s\n", t + 1 < kTests ? "," : "");
  }
  printf("], \"sqrt_range\": [\"0x0f800000\", \"0x7f800000\"], \"div_pairs\": %llu}\n", 64ull << 30);
  return 0;
}
