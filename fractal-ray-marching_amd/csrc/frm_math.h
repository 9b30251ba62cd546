// frm_math.h — the deterministic f32 math layer ("frm semantics") shared by the gfx950
// kernel and by libfrm's host-side uniform precompute.
//
// Why this exists: fragment.wgsl (the reference hot path) uses WGSL builtins whose
// precision is implementation-defined (sin/cos/acos/atan2/pow/log; WGSL only bounds
// them, e.g. sin/cos absolute error <= 2^-11). To make the GPU render bit-reproducible
// and checkable against a CPU restatement, every builtin is defined here in terms of
// operations that IEEE-754 specifies exactly and that gfx950 and x86-64 both implement
// exactly: +, -, *, fma, correctly-rounded / and sqrt, floor, rint, frexp, ldexp,
// minNum/maxNum, comparisons and selects. No hardware transcendental instruction
// (v_sin/v_cos/v_exp/v_log/v_rcp/v_rsq) ever contributes to a result bit.
//
// frm semantics v2 (round 5): the polynomial kernels and their constants are specified in
// DESIGN.md section 2 (fitted by tools/v2fit.py); oracle/frm_oracle.c restates them
// independently for the CPU. Accuracy (tests/test_oracle_math.py, against float64 libm):
// sin/cos/acos/atan2/log/log2/exp2 within a few f32 ulp on the ranges the path uses —
// tighter than WGSL requires.
//
// Compile with -ffp-contract=off on both host and device: every fusion below is an
// explicit fma.
#pragma once
#if !defined(__HIPCC_RTC__)  // hiprtc (frm_reload) provides these itself
#include <stdint.h>
#include <string.h>
#include <math.h>
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#endif
#define FRM_HD __host__ __device__ __forceinline__
#else
#define FRM_HD static inline
#endif

namespace frm {

// ---- constants (WGSL abstract-float constants rounded once to f32) -------------
constexpr float kPi = 3.14159274101257324219f;         // f32(pi)
constexpr float kHalfPi = 1.57079637050628662109f;     // f32(pi/2)
constexpr float kInvPiHi = 0x1.45f306p-2f;             // f32(1/pi)
constexpr float kInvPiLo = 0x1.b93910p-27f;            // f32(1/pi - kInvPiHi)
constexpr float kRoundK = 0x1.8p23f;                   // 1.5 * 2^23: x + K rounds x to an integer
constexpr float kSqrtHalf = 0.707106769084930419922f;  // f32(sqrt(1/2))
constexpr float kInf = __builtin_huge_valf();

// ---- exact primitives -------------------------------------------------------
FRM_HD float fma_(float a, float b, float c) { return fmaf(a, b, c); }
FRM_HD float sqrt_(float x) { return sqrtf(x); }  // correctly rounded (hipcc default)
FRM_HD float min_(float a, float b) { return fminf(a, b); }  // IEEE minNum
FRM_HD float max_(float a, float b) { return fmaxf(a, b); }  // IEEE maxNum
FRM_HD float fract_(float x) { return x - floorf(x); }       // WGSL fract(e) = e - floor(e)
FRM_HD float clamp_(float x, float lo, float hi) { return min_(max_(x, lo), hi); }
// WGSL mix(e1,e2,e3) = e1*(1-e3) + e2*e3: two products and an add, no fusion.
FRM_HD float mix_(float a, float b, float t) { return a * (1.0f - t) + b * t; }
FRM_HD uint32_t bits_(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }

// ---- frm semantics v2 polynomial kernels (minimax fits, tools/v2fit.py) ------------
// Horner with fma, lowest-order coefficient first in the name: c0 + x (c1 + x (c2 + ...)).
// sin(pi r) / r and cos(pi r) in u = r^2, r in [-1/2, 1/2]
FRM_HD float sinpi_poly(float u) {
  return fma_(fma_(fma_(fma_(0x1.3daffap-4f, u, -0x1.324cccp-1f), u, 0x1.4668b0p+1f), u, -0x1.4abbc2p+2f), u,
              0x1.921fb6p+1f);
}
FRM_HD float cospi_poly(float u) {
  return fma_(fma_(fma_(fma_(0x1.c2b9aap-3f, u, -0x1.55041ap+0f), u, 0x1.03bdaap+2f), u, -0x1.3bd3b0p+2f), u, 1.0f);
}
// acos(a) / sqrt(1 - a), a in [0, 1], with P(0) = f32(pi/2)
FRM_HD float acos_poly(float a) {
  return fma_(fma_(fma_(fma_(fma_(fma_(0x1.35deb4p-9f, a, -0x1.748422p-7f), a, 0x1.bd48d6p-6f), a, -0x1.912814p-5f),
                        a, 0x1.6bbdc6p-4f), a, -0x1.b77b98p-3f), a, 0x1.921fb6p+0f);
}
// (atan(a) - a) / a^3 in s = a^2, a in [0, 1]
FRM_HD float atan_poly(float s) {
  return fma_(fma_(fma_(fma_(fma_(fma_(-0x1.3c0c38p-8f, s, 0x1.953dcap-6f), s, -0x1.ed2edep-5f), s, 0x1.984ef0p-4f),
                        s, -0x1.1f90fcp-3f), s, 0x1.991268p-3f), s, -0x1.5552dep-2f);
}
// log2(1 + f) / f and ln(1 + f) / f, f in [sqrt(1/2) - 1, sqrt(2) - 1]
FRM_HD float log2_poly(float f) {
  return fma_(fma_(fma_(fma_(fma_(fma_(fma_(-0x1.2a9f30p-3f, f, 0x1.df5156p-3f), f, -0x1.fdb316p-3f), f,
                                  0x1.25fd38p-2f), f, -0x1.70e2aap-2f), f, 0x1.ec7724p-2f), f, -0x1.715528p-1f), f,
              0x1.715476p+0f);
}
FRM_HD float ln_poly(float f) {
  return fma_(fma_(fma_(fma_(fma_(fma_(fma_(-0x1.9dfa4ep-4f, f, 0x1.4c3cdcp-3f), f, -0x1.614bfcp-3f), f,
                                  0x1.978e32p-3f), f, -0x1.ff623ep-3f), f, 0x1.5559dcp-2f), f, -0x1.00007ap-1f), f,
              0x1.fffffep-1f);
}
// (2^f - 1) / f, f in [-1/2, 1/2]
FRM_HD float exp2_poly(float f) {
  return fma_(fma_(fma_(fma_(0x1.5bb9f4p-10f, f, 0x1.3cea80p-7f), f, 0x1.c6b752p-5f), f, 0x1.ebf9bcp-3f), f,
              0x1.62e42ap-1f);
}

// ---- sin / cos --------------------------------------------------------------
// Half-turn reduction: r = x/pi - j, j the nearest integer (|r| <= 1/2, the 1/pi product in
// two parts); sin x = (-1)^j r S(r^2), cos x = (-1)^j C(r^2). For |x| <= 2^20, j is rint of the
// exact product x * kInvPiHi, taken from t = fma(x, kInvPiHi, K), whose ulp is 1 (its low bit
// is j's parity); larger and non-finite x take j = rint(RN(x * kInvPiHi)) (defined but not
// accurate there: WGSL bounds sin/cos on [-pi, pi] only; NaN and inf give NaN).
FRM_HD void sincos_(float x, float* s_out, float* c_out) {
  const float t = fma_(x, kInvPiHi, kRoundK);
  float j;
  uint32_t odd;
  if (fabsf(x) <= 0x1p20f) {
    j = t - kRoundK;
    odd = bits_(t) & 1u;
  } else {
    j = rintf(x * kInvPiHi);
    odd = fabsf(j) < 0x1p24f ? (uint32_t)((int32_t)j & 1) : 0u;
  }
  float r = fma_(x, kInvPiHi, -j);
  r = fma_(x, kInvPiLo, r);
  const float u = r * r;
  const float s = r * sinpi_poly(u);
  const float c = cospi_poly(u);
  *s_out = odd ? -s : s;
  *c_out = odd ? -c : c;
}
FRM_HD float sin_(float x) { float s, c; sincos_(x, &s, &c); return s; }
FRM_HD float cos_(float x) { float s, c; sincos_(x, &s, &c); return c; }

// ---- acos -------------------------------------------------------------------
// acos(t) = sqrt(1 - |t|) P(|t|) for t >= 0 (+-0 included), pi - that for t < 0.
FRM_HD float acos_(float t) {
  const float a = fabsf(t);
  const float r = sqrt_(1.0f - a) * acos_poly(a);
  return t < 0.0f ? kPi - r : r;
}

// ---- atan2 ------------------------------------------------------------------
// a = min(|x|,|y|) * RN(1 / max(|x|,|y|)) in [0,1] (0 when both are 0); atan(a) = a + a s Q(s),
// s = a^2; octant/quadrant fix-up. atan2(+-0, +-0) = +-0.
FRM_HD float atan2_(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  float mx = max_(ax, ay), mn = min_(ax, ay);
  float a = mn * (1.0f / mx);
  a = (mx == 0.0f) ? 0.0f : a;
  float s = a * a;
  float r = fma_(a * s, atan_poly(s), a);
  r = (ay > ax) ? kHalfPi - r : r;
  r = (x < 0.0f) ? kPi - r : r;
  return copysignf(r, y);
}

// ---- log / log2 -------------------------------------------------------------
// x = m*2^e with m in [sqrt(1/2), sqrt(2)) (frexp + one exact doubling); f = m-1 (exact);
// log2 x = e + f Q(f) (one fma); ln x = e ln2 + f L(f) (ln 2 in two parts).
// Special values: log(+0/-0) = -inf, log(x<0) = NaN, log(+inf) = +inf, log(NaN) = NaN.
FRM_HD void log_split_(float x, float* f_out, float* e_out) {
  int e;
  float m = frexpf(x, &e);  // m in [0.5, 1), exact
  bool lo = m < kSqrtHalf;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  *f_out = m - 1.0f;
  *e_out = (float)e;
}
FRM_HD float log_special_(float x, float r) {
  r = (x == kInf) ? x : r;
  r = (x == 0.0f) ? -kInf : r;
  r = (x < 0.0f || x != x) ? __builtin_nanf("") : r;
  return r;
}
FRM_HD float log2_(float x) {
  float f, fe;
  log_split_(x, &f, &fe);
  return log_special_(x, fma_(f, log2_poly(f), fe));
}
// ln of m 2^e from its split
FRM_HD float ln_from_split_(float f, float fe) {
  return fma_(fe, 0.693359375f, fma_(fe, -2.12194440e-4f, f * ln_poly(f)));
}
// log_ for positive finite x (normal or subnormal), where log_special_ changes nothing.
FRM_HD float log_posfinite_(float x) {
  float f, fe;
  log_split_(x, &f, &fe);
  return ln_from_split_(f, fe);
}
FRM_HD float log_(float x) { return log_special_(x, log_posfinite_(x)); }

// ---- exp2 / pow -------------------------------------------------------------
// k = rint(y) after clamping y to [-151, 129]; f = y - k in [-1/2, 1/2] (exact);
// 2^f = 1 + f P(f); result = ldexp(2^f, k) (exact scaling, one rounding for subnormal
// results). NaN in -> NaN out.
FRM_HD float exp2_(float y) {
  float yc = min_(max_(y, -151.0f), 129.0f);
  float k = rintf(yc);
  float f = yc - k;
  float r = ldexpf(fma_(f, exp2_poly(f), 1.0f), (int)k);
  return (y != y) ? y : r;
}
// WGSL pow accuracy is "inherited from exp2(e2 * log2(e1))"; frm defines it as exactly that.
FRM_HD float pow_(float x, float y) { return exp2_(y * log2_(x)); }

// ---- vec3 -------------------------------------------------------------------
struct v3 {
  float x, y, z;
};
FRM_HD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
FRM_HD v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
FRM_HD v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
FRM_HD v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
FRM_HD v3 operator*(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
FRM_HD v3 operator*(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
FRM_HD v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
// dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
FRM_HD float dot(v3 a, v3 b) { return fma_(a.z, b.z, fma_(a.y, b.y, a.x * b.x)); }
FRM_HD float length(v3 a) { return sqrt_(dot(a, a)); }
// WGSL normalize(e) = e / length(e): three correctly-rounded divisions.
FRM_HD v3 normalize(v3 a) {
  float l = length(a);
  return mk(a.x / l, a.y / l, a.z / l);
}
// cross(u,v): two products and a subtraction per component, no fusion.
FRM_HD v3 cross(v3 u, v3 v) {
  return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
// a + s*b with the multiply-add fused (WGSL `a + s * b` contracted).
FRM_HD v3 fma3(float s, v3 b, v3 a) { return mk(fma_(s, b.x, a.x), fma_(s, b.y, a.y), fma_(s, b.z, a.z)); }
FRM_HD v3 fma3v(v3 s, v3 b, v3 a) { return mk(fma_(s.x, b.x, a.x), fma_(s.y, b.y, a.y), fma_(s.z, b.z, a.z)); }
FRM_HD v3 abs3(v3 a) { return mk(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
FRM_HD v3 max3s(v3 a, float s) { return mk(max_(a.x, s), max_(a.y, s), max_(a.z, s)); }
FRM_HD v3 min3s(v3 a, float s) { return mk(min_(a.x, s), min_(a.y, s), min_(a.z, s)); }
// colorize(p) = min(Color(1), p + 0.5)   fragment.wgsl:118-120
FRM_HD v3 colorize(v3 p) { return min3s(mk(p.x + 0.5f, p.y + 0.5f, p.z + 0.5f), 1.0f); }

}  // namespace frm
