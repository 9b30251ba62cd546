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
// The polynomial kernels and their constants are specified in DESIGN.md §"frm math";
// oracle/frm_oracle.c restates them independently for the CPU. Accuracy (measured by
// tests/test_oracle_math.py against float64 libm): sin/cos/acos/atan2/log/log2/exp2
// within a few f32 ulp on the ranges the path uses — tighter than WGSL requires.
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
constexpr float kHalfPiLo = -4.37113900018624283e-8f;  // f32(pi/2 - f32(pi/2))
constexpr float kTwoOverPi = 0.636619746685028076172f; // f32(2/pi)
constexpr float kLog2e = 1.44269502162933349609f;      // f32(log2(e))
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

// ---- sin / cos --------------------------------------------------------------
// j = rint(x*2/pi); r = x - j*pi/2 (two fma, Cody-Waite); minimax polynomials on
// [-pi/4, pi/4]; quadrant select. j is clamped to +-2^22 before the int conversion so
// NaN/inf inputs are well defined (they yield NaN through r).
FRM_HD void sincos_(float x, float* s_out, float* c_out) {
  float j = rintf(x * kTwoOverPi);
  float r = fma_(-j, kHalfPi, x);
  r = fma_(-j, kHalfPiLo, r);
  int q = (int)min_(max_(j, -4194304.0f), 4194304.0f);
  float z = r * r;
  float ps = fma_(fma_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  float s = fma_(r * z, ps, r);
  float pc = fma_(fma_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                  4.166664568298827e-2f);
  float c = fma_(z * z, pc, fma_(-0.5f, z, 1.0f));
  float sv = (q & 1) ? c : s;
  float cv = (q & 1) ? s : c;
  *s_out = (q & 2) ? -sv : sv;
  *c_out = ((q + 1) & 2) ? -cv : cv;
}
FRM_HD float sin_(float x) { float s, c; sincos_(x, &s, &c); return s; }
FRM_HD float cos_(float x) { float s, c; sincos_(x, &s, &c); return c; }

// ---- acos -------------------------------------------------------------------
// asin kernel on w in [0, 1/2]: asin(w) = w + w*z*P(z); |t| > 1/2 uses
// w = sqrt((1-|t|)/2), z = w^2 (computed as (1-|t|)/2 directly).
FRM_HD float acos_(float t) {
  float a = fabsf(t);
  bool big = a > 0.5f;
  float zb = 0.5f * (1.0f - a);
  float z = big ? zb : a * a;
  float w = big ? sqrt_(zb) : a;
  float p = fma_(fma_(fma_(fma_(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                      7.4953002686e-2f), z, 1.6666752422e-1f);
  float s = fma_(w * z, p, w);
  float rb = (t > 0.0f) ? 2.0f * s : kPi - 2.0f * s;
  float rs = kHalfPi - copysignf(s, t);
  return big ? rb : rs;
}

// ---- atan2 ------------------------------------------------------------------
// a = min(|x|,|y|)/max(|x|,|y|) in [0,1]; atan(a) = a + a*s*Q(s), s = a^2, Q a degree-7
// minimax fit (Remez, relative error 1.5e-8 on [0,1]); octant/quadrant fix-up.
// atan2(+-0, +-0) = +-0 (a := 0).
FRM_HD float atan2_(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  float mx = max_(ax, ay), mn = min_(ax, ay);
  float a = mn / mx;
  a = (mx == 0.0f) ? 0.0f : a;
  float s = a * a;
  float q = fma_(fma_(fma_(fma_(fma_(fma_(fma_(0.002974590389872539f, s, -0.016581183968493302f), s,
                                      0.04355353931255974f), s, -0.07580578130128461f), s,
                          0.10678940285181907f), s, -0.14214209135918496f), s,
                0.1999413720560495f), s, -0.3333316696611865f);
  float r = fma_(a * s, q, a);
  r = (ay > ax) ? kHalfPi - r : r;
  r = (x < 0.0f) ? kPi - r : r;
  return copysignf(r, y);
}

// ---- log / log2 -------------------------------------------------------------
// x = m*2^e with m in [sqrt(1/2), sqrt(2)) (frexp + one exact doubling); f = m-1 (exact);
// ln(1+f) = f - z/2 + f*z*P(f), z = f^2, P degree 8.
// Special values: log(+0/-0) = -inf, log(x<0) = NaN, log(+inf) = +inf, log(NaN) = NaN.
FRM_HD float log1p_kernel_(float f) {
  float z = f * f;
  float p = fma_(fma_(fma_(fma_(fma_(fma_(fma_(fma_(7.0376836292e-2f, f, -1.1514610310e-1f), f,
        1.1676998740e-1f), f, -1.2420140846e-1f), f, 1.4249322787e-1f), f, -1.6668057665e-1f), f,
        2.0000714765e-1f), f, -2.4999993993e-1f), f, 3.3333331174e-1f);
  float y = fma_(-0.5f, z, (f * z) * p);
  return f + y;
}
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
  float r = fma_(log1p_kernel_(f), kLog2e, fe);
  return log_special_(x, r);
}
// log_ for positive finite x (normal or subnormal), where log_special_ changes nothing.
FRM_HD float log_posfinite_(float x) {
  float f, fe;
  log_split_(x, &f, &fe);
  float l = log1p_kernel_(f);
  return fma_(fe, 0.693359375f, fma_(fe, -2.12194440e-4f, l));
}
FRM_HD float log_(float x) { return log_special_(x, log_posfinite_(x)); }

// ---- exp2 / pow -------------------------------------------------------------
// k = rint(y) after clamping y to [-151, 129]; f = y - k in [-1/2, 1/2] (exact);
// 2^f = 1 + f*P(f), P degree 5; result = ldexp(2^f, k) (exact scaling, one rounding for
// subnormal results). NaN in -> NaN out.
FRM_HD float exp2_(float y) {
  float yc = min_(max_(y, -151.0f), 129.0f);
  float k = rintf(yc);
  float f = yc - k;
  float p = fma_(fma_(fma_(fma_(fma_(1.535336188319500e-4f, f, 1.339887440266574e-3f), f,
                               9.618437357674640e-3f), f, 5.550332471162809e-2f), f,
                     2.402264791363012e-1f), f, 6.931472028550421e-1f);
  float r = ldexpf(fma_(f, p, 1.0f), (int)k);
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
