// frm_fast.h — device-only fast paths of the frm builtins that are BIT-IDENTICAL to the
// exact definitions in frm_math.h on restricted operand ranges. The persistent kernel
// runs mb_body_tame() only when every active lane of the wave has tame operands
// (mb_tame()); otherwise it runs the exact mb_body(). Results never depend on which
// path ran (tests/test_gpu_de.py checks the tame path against the oracle).
//
// Where the savings come from (hipcc's correctly rounded lowerings, gfx950):
//  * sqrt: v_rsq_f32 + one residual correction is the correctly rounded sqrt on [2^-96, 2^126]
//    (exhaustively checked, below), in place of LLVM's v_sqrt + two-sided correction + the rescale
//    of inputs below 2^-96.
//  * 1 / b: v_rcp_f32 + one Newton step is RN(1 / b) for every |b| in [2^-125, 2^125]
//    (checked over all 4.2 G such encodings on gfx950, tools/micro/hw_exact_probe.hip,
//    profiles/round5/hw_exact.json): the correctly rounded reciprocal in three instructions.
//  * a / b: a * RN(1 / b) corrected once (Markstein), in place of LLVM's division sequence
//    (v_div_scale, v_rcp, Newton steps, v_div_fmas, v_div_fixup).
//  * log2 / exp2: the special-value selects are dead for positive normal finite inputs /
//    finite exponents; the exponent split of log2 and the scaling of exp2 are integer
//    arithmetic on the encodings where the operand (log2) / result (exp2) is normal.
#pragma once
#include "frm_math.h"

namespace frm {

#if defined(__HIP_DEVICE_COMPILE__)

// Correctly rounded sqrt for x in [2^-96, 2^126] from the hardware reciprocal square root: s =
// x y, one residual e = x - s^2 (fma, exact) and s + e (y / 2). Exhaustively checked equal to the
// correctly rounded sqrtf for every x in [2^-96, 2^128) on gfx950 (tools/micro/hw_exact_probe2.hip,
// profiles/round5/hw_exact2.json): 5 instructions, one transcendental, no compares or selects
// (LLVM's correctly rounded expansion: v_sqrt + two neighbour residuals + compares + selects).
__device__ __forceinline__ float sqrt_rsq(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y;
  return fmaf(fmaf(-s, s, x), 0.5f * y, s);
}

// Correctly rounded sqrt for x in {+-0} U [2^-96, 2^126], x <= -2^-126 and NaN (NaN out, as
// sqrtf): sqrt_rsq with the reciprocal square root taken of x + 2^-126, which is x itself on that
// domain except at +-0 (2^-126 is below half an ulp of 2^-96), where it makes the reciprocal finite
// (instead of rsq(0) = inf), so that s = x * y is the signed zero sqrt(+-0) is and the correction
// keeps it. One add instead of a compare and a select.
__device__ __forceinline__ float sqrt_nosmall(float x) {
  const float y = __builtin_amdgcn_rsqf(x + 0x1p-126f);
  const float s = x * y;
  return fmaf(fmaf(-s, s, x), 0.5f * y, s);
}

// RN(1 / b) for |b| in [2^-125, 2^125] (exhaustively checked, see above).
__device__ __forceinline__ float rcp_rn(float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  return fmaf(fmaf(-b, r, 1.0f), r, r);
}

// Correctly rounded a / b for a in {+-0} U +-[2^-60, 2^40], b in +-[2^-60, 2^40]: from the
// correctly rounded reciprocal y = RN(1/b), q = RN(a y) is within one ulp of a / b and one
// Markstein correction RN(q + RN(a - b q) y) (the remainder is exact) is RN(a / b)
// (Markstein's theorem; no operand, quotient or remainder near the exponent limits here).
// Zero numerators are handled exactly: 0 / b = +-0 with sign(a) ^ sign(b).
__device__ __forceinline__ float div_tame(float a, float b) {
  const float y = rcp_rn(b);
  const float q = a * y;
  const float r = fmaf(fmaf(-b, q, a), y, q);
  return (a == 0.0f) ? q : r;
}

// div_tame without the zero-numerator fix-up: for a = -0 the correction gives +0 where a / b
// is -0. Used where that sign cannot matter (acos_dev(+-0)).
__device__ __forceinline__ float div_tame_nz(float a, float b) {
  const float y = rcp_rn(b);
  const float q = a * y;
  return fmaf(fmaf(-b, q, a), y, q);
}

// max_(a, b) for operands that are never signalling NaNs (values computed here): plain v_max_f32,
// without the quieting canonicalize the compiler puts in front of fmaxf in IEEE mode (same value)
__device__ __forceinline__ float max_quiet(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// a / b from the precomputed y = RN(1 / b) (b > 0, the Menger scales; a in {+-0} U
// +-[2^-60, 2^40]): div_tame's correction, with the sign of a zero quotient kept (0 / b = a).
__device__ __forceinline__ float div_by_rcp(float a, float b, float y) {
  const float q = a * y;
  const float r = fmaf(fmaf(-b, q, a), y, q);
  return (a == 0.0f) ? a : r;
}

// v ^ (m & 0x80000000) in one v_bitop3_b32 (truth table 0x6c: (src0 & src2) ^ src1); left to
// itself the compiler sometimes splits it into v_and + v_xor
__device__ __forceinline__ uint32_t xor_sign_(uint32_t v, uint32_t m) {
#if defined(__gfx950__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c" : "=v"(r) : "v"(m), "v"(v), "s"(0x80000000u));
  return r;
#else  // v_bitop3 is gfx950-only (ARCH overrides, frm_reload on another device)
  return v ^ (m & 0x80000000u);
#endif
}
__device__ __forceinline__ uint32_t bfi_(uint32_t mask, uint32_t a, uint32_t b) {  // (mask & a) | (~mask & b)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
}

// sincos_ for |x| <= 2^20 (the branch sincos_ takes there): t = fma(x, 1/pi, K), j = t - K,
// and j's parity is t's low bit, so both results carry the sign (-1)^j = bit 0 of t moved to
// bit 31. sincos_unsigned returns the unsigned pair and t's encoding (*t_out): the Mandelbulb body
// applies the signs to its products (sincos_small applies them itself).
__device__ __forceinline__ void sincos_unsigned(float x, float* s_out, float* c_out, uint32_t* t_out) {
  const float t = fma_(x, kInvPiHi, kRoundK);
  const float j = t - kRoundK;
  float r = fma_(x, kInvPiHi, -j);
  r = fma_(x, kInvPiLo, r);
  const float u = r * r;
  *s_out = r * sinpi_poly(u);
  *c_out = cospi_poly(u);
  *t_out = __float_as_uint(t);
}
__device__ __forceinline__ void sincos_small(float x, float* s_out, float* c_out) {
  float s, c;
  uint32_t t;
  sincos_unsigned(x, &s, &c, &t);
  const uint32_t sg = t << 31;
  *s_out = __uint_as_float(__float_as_uint(s) ^ sg);
  *c_out = __uint_as_float(__float_as_uint(c) ^ sg);
}

// acos_ with the exact-for-its-range sqrt (1 - |t| is 0 or >= 2^-24 for |t| <= 1; NaN/negative
// inputs propagate NaN exactly as sqrtf does). The t < 0 branch pi - r as fma(r, sg, off) with
// sg = t < 0 ? -1 : 1 (t's sign bit) and off = fma(sg, -pi/2, pi/2) in {+0, pi}: one rounding
// either way; t = -0 gives pi - pi/2 = pi/2 exactly, the value of the t >= 0 branch.
__device__ __forceinline__ float acos_dev(float t) {
  const float a = fabsf(t);
  const float r = sqrt_nosmall(1.0f - a) * acos_poly(a);
  const float sg = __uint_as_float(bfi_(0x80000000u, __float_as_uint(t), 0x3f800000u));
  return fma_(r, sg, fma_(sg, -0.5f * kPi, 0.5f * kPi));
}

// atan2_ for tame x, y (each 0 or with magnitude in [2^-60, 2^40]).
__device__ __forceinline__ float atan2_tame(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  // mx = max_(ax, ay, 2^-100), mn = min_(ax, ay) for finite x, y: plain v_max3 / v_min with
  // |.| source modifiers, without the NaN-quieting canonicalizes the compiler adds to
  // fmaxf / fminf in IEEE mode (same values for non-NaN operands). Tame non-zero
  // magnitudes are >= 2^-60, so the 2^-100 floor only replaces mx = 0 (x = y = 0), where
  // a = 0 * RN(2^100) = +0: the value atan2's mx = 0 branch sets.
  float mx, mn;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(mx) : "v"(x), "v"(y), "s"(0x1p-100f));
  asm("v_min_f32 %0, |%1|, |%2|" : "=v"(mn) : "v"(x), "v"(y));
  const float a = mn * rcp_rn(mx);
  const float s = a * a;
  float r = fma_(a * s, atan_poly(s), a);
  // the octant fix-ups without compares: (c ? h - r : r) == fma(r, c ? -1 : 1, c ? h : 0), one
  // rounding either way (r >= +0); the +-1 is a bit-field insert of c's sign bit into 1.0.
  // c = sign bit of ax - ay (exact difference: negative iff ay > ax, +0 when equal) and of
  // x + 0 (-0 + 0 = +0: negative iff x < 0).
  const uint32_t c1 = __float_as_uint(ax - ay), c2 = __float_as_uint(x + 0.0f);
  const float s1 = __uint_as_float(bfi_(0x80000000u, c1, 0x3f800000u));
  const float s2 = __uint_as_float(bfi_(0x80000000u, c2, 0x3f800000u));
  // offsets (c ? h : 0) as fma(s, -h/2, h/2): exact (+0 or h)
  r = fma_(r, s1, fma_(s1, -0.5f * kHalfPi, 0.5f * kHalfPi));
  r = fma_(r, s2, fma_(s2, -0.5f * kPi, 0.5f * kPi));
  return copysignf(r, y);
}

// log_split_ for positive normal finite x by integer arithmetic (the musl logf split):
// ix = bits(x) - bits(sqrt(1/2)); k = ix >> 23 (arithmetic) is the exponent for a mantissa
// in [sqrt(1/2), sqrt(2)) and bits(x) - (ix & 0xff800000) that mantissa: the same m and e
// as frexp + the doubling below sqrt(1/2) (x = m0 * 2^e, m0 in [1/2, 1): m0 >= sqrt(1/2)
// keeps m0, else 2 m0 with e - 1), without v_frexp, the compare and the selects.
__device__ __forceinline__ void log_split_normal(float x, float* f_out, float* e_out) {
  const uint32_t ix = __float_as_uint(x) - 0x3f3504f3u;  // bits of kSqrtHalf
  *f_out = __uint_as_float(__float_as_uint(x) - (ix & 0xff800000u)) - 1.0f;
  *e_out = (float)((int32_t)ix >> 23);
}

// log2_ for positive normal finite x.
__device__ __forceinline__ float log2_tame(float x) {
  float f, fe;
  log_split_normal(x, &f, &fe);
  return fma_(f, log2_poly(f), fe);
}

// log_ for positive normal finite x (log_posfinite_ with the integer split).
__device__ __forceinline__ float log_posnormal(float x) {
  float f, fe;
  log_split_normal(x, &f, &fe);
  return ln_from_split_(f, fe);
}

// exp2_ for finite y whose rint lies in [-125, 127] (y in [-125.5, 127.5)): there the
// result 2^f * 2^k is a normal number (2^f in [2^-1/2, 2^1/2]), so ldexp is an add of k to
// the exponent field, and rint(y) comes from the 1.5 * 2^23 rounding constant: the low 9
// bits of t = y + K's encoding are k mod 512, so (bits(t) << 23) == k << 23 mod 2^32
// (one v_lshl_add_u32 in place of v_rndne, v_cvt and v_ldexp). The clamp to [-151, 129]
// cannot fire there.
__device__ __forceinline__ float exp2_tame(float y) {
  const float t = y + kRoundK;
  const float k = t - kRoundK;
  const float f = y - k;
  return __uint_as_float(__float_as_uint(fma_(f, exp2_poly(f), 1.0f)) + (__float_as_uint(t) << 23));
}

#endif  // __HIP_DEVICE_COMPILE__

}  // namespace frm
