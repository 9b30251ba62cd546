// frm_fast.h — device-only fast paths of the frm builtins that are BIT-IDENTICAL to the
// exact definitions in frm_math.h on restricted operand ranges. The persistent kernel
// runs mb_body_tame() only when every active lane of the wave has tame operands
// (mb_tame()); otherwise it runs the exact mb_body(). Results never depend on which
// path ran (tests/test_gpu_de.py checks the tame path against the oracle).
//
// Where the savings come from (hipcc's correctly rounded lowerings, gfx950):
//  * sqrt: v_sqrt_f32 + a one-ulp correction; the exact lowering also rescales inputs
//    below 2^-96 (5 instructions) — not needed when x == 0 or x >= 2^-96.
//  * a / b: the same Newton sequence as the exact lowering, without v_div_scale (returns
//    its input unchanged when no operand or quotient is near the exponent limits),
//    v_div_fmas (a plain fma when v_div_scale did not scale) and v_div_fixup (for
//    finite non-zero operands with a normal quotient it only re-applies the sign).
//    Zero numerators are handled exactly: 0 / b = +-0 with sign(a) ^ sign(b).
//  * log2 / exp2: the special-value selects are dead for positive normal finite inputs /
//    finite exponents; the exponent split of log2 and the scaling of exp2 are integer
//    arithmetic on the encodings where the operand (log2) / result (exp2) is normal.
#pragma once
#include "frm_math.h"

namespace frm {

#if defined(__HIP_DEVICE_COMPILE__)

// Correctly rounded sqrt, exact for x == +-0, x >= 2^-96, +inf, NaN and x < 0 (all x
// except subnormals and normals below 2^-96). Mirrors LLVM's expansion minus the rescale
// and minus its +-0/+inf pass-through: there the one-ulp corrections cannot fire
// (s = +-0: s_dn is NaN, the s_up residual is +-0; s = +inf: both residuals are NaN).
__device__ __forceinline__ float sqrt_nosmall(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
  float s_up = __uint_as_float(__float_as_uint(s) + 1u);
  float r_dn = fmaf(-s_dn, s, x);
  float r_up = fmaf(-s_up, s, x);
  s = (r_dn <= 0.0f) ? s_dn : s;
  return (r_up > 0.0f) ? s_up : s;
}

// Correctly rounded a / b for a in {+-0} U +-[2^-60, 2^40], b in +-[2^-60, 2^40].
__device__ __forceinline__ float div_tame(float a, float b) {
  float r = __builtin_amdgcn_rcpf(b);
  float e = fmaf(-b, r, 1.0f);
  r = fmaf(e, r, r);
  float q = a * r;
  float rem = fmaf(-b, q, a);
  q = fmaf(rem, r, q);
  rem = fmaf(-b, q, a);
  q = fmaf(rem, r, q);
  const float zero = __uint_as_float((__float_as_uint(a) ^ __float_as_uint(b)) & 0x80000000u);
  return (a == 0.0f) ? zero : q;
}

// div_tame without the zero-numerator fix-up: for a = +0 the Newton sequence already
// gives +0; for a = -0 it gives +0 where a / b is -0. Used where that sign cannot matter
// (acos_dev(+-0) and atan2's min/max ratio, whose numerator is never -0).
__device__ __forceinline__ float div_tame_nz(float a, float b) {
  float r = __builtin_amdgcn_rcpf(b);
  float e = fmaf(-b, r, 1.0f);
  r = fmaf(e, r, r);
  float q = a * r;
  float rem = fmaf(-b, q, a);
  q = fmaf(rem, r, q);
  rem = fmaf(-b, q, a);
  return fmaf(rem, r, q);
}

// max_(a, b) for operands that are never signalling NaNs (values computed here): plain v_max_f32,
// without the quieting canonicalize the compiler puts in front of fmaxf in IEEE mode (same value)
__device__ __forceinline__ float max_quiet(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// a / b from a precomputed reciprocal r within one ulp of 1 / b: div_tame's two Newton
// corrections (the same domain: a in {+-0} U +-[2^-60, 2^40], b in +-[2^-60, 2^40]), with the
// sign of a zero quotient restored; b > 0 here (the Menger scales), so 0 / b keeps a's sign.
__device__ __forceinline__ float div_by_rcp(float a, float b, float r) {
  float q = a * r;
  float rem = fmaf(-b, q, a);
  q = fmaf(rem, r, q);
  rem = fmaf(-b, q, a);
  q = fmaf(rem, r, q);
  return (a == 0.0f) ? a : q;
}

// sincos_ for finite |x| <= 2^22 * pi/2 (the quadrant clamp is a no-op there); negating through
// the sign bit: (q & 2) ? -v : v == v ^ (bit 1 of q moved to bit 31). Bit-identical.
// rint(x * 2/pi) by the 1.5 * 2^23 rounding constant: |x * 2/pi| < 2^22, so t = x * 2/pi + K
// rounds to an integer (to nearest even, as rint does), j = t - K is exact and the low bits
// of t's encoding are j mod 2^22 (two v_add in place of v_rndne + v_cvt). The odd-quadrant
// swap is a bit-field select on a sign-extended bit 0 (no compare, no v_cndmask).
__device__ __forceinline__ uint32_t bfi_(uint32_t mask, uint32_t a, uint32_t b) {  // (mask & a) | (~mask & b)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
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
__device__ __forceinline__ void sincos_small(float x, float* s_out, float* c_out) {
  const float tq = x * kTwoOverPi + 0x1.8p23f;
  const float j = tq - 0x1.8p23f;
  const uint32_t q = __float_as_uint(tq);
  float r = fma_(-j, kHalfPi, x);
  r = fma_(-j, kHalfPiLo, r);
  float z = r * r;
  float ps = fma_(fma_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  float s = fma_(r * z, ps, r);
  float pc = fma_(fma_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                  4.166664568298827e-2f);
  float c = fma_(z * z, pc, fma_(-0.5f, z, 1.0f));
  const uint32_t odd = (uint32_t)((int32_t)(q << 31) >> 31);  // v_bfe_i32 q, 0, 1
  const float sv = __uint_as_float(bfi_(odd, __float_as_uint(c), __float_as_uint(s)));
  const float cv = __uint_as_float(bfi_(odd, __float_as_uint(s), __float_as_uint(c)));
  *s_out = __uint_as_float(xor_sign_(__float_as_uint(sv), q << 30));
  *c_out = __uint_as_float(xor_sign_(__float_as_uint(cv), (q + 1u) << 30));
}

// acos_ with the exact-for-its-range sqrt (zb is 0 or >= 2^-25 for |t| <= 1; NaN/negative
// inputs propagate NaN exactly as sqrtf does).
__device__ __forceinline__ float acos_dev(float t) {
  float a = fabsf(t);
  bool big = a > 0.5f;
  float zb = 0.5f * (1.0f - a);
  float z = big ? zb : a * a;
  float w = big ? sqrt_nosmall(zb) : a;
  float p = fma_(fma_(fma_(fma_(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                      7.4953002686e-2f), z, 1.6666752422e-1f);
  float s = fma_(w * z, p, w);
  // rb is used only for |t| > 1/2 (t != 0): t > 0 is t's sign bit, and (t > 0 ? 2s : pi - 2s)
  // == fma(2s, t < 0 ? -1 : 1, t < 0 ? pi : 0), one rounding either way
  const uint32_t tb = __float_as_uint(t);
  const float sg = __uint_as_float(bfi_(0x80000000u, tb, 0x3f800000u));  // t < 0 ? -1 : 1
  // the offset (t < 0 ? pi : 0) as fma(sg, -pi/2, pi/2): exact (+0 or pi), one FMA-class
  // instruction instead of a shift and a mask
  float rb = fma_(2.0f * s, sg, fma_(sg, -0.5f * kPi, 0.5f * kPi));
  // pi/2 - copysign(s, t) == fma(-sg, s, pi/2): sg * s is exact (+-s; t = -0 gives sg = -1)
  float rs = fma_(-sg, s, kHalfPi);
  return big ? rb : rs;
}

// atan2_ for tame x, y (each 0 or with magnitude in [2^-60, 2^40]).
__device__ __forceinline__ float atan2_tame(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  // mx = max_(ax, ay, 2^-100), mn = min_(ax, ay) for finite x, y: plain v_max3 / v_min with
  // |.| source modifiers, without the NaN-quieting canonicalizes the compiler adds to
  // fmaxf / fminf in IEEE mode (same values for non-NaN operands). Tame non-zero
  // magnitudes are >= 2^-60, so the 2^-100 floor only replaces mx = 0 (x = y = 0), where
  // the Newton division then gives 0 / 2^-100 = +0: the value atan2's a = 0 branch needs.
  float mx, mn;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(mx) : "v"(x), "v"(y), "s"(0x1p-100f));
  asm("v_min_f32 %0, |%1|, |%2|" : "=v"(mn) : "v"(x), "v"(y));
  const float a = div_tame_nz(mn, mx);  // mn >= +0
  float s = a * a;
  float q = fma_(fma_(fma_(fma_(fma_(fma_(fma_(0.002974590389872539f, s, -0.016581183968493302f), s,
                                      0.04355353931255974f), s, -0.07580578130128461f), s,
                          0.10678940285181907f), s, -0.14214209135918496f), s,
                0.1999413720560495f), s, -0.3333316696611865f);
  float r = fma_(a * s, q, a);
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
  return fma_(log1p_kernel_(f), kLog2e, fe);
}

// log_ for positive normal finite x (log_posfinite_ with the integer split).
__device__ __forceinline__ float log_posnormal(float x) {
  float f, fe;
  log_split_normal(x, &f, &fe);
  float l = log1p_kernel_(f);
  return fma_(fe, 0.693359375f, fma_(fe, -2.12194440e-4f, l));
}

// exp2_ for finite y whose rint lies in [-125, 127] (y in [-125.5, 127.5)): there the
// result 2^f * 2^k is a normal number (2^f in [2^-1/2, 2^1/2]), so ldexp is an add of k to
// the exponent field, and rint(y) comes from the 1.5 * 2^23 rounding constant: the low 9
// bits of t = y + K's encoding are k mod 512, so (bits(t) << 23) == k << 23 mod 2^32
// (one v_lshl_add_u32 in place of v_rndne, v_cvt and v_ldexp). The clamp to [-151, 129]
// cannot fire there.
__device__ __forceinline__ float exp2_tame(float y) {
  const float t = y + 0x1.8p23f;
  const float k = t - 0x1.8p23f;
  float f = y - k;
  float p = fma_(fma_(fma_(fma_(fma_(1.535336188319500e-4f, f, 1.339887440266574e-3f), f,
                               9.618437357674640e-3f), f, 5.550332471162809e-2f), f,
                     2.402264791363012e-1f), f, 6.931472028550421e-1f);
  return __uint_as_float(__float_as_uint(fma_(f, p, 1.0f)) + (__float_as_uint(t) << 23));
}

#endif  // __HIP_DEVICE_COMPILE__

}  // namespace frm
