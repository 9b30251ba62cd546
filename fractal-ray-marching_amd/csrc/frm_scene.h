// frm_scene.h — per-frame uniforms and the per-pixel hot path of src/fragment.wgsl
// (scene dispatch 18-78, distance estimators 118-271, march 273-304, normal 306-313,
// camera 315-325, shading 327-349) restated for a gfx950 compute kernel.
//
// Design: everything that depends only on Parameters (fractal family, animated
// constants, plane normals, camera rows) is hoisted to the host once per frame
// (SceneUniforms / FrameUniforms, filled by frm_host.cpp) and reaches the kernel by
// value in the kernarg segment (scalar registers). The device code is templated on the
// fractal family so the scene switch (fragment.wgsl:19) costs nothing per step.
#pragma once
#include "frm_math.h"
#include "frm_fast.h"

// FRM_ASSUME(c): tell the optimizer c holds (see "ITERS" below).
#if defined(__clang__)
#define FRM_ASSUME(c) __builtin_assume(c)
#else
#define FRM_ASSUME(c) \
  do {                \
    if (!(c)) __builtin_unreachable(); \
  } while (0)
#endif

namespace frm {

// ITERS template flag: false <=> num_iterations == 0. The fractal loops of every family
// are compiled twice: without a loop (ITERS = false) and with the trip count asserted
// to be >= 1 (ITERS = true; any u32 above that, as the reference's Parameters allows),
// so no device code ever evaluates the uniform guard
// "num_iterations > 0" inside the divergent march loop. ROCm 7.2's AMDGPU backend
// miscompiles that guard (it is rematerialised as a lane mask under the loop's exec
// mask and reused after the loop with a different exec mask), which re-entered the
// fold loop for lanes that had left the march early (DESIGN.md §"Compiler workaround").
template <bool ITERS>
FRM_HD uint32_t iterations(uint32_t n) {
  if (!ITERS) return 0u;
  FRM_ASSUME(n >= 1u);
  return n;
}

enum Family : uint32_t {
  kMenger = 0,      // scenes 0-14          fragment.wgsl:202-211
  kSierpinski = 1,  // scene 15             fragment.wgsl:164-188
  kKoch = 2,        // scenes 16-17         fragment.wgsl:213-238
  kMandelbulb = 3,  // scene 18             fragment.wgsl:240-271
  kSphere = 4,      // build extension (BASELINE config C1), not in the reference
  kMandelbulbHw = 5,  // scene 18 with FRM_FLAG_HW_MATH: hardware transcendentals (not bit-exact)
};
// the Mandelbulb family, in either math (frm builtins / hardware transcendentals)
constexpr bool is_mandelbulb(uint32_t fam) { return fam == kMandelbulb || fam == kMandelbulbHw; }

// Constants of fragment.wgsl:1-16 and 92-94 (abstract floats rounded once to f32).
constexpr float kMaxTotalDistance = 1000.0f;          // :2
constexpr float kMinDistance = 4.99999987376214e-07f; // :3  f32(5e-7)
constexpr float kInfinity = 1.00000002004087734e+20f; // :94 f32(pow(10,20))
constexpr float kCameraDirectionZ = 0x1.fe04c8p-1f;  // :329 f32(1/atan(pi/2)) = 0.99613023
constexpr float kToSunX = 0.666666686534881592f;      // :337 normalize(-SUN_DIRECTION)
constexpr float kToSunY = 0.333333343267440796f;
constexpr float kToSunZ = -0.666666686534881592f;
constexpr float kShadowFactor = 0.699999988079071045f;   // :11 f32(0.7)
constexpr float kShadowSharpness = 32.0f;               // :12
constexpr float kSpecularFactor = 0.150000005960464478f; // :13 f32(0.15)
constexpr float kSpecularSharpness = 16.0f;             // :14
constexpr float kAOFactor = 0.200000002980232239f;      // :15 f32(0.2)
constexpr float kAOSharpness = 100.0f;                  // :16

struct Plane {
  v3 anchor, normal;
};

constexpr uint32_t kMengerFastMax = 16;  // iterations with a precomputed reciprocal scale

struct SceneUniforms {
  uint32_t family;
  uint32_t n;            // parameters.num_iterations
  // Menger (cross_size, scale_factor), fragment.wgsl:21-63
  float menger_cross, menger_factor;
  // Menger: menger_rcp[i] = RN(1 / scale_i) for the DE's scales (scale_0 = 1, scale_i+1 =
  // scale_i * factor), set with menger_fast when every division (-ci) / scale_i of the frame lies
  // in div_tame's domain (frm_host.cpp set_menger): the GPU then divides by Newton steps from
  // that reciprocal (frm_fast.h div_by_rcp), which give the correctly rounded quotient there
  uint32_t menger_fast;
  float menger_rcp[kMengerFastMax];
  // Mandelbulb power = animate_between(4, 9), bailout 100, fragment.wgsl:75
  float mb_power, mb_power_m1, mb_bailout;
  // Sierpinski: TOP.y, HEIGHT*BASE_SCALE_FACTOR*0.5, a/b/c - TOP, fold normals
  float sp_top_y, sp_yoff;
  v3 sp_top[3];
  v3 sp_normal[3];
  // Koch: mirror normals, OFFSET, final scale_factor
  v3 koch_n1, koch_n2;
  float koch_offset, koch_scale;
  // tetrahedron() planes (Sierpinski: TOP,a,b,c; Koch: TOP,LEFT,RIGHT,BACK)
  Plane tet[4];
};

struct FrameUniforms {
  float row[3][4];    // camera_matrix columns 0..2 (= rows of the cgmath matrix)
  v3 origin;          // transform_position(Position(0)), fragment.wgsl:331
  float aspect_x, aspect_y;
  uint32_t width, height;
  uint32_t max_steps;
  float max_steps_f;  // Scalar(MAX_ITERATIONS)
};

// ---- distance estimators -----------------------------------------------------
// Mandelbulb work counters (data dependent); the other families' work is a fixed
// function of num_iterations.
struct DeCount {
  uint32_t bodies;
  uint32_t bailouts;
};

// mirror(position, anchor, normal), fragment.wgsl:159-162
FRM_HD v3 mirror(v3 p, v3 anchor, v3 n) {
  float d = dot(p - anchor, n);
  return fma3(fabsf(d) - d, n, p);
}
// mirror about a plane through the origin: position - Position(0) == position exactly.
FRM_HD v3 mirror0(v3 p, v3 n) {
  float d = dot(p, n);
  return fma3(fabsf(d) - d, n, p);
}
// tetrahedron(...), fragment.wgsl:151-157 (planes precomputed on the host)
FRM_HD float tetrahedron(const SceneUniforms& u, v3 p) {
  float h0 = dot(p - u.tet[0].anchor, u.tet[0].normal);
  float h1 = dot(p - u.tet[1].anchor, u.tet[1].normal);
  float h2 = dot(p - u.tet[2].anchor, u.tet[2].normal);
  float h3 = dot(p - u.tet[3].anchor, u.tet[3].normal);
  return max_(max_(max_(h0, h1), h2), h3);
}

// menger_sponge(position, cross_size, scale_factor), fragment.wgsl:202-211, with
// box (138-141), repeat (190-192), cross_inside (194-200). FAST (GPU, u.menger_fast): the
// division by the scale uses the precomputed reciprocal (the next one is loaded an iteration
// ahead); same bits.
template <bool ITERS, bool FAST>
FRM_HD float menger_folds(const SceneUniforms& u, v3 p, float d) {
  const uint32_t n = iterations<ITERS>(u.n);
  float scale = 1.0f;
  float rcp = FAST ? u.menger_rcp[0] : 0.0f;
  for (uint32_t i = 0; i < n; ++i) {
    const float rcp_next = FAST ? u.menger_rcp[i + 1u < kMengerFastMax ? i + 1u : kMengerFastMax - 1u] : 0.0f;
    v3 r = p * scale;
    v3 c = mk(fract_(r.x + 0.5f) - 0.5f, fract_(r.y + 0.5f) - 0.5f, fract_(r.z + 0.5f) - 0.5f);
    v3 a = abs3(c);
    float cx = max_(a.y, a.z), cy = max_(a.z, a.x), cz = max_(a.x, a.y);
    float ci = min_(min_(cx, cy), cz) - u.menger_cross;
#if defined(__HIP_DEVICE_COMPILE__)
    const float q = FAST ? div_by_rcp(-ci, scale, rcp) : (-ci) / scale;
    if constexpr (FAST)
      d = max_quiet(d, q);
    else
      d = max_(d, q);
#else
    (void)rcp;
    const float q = (-ci) / scale;
    d = max_(d, q);
#endif
    scale = scale * u.menger_factor;
    rcp = rcp_next;
  }
  return d;
}
template <bool ITERS>
FRM_HD float de_menger(const SceneUniforms& u, v3 p) {
  v3 q = mk(fabsf(p.x) - 0.5f, fabsf(p.y) - 0.5f, fabsf(p.z) - 0.5f);
  float d = length(max3s(q, 0.0f)) + min_(max_(max_(q.x, q.y), q.z), 0.0f);
#if defined(__HIP_DEVICE_COMPILE__)
  if (u.menger_fast) return menger_folds<ITERS, true>(u, p, d);
#endif
  return menger_folds<ITERS, false>(u, p, d);
}

// sierpinski_tetrahedron(position), fragment.wgsl:164-188. The loop runs i = N-1 .. 0; for
// N >= 2^31, i32(N) - 1 < 0 and WGSL's loop runs zero times: the host then passes n = 0
// (compute_scene_uniforms).
template <bool ITERS>
FRM_HD float de_sierpinski(const SceneUniforms& u, v3 p) {
  const uint32_t n = iterations<ITERS>(u.n);
  v3 q = mk(p.x, p.y + u.sp_yoff, p.z);
  v3 top = mk(0.0f, u.sp_top_y, 0.0f);
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t i = n - 1u - j;
    float dist = (float)(int32_t)(1u << (i & 31u));  // Scalar(1 << u32(i)), i32
    q = mirror(q, fma3(dist, u.sp_top[0], top), u.sp_normal[0]);
    q = mirror(q, fma3(dist, u.sp_top[1], top), u.sp_normal[1]);
    q = mirror(q, fma3(dist, u.sp_top[2], top), u.sp_normal[2]);
  }
  return tetrahedron(u, q);
}

// koch3D(position, normal_z), fragment.wgsl:213-238.
template <bool ITERS>
FRM_HD float de_koch(const SceneUniforms& u, v3 p) {
  const uint32_t n = iterations<ITERS>(u.n);
  v3 q = p * 2.0f;
  for (uint32_t i = 0; i < n; ++i) {
    q = q * 1.5f;
    q = mk(q.y, q.x, q.z);
    q = mirror0(q, u.koch_n1);
    q = mirror0(q, u.koch_n2);
    q.z = q.z - u.koch_offset;
  }
  q.y = fabsf(q.y);
  return tetrahedron(u, q) / u.koch_scale;
}

// One Mandelbulb loop body (fragment.wgsl:251-267) at magnitude r = length(z) <= bailout:
// updates z and dr in place. pow(r, y) is exp2(y*log2(r)) (frm semantics), and the body's
// second pow, pow(r, P), is pow(r, P - 1) * r (frm v3, DESIGN.md section 2: P >= 4 here, so
// the identity is exact in real arithmetic for every r >= 0, and the one extra rounding is
// smaller than the exp2's amplified log2 error it replaces). P = power, Pm1 = power - 1
// (SceneUniforms::mb_power / mb_power_m1, or one frame's of a multi-frame launch with
// per-frame powers).
FRM_HD void mb_body(float P, float Pm1, v3 c, float r, v3& z, float& dr) {
  float theta = acos_(z.z / r);
  float phi = atan2_(z.y, z.x);
  float l2 = log2_(r);
  const float pm1 = exp2_(Pm1 * l2);
  dr = fma_(pm1 * P, dr, 1.0f);
  float er = pm1 * r;
  float st, ct, sp, cp;
  sincos_(theta * P, &st, &ct);
  sincos_(phi * P, &sp, &cp);
  z = mk(fma_(er, st * cp, c.x), fma_(er, sp * st, c.y), fma_(er, ct, c.z));
}
#if defined(__HIP_DEVICE_COMPILE__)
// FRM_FLAG_HW_MATH (opt-in, never the default; kMandelbulbHw): the Mandelbulb body, magnitude and
// distance on gfx950's hardware transcendentals, as a Vulkan driver lowers fragment.wgsl's
// builtins: log2/exp2 -> v_log_f32/v_exp_f32, sin/cos -> v_sin/v_cos (argument in revolutions),
// sqrt -> v_sqrt_f32, a / b -> a * v_rcp_f32(b); acos and atan2 keep their polynomials on those
// primitives. Within WGSL's builtin accuracy bounds but not bit-exact with the oracle: its frames
// are gated by the classified P1 comparison against precise builtins (tests/test_gpu_hw_math.py,
// DESIGN.md section 3) instead of P0.
__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float hw_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ void hw_sincos(float x, float* s, float* c) {
  const float rev = x * 0.15915494309189535f;
  *s = __builtin_amdgcn_sinf(rev);
  *c = __builtin_amdgcn_cosf(rev);
}
__device__ __forceinline__ float hw_acos(float t) {
  float a = fabsf(t);
  bool big = a > 0.5f;
  float zb = 0.5f * (1.0f - a);
  float z = big ? zb : a * a;
  float w = big ? hw_sqrt(zb) : a;
  float p = fma_(fma_(fma_(fma_(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                      7.4953002686e-2f), z, 1.6666752422e-1f);
  float s = fma_(w * z, p, w);
  float rb = (t > 0.0f) ? 2.0f * s : kPi - 2.0f * s;
  return big ? rb : kHalfPi - copysignf(s, t);
}
__device__ __forceinline__ float hw_atan2(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float a = mx == 0.0f ? 0.0f : hw_div(mn, mx);
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
__device__ __forceinline__ void mb_body_hw(float P, float Pm1, v3 c, float r, v3& z, float& dr) {
  float theta = hw_acos(hw_div(z.z, r));
  float phi = hw_atan2(z.y, z.x);
  float l2 = __builtin_amdgcn_logf(r);
  dr = fma_(__builtin_amdgcn_exp2f(Pm1 * l2) * P, dr, 1.0f);
  float er = __builtin_amdgcn_exp2f(P * l2);
  float st, ct, sp, cp;
  hw_sincos(theta * P, &st, &ct);
  hw_sincos(phi * P, &sp, &cp);
  z = mk(fma_(er, st * cp, c.x), fma_(er, sp * st, c.y), fma_(er, ct, c.z));
}
__device__ __forceinline__ float mb_distance_hw(float r, float dr) {
  return hw_div((0.5f * (__builtin_amdgcn_logf(r) * 0.6931471805599453f)) * r, dr);
}
#endif

// distance = 0.5 * log(magnitude) * magnitude / magnitude_derivative, fragment.wgsl:269
FRM_HD float mb_distance(float r, float dr) { return ((0.5f * log_(r)) * r) / dr; }
// mb_distance for positive finite r (log_'s special-value selects cannot fire): same bits.
FRM_HD float mb_distance_posfinite(float r, float dr) { return ((0.5f * log_posfinite_(r)) * r) / dr; }
#if defined(__HIP_DEVICE_COMPILE__)
// mb_distance for positive normal finite r (integer exponent split, frm_fast.h): same bits.
__device__ __forceinline__ float mb_distance_posnormal(float r, float dr) {
  return ((0.5f * log_posnormal(r)) * r) / dr;
}
#endif

#if defined(__HIPCC__)
// Lane mask of a per-lane predicate (no int round trip, unlike HIP's __ballot(int)).
__device__ __forceinline__ uint64_t ballot(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(b);
#else
  return b;
#endif
}
// This lane's bit of a wave-uniform lane mask. The inverse ballot makes the mask the exec
// predicate directly (no VALU); older compilers (the ROCm 7.0 hiprtc bundled with torch,
// used by frm_reload) lack it and test the bit.
__device__ __forceinline__ bool lane_in(uint64_t mask) {
#if defined(__HIP_DEVICE_COMPILE__) && __has_builtin(__builtin_amdgcn_inverse_ballot_w64)
  return __builtin_amdgcn_inverse_ballot_w64(mask);
#else
  return (mask >> (threadIdx.x & 63u)) & 1u;
#endif
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// Operands of one Mandelbulb body are tame when r = length(z) is in [2^-13, bailout]
// and every component of z is 0 or has magnitude >= 2^-60: then z.z / r and
// min/max(|x|,|y|) are tame divisions, log2(r) has a positive normal argument and the
// exp2 argument (P-1)*log2 r (P in [4, 9], log2 r in [-13, log2 100]) lies in [-104, 54],
// where exp2_tame's result is normal (and so is its product with r, pow(r, P): >= 2^-117).
// The test is stricter than that domain: every |component| >= 2^-60 (one v_min3_f32 with |.|
// modifiers; a NaN component loses the minNum, but then r is NaN and fails r >= 2^-13), so an exact
// zero component also takes the exact body (same bits, slower). Such zeros came from step 0 of the
// primary rays, which samples the camera origin itself (P1: (0, 0, -1.6)): 14.5 % of body-loop
// iterations went exact (profiles/round6/ab_tame). That step now runs once per frame on the host
// (frm_kernels.hip first_steps), and the headline's body loop runs no exact body at all; the
// integer-key test that let zeros pass cost 3 VALU more per iteration.
__device__ __forceinline__ bool mb_tame(v3 z, float r) {
  float m;
  asm("v_min3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m) : "v"(z.x), "v"(z.y), "v"(z.z));
  return (r >= 0x1p-13f) & (m >= 0x1p-60f);
}

// mb_body (frm_scene.h) with the tame primitives: the same operations in the same order.
__device__ __forceinline__ void mb_body_tame(float P, float Pm1, v3 c, float r, v3& z, float& dr) {
  float theta = acos_dev(div_tame_nz(z.z, r));  // acos_dev(-0) == acos_dev(+0)
  float phi = atan2_tame(z.y, z.x);
  float l2 = log2_tame(r);
  const float pm1 = exp2_tame(Pm1 * l2);
  dr = fma_(pm1 * P, dr, 1.0f);
  float er = pm1 * r;  // pow(r, P) = pow(r, P - 1) * r (frm v3)
  // |theta * P|, |phi * P| <= 9 pi (P in [4, 9]): sincos_'s |x| <= 2^20 branch. The signs
  // (-1)^j of the two pairs go onto er (a sign flip commutes with the rounding of fma):
  // x, y take sign(theta pair) ^ sign(phi pair) = bit 31 of (t_theta + t_phi) << 31, z the
  // theta pair's
  float st, ct, sp, cp;
  uint32_t tt, tp;
  sincos_unsigned(theta * P, &st, &ct, &tt);
  sincos_unsigned(phi * P, &sp, &cp, &tp);
  const float er_xy = __uint_as_float(__float_as_uint(er) ^ ((tt + tp) << 31));
  const float er_z = __uint_as_float(__float_as_uint(er) ^ (tt << 31));
  z = mk(fma_(er_xy, st * cp, c.x), fma_(er_xy, sp * st, c.y), fma_(er_z, ct, c.z));
}

// length() through sqrt_rsq: exact when dot(a, a) lies in [2^-96, 2^126]. length_wide: whether
// a lane's dot(a, a) lies outside it (0, tiny, huge, inf, NaN): one integer range test on the
// encoding (bits - bits(2^-96), unsigned, above the range's width); such a wave takes length().
__device__ __forceinline__ float length_rsq(v3 a) { return sqrt_rsq(dot(a, a)); }
__device__ __forceinline__ bool length_wide(v3 a) {
  constexpr uint32_t kLo = 0x0f800000u, kHi = 0x7e800000u;  // bits of 2^-96, 2^126
  return __float_as_uint(dot(a, a)) - kLo > kHi - kLo;
}

#endif


// One Mandelbulb body; on the GPU the wave takes the tame fast path (frm_fast.h) when all
// its active lanes have tame operands. Bit-identical to mb_body either way. HW: the hardware-
// transcendental body (FRM_FLAG_HW_MATH; host builds have no such math and run mb_body).
template <bool HW = false>
FRM_HD void mb_step(float P, float Pm1, v3 c, float r, v3& z, float& dr) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (HW) {
    mb_body_hw(P, Pm1, c, r, z, dr);
    return;
  }
  if (ballot(!mb_tame(z, r)) == 0) {
    mb_body_tame(P, Pm1, c, r, z, dr);
    return;
  }
#endif
  mb_body(P, Pm1, c, r, z, dr);
}
template <bool HW = false>
FRM_HD void mb_step(const SceneUniforms& u, v3 c, float r, v3& z, float& dr) {
  mb_step<HW>(u.mb_power, u.mb_power_m1, c, r, z, dr);
}
// length(z) for the Mandelbulb magnitude; fast sqrt unless a lane's |z|^2 lies outside
// [2^-96, 2^126] (z = 0 included: the exact sqrtf gives its 0).
template <bool HW = false>
FRM_HD float mb_length(v3 z) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (HW) return hw_sqrt(dot(z, z));
  if (ballot(length_wide(z)) == 0) return length_rsq(z);
#endif
  return length(z);
}

// mandelbulb(position, power, bailout), fragment.wgsl:240-271: N+1 bodies; the distance
// uses the last magnitude computed at the top of the loop.
template <bool ITERS, bool HW = false>
FRM_HD float de_mandelbulb(const SceneUniforms& u, v3 p, DeCount& cnt) {
  const uint32_t n = iterations<ITERS>(u.n);
  v3 z = p;
  float dr = 1.0f;
  float r = 0.0f;
  for (uint32_t i = 0;; ++i) {
    r = mb_length<HW>(z);
    if (r > u.mb_bailout) {
      cnt.bailouts++;
      break;
    }
    mb_step<HW>(u, p, r, z, dr);
    cnt.bodies++;
    if (i == n) break;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (HW) return mb_distance_hw(r, dr);
#endif
  return mb_distance(r, dr);
}

FRM_HD float de_sphere(v3 p) { return length(p) - 0.5f; }

template <uint32_t FAM, bool ITERS>
FRM_HD float scene_de(const SceneUniforms& u, v3 p, DeCount& cnt) {
  if constexpr (FAM == kMenger) return de_menger<ITERS>(u, p);
  else if constexpr (FAM == kSierpinski) return de_sierpinski<ITERS>(u, p);
  else if constexpr (FAM == kKoch) return de_koch<ITERS>(u, p);
  else if constexpr (FAM == kMandelbulb) return de_mandelbulb<ITERS>(u, p, cnt);
  else if constexpr (FAM == kMandelbulbHw) return de_mandelbulb<ITERS, true>(u, p, cnt);
  else return de_sphere(p);
}

// Object colour at a hit: colorize(position), or colorize(1.5*position) for Sierpinski.
template <uint32_t FAM>
FRM_HD v3 scene_color(v3 p) {
  if constexpr (FAM == kSierpinski) return colorize(p * 1.5f);
  else return colorize(p);
}

// ---- camera / ray generation ----------------------------------------------------
// Pixel centre of the full-screen quad (vertex.wgsl:6-17, WebGPU y-up NDC, row 0 = top).
FRM_HD float screen_x(uint32_t x, uint32_t w) { return (float)(2u * x + 1u) / (float)w - 1.0f; }
FRM_HD float screen_y(uint32_t y, uint32_t h) { return 1.0f - (float)(2u * y + 1u) / (float)h; }

// (vec4(d, 0) * camera_matrix).xyz, fragment.wgsl:315-325; dot4 = fma chain. `row` = the
// camera_matrix rows of the frame (f.row, or one frame's of a batch).
FRM_HD v3 camera_ray_rows(const FrameUniforms& f, const float (&row)[3][4], uint32_t x, uint32_t y) {
  float sx = screen_x(x, f.width), sy = screen_y(y, f.height);
  v3 d = normalize(mk(sx * f.aspect_x, sy * f.aspect_y, kCameraDirectionZ));
  v3 o;
  o.x = fma_(0.0f, row[0][3], fma_(d.z, row[0][2], fma_(d.y, row[0][1], d.x * row[0][0])));
  o.y = fma_(0.0f, row[1][3], fma_(d.z, row[1][2], fma_(d.y, row[1][1], d.x * row[1][0])));
  o.z = fma_(0.0f, row[2][3], fma_(d.z, row[2][2], fma_(d.y, row[2][1], d.x * row[2][0])));
  return o;
}
FRM_HD v3 camera_ray(const FrameUniforms& f, uint32_t x, uint32_t y) { return camera_ray_rows(f, f.row, x, y); }

// The camera of one frame of a multi-frame launch (frm_render_bands_batch): the rows of its
// camera_matrix and transform_position(Position(0)). Frames of a batch share everything
// else (size, aspect, step cap, scene uniforms).
struct FrameCamera {
  float row[3][4];
  v3 origin;
};

// ---- shading helpers (fragment.wgsl:336-346) ----------------------------------------
FRM_HD v3 to_sun() { return mk(kToSunX, kToSunY, kToSunZ); }

// Normal from the four tetrahedral taps d0..d3 (k.xyy, k.yyx, k.yxy, k.xxx),
// fragment.wgsl:306-313: sum left to right, then normalize.
FRM_HD v3 normal_from_taps(float d0, float d1, float d2, float d3) {
  v3 s = mk(((d0 - d1) - d2) + d3, ((-d0 - d1) + d2) + d3, ((-d0 + d1) - d2) + d3);
  return normalize(s);
}
FRM_HD v3 normal_tap_pos(v3 p, int k) {
  const float e = kMinDistance;
  switch (k) {
    case 0: return mk(p.x + e, p.y + -e, p.z + -e);
    case 1: return mk(p.x + -e, p.y + -e, p.z + e);
    case 2: return mk(p.x + -e, p.y + e, p.z + -e);
    default: return mk(p.x + e, p.y + e, p.z + e);
  }
}

// Shading of a hit pixel, fragment.wgsl:337-346, split at the shadow march:
// shade_hit_pre runs before it (specular term, ambient occlusion), shade_hit_post after.
FRM_HD v3 shade_hit_pre(const FrameUniforms& f, v3 color, v3 dir, v3 n, uint32_t steps, float* specular) {
  v3 halfway = normalize(-dir + to_sun());
  *specular = pow_(max_(dot(halfway, n), 0.0f), kSpecularSharpness);
  float ao = pow_(1.0f - (float)steps / f.max_steps_f, kAOSharpness);
  return color * mix_(kAOFactor, 1.0f, ao);
}
FRM_HD v3 shade_hit_post(v3 color, float specular, float sun_distance, float sun_closeness) {
  float shadow = ((sun_distance < 0.0f ? 1.0f : 0.0f) * kShadowSharpness) * sun_closeness;
  color = color * mix_(kShadowFactor, 1.0f, clamp_(shadow, 0.0f, 1.0f));
  float add = ((kSpecularFactor * shadow) * specular) * 1.0f;
  return mk(color.x + add, color.y + add, color.z + add);
}

// Shadow-ray origin: object_position + object_normal * 2 * MIN_DISTANCE (contracted).
FRM_HD v3 shadow_origin(v3 pos, v3 n) {
  return mk(fma_(n.x * 2.0f, kMinDistance, pos.x), fma_(n.y * 2.0f, kMinDistance, pos.y),
            fma_(n.z * 2.0f, kMinDistance, pos.z));
}
// start_position + total_distance * direction (contracted), fragment.wgsl:290.
FRM_HD v3 ray_at(v3 o, float t, v3 d) { return mk(fma_(t, d.x, o.x), fma_(t, d.y, o.y), fma_(t, d.z, o.z)); }

// ---- march + fragment_main ------------------------------------------------------------
struct MarchState {
  v3 pos;
  float total;
  float closeness;
  uint32_t steps;
  bool hit;
};

// march(start_position, direction), fragment.wgsl:281-304. `evals` counts scene()
// calls in the loop (= steps, +1 on a hit). Closeness is only needed by the shadow ray.
template <uint32_t FAM, bool ITERS, bool CLOSENESS>
FRM_HD MarchState march(const SceneUniforms& su, uint32_t max_steps, v3 o, v3 d, DeCount& cnt,
                        uint32_t& evals) {
  MarchState m;
  m.pos = o;
  m.hit = false;
  float total = 0.0f, closeness = kInfinity;
  uint32_t it = 0;
  for (; it < max_steps && total < kMaxTotalDistance; ++it) {
    v3 p = ray_at(o, total, d);
    float de = scene_de<FAM, ITERS>(su, p, cnt);
    evals++;
    if (CLOSENESS) closeness = min_(closeness, de / total);
    if (de <= kMinDistance) {
      m.hit = true;
      m.pos = p;
      break;
    }
    total = total + de;
  }
  m.total = total;
  m.closeness = closeness;
  m.steps = it;
  return m;
}

struct PixelCount {
  uint32_t hit, primary, shadow, normal;
  DeCount de;
};

// fragment_main(screen_position) for pixel (x, y): the linear colour. fragment.wgsl:327-349.
template <uint32_t FAM, bool ITERS>
FRM_HD v3 shade_pixel(const FrameUniforms& f, const SceneUniforms& su, uint32_t x, uint32_t y,
                      PixelCount& pc) {
  v3 dir = camera_ray(f, x, y);
  MarchState m = march<FAM, ITERS, false>(su, f.max_steps, f.origin, dir, pc.de, pc.primary);
  v3 color = mk(0.0f, 0.0f, 0.0f);
  if (m.hit) {  // object_result.distance >= 0
    pc.hit = 1;
    color = scene_color<FAM>(m.pos);
    float d0 = scene_de<FAM, ITERS>(su, normal_tap_pos(m.pos, 0), pc.de);
    float d1 = scene_de<FAM, ITERS>(su, normal_tap_pos(m.pos, 1), pc.de);
    float d2 = scene_de<FAM, ITERS>(su, normal_tap_pos(m.pos, 2), pc.de);
    float d3 = scene_de<FAM, ITERS>(su, normal_tap_pos(m.pos, 3), pc.de);
    pc.normal += 4;
    v3 n = normal_from_taps(d0, d1, d2, d3);
    float spec;
    color = shade_hit_pre(f, color, dir, n, m.steps, &spec);
    MarchState sun = march<FAM, ITERS, true>(su, f.max_steps, shadow_origin(m.pos, n), to_sun(), pc.de, pc.shadow);
    color = shade_hit_post(color, spec, sun.hit ? sun.total : -kInfinity, sun.closeness);
  }
  return color;
}

// Linear colour -> sRGB 8-bit code: the number of thresholds T[1..255] that c reaches.
// T[k] is the smallest f32 whose exact sRGB encoding rounds to >= k (frm_srgb_table.h),
// so this equals round(255 * srgb(clamp(c, 0, 1))) exactly; NaN -> 0 (UNORM rule).
// On the GPU the search is replaced by a candidate code from the sRGB curve evaluated with the
// hardware log/exp (within one code of the exact code for every f32, tests/test_gpu_present.py
// checks all of [0, 1] and the special values) and one comparison on each side of it: two
// table reads instead of eight dependent ones (the table sits in LDS, where data-dependent
// reads conflict on banks). The table alone decides the code, so the result is the same.
FRM_HD uint32_t encode_srgb(float c, const float* table) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float cc = __builtin_fminf(__builtin_fmaxf(c, 0.0f), 1.0f);  // NaN -> 0
  const float s = cc <= 0.0031308f
                      ? cc * 12.92f
                      : fmaf(1.055f, __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(cc) * 0.41666666f), -0.055f);
  const uint32_t k = min((uint32_t)fmaf(s, 255.0f, 0.5f), 254u);
  const float lo = table[k], hi = table[k + 1u];
  // table[k + 1] <= c: one up; c < table[k] (then also c < table[k + 1]): one down, except at 0
  // (NaN stays at 0); branch-free
  return k + (c >= hi ? 1u : 0u) - ((k > 0u && !(c >= lo)) ? 1u : 0u);
#else
  uint32_t i = 0;
#pragma unroll
  for (uint32_t step = 128; step >= 1; step >>= 1)
    if (c >= table[i + step]) i += step;
  return i;
#endif
}

FRM_HD uint32_t pack_rgba(v3 c, const float* table) {
  return encode_srgb(c.x, table) | (encode_srgb(c.y, table) << 8) | (encode_srgb(c.z, table) << 16) |
         (255u << 24);
}

}  // namespace frm
