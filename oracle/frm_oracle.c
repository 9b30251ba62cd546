/*
 * frm_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
 *
 * A plain-C restatement of the reference hot path, MariusDoe/fractal-ray-marching
 * src/fragment.wgsl (fragment_main :327-349, march :281-304, calculate_normal :306-313,
 * scene :18-82, DEs :118-271, camera :315-325) plus the pixel-centre rule of
 * src/vertex.wgsl:6-17 and the Rgba8UnormSrgb store of src/blit_graphics.rs:14.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (libfrm.so) never links or calls it.
 *
 * Two math modes:
 *   OM_FRM  — the builtins as specified in DESIGN.md §"frm math" (restated here from the
 *             spec, not shared with the kernel source): the GPU must match this mode BIT FOR
 *             BIT (parity gate P0).
 *   OM_LIBM — sin/cos/acos/atan2/log/log2/exp2/pow evaluated in double precision by libm
 *             and rounded once to f32: the "precise WGSL" semantic cross-check (gate P1).
 * Everything else (IEEE f32 +-*, fma, correctly rounded / and sqrt, minNum/maxNum) is the
 * same in both modes. Compile with -ffp-contract=off (see oracle/Makefile).
 *
 * Parity status: the reference ships no tests, fixtures or golden outputs, and neither
 * its Rust host nor its WGSL can be built or executed in this environment (no cargo,
 * naga or Vulkan). The oracle is therefore pinned by closed-form known answers
 * (tests/test_oracle_kat.py) and by the OM_LIBM cross-check, not by reference outputs.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OM_FRM 0
#define OM_LIBM 1

typedef struct {
  float x, y, z;
} vec3;

static vec3 V(float x, float y, float z) {
  vec3 r = {x, y, z};
  return r;
}
static vec3 vadd(vec3 a, vec3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static vec3 vsub(vec3 a, vec3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static vec3 vscale(vec3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static vec3 vmul(vec3 a, vec3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static vec3 vneg(vec3 a) { return V(-a.x, -a.y, -a.z); }
/* dot = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)) */
static float vdot(vec3 a, vec3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static float vlength(vec3 a) { return sqrtf(vdot(a, a)); }
static vec3 vnormalize(vec3 a) {
  float l = vlength(a);
  return V(a.x / l, a.y / l, a.z / l);
}
static vec3 vcross(vec3 u, vec3 v) {
  return V(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
/* a + s*b, contracted */
static vec3 vmadd(float s, vec3 b, vec3 a) {
  return V(fmaf(s, b.x, a.x), fmaf(s, b.y, a.y), fmaf(s, b.z, a.z));
}
static float wmin(float a, float b) { return fminf(a, b); }
static float wmax(float a, float b) { return fmaxf(a, b); }
static float wclamp(float x, float lo, float hi) { return wmin(wmax(x, lo), hi); }
static float wmix(float a, float b, float t) { return a * (1.0f - t) + b * t; }
static float wfract(float x) { return x - floorf(x); }

/* ======================= builtins, OM_FRM (frm semantics v2; v3 in mandelbulb) ========= */
static const float PI_F = 3.14159274101257324219f;
static const float HALF_PI_F = 1.57079637050628662109f;
static const float INV_PI_HI = 0x1.45f306p-2f; /* RN(1/pi) */
static const float INV_PI_LO = 0x1.b93910p-27f; /* RN(1/pi - INV_PI_HI) */
static const float ROUND_K = 0x1.8p23f;         /* 1.5 * 2^23: x + K rounds x to an integer */

static float horner(const float* c, int n, float x) { /* c[0] + x (c[1] + x (... c[n-1])) */
  float p = c[n - 1];
  for (int i = n - 2; i >= 0; --i) p = fmaf(p, x, c[i]);
  return p;
}

/* sin/cos: half-turn reduction r = x/pi - j, j the nearest integer (|r| <= 1/2);
 * sin(x) = (-1)^j r S(r^2), cos(x) = (-1)^j C(r^2), minimax fits of sin(pi r)/r and cos(pi r)
 * (tools/v2fit.py). For |x| <= 2^20, j = rint of the exact product x * INV_PI_HI, taken from
 * t = fma(x, INV_PI_HI, K) (t's unit in the last place is 1); larger or non-finite x take
 * j = rint(RN(x * INV_PI_HI)) (defined, not accurate: WGSL bounds sin/cos on [-pi, pi] only). */
static const float SIN_C[5] = {0x1.921fb6p+1f, -0x1.4abbc2p+2f, 0x1.4668b0p+1f, -0x1.324cccp-1f, 0x1.3daffap-4f};
static const float COS_C[5] = {1.0f, -0x1.3bd3b0p+2f, 0x1.03bdaap+2f, -0x1.55041ap+0f, 0x1.c2b9aap-3f};
static void frm_sincos(float x, float* so, float* co) {
  float j;
  int odd;
  if (fabsf(x) <= 0x1p20f) {
    float t = fmaf(x, INV_PI_HI, ROUND_K);
    uint32_t tb;
    memcpy(&tb, &t, 4);
    j = t - ROUND_K;
    odd = (int)(tb & 1u);
  } else {
    j = rintf(x * INV_PI_HI);
    odd = fabsf(j) < 0x1p24f ? (int)((int64_t)j & 1) : 0; /* NaN: 0 */
  }
  float r = fmaf(x, INV_PI_HI, -j);
  r = fmaf(x, INV_PI_LO, r);
  float u = r * r;
  float s = r * horner(SIN_C, 5, u);
  float c = horner(COS_C, 5, u);
  *so = odd ? -s : s;
  *co = odd ? -c : c;
}

/* acos(t) = sqrt(1 - |t|) P(|t|) for t >= 0 and pi - that for t < 0; P a relative minimax fit
 * with P(0) = RN(pi/2). */
static const float ACOS_C[7] = {0x1.921fb6p+0f, -0x1.b77b98p-3f, 0x1.6bbdc6p-4f, -0x1.912814p-5f,
                                0x1.bd48d6p-6f, -0x1.748422p-7f, 0x1.35deb4p-9f};
static float frm_acos(float t) {
  float a = fabsf(t);
  float r = sqrtf(1.0f - a) * horner(ACOS_C, 7, a);
  return t < 0.0f ? PI_F - r : r;
}

/* atan2: a = min(|x|,|y|) * RN(1 / max(|x|,|y|)) in [0, 1] (0 when both are 0);
 * atan(a) = a + a s Q(s), s = a^2, Q a relative minimax fit; octant and quadrant fix-ups;
 * atan2(+-0, +-0) = +-0. */
static const float ATAN_C[7] = {-0x1.5552dep-2f, 0x1.991268p-3f, -0x1.1f90fcp-3f, 0x1.984ef0p-4f,
                                -0x1.ed2edep-5f, 0x1.953dcap-6f, -0x1.3c0c38p-8f};
static float frm_atan2(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float a = mn * (1.0f / mx);
  if (mx == 0.0f) a = 0.0f;
  float s = a * a;
  float r = fmaf(a * s, horner(ATAN_C, 7, s), a);
  if (ay > ax) r = HALF_PI_F - r;
  if (x < 0.0f) r = PI_F - r;
  return copysignf(r, y);
}

/* x = m 2^e, m in [sqrt(1/2), sqrt(2)); returns f = m - 1 (exact) and e */
static float frm_split(float x, float* e_out) {
  int e;
  float m = frexpf(x, &e);
  if (m < 0.707106769084930419922f) {
    m = m + m;
    e = e - 1;
  }
  *e_out = (float)e;
  return m - 1.0f;
}
static float frm_log_special(float x, float r) {
  if (x != x || x < 0.0f) return NAN;
  if (x == 0.0f) return -INFINITY;
  if (x == INFINITY) return INFINITY;
  return r;
}
/* log2(x) = e + f Q(f), Q a relative minimax fit of log2(1 + f) / f */
static const float LOG2_C[8] = {0x1.715476p+0f, -0x1.715528p-1f, 0x1.ec7724p-2f, -0x1.70e2aap-2f,
                                0x1.25fd38p-2f, -0x1.fdb316p-3f, 0x1.df5156p-3f, -0x1.2a9f30p-3f};
static float frm_log2(float x) {
  float e;
  float f = frm_split(x, &e);
  return frm_log_special(x, fmaf(f, horner(LOG2_C, 8, f), e));
}
/* log(x) = e ln2 + f L(f) (ln 2 in two parts), L a relative minimax fit of ln(1 + f) / f */
static const float LN_C[8] = {0x1.fffffep-1f, -0x1.00007ap-1f, 0x1.5559dcp-2f, -0x1.ff623ep-3f,
                              0x1.978e32p-3f, -0x1.614bfcp-3f, 0x1.4c3cdcp-3f, -0x1.9dfa4ep-4f};
static float frm_log(float x) {
  float e;
  float f = frm_split(x, &e);
  float l = f * horner(LN_C, 8, f);
  return frm_log_special(x, fmaf(e, 0.693359375f, fmaf(e, -2.12194440e-4f, l)));
}
/* exp2: k = rint(y) after clamping y to [-151, 129], f = y - k in [-1/2, 1/2] (exact);
 * 2^f = 1 + f P(f) (relative minimax fit); ldexp (one rounding for subnormal results). */
static const float EXP2_C[5] = {0x1.62e42ap-1f, 0x1.ebf9bcp-3f, 0x1.c6b752p-5f, 0x1.3cea80p-7f, 0x1.5bb9f4p-10f};
static float frm_exp2(float y) {
  if (y != y) return y;
  float yc = fminf(fmaxf(y, -151.0f), 129.0f);
  float k = rintf(yc);
  float f = yc - k;
  return ldexpf(fmaf(f, horner(EXP2_C, 5, f), 1.0f), (int)k);
}

/* ======================= builtin dispatch ======================================== */
static void b_sincos(int mode, float x, float* s, float* c) {
  if (mode == OM_LIBM) {
    *s = (float)sin((double)x);
    *c = (float)cos((double)x);
  } else {
    frm_sincos(x, s, c);
  }
}
static float b_sin(int mode, float x) {
  float s, c;
  b_sincos(mode, x, &s, &c);
  return s;
}
static float b_acos(int mode, float x) { return mode == OM_LIBM ? (float)acos((double)x) : frm_acos(x); }
static float b_atan2(int mode, float y, float x) {
  if (mode == OM_LIBM) return (x == 0.0f && y == 0.0f) ? copysignf(0.0f, y) : (float)atan2((double)y, (double)x);
  return frm_atan2(y, x);
}
static float b_log(int mode, float x) { return mode == OM_LIBM ? (float)log((double)x) : frm_log(x); }
static float b_log2(int mode, float x) { return mode == OM_LIBM ? (float)log2((double)x) : frm_log2(x); }
static float b_exp2(int mode, float x) { return mode == OM_LIBM ? (float)exp2((double)x) : frm_exp2(x); }
/* WGSL pow: accuracy inherited from exp2(y*log2(x)); frm defines it as exactly that. */
static float b_pow(int mode, float x, float y) {
  if (mode == OM_LIBM) return (float)pow((double)x, (double)y);
  return frm_exp2(y * frm_log2(x));
}

/* ======================= frame state ============================================ */
typedef struct {
  vec3 a;
  vec3 n;
} plane;

typedef struct {
  int mode;
  uint32_t width, height, max_steps, num_iterations, scene_index, sphere;
  float M[16], aspect[2], time;
  /* scene() uniforms (Parameters-only subexpressions, hoisted once per frame) */
  int family; /* 0 menger, 1 sierpinski, 2 koch, 3 mandelbulb, 4 sphere */
  float menger_cross, menger_scale;
  float mb_power;
  float koch_normal_z;
  /* sierpinski / koch constants */
  vec3 s_top, s_a, s_b, s_c, s_a_top, s_b_top, s_c_top, s_a_n, s_b_n, s_c_n;
  vec3 k_top, k_left, k_right, k_back, k_n1, k_n2;
  float k_offset;
  plane tet[4];
  vec3 origin;
} om_frame;

typedef struct {
  uint64_t primary, shadow, normal, hits, pixels, bodies, bailouts;
} om_counts;

/* animate_between, fragment.wgsl:80-82 (0.5 + 0.5*s and a + (b-a)*w contracted) */
static float animate_between(const om_frame* F, float a, float b) {
  float s = b_sin(F->mode, F->time * 0.2f);
  return fmaf(b - a, fmaf(0.5f, s, 0.5f), a);
}

static vec3 plane_normal(vec3 a, vec3 b, vec3 c) { return vnormalize(vcross(vsub(c, a), vsub(b, a))); }

static void set_tet(om_frame* F, vec3 a, vec3 b, vec3 c, vec3 d) {
  F->tet[0].a = a; F->tet[0].n = plane_normal(a, b, c);
  F->tet[1].a = a; F->tet[1].n = plane_normal(a, c, d);
  F->tet[2].a = a; F->tet[2].n = plane_normal(a, d, b);
  F->tet[3].a = b; F->tet[3].n = plane_normal(b, d, c);
}

/* scene() switch, fragment.wgsl:18-78 ("case 0, default") */
static void frame_setup(om_frame* F) {
  const float t6 = (float)(1.0 / 6.0), t5 = (float)(1.0 / 5.0), t4 = (float)(1.0 / 4.0);
  const float t3 = (float)(1.0 / 3.0), t8 = (float)(1.0 / 8.0);
  F->family = 0;
  F->menger_cross = t6;
  F->menger_scale = 3.0f;
  if (F->sphere) {
    F->family = 4;
  } else {
    switch (F->scene_index) {
      case 1: F->menger_cross = t5; F->menger_scale = 3.0f; break;
      case 2: F->menger_cross = t4; F->menger_scale = 3.0f; break;
      case 3: F->menger_cross = t3; F->menger_scale = 3.0f; break;
      case 4: F->menger_cross = 1.0f / animate_between(F, 2.0f, 8.0f); F->menger_scale = 3.0f; break;
      case 5: F->menger_cross = t6; F->menger_scale = 2.0f; break;
      case 6: F->menger_cross = t4; F->menger_scale = 2.0f; break;
      case 7: F->menger_cross = t8; F->menger_scale = 2.0f; break;
      case 8: F->menger_cross = 1.0f / animate_between(F, 3.0f, 10.0f); F->menger_scale = 2.0f; break;
      case 9: F->menger_cross = t4; F->menger_scale = 4.0f; break;
      case 10: F->menger_cross = t5; F->menger_scale = 5.0f; break;
      case 11: F->menger_cross = t4; F->menger_scale = 6.0f; break;
      case 12: F->menger_cross = t3; F->menger_scale = animate_between(F, 3.0f, 5.0f); break;
      case 13: F->menger_cross = t4; F->menger_scale = animate_between(F, 2.0f, 4.0f); break;
      case 14: F->menger_cross = t6; F->menger_scale = animate_between(F, 1.2f, 3.0f); break;
      case 15: F->family = 1; break;
      case 16: F->family = 2; F->koch_normal_z = (float)sqrt(3.0); break;
      case 17: F->family = 2; F->koch_normal_z = animate_between(F, (float)sqrt(3.0), 4.0f); break;
      case 18: F->family = 3; F->mb_power = animate_between(F, 4.0f, 9.0f); break;
      default: break; /* 0 and out of range: classic Menger */
    }
  }
  if (F->family == 1) { /* sierpinski_tetrahedron consts, fragment.wgsl:165-178 */
    const double HEIGHT = 4.0 / sqrt(6.0), ONE_OVER_SQRT_3 = 1.0 / sqrt(3.0);
    float scale_factor = 0.5f / (float)(int32_t)(1u << (F->num_iterations % 32u));
    F->s_top = V(0.0f, (float)(HEIGHT * 0.5), 0.0f);
    F->s_a = vmadd(scale_factor, V(-1.0f, (float)-HEIGHT, (float)-ONE_OVER_SQRT_3), F->s_top);
    F->s_b = vmadd(scale_factor, V(1.0f, (float)-HEIGHT, (float)-ONE_OVER_SQRT_3), F->s_top);
    F->s_c = vmadd(scale_factor, V(0.0f, (float)-HEIGHT, (float)(2.0 * ONE_OVER_SQRT_3)), F->s_top);
    F->s_a_top = vsub(F->s_a, F->s_top);
    F->s_b_top = vsub(F->s_b, F->s_top);
    F->s_c_top = vsub(F->s_c, F->s_top);
    F->s_a_n = vnormalize(vsub(F->s_top, F->s_a));
    F->s_b_n = vnormalize(vsub(F->s_top, F->s_b));
    F->s_c_n = vnormalize(vsub(F->s_top, F->s_c));
    set_tet(F, F->s_top, F->s_a, F->s_b, F->s_c);
  }
  if (F->family == 2) { /* koch3D consts, fragment.wgsl:214-223 (typed f32 consts) */
    const float SIDE = 3.0f, HALF = SIDE / 2.0f, SIDE_SQRT = sqrtf(SIDE);
    F->k_offset = sqrtf(SIDE * SIDE - HALF * HALF) - SIDE_SQRT;
    F->k_top = V(0.0f, 1.0f, 0.0f);
    F->k_left = V(-HALF, 0.0f, -F->k_offset);
    F->k_right = V(HALF, 0.0f, -F->k_offset);
    F->k_back = V(0.0f, 0.0f, SIDE_SQRT);
    F->k_n1 = vnormalize(V(0.0f, 1.0f, F->koch_normal_z));
    F->k_n2 = vmul(F->k_n1, V(1.0f, -1.0f, 1.0f));
    set_tet(F, F->k_top, F->k_left, F->k_right, F->k_back);
  }
  /* transform_position(Position(0)): dot4 fma chain with (0,0,0,1) */
  float o[3];
  for (int j = 0; j < 3; ++j) {
    const float* c = &F->M[4 * j];
    o[j] = fmaf(1.0f, c[3], fmaf(0.0f, c[2], fmaf(0.0f, c[1], 0.0f * c[0])));
  }
  F->origin = V(o[0], o[1], o[2]);
}

/* ======================= distance estimators ===================================== */
static float half_space(vec3 p, vec3 anchor, vec3 normal) { return vdot(vsub(p, anchor), normal); }
static float tetrahedron(const om_frame* F, vec3 p) {
  return wmax(wmax(wmax(half_space(p, F->tet[0].a, F->tet[0].n), half_space(p, F->tet[1].a, F->tet[1].n)),
                   half_space(p, F->tet[2].a, F->tet[2].n)),
              half_space(p, F->tet[3].a, F->tet[3].n));
}
static vec3 mirror(vec3 p, vec3 anchor, vec3 normal) {
  float d = vdot(vsub(p, anchor), normal);
  return vmadd(fabsf(d) - d, normal, p);
}
static vec3 colorize(vec3 p) {
  return V(wmin(1.0f, p.x + 0.5f), wmin(1.0f, p.y + 0.5f), wmin(1.0f, p.z + 0.5f));
}
static float max_c3(vec3 a) { return wmax(wmax(a.x, a.y), a.z); }
static float min_c3(vec3 a) { return wmin(wmin(a.x, a.y), a.z); }

static float box(vec3 p, float size) {
  vec3 q = V(fabsf(p.x) - size, fabsf(p.y) - size, fabsf(p.z) - size);
  return vlength(V(wmax(q.x, 0.0f), wmax(q.y, 0.0f), wmax(q.z, 0.0f))) + wmin(max_c3(q), 0.0f);
}
static vec3 repeat(vec3 p) { return V(wfract(p.x + 0.5f) - 0.5f, wfract(p.y + 0.5f) - 0.5f, wfract(p.z + 0.5f) - 0.5f); }
static float cross_inside(vec3 p, float size) {
  vec3 a = V(fabsf(p.x), fabsf(p.y), fabsf(p.z));
  return min_c3(V(wmax(a.y, a.z), wmax(a.z, a.x), wmax(a.x, a.y))) - size;
}
static float menger_sponge(const om_frame* F, vec3 p) {
  float distance = box(p, 0.5f);
  float scale = 1.0f; /* 0.5 / SIZE */
  for (uint32_t i = 0; i < F->num_iterations; ++i) {
    distance = wmax(distance, -cross_inside(repeat(vscale(p, scale)), F->menger_cross) / scale);
    scale *= F->menger_scale;
  }
  return distance;
}
static float sierpinski(const om_frame* F, vec3 position) {
  vec3 p = position;
  p.y += (float)(4.0 / sqrt(6.0) * 0.5 * 0.5);
  for (int32_t i = (int32_t)F->num_iterations - 1; i >= 0; i--) {
    float distance = (float)(int32_t)(1u << ((uint32_t)i % 32u));
    p = mirror(p, vmadd(distance, F->s_a_top, F->s_top), F->s_a_n);
    p = mirror(p, vmadd(distance, F->s_b_top, F->s_top), F->s_b_n);
    p = mirror(p, vmadd(distance, F->s_c_top, F->s_top), F->s_c_n);
  }
  return tetrahedron(F, p);
}
static float koch(const om_frame* F, vec3 position) {
  vec3 p = vscale(position, 2.0f);
  float scale_factor = 2.0f;
  for (uint32_t i = 0; i < F->num_iterations; ++i) {
    scale_factor *= 1.5f;
    p = vscale(p, 1.5f);
    p = V(p.y, p.x, p.z);
    p = mirror(p, V(0.0f, 0.0f, 0.0f), F->k_n1);
    p = mirror(p, V(0.0f, 0.0f, 0.0f), F->k_n2);
    p.z -= F->k_offset;
  }
  p.y = fabsf(p.y);
  return tetrahedron(F, p) / scale_factor;
}
static float mandelbulb(const om_frame* F, vec3 position, om_counts* C) {
  const float power = F->mb_power, bailout = 100.0f;
  const int m = F->mode;
  vec3 current = position;
  float magnitude_derivative = 1.0f, magnitude = 0.0f;
  for (uint32_t i = 0; i <= F->num_iterations; i++) {
    magnitude = vlength(current);
    if (magnitude > bailout) {
      C->bailouts++;
      break;
    }
    float theta = b_acos(m, current.z / magnitude);
    float phi = b_atan2(m, current.y, current.x);
    /* fragment.wgsl:254, 257; frm v3: pow(magnitude, power) evaluated as
       pow(magnitude, power - 1) * magnitude; OM_LIBM keeps the float64 pow */
    const float pow_m1 = b_pow(m, magnitude, power - 1.0f);
    magnitude_derivative = fmaf(pow_m1 * power, magnitude_derivative, 1.0f);
    float exp_magnitude = m == OM_LIBM ? b_pow(m, magnitude, power) : pow_m1 * magnitude;
    float st, ct, sp, cp;
    b_sincos(m, theta * power, &st, &ct);
    b_sincos(m, phi * power, &sp, &cp);
    current = vmadd(exp_magnitude, V(st * cp, sp * st, ct), position);
    C->bodies++;
  }
  return ((0.5f * b_log(m, magnitude)) * magnitude) / magnitude_derivative;
}

static float scene(const om_frame* F, vec3 p, vec3* color, om_counts* C) {
  float d;
  switch (F->family) {
    case 1: d = sierpinski(F, p); if (color) *color = colorize(vscale(p, 1.5f)); return d;
    case 2: d = koch(F, p); break;
    case 3: d = mandelbulb(F, p, C); break;
    case 4: d = vlength(p) - 0.5f; break;
    default: d = menger_sponge(F, p); break;
  }
  if (color) *color = colorize(p);
  return d;
}

/* ======================= march / normal / fragment ================================ */
static const float MAX_TOTAL_DISTANCE = 1000.0f;
static const float MIN_DISTANCE = 5e-7f;
static const float INF_1E20 = 1e20f;

typedef struct {
  vec3 position, color;
  float distance, closeness;
  uint32_t steps;
} march_result;

static march_result march(const om_frame* F, vec3 start, vec3 dir, uint64_t* evals, om_counts* C) {
  march_result r;
  r.position = start;
  r.distance = -INF_1E20;
  r.color = V(0.0f, 0.0f, 0.0f);
  float total = 0.0f, closeness = INF_1E20;
  uint32_t it = 0;
  for (; it < F->max_steps && total < MAX_TOTAL_DISTANCE; it++) {
    vec3 p = vmadd(total, dir, start);
    vec3 col;
    float d = scene(F, p, &col, C);
    (*evals)++;
    closeness = wmin(closeness, d / total);
    if (d <= MIN_DISTANCE) {
      r.color = col;
      r.distance = total;
      r.position = p;
      break;
    }
    total += d;
  }
  r.closeness = closeness;
  r.steps = it;
  return r;
}

static vec3 calculate_normal(const om_frame* F, vec3 p, om_counts* C) {
  const float e = MIN_DISTANCE;
  float d0 = scene(F, V(p.x + e, p.y + -e, p.z + -e), NULL, C);
  float d1 = scene(F, V(p.x + -e, p.y + -e, p.z + e), NULL, C);
  float d2 = scene(F, V(p.x + -e, p.y + e, p.z + -e), NULL, C);
  float d3 = scene(F, V(p.x + e, p.y + e, p.z + e), NULL, C);
  C->normal += 4;
  /* k.xyy*d0 + k.yyx*d1 + k.yxy*d2 + k.xxx*d3, left to right */
  vec3 s = V(d0, -d0, -d0);
  s = vadd(s, V(-d1, -d1, d1));
  s = vadd(s, V(-d2, d2, -d2));
  s = vadd(s, V(d3, d3, d3));
  return vnormalize(s);
}

#define INFO_HIT 1u
#define INFO_SUN_HIT 2u
#define INFO_NAN 4u
#define INFO_SHADOW_FIRST_NONPOS 8u
#define INFO_ZERO_NORMAL 16u

/* Camera ray of pixel (x, y): fragment.wgsl:329-330 with vertex.wgsl's pixel centre. */
static vec3 camera_dir(const om_frame* F, uint32_t x, uint32_t y) {
  const float CAMERA_DIRECTION_Z = (float)(1.0 / atan(90.0 * 3.141592653589793238 / 180.0));
  float sx = (float)(2u * x + 1u) / (float)F->width - 1.0f;
  float sy = 1.0f - (float)(2u * y + 1u) / (float)F->height;
  vec3 d0 = vnormalize(V(sx * F->aspect[0], sy * F->aspect[1], CAMERA_DIRECTION_Z));
  float dir[3];
  for (int j = 0; j < 3; ++j) {
    const float* c = &F->M[4 * j];
    dir[j] = fmaf(0.0f, c[3], fmaf(d0.z, c[2], fmaf(d0.y, c[1], d0.x * c[0])));
  }
  return V(dir[0], dir[1], dir[2]);
}

static const vec3 TO_SUN = {0.666666686534881592f, 0.333333343267440796f, -0.666666686534881592f};

/* Shading of a hit, fragment.wgsl:336-346, from the march's geometric results: the object
 * colour, primary steps, normal and the shadow march's distance and closeness. The only
 * builtins are the two pows (specular, ambient occlusion), in the frame's math mode. */
static vec3 shade_hit(const om_frame* F, vec3 camera_direction, vec3 color, uint32_t steps, vec3 n,
                      float sun_distance, float sun_closeness) {
  vec3 halfway = vnormalize(vadd(vneg(camera_direction), TO_SUN));
  float specular = b_pow(F->mode, wmax(vdot(halfway, n), 0.0f), 16.0f);
  float ao = b_pow(F->mode, 1.0f - (float)steps / (float)F->max_steps, 100.0f);
  color = vscale(color, wmix(0.2f, 1.0f, ao));
  float shadow = ((sun_distance < 0.0f ? 1.0f : 0.0f) * 32.0f) * sun_closeness;
  color = vscale(color, wmix(0.7f, 1.0f, wclamp(shadow, 0.0f, 1.0f)));
  float add = ((0.15f * shadow) * specular) * 1.0f;
  return vadd(color, V(add, add, add));
}

/* Per-pixel trace of the geometric inputs of the shading (parity classification, P1):
 * hit, primary steps, normal xyz, sun hit, sun closeness, object colour xyz. */
#define OM_TRACE_FLOATS 10

/* fragment_main; returns linear colour, fills counters, a per-pixel info word and (if
 * trace) the OM_TRACE_FLOATS geometric shading inputs */
static vec3 fragment(const om_frame* F, uint32_t x, uint32_t y, om_counts* C, uint32_t* info, float* trace) {
  vec3 camera_direction = camera_dir(F, x, y);
  march_result obj = march(F, F->origin, camera_direction, &C->primary, C);
  vec3 color = obj.color;
  uint32_t inf = obj.steps << 8;
  if (trace) {
    memset(trace, 0, OM_TRACE_FLOATS * sizeof(float));
    trace[1] = (float)obj.steps;
  }
  if (obj.distance >= 0.0f) {
    inf |= INFO_HIT;
    C->hits++;
    vec3 n = calculate_normal(F, obj.position, C);
    if (n.x != n.x) inf |= INFO_ZERO_NORMAL;
    vec3 start = V(fmaf(n.x * 2.0f, MIN_DISTANCE, obj.position.x), fmaf(n.y * 2.0f, MIN_DISTANCE, obj.position.y),
                   fmaf(n.z * 2.0f, MIN_DISTANCE, obj.position.z));
    march_result sun = march(F, start, TO_SUN, &C->shadow, C);
    if (sun.distance >= 0.0f) inf |= INFO_SUN_HIT;
    if (sun.closeness != sun.closeness || sun.closeness == -INFINITY) inf |= INFO_SHADOW_FIRST_NONPOS;
    if (trace) {
      const float t[OM_TRACE_FLOATS] = {1.0f, (float)obj.steps, n.x, n.y, n.z, sun.distance >= 0.0f ? 1.0f : 0.0f,
                                        sun.closeness, color.x, color.y, color.z};
      memcpy(trace, t, sizeof(t));
    }
    color = shade_hit(F, camera_direction, color, obj.steps, n, sun.distance, sun.closeness);
    if (color.x != color.x || color.y != color.y || color.z != color.z) inf |= INFO_NAN;
  }
  *info = inf;
  return color;
}

/* ======================= sRGB encode (Rgba8UnormSrgb store) ====================== */
static float g_srgb_t[256];
static pthread_once_t g_srgb_once = PTHREAD_ONCE_INIT;

static double srgb_exact(double c) { return c <= 0.0031308 ? 12.92 * c : 1.055 * pow(c, 1.0 / 2.4) - 0.055; }
static void srgb_init(void) {
  g_srgb_t[0] = -INFINITY;
  for (int k = 1; k < 256; ++k) { /* smallest f32 c >= 0 with round(255*srgb(c)) >= k */
    uint32_t lo = 0, hi = 0x3f800000u;
    while (lo < hi) {
      uint32_t mid = lo + (hi - lo) / 2;
      float c;
      memcpy(&c, &mid, 4);
      if (floor(srgb_exact((double)c) * 255.0 + 0.5) >= (double)k) hi = mid;
      else lo = mid + 1;
    }
    memcpy(&g_srgb_t[k], &lo, 4);
  }
}
static uint8_t encode(float c) {
  int k = 0;
  for (int i = 1; i < 256; ++i)
    if (c >= g_srgb_t[i]) k = i; /* thresholds are increasing */
  return (uint8_t)k;
}

/* ======================= public API ============================================== */
typedef struct {
  const om_frame* F;
  const uint32_t* rows;
  uint32_t nrows;
  uint8_t* rgba;
  float* linear;
  uint32_t* info;
  float* trace;
  uint32_t next; /* atomic row cursor (rayon-like dynamic schedule) */
  pthread_mutex_t mu;
  om_counts total;
} job;

static void* worker(void* arg) {
  job* J = (job*)arg;
  om_counts C;
  memset(&C, 0, sizeof(C));
  const uint32_t W = J->F->width;
  for (;;) {
    uint32_t r = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
    if (r >= J->nrows) break;
    uint32_t y = J->rows ? J->rows[r] : r;
    for (uint32_t x = 0; x < W; ++x) {
      uint32_t inf;
      const size_t i = (size_t)r * W + x;
      vec3 c = fragment(J->F, x, y, &C, &inf, J->trace ? J->trace + OM_TRACE_FLOATS * i : NULL);
      C.pixels++;
      uint8_t* px = J->rgba + 4 * i;
      px[0] = encode(c.x);
      px[1] = encode(c.y);
      px[2] = encode(c.z);
      px[3] = 255;
      if (J->linear) {
        J->linear[3 * i] = c.x;
        J->linear[3 * i + 1] = c.y;
        J->linear[3 * i + 2] = c.z;
      }
      if (J->info) J->info[i] = inf;
    }
  }
  pthread_mutex_lock(&J->mu);
  J->total.primary += C.primary;
  J->total.shadow += C.shadow;
  J->total.normal += C.normal;
  J->total.hits += C.hits;
  J->total.pixels += C.pixels;
  J->total.bodies += C.bodies;
  J->total.bailouts += C.bailouts;
  pthread_mutex_unlock(&J->mu);
  return NULL;
}

static void frame_from_params(om_frame* F, const uint8_t* params96, uint32_t width, uint32_t height,
                              uint32_t max_steps, uint32_t flags, int mode) {
  memset(F, 0, sizeof(*F));
  memcpy(F->M, params96, 64);
  memcpy(F->aspect, params96 + 64, 8);
  memcpy(&F->time, params96 + 72, 4);
  memcpy(&F->num_iterations, params96 + 76, 4);
  memcpy(&F->scene_index, params96 + 80, 4);
  F->width = width;
  F->height = height;
  F->max_steps = max_steps ? max_steps : 5000u;
  F->sphere = (flags & 1u) ? 1u : 0u;
  F->mode = mode;
  frame_setup(F);
}

/* Render `nrows` rows (rows[i], or 0..nrows-1 when rows == NULL) of a width x height frame.
 * counters (8 x u64, same order as libfrm's device counters): pixels, hits, primary
 * steps, shadow steps, normal evals, Mandelbulb bodies, bailouts, 0. */
int om_render_trace(const uint8_t* params96, uint32_t width, uint32_t height, uint32_t max_steps,
                    uint32_t flags, int mode, const uint32_t* rows, uint32_t nrows, int threads,
                    uint8_t* out_rgba, uint64_t* counters, float* out_linear, uint32_t* out_info,
                    float* out_trace) {
  if (!params96 || !out_rgba || width == 0 || height == 0 || threads < 1) return 1;
  for (uint32_t i = 0; rows && i < nrows; ++i)
    if (rows[i] >= height) return 1;
  pthread_once(&g_srgb_once, srgb_init);
  om_frame F;
  frame_from_params(&F, params96, width, height, max_steps, flags, mode);
  job J;
  memset(&J, 0, sizeof(J));
  J.F = &F;
  J.rows = rows;
  J.nrows = nrows;
  J.rgba = out_rgba;
  J.linear = out_linear;
  J.info = out_info;
  J.trace = out_trace;
  pthread_mutex_init(&J.mu, NULL);
  pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!tid) return 2;
  char* live = (char*)calloc((size_t)threads, 1);
  for (int t = 1; t < threads; ++t) live[t] = pthread_create(&tid[t], NULL, worker, &J) == 0;
  worker(&J); /* the calling thread works too */
  for (int t = 1; t < threads; ++t)
    if (live[t]) pthread_join(tid[t], NULL);
  free(live);
  free(tid);
  pthread_mutex_destroy(&J.mu);
  if (counters) {
    counters[0] = J.total.pixels;
    counters[1] = J.total.hits;
    counters[2] = J.total.primary;
    counters[3] = J.total.shadow;
    counters[4] = J.total.normal;
    counters[5] = J.total.bodies;
    counters[6] = J.total.bailouts;
    counters[7] = 0;
  }
  return 0;
}

int om_render(const uint8_t* params96, uint32_t width, uint32_t height, uint32_t max_steps, uint32_t flags,
              int mode, const uint32_t* rows, uint32_t nrows, int threads, uint8_t* out_rgba,
              uint64_t* counters, float* out_linear, uint32_t* out_info) {
  return om_render_trace(params96, width, height, max_steps, flags, mode, rows, nrows, threads, out_rgba, counters,
                         out_linear, out_info, NULL);
}

/* Re-shade n pixels (x, y interleaved in xy) from traces (OM_TRACE_FLOATS each, as
 * om_render_trace writes them) with the shading of `mode`, and encode them: the colour the
 * pixel would have with those geometric inputs. */
int om_shade_trace(const uint8_t* params96, uint32_t width, uint32_t height, uint32_t max_steps, uint32_t flags,
                   int mode, const uint32_t* xy, uint32_t n, const float* trace, uint8_t* out_rgba) {
  if (!params96 || !xy || !trace || !out_rgba || width == 0 || height == 0) return 1;
  pthread_once(&g_srgb_once, srgb_init);
  om_frame F;
  frame_from_params(&F, params96, width, height, max_steps, flags, mode);
  for (uint32_t i = 0; i < n; ++i) {
    const float* t = trace + (size_t)OM_TRACE_FLOATS * i;
    if (xy[2 * i] >= width || xy[2 * i + 1] >= height) return 1;
    vec3 c = V(0.0f, 0.0f, 0.0f);
    if (t[0] != 0.0f)
      c = shade_hit(&F, camera_dir(&F, xy[2 * i], xy[2 * i + 1]), V(t[7], t[8], t[9]), (uint32_t)t[1],
                    V(t[2], t[3], t[4]), t[5] != 0.0f ? 0.0f : -INF_1E20, t[6]);
    uint8_t* px = out_rgba + 4 * (size_t)i;
    px[0] = encode(c.x);
    px[1] = encode(c.y);
    px[2] = encode(c.z);
    px[3] = 255;
  }
  return 0;
}

/* scene() at n points (xyz interleaved): distance, colour, Mandelbulb counts. */
int om_scene_de(const uint8_t* params96, uint32_t flags, int mode, const float* pts, uint32_t n, float* out_d,
                float* out_color, uint64_t* out_counts) {
  om_frame F;
  frame_from_params(&F, params96, 1, 1, 0, flags, mode);
  om_counts C;
  memset(&C, 0, sizeof(C));
  for (uint32_t i = 0; i < n; ++i) {
    vec3 col;
    out_d[i] = scene(&F, V(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), &col, &C);
    if (out_color) {
      out_color[3 * i] = col.x;
      out_color[3 * i + 1] = col.y;
      out_color[3 * i + 2] = col.z;
    }
  }
  if (out_counts) {
    out_counts[0] = C.bodies;
    out_counts[1] = C.bailouts;
  }
  return 0;
}

/* Builtins on arrays: fn 0 sin, 1 cos, 2 acos, 3 atan2(a,b), 4 log, 5 log2, 6 exp2,
 * 7 pow(a,b), 8 sqrt, 9 div(a,b). */
int om_math(int fn, int mode, const float* a, const float* b, uint32_t n, float* out) {
  for (uint32_t i = 0; i < n; ++i) {
    float s, c, x = a[i], y = b ? b[i] : 0.0f;
    switch (fn) {
      case 0: b_sincos(mode, x, &s, &c); out[i] = s; break;
      case 1: b_sincos(mode, x, &s, &c); out[i] = c; break;
      case 2: out[i] = b_acos(mode, x); break;
      case 3: out[i] = b_atan2(mode, x, y); break;
      case 4: out[i] = b_log(mode, x); break;
      case 5: out[i] = b_log2(mode, x); break;
      case 6: out[i] = b_exp2(mode, x); break;
      case 7: out[i] = b_pow(mode, x, y); break;
      case 8: out[i] = sqrtf(x); break;
      case 9: out[i] = x / y; break;
      default: return 1;
    }
  }
  return 0;
}

void om_srgb_thresholds(float* out256) {
  pthread_once(&g_srgb_once, srgb_init);
  memcpy(out256, g_srgb_t, sizeof(g_srgb_t));
}

int om_encode_srgb(const float* c, uint32_t n, uint8_t* out) {
  pthread_once(&g_srgb_once, srgb_init);
  for (uint32_t i = 0; i < n; ++i) out[i] = encode(c[i]);
  return 0;
}

/* Per-frame uniforms the oracle derived (for host-logic tests): family, Mandelbulb power,
 * Menger cross/scale, Koch normal_z, camera origin. */
int om_frame_info(const uint8_t* params96, uint32_t flags, int mode, float* out8) {
  om_frame F;
  frame_from_params(&F, params96, 1, 1, 0, flags, mode);
  out8[0] = (float)F.family;
  out8[1] = F.mb_power;
  out8[2] = F.menger_cross;
  out8[3] = F.menger_scale;
  out8[4] = F.koch_normal_z;
  out8[5] = F.origin.x;
  out8[6] = F.origin.y;
  out8[7] = F.origin.z;
  return 0;
}

/* ---- presentation resample: blit.wgsl:6-11 through the sampler of
 * persistent_graphics.rs:55-64 (clamp to edge, linear magnification, nearest
 * minification), texels of the Rgba8UnormSrgb render texture (blit_graphics.rs:14) read as
 * linear light. Restated independently of the kernel: the decode table is the closed-form
 * inverse transfer function in long double, rounded once to f32. flags: 1 = encode the
 * output as sRGB (an ...Srgb surface), else linear unorm; 2 = B,G,R,A byte order. */
static float g_srgb_dec[256];
static pthread_once_t g_dec_once = PTHREAD_ONCE_INIT;
static void dec_init(void) {
  for (int k = 0; k < 256; ++k) {
    long double s = (long double)k / 255.0L;
    long double lin = s <= 0.04045L ? s / 12.92L : powl((s + 0.055L) / 1.055L, 2.4L);
    g_srgb_dec[k] = (float)lin;
  }
}
static float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
static uint8_t out_channel(float c, uint32_t flags) {
  if (flags & 1u) return encode(c);
  return (uint8_t)rintf(fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f);
}
static uint32_t clampi(int v, uint32_t n) { return v < 0 ? 0u : ((uint32_t)v >= n ? n - 1u : (uint32_t)v); }

void om_srgb_decode(float* out256) {
  pthread_once(&g_dec_once, dec_init);
  memcpy(out256, g_srgb_dec, sizeof(g_srgb_dec));
}

int om_blit(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh,
            uint32_t flags) {
  if (!src || !dst || !sw || !sh || !dw || !dh) return 1;
  pthread_once(&g_srgb_once, srgb_init);
  pthread_once(&g_dec_once, dec_init);
  const int magnify = (float)sw / (float)dw <= 1.0f && (float)sh / (float)dh <= 1.0f;
  for (uint32_t y = 0; y < dh; ++y)
    for (uint32_t x = 0; x < dw; ++x) {
      /* vertex.wgsl's varyings at the pixel centre, then blit.wgsl:8-9 */
      const float sx = (float)(2u * x + 1u) / (float)dw - 1.0f;
      const float sy = 1.0f - (float)(2u * y + 1u) / (float)dh;
      const float u = (sx + 1.0f) * 0.5f, v = 1.0f - (sy + 1.0f) * 0.5f;
      float ch[3];
      if (magnify) {
        const float tu = u * (float)sw - 0.5f, tv = v * (float)sh - 0.5f;
        const float fu = floorf(tu), fv = floorf(tv), a = tu - fu, c = tv - fv;
        const uint32_t x0 = clampi((int)fu, sw), x1 = clampi((int)fu + 1, sw);
        const uint32_t y0 = clampi((int)fv, sh), y1 = clampi((int)fv + 1, sh);
        for (int k = 0; k < 3; ++k) {
          const float t00 = g_srgb_dec[src[4 * ((size_t)y0 * sw + x0) + k]];
          const float t10 = g_srgb_dec[src[4 * ((size_t)y0 * sw + x1) + k]];
          const float t01 = g_srgb_dec[src[4 * ((size_t)y1 * sw + x0) + k]];
          const float t11 = g_srgb_dec[src[4 * ((size_t)y1 * sw + x1) + k]];
          ch[k] = mixf(mixf(t00, t10, a), mixf(t01, t11, a), c);
        }
      } else {
        const uint32_t ix = clampi((int)floorf(u * (float)sw), sw), iy = clampi((int)floorf(v * (float)sh), sh);
        for (int k = 0; k < 3; ++k) ch[k] = g_srgb_dec[src[4 * ((size_t)iy * sw + ix) + k]];
      }
      uint8_t* o = dst + 4 * ((size_t)y * dw + x);
      const uint8_t r = out_channel(ch[0], flags), g = out_channel(ch[1], flags), b = out_channel(ch[2], flags);
      o[0] = (flags & 2u) ? b : r;
      o[1] = g;
      o[2] = (flags & 2u) ? r : b;
      o[3] = 255;
    }
  return 0;
}
