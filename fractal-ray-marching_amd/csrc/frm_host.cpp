// frm_host.cpp — host side of libfrm: the Parameters mutators of src/parameters.rs and
// the per-frame uniform precompute (the WGSL `scene()` switch and every
// Parameters-only subexpression of src/fragment.wgsl, hoisted out of the per-pixel path).
#include <math.h>
#include <string.h>

#include "frm.h"
#include "frm_uniforms.h"

using namespace frm;

namespace {

// animate_between(a, b) = a + (b - a) * (0.5 + 0.5 * sin(time * 0.2))   fragment.wgsl:80-82
float animate_between(float time, float a, float b) {
  float w = fma_(0.5f, sin_(time * 0.2f), 0.5f);
  return fma_(b - a, w, a);
}

// plane_normal(a, b, c) = normalize(cross(c - a, b - a))   fragment.wgsl:147-149
v3 plane_normal(v3 a, v3 b, v3 c) { return normalize(cross(c - a, b - a)); }

// tetrahedron(position, a, b, c, d) planes, fragment.wgsl:151-157
void set_tetrahedron(SceneUniforms* u, v3 a, v3 b, v3 c, v3 d) {
  u->tet[0].anchor = a; u->tet[0].normal = plane_normal(a, b, c);
  u->tet[1].anchor = a; u->tet[1].normal = plane_normal(a, c, d);
  u->tet[2].anchor = a; u->tet[2].normal = plane_normal(a, d, b);
  u->tet[3].anchor = b; u->tet[3].normal = plane_normal(b, d, c);
}

void set_menger(SceneUniforms* u, float cross, float factor) {
  u->family = kMenger;
  u->menger_cross = cross;
  u->menger_factor = factor;
  // Reciprocal scales for the GPU's division (-ci) / scale_i (frm_scene.h de_menger). Its domain
  // (div_tame's): scale_i in [1, 2^40], and -ci either +-0 or of magnitude in [2^-60, 2^40]. ci
  // = m - cross with m in [0, 1/2] (a min of maxima of |fract(.) - 1/2|), so |ci| <= 1/2 + cross,
  // and a non-zero difference of two floats of which one is cross >= 2^-34 is at least
  // ulp(cross) / 2 >= 2^-60 when m is within a factor of two of cross (Sterbenz: exact) and
  // larger than cross / 2 otherwise.
  const uint32_t n = u->n;
  bool fast = n <= kMengerFastMax && cross >= 0x1p-34f && cross <= 0x1p39f;
  float scale = 1.0f;
  for (uint32_t i = 0; fast && i < n; ++i) {
    if (!(scale >= 1.0f && scale <= 0x1p40f)) fast = false;
    else u->menger_rcp[i] = (float)(1.0 / (double)scale);
    scale = scale * factor;
  }
  u->menger_fast = fast ? 1u : 0u;
}

// sierpinski_tetrahedron uniforms, fragment.wgsl:165-178
void set_sierpinski(SceneUniforms* u, uint32_t n) {
  u->family = kSierpinski;
  const double height = 4.0 / sqrt(6.0);       // HEIGHT (abstract float)
  const double one_over_sqrt3 = 1.0 / sqrt(3.0);
  // Scalar(1 << num_iterations): i32 shift, amount taken modulo 32.
  float scale = 0.5f / (float)(int32_t)(1u << (n & 31u));
  v3 top = mk(0.0f, (float)(height * 0.5), 0.0f);
  v3 da = mk(-1.0f, (float)(-height), (float)(-one_over_sqrt3));
  v3 db = mk(1.0f, (float)(-height), (float)(-one_over_sqrt3));
  v3 dc = mk(0.0f, (float)(-height), (float)(2.0 * one_over_sqrt3));
  v3 a = fma3(scale, da, top), b = fma3(scale, db, top), c = fma3(scale, dc, top);
  u->sp_top_y = top.y;
  u->sp_yoff = (float)(height * 0.5 * 0.5);
  u->sp_top[0] = a - top; u->sp_top[1] = b - top; u->sp_top[2] = c - top;
  u->sp_normal[0] = normalize(top - a);
  u->sp_normal[1] = normalize(top - b);
  u->sp_normal[2] = normalize(top - c);
  set_tetrahedron(u, top, a, b, c);
}

// koch3D uniforms, fragment.wgsl:214-223 (SIDE_LENGTH is a typed f32 constant)
void set_koch(SceneUniforms* u, uint32_t n, float normal_z) {
  u->family = kKoch;
  const float side = 3.0f, half = side / 2.0f;
  const float side_sqrt = sqrtf(side);
  const float offset = sqrtf(side * side - half * half) - side_sqrt;
  v3 top = mk(0.0f, 1.0f, 0.0f);
  v3 left = mk(-half, 0.0f, -offset), right = mk(half, 0.0f, -offset);
  v3 back = mk(0.0f, 0.0f, side_sqrt);
  u->koch_n1 = normalize(mk(0.0f, 1.0f, normal_z));
  u->koch_n2 = u->koch_n1 * mk(1.0f, -1.0f, 1.0f);
  u->koch_offset = offset;
  float scale = 2.0f;
  // 2 * 1.5^n in f32; once it overflows it stays +inf (the loop need not run to n ~ 2^32)
  for (uint32_t i = 0; i < n && !isinf(scale); ++i) scale = scale * 1.5f;
  u->koch_scale = scale;
  set_tetrahedron(u, top, left, right, back);
}

}  // namespace

namespace frm {

void compute_scene_uniforms(const frm_parameters& p, uint32_t flags, SceneUniforms* u) {
  memset(u, 0, sizeof(*u));
  u->n = p.num_iterations;
  const float t = p.time;
  if (flags & FRM_FLAG_SCENE_SPHERE) {
    u->family = kSphere;
    return;
  }
  switch (p.scene_index) {  // fragment.wgsl:19-77; `case 0, default`
    case 1: set_menger(u, (float)(1.0 / 5.0), 3.0f); break;
    case 2: set_menger(u, (float)(1.0 / 4.0), 3.0f); break;
    case 3: set_menger(u, (float)(1.0 / 3.0), 3.0f); break;
    case 4: set_menger(u, 1.0f / animate_between(t, 2.0f, 8.0f), 3.0f); break;
    case 5: set_menger(u, (float)(1.0 / 6.0), 2.0f); break;
    case 6: set_menger(u, (float)(1.0 / 4.0), 2.0f); break;
    case 7: set_menger(u, (float)(1.0 / 8.0), 2.0f); break;
    case 8: set_menger(u, 1.0f / animate_between(t, 3.0f, 10.0f), 2.0f); break;
    case 9: set_menger(u, (float)(1.0 / 4.0), 4.0f); break;
    case 10: set_menger(u, (float)(1.0 / 5.0), 5.0f); break;
    case 11: set_menger(u, (float)(1.0 / 4.0), 6.0f); break;
    case 12: set_menger(u, (float)(1.0 / 3.0), animate_between(t, 3.0f, 5.0f)); break;
    case 13: set_menger(u, (float)(1.0 / 4.0), animate_between(t, 2.0f, 4.0f)); break;
    case 14: set_menger(u, (float)(1.0 / 6.0), animate_between(t, 1.2f, 3.0f)); break;
    case 15:
      set_sierpinski(u, p.num_iterations);
      // `for (var i = i32(N) - 1; i >= 0; i--)` (fragment.wgsl:181): no fold for N >= 2^31
      if ((int32_t)p.num_iterations < 0) u->n = 0;
      break;
    case 16: set_koch(u, p.num_iterations, (float)sqrt(3.0)); break;
    case 17: set_koch(u, p.num_iterations, animate_between(t, (float)sqrt(3.0), 4.0f)); break;
    case 18:
      u->family = (flags & FRM_FLAG_HW_MATH) ? kMandelbulbHw : kMandelbulb;
      u->mb_power = animate_between(t, 4.0f, 9.0f);
      u->mb_power_m1 = u->mb_power - 1.0f;
      u->mb_bailout = 100.0f;
      break;
    default: set_menger(u, (float)(1.0 / 6.0), 3.0f); break;
  }
}

void compute_frame_uniforms(const frm_parameters& p, uint32_t width, uint32_t height,
                            uint32_t max_steps, FrameUniforms* f) {
  memset(f, 0, sizeof(*f));
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 4; ++i) f->row[j][i] = p.camera_matrix[4 * j + i];
  // transform_position(Position(0)) = (vec4(0,0,0,1) * M).xyz with the dot4 fma chain.
  for (int j = 0; j < 3; ++j) {
    const float* c = &p.camera_matrix[4 * j];
    float v = fma_(1.0f, c[3], fma_(0.0f, c[2], fma_(0.0f, c[1], 0.0f * c[0])));
    if (j == 0) f->origin.x = v;
    if (j == 1) f->origin.y = v;
    if (j == 2) f->origin.z = v;
  }
  f->aspect_x = p.aspect_scale[0];
  f->aspect_y = p.aspect_scale[1];
  f->width = width;
  f->height = height;
  f->max_steps = max_steps;
  f->max_steps_f = (float)max_steps;
}

// Algorithmic VALU lane-op model ("WOM"): ops counted from the
// WGSL source with uniform subexpressions hoisted; transcendentals count 1.
uint64_t wom_ops(const SceneUniforms& u, const uint64_t* c) {
  const uint64_t n = u.n;
  const uint64_t steps = c[kCntPrimary] + c[kCntShadow];
  const uint64_t de_calls = steps + c[kCntNormal];
  uint64_t de_ops = 0;
  switch (u.family) {
    case kMenger: de_ops = de_calls * (14 + 21 * n); break;
    case kSierpinski: de_ops = de_calls * (28 + 30 * n); break;
    case kKoch: de_ops = de_calls * (32 + 18 * n); break;
    case kMandelbulb:
    case kMandelbulbHw: de_ops = c[kCntBodies] * 57 + c[kCntBailouts] * 5 + de_calls * 6; break;
    default: de_ops = de_calls * 5; break;
  }
  // march-step overhead 10 per step; per pixel ray generation 28; per hit the normal
  // overhead 31 plus shading 60.
  return de_ops + steps * 10 + c[kCntPixels] * 28 + c[kCntHits] * 91;
}

}  // namespace frm

// ---- C ABI: Parameters mutators (src/parameters.rs) ------------------------------

extern "C" void frm_parameters_default(frm_parameters* p) {
  if (p) memset(p, 0, sizeof(*p));
}

extern "C" void frm_parameters_update_aspect(frm_parameters* p, uint32_t w, uint32_t h) {
  if (!p) return;
  float m = (float)(w < h ? w : h);  // min(width, height) as f32
  p->aspect_scale[0] = (float)w / m;
  p->aspect_scale[1] = (float)h / m;
}

extern "C" void frm_parameters_update_time(frm_parameters* p, float delta) {
  if (p) p->time += delta;
}

extern "C" void frm_parameters_update_num_iterations(frm_parameters* p, int32_t delta) {
  if (!p) return;  // u32::saturating_add_signed
  int64_t v = (int64_t)p->num_iterations + (int64_t)delta;
  if (v < 0) v = 0;
  if (v > (int64_t)UINT32_MAX) v = UINT32_MAX;
  p->num_iterations = (uint32_t)v;
}

extern "C" void frm_parameters_update_scene_index(frm_parameters* p, int32_t delta) {
  if (!p) return;  // (scene_index as i32 + delta).rem_euclid(19) as u32
  int64_t v = ((int64_t)(int32_t)p->scene_index + (int64_t)delta) % (int64_t)FRM_NUM_SCENES;
  if (v < 0) v += FRM_NUM_SCENES;
  p->scene_index = (uint32_t)v;
}

extern "C" void frm_parameters_update_camera(frm_parameters* p, const float position[3],
                                             float yaw, float pitch) {
  if (!p || !position) return;
  // C = T(position) * Ry(yaw) * Rx(pitch) (cgmath, camera.rs:26-44); every entry is a
  // single product, so evaluation order does not matter. Stored as C^T column-major,
  // i.e. camera_matrix[4*row + col] = C[row][col].
  const float sy = sinf(yaw), cy = cosf(yaw), sx = sinf(pitch), cx = cosf(pitch);
  const float c[4][4] = {
      {cy, sy * sx, sy * cx, position[0]},
      {0.0f, cx, -sx, position[1]},
      {-sy, cy * sx, cy * cx, position[2]},
      {0.0f, 0.0f, 0.0f, 1.0f},
  };
  for (int r = 0; r < 4; ++r)
    for (int k = 0; k < 4; ++k) p->camera_matrix[4 * r + k] = c[r][k];
}

// ---- animation driver: src/camera.rs + src/timing.rs -----------------
// Plain f32 arithmetic in cgmath's operation order (no contraction: -ffp-contract=off),
// f32 libm for sin/cos/atan2/exp like Rust's f32 methods.
namespace {

constexpr float kFullTurn = 6.2831855f;        // Rad::<f32>::full_turn() = f32(2 pi)
constexpr float kMaxPitch = 1.5707964f;        // FRAC_PI_2, camera.rs:156
constexpr float kRotationPerSecond = 0.5f;     // camera.rs:46
constexpr float kRotationPerPixel = 0.0003f;   // camera.rs:149

// utils.rs:62-69
float limited_quadratic_delta(float current, float delta) {
  float factor = current == 0.0f ? 0.025f : fminf(fmaxf(fabsf(current), 0.0001f), 0.1f);
  return 0.2f * delta * factor;
}

// held_keys.rs:32-34: i8 difference of two held flags
float magnitude(uint32_t keys, uint32_t positive, uint32_t negative) {
  return (float)((int)((keys & positive) != 0) - (int)((keys & negative) != 0));
}

void add_pitch(frm_camera* c, float pitch) {  // camera.rs:159-169 (num_traits::clamp)
  float v = c->pitch + pitch;
  c->pitch = v < -kMaxPitch ? -kMaxPitch : (v > kMaxPitch ? kMaxPitch : v);
}

void add_yaw(frm_camera* c, float yaw) {  // camera.rs:163-173: Rad % Rad is f32 fmod
  c->yaw = fmodf(c->yaw + yaw, kFullTurn);
}

}  // namespace

extern "C" void frm_camera_default(frm_camera* c) {
  if (!c) return;
  memset(c, 0, sizeof(*c));
  c->movement_per_second = 1.0f;
  c->position[2] = -1.0f;
  c->lock_yaw_mode = FRM_LOCK_YAW_NONE;
}

extern "C" void frm_camera_update(frm_camera* c, uint32_t keys, float seconds) {
  if (!c) return;
  // do_movement (camera.rs:107-117): forward = yaw_matrix().z, right = yaw_matrix().x
  const float sy = sinf(c->yaw), cy = cosf(c->yaw);
  const float fm = magnitude(keys, FRM_KEY_MOVE_FORWARD, FRM_KEY_MOVE_BACKWARD);
  const float rm = magnitude(keys, FRM_KEY_MOVE_RIGHT, FRM_KEY_MOVE_LEFT);
  const float um = magnitude(keys, FRM_KEY_MOVE_UP, FRM_KEY_MOVE_DOWN);
  const float mv[3] = {(sy * fm + cy * rm) + 0.0f * um, (0.0f * fm + 0.0f * rm) + 1.0f * um,
                       (cy * fm + -sy * rm) + 0.0f * um};
  if (!(mv[0] == 0.0f && mv[1] == 0.0f && mv[2] == 0.0f)) {
    // normalize_to(m) = v * (m / |v|), |v| = sqrt((x*x + y*y) + z*z)
    const float len = sqrtf((mv[0] * mv[0] + mv[1] * mv[1]) + mv[2] * mv[2]);
    const float s = (c->movement_per_second * seconds) / len;
    for (int k = 0; k < 3; ++k) c->position[k] = c->position[k] + mv[k] * s;
  }
  const float rot = kRotationPerSecond * seconds;
  add_pitch(c, rot * magnitude(keys, FRM_KEY_PITCH_DOWN, FRM_KEY_PITCH_UP));
  add_yaw(c, rot * magnitude(keys, FRM_KEY_YAW_RIGHT, FRM_KEY_YAW_LEFT));
  // do_orbit (camera.rs:119-122): Matrix3::from_angle_y(a) * p, rows (c,0,s),(0,1,0),(-s,0,c)
  const float a = c->orbit_angle_per_second * seconds;
  const float so = sinf(a), co = cosf(a);
  const float p0 = c->position[0], p1 = c->position[1], p2 = c->position[2];
  c->position[0] = (co * p0 + 0.0f * p1) + so * p2;
  c->position[1] = (0.0f * p0 + 1.0f * p1) + 0.0f * p2;
  c->position[2] = (-so * p0 + 0.0f * p1) + co * p2;
  // do_lock_rotation (camera.rs:124-147)
  if (c->lock_yaw_mode != FRM_LOCK_YAW_NONE) {
    float offset = 0.0f;
    switch (c->lock_yaw_mode) {
      case FRM_LOCK_YAW_INWARDS: offset = -kFullTurn / 2.0f; break;
      case FRM_LOCK_YAW_RIGHT: offset = -kFullTurn / 4.0f; break;
      case FRM_LOCK_YAW_LEFT: offset = kFullTurn / 4.0f; break;
      default: offset = 0.0f; break;  // Outwards
    }
    c->yaw = atan2f(c->position[0], c->position[2]) + offset;
  }
  if (c->lock_pitch) {
    const float radius = sqrtf(c->position[0] * c->position[0] + c->position[2] * c->position[2]);
    c->pitch = atan2f(c->position[1], radius);
  }
}

extern "C" void frm_camera_update_speed(frm_camera* c, float delta) {
  if (c) c->movement_per_second = c->movement_per_second * expf(delta * 0.1f);
}

extern "C" void frm_camera_update_orbit_speed(frm_camera* c, float delta) {
  if (c) c->orbit_angle_per_second = c->orbit_angle_per_second + limited_quadratic_delta(c->orbit_angle_per_second, delta);
}

extern "C" void frm_camera_reset_orbit_speed(frm_camera* c) {
  if (c) c->orbit_angle_per_second = 0.0f;
}

extern "C" void frm_camera_toggle_lock_pitch(frm_camera* c) {
  if (c) c->lock_pitch = !c->lock_pitch;
}

extern "C" void frm_camera_cycle_lock_yaw_mode(frm_camera* c, int32_t backwards) {
  if (!c) return;
  // None -> Inwards -> Right -> Outwards -> Left -> None (backwards: the reverse)
  const int32_t m = c->lock_yaw_mode < 0 || c->lock_yaw_mode > 4 ? 0 : c->lock_yaw_mode;
  c->lock_yaw_mode = backwards ? (m + 4) % 5 : (m + 1) % 5;
}

extern "C" void frm_camera_rotate_from_cursor(frm_camera* c, float yaw_pixels, float pitch_pixels) {
  if (!c) return;
  add_pitch(c, kRotationPerPixel * pitch_pixels);
  add_yaw(c, kRotationPerPixel * yaw_pixels);
}

extern "C" void frm_parameters_update_camera_from(frm_parameters* p, const frm_camera* c) {
  if (p && c) frm_parameters_update_camera(p, c->position, c->yaw, c->pitch);
}

extern "C" void frm_timing_init(frm_timing* t) {
  if (t) t->time_factor = 1.0f;
}

extern "C" float frm_timing_update(frm_timing* t, frm_parameters* p, float delta_seconds) {
  if (t && p) frm_parameters_update_time(p, t->time_factor * delta_seconds);
  return delta_seconds;
}

extern "C" void frm_timing_update_time_factor(frm_timing* t, float delta) {
  if (t) t->time_factor = t->time_factor + limited_quadratic_delta(t->time_factor, delta);
}

extern "C" void frm_timing_stop_time(frm_timing* t) {
  if (t) t->time_factor = 0.0f;
}
