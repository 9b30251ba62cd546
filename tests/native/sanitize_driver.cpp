// Sanitizer driver (tests/test_sanitizers.py): exercises the host-side C code under
// AddressSanitizer + UndefinedBehaviorSanitizer (or ThreadSanitizer): libfrm's host mirrors
// of parameters.rs / camera.rs / timing.rs (csrc/frm_host.cpp) and the CPU oracle
// (oracle/frm_oracle.c: the threaded renderer, DE/maths entry points, the blit). Host code
// only: GPU sanitizers are not available for gfx950 here. Exit status 0 = clean.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "frm.h"

extern "C" {
int om_render(const uint8_t* params96, uint32_t width, uint32_t height, uint32_t max_steps, uint32_t flags,
              int mode, const uint32_t* rows, uint32_t nrows, int threads, uint8_t* out_rgba,
              uint64_t* counters, float* out_linear, uint32_t* out_info);
int om_scene_de(const uint8_t* params96, uint32_t flags, int mode, const float* pts, uint32_t n, float* out_d,
                float* out_color, uint64_t* out_counts);
int om_math(int fn, int mode, const float* a, const float* b, uint32_t n, float* out);
int om_blit(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh, uint32_t flags);
}

static int fail(const char* what) {
  fprintf(stderr, "sanitize_driver: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  // host mirrors: a short fly-through with every key, orbit, locks and time control
  frm_parameters p;
  frm_parameters_default(&p);
  frm_camera cam;
  frm_camera_default(&cam);
  frm_timing tim;
  frm_timing_init(&tim);
  for (int i = 0; i < 200; ++i) {
    frm_camera_update(&cam, (uint32_t)(i * 2654435761u) & 0x3FFu, 1.0f / 60.0f);
    if (i % 17 == 0) frm_camera_cycle_lock_yaw_mode(&cam, i % 2);
    if (i % 23 == 0) frm_camera_toggle_lock_pitch(&cam);
    if (i % 7 == 0) frm_camera_rotate_from_cursor(&cam, (float)(i % 13) - 6.0f, (float)(i % 5) - 2.0f);
    frm_camera_update_speed(&cam, (i % 3) - 1.0f);
    frm_camera_update_orbit_speed(&cam, (i % 5) - 2.0f);
    frm_parameters_update_camera_from(&p, &cam);
    frm_timing_update(&tim, &p, 1.0f / 60.0f);
    if (i % 11 == 0) frm_timing_update_time_factor(&tim, 0.5f);
  }
  frm_camera_reset_orbit_speed(&cam);
  frm_timing_stop_time(&tim);
  frm_parameters_update_num_iterations(&p, -100);
  frm_parameters_update_num_iterations(&p, 7);
  frm_parameters_update_scene_index(&p, 40);
  frm_parameters_update_scene_index(&p, -3);
  frm_parameters_update_time(&p, 2.5f);

  // oracle: every scene, iteration counts including the i32 shift wrap, sphere flag, both
  // math modes, a row subset, ragged sizes
  const uint32_t sizes[][2] = {{1, 1}, {33, 17}, {48, 27}};
  for (uint32_t scene = 0; scene < 20; ++scene) {
    for (int32_t iters : {0, 3, 33}) {
      frm_parameters q = p;
      q.scene_index = scene;
      q.num_iterations = (uint32_t)iters;
      for (const auto& wh : sizes) {
        const uint32_t w = wh[0], h = wh[1];
        frm_parameters_update_aspect(&q, w, h);
        const float pos[3] = {0.2f, 0.1f, -2.0f};
        frm_parameters_update_camera(&q, pos, 0.1f, 0.05f);
        std::vector<uint8_t> rgba((size_t)w * h * 4);
        std::vector<float> lin((size_t)w * h * 3);
        std::vector<uint32_t> info((size_t)w * h * 4);
        uint64_t c[8];
        for (int mode = 0; mode < 2; ++mode)
          for (uint32_t flags : {0u, FRM_FLAG_SCENE_SPHERE})
            if (om_render((const uint8_t*)&q, w, h, 64, flags, mode, nullptr, h, threads, rgba.data(), c, lin.data(),
                          info.data()))
              return fail("om_render");
        const uint32_t rows[2] = {0, h - 1};  // the output holds the 2 rendered rows
        std::vector<uint8_t> two_rows((size_t)2 * w * 4);
        if (om_render((const uint8_t*)&q, w, h, 32, 0, 0, rows, 2, threads, two_rows.data(), c, nullptr, nullptr))
          return fail("om_render rows");
      }
    }
  }
  // DE and builtins at points including specials
  std::vector<float> pts = {0, 0, 0, 1e-30f, 0, 0, 1e30f, -1e30f, 0, 0.5f, 0.25f, -0.75f, NAN, 1, 2, INFINITY, 0, 0};
  std::vector<float> d(pts.size() / 3), col(pts.size()), a(64), b(64), out(64);
  uint64_t counts[2];
  for (uint32_t scene = 0; scene < 19; ++scene) {
    frm_parameters q = p;
    q.scene_index = scene;
    q.num_iterations = 5;
    for (int mode = 0; mode < 2; ++mode)
      if (om_scene_de((const uint8_t*)&q, 0, mode, pts.data(), (uint32_t)d.size(), d.data(), col.data(), counts))
        return fail("om_scene_de");
  }
  for (int i = 0; i < 64; ++i) {
    a[i] = (i - 32) * 0.37f;
    b[i] = (i % 7) * 1.3f - 2.0f;
  }
  a[0] = NAN;
  a[1] = INFINITY;
  a[2] = -0.0f;
  for (int fn = 0; fn < 12; ++fn)
    for (int mode = 0; mode < 2; ++mode) om_math(fn, mode, a.data(), b.data(), 64, out.data());
  // blit: up-, down- and mixed scaling, every flag
  std::vector<uint8_t> src(7 * 5 * 4, 128), dst(13 * 3 * 4);
  for (uint32_t flags = 0; flags < 4; ++flags)
    if (om_blit(src.data(), 7, 5, dst.data(), 13, 3, flags)) return fail("om_blit");
  printf("sanitize_driver ok\n");
  return 0;
}
