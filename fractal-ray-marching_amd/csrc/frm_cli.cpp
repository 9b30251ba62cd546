// frm_render — offscreen CLI over libfrm: renders frames of a
// reference scene and writes binary PPMs (P6, sRGB bytes), replacing the reference's
// `present` (graphics.rs:101-108) for offline use. With --frames F > 1 it is a scripted
// fly-through: each frame runs the reference's update order (initialized_app.rs:43-48)
// through libfrm's restatement of Timing and Camera (frm_timing_*, frm_camera_*):
// time += time_factor * dt; camera.update(held keys, dt); parameters.update_camera.
//   frm_render [--width W] [--height H] [--scene S] [--iters N] [--time T]
//              [--max-steps M] [--pos X Y Z] [--yaw A] [--pitch B] [--device D]
//              [--simple] [--sphere] [--out file.ppm | pattern_%04d.ppm]
//              [--frames F] [--dt S] [--keys BITS] [--orbit RAD_PER_S]
//              [--lock-yaw 0..4] [--lock-pitch] [--time-factor X]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "frm.h"

static int check(int rc, frm_ctx* ctx, const char* what) {
  if (rc != FRM_OK) {
    fprintf(stderr, "frm_render: %s failed (%d): %s\n", what, rc, frm_last_error(ctx));
    exit(1);
  }
  return rc;
}

int main(int argc, char** argv) {
  uint32_t width = 1920, height = 1080, scene = 18, iters = 12, max_steps = 256;
  float time = 3.2175055f, pos[3] = {0.0f, 0.0f, -1.6f}, yaw = 0.0f, pitch = 0.0f;
  int device = 0;
  uint32_t flags = 0;
  const char* out = "frame.ppm";
  uint32_t frames = 1, keys = 0;
  float dt = 1.0f / 60.0f, orbit = 0.0f, time_factor = 1.0f;
  int lock_yaw = FRM_LOCK_YAW_NONE, lock_pitch = 0;
  for (int i = 1; i < argc; ++i) {
    const char* a = argv[i];
    auto next = [&](void) -> const char* {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a); exit(2); }
      return argv[++i];
    };
    if (!strcmp(a, "--width")) width = (uint32_t)atoi(next());
    else if (!strcmp(a, "--height")) height = (uint32_t)atoi(next());
    else if (!strcmp(a, "--scene")) scene = (uint32_t)atoi(next());
    else if (!strcmp(a, "--iters")) iters = (uint32_t)atoi(next());
    else if (!strcmp(a, "--time")) time = (float)atof(next());
    else if (!strcmp(a, "--max-steps")) max_steps = (uint32_t)atoi(next());
    else if (!strcmp(a, "--pos")) { pos[0] = (float)atof(next()); pos[1] = (float)atof(next()); pos[2] = (float)atof(next()); }
    else if (!strcmp(a, "--yaw")) yaw = (float)atof(next());
    else if (!strcmp(a, "--pitch")) pitch = (float)atof(next());
    else if (!strcmp(a, "--device")) device = atoi(next());
    else if (!strcmp(a, "--simple")) flags |= FRM_FLAG_SIMPLE_KERNEL;
    else if (!strcmp(a, "--sphere")) flags |= FRM_FLAG_SCENE_SPHERE;
    else if (!strcmp(a, "--out")) out = next();
    else if (!strcmp(a, "--frames")) frames = (uint32_t)atoi(next());
    else if (!strcmp(a, "--dt")) dt = (float)atof(next());
    else if (!strcmp(a, "--keys")) keys = (uint32_t)strtoul(next(), nullptr, 0);
    else if (!strcmp(a, "--orbit")) orbit = (float)atof(next());
    else if (!strcmp(a, "--lock-yaw")) lock_yaw = atoi(next());
    else if (!strcmp(a, "--lock-pitch")) lock_pitch = 1;
    else if (!strcmp(a, "--time-factor")) time_factor = (float)atof(next());
    else { fprintf(stderr, "unknown argument %s\n", a); return 2; }
  }
  frm_config cfg = {device, max_steps, flags, 0};
  frm_ctx* ctx = nullptr;
  check(frm_create(&ctx, &cfg), nullptr, "frm_create");
  frm_parameters p;
  frm_parameters_default(&p);
  frm_parameters_update_aspect(&p, width, height);
  p.time = time;
  p.num_iterations = iters;
  p.scene_index = scene;
  frm_camera cam;
  frm_camera_default(&cam);
  for (int k = 0; k < 3; ++k) cam.position[k] = pos[k];
  cam.yaw = yaw;
  cam.pitch = pitch;
  cam.orbit_angle_per_second = orbit;
  cam.lock_yaw_mode = lock_yaw;
  cam.lock_pitch = lock_pitch;
  frm_timing timing;
  frm_timing_init(&timing);
  timing.time_factor = time_factor;
  frm_parameters_update_camera_from(&p, &cam);
  check(frm_resize(ctx, width, height), ctx, "frm_resize");
  std::vector<uint8_t> rgba((size_t)width * height * 4);
  for (uint32_t fr = 0; fr < frames; ++fr) {
    if (fr > 0) {  // initialized_app.rs:43-48, with a fixed frame time
      const float delta = frm_timing_update(&timing, &p, dt);
      frm_camera_update(&cam, keys, delta);
      frm_parameters_update_camera_from(&p, &cam);
    }
    check(frm_set_parameters(ctx, &p), ctx, "frm_set_parameters");
    frm_stats st;
    check(frm_render(ctx, &st), ctx, "frm_render");
    check(frm_read_frame(ctx, rgba.data(), rgba.size()), ctx, "frm_read_frame");
    char name[4096];
    if (strchr(out, '%')) snprintf(name, sizeof(name), out, fr);
    else snprintf(name, sizeof(name), "%s", out);
    FILE* f = fopen(name, "wb");
    if (!f) { perror(name); return 1; }
    fprintf(f, "P6\n%u %u\n255\n", width, height);
    for (size_t i = 0; i < (size_t)width * height; ++i) fwrite(&rgba[4 * i], 1, 3, f);
    fclose(f);
    printf("{\"frame\": %u, \"out\": \"%s\", \"width\": %u, \"height\": %u, \"time\": %.6f, "
           "\"pos\": [%.5f, %.5f, %.5f], \"yaw\": %.5f, \"pitch\": %.5f, \"kernel_ms\": %.3f, "
           "\"march_steps\": %llu, \"hit_pixels\": %llu, \"gsteps_per_s\": %.3f}\n",
           fr, name, width, height, p.time, cam.position[0], cam.position[1], cam.position[2], cam.yaw,
           cam.pitch, st.kernel_ms, (unsigned long long)st.march_steps, (unsigned long long)st.hit_pixels,
           st.march_steps / (st.kernel_ms * 1e-3) / 1e9);
  }
  frm_destroy(ctx);
  return 0;
}
