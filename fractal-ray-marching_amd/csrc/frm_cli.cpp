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
//              [--lock-yaw 0..4] [--lock-pitch] [--time-factor X] [--gpus N] [--batch B]
// With --batch B (one context) the fly-through's frames are rendered B per launch
// (frm_render_bands_batch: one work queue for B frames whose camera and, for the Mandelbulb,
// time differ), so a launch's tail is paid once per B frames; the frames' bytes are the same.
// With --gpus N every frame is row-tiled across devices 0..N-1 from this one process: the CLI
// creates a group context (frm_config.device_count = N, include/frm.h), in which device r renders
// the interleaved bands r, r+N, ..., RCCL point-to-point transfers gather the bands on device 0
// over xGMI and device 0 reassembles the frame. Everything else is the one-GPU
// loop: frm_render + frm_read_frame, the config alone selects the GPUs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "frm.h"

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    fprintf(stderr, "frm_render: %s failed: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}

static int check(int rc, frm_ctx* ctx, const char* what) {
  if (rc != FRM_OK) {
    fprintf(stderr, "frm_render: %s failed (%d): %s\n", what, rc, frm_last_error(ctx));
    exit(1);
  }
  return rc;
}

static int write_ppm(const char* out, uint32_t fr, const uint8_t* rgba, uint32_t width, uint32_t height,
                     char* name, size_t name_len) {
  if (strchr(out, '%')) snprintf(name, name_len, out, fr);
  else snprintf(name, name_len, "%s", out);
  FILE* f = fopen(name, "wb");
  if (!f) {
    perror(name);
    return 1;
  }
  fprintf(f, "P6\n%u %u\n255\n", width, height);
  for (size_t i = 0; i < (size_t)width * height; ++i) fwrite(&rgba[4 * i], 1, 3, f);
  fclose(f);
  return 0;
}

// --batch: the fly-through's Parameters first (the same update order as the per-frame loop),
// then B frames per frm_render_bands_batch launch into a device buffer, each written as a PPM.
// kernel_ms is the launch's wall time (frm_synchronize) over its frames; the work counters are
// the launch's, reported per launch.
static int render_batched(frm_ctx* ctx, frm_parameters p, frm_camera cam, frm_timing timing, uint32_t keys,
                          float dt, uint32_t frames, uint32_t batch, uint32_t width, uint32_t height,
                          const char* out) {
  std::vector<frm_parameters> ps(frames);
  std::vector<frm_camera> cams(frames);
  for (uint32_t fr = 0; fr < frames; ++fr) {
    if (fr > 0) {
      const float delta = frm_timing_update(&timing, &p, dt);
      frm_camera_update(&cam, keys, delta);
      frm_parameters_update_camera_from(&p, &cam);
    }
    ps[fr] = p;
    cams[fr] = cam;
  }
  const size_t fb = (size_t)width * height * 4;
  uint8_t* dev = nullptr;
  uint64_t* dcnt = nullptr;
  hip_check(hipMalloc(&dev, fb * batch), "hipMalloc");
  hip_check(hipMalloc(&dcnt, FRM_NUM_COUNTERS * sizeof(uint64_t)), "hipMalloc");
  std::vector<uint8_t> host(fb * batch);
  char name[4096];
  for (uint32_t g = 0; g < frames; g += batch) {
    const uint32_t n = frames - g < batch ? frames - g : batch;
    hip_check(hipMemset(dcnt, 0, FRM_NUM_COUNTERS * sizeof(uint64_t)), "hipMemset");
    const auto t0 = std::chrono::steady_clock::now();
    check(frm_render_bands_batch(ctx, n, &ps[g], dev, fb * n, fb, height, 0, 1, nullptr, dcnt), ctx,
          "frm_render_bands_batch");
    check(frm_synchronize(ctx), ctx, "frm_synchronize");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t c[FRM_NUM_COUNTERS];
    hip_check(hipMemcpy(c, dcnt, sizeof(c), hipMemcpyDeviceToHost), "hipMemcpy");
    hip_check(hipMemcpy(host.data(), dev, fb * n, hipMemcpyDeviceToHost), "hipMemcpy");
    for (uint32_t b = 0; b < n; ++b) {
      const uint32_t fr = g + b;
      if (write_ppm(out, fr, &host[fb * b], width, height, name, sizeof(name))) return 1;
      printf("{\"frame\": %u, \"out\": \"%s\", \"width\": %u, \"height\": %u, \"time\": %.6f, "
             "\"pos\": [%.5f, %.5f, %.5f], \"yaw\": %.5f, \"pitch\": %.5f, \"kernel_ms\": %.3f, "
             "\"batch\": %u, \"launch_march_steps\": %llu, \"launch_hit_pixels\": %llu, \"gsteps_per_s\": %.3f}\n",
             fr, name, width, height, ps[fr].time, cams[fr].position[0], cams[fr].position[1], cams[fr].position[2],
             cams[fr].yaw, cams[fr].pitch, ms / n, n, (unsigned long long)(c[2] + c[3]), (unsigned long long)c[1],
             (double)(c[2] + c[3]) / (ms * 1e-3) / 1e9);
    }
  }
  (void)hipFree(dev);
  (void)hipFree(dcnt);
  frm_destroy(ctx);
  return 0;
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
  uint32_t gpus = 0;  // 0: one GPU (--device); >= 1: a group context over devices 0..gpus-1
  uint32_t batch = 1;  // frames per launch (one context)
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
    else if (!strcmp(a, "--gpus")) gpus = (uint32_t)atoi(next());
    else if (!strcmp(a, "--batch")) batch = (uint32_t)atoi(next());
    else { fprintf(stderr, "unknown argument %s\n", a); return 2; }
  }
  frm_ctx* ctx = nullptr;
  frm_config cfg = {device, max_steps, flags, 0, 0, {0}};
  if (gpus > 0) {
    int count = 0;
    hip_check(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if ((int)gpus > count || gpus > FRM_MAX_DEVICES) {
      fprintf(stderr, "frm_render: --gpus %u but %d devices (at most %u)\n", gpus, count, FRM_MAX_DEVICES);
      return 2;
    }
    cfg.device_count = gpus;  // a group context: devices 0..gpus-1
    for (uint32_t r = 0; r < gpus; ++r) cfg.devices[r] = (int32_t)r;
  }
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
  if (batch < 1 || batch > FRM_MAX_BATCH) {
    fprintf(stderr, "frm_render: --batch %u outside [1, %u]\n", batch, FRM_MAX_BATCH);
    return 2;
  }
  if (batch > 1 && gpus > 0) {
    fprintf(stderr, "frm_render: --batch renders on one GPU (frm_render_bands_batch is a per-device entry point)\n");
    return 2;
  }
  if (batch > 1) return render_batched(ctx, p, cam, timing, keys, dt, frames, batch, width, height, out);
  for (uint32_t fr = 0; fr < frames; ++fr) {
    if (fr > 0) {  // initialized_app.rs:43-48, with a fixed frame time
      const float delta = frm_timing_update(&timing, &p, dt);
      frm_camera_update(&cam, keys, delta);
      frm_parameters_update_camera_from(&p, &cam);
    }
    frm_stats st;
    memset(&st, 0, sizeof(st));
    check(frm_set_parameters(ctx, &p), ctx, "frm_set_parameters");
    check(frm_render(ctx, &st), ctx, "frm_render");  // a group: render, gather and reassembly
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
