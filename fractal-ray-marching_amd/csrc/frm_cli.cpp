// frm_render — offscreen CLI over libfrm: renders one frame of a
// reference scene for a fixed camera pose and writes a binary PPM (P6, sRGB bytes).
// Replaces the reference's `present` (graphics.rs:101-108) for offline use.
//   frm_render [--width W] [--height H] [--scene S] [--iters N] [--time T]
//              [--max-steps M] [--pos X Y Z] [--yaw A] [--pitch B] [--device D]
//              [--simple] [--sphere] [--out file.ppm]
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
    else { fprintf(stderr, "unknown argument %s\n", a); return 2; }
  }
  frm_config cfg = {device, max_steps, flags, 0};
  frm_ctx* ctx = nullptr;
  check(frm_create(&ctx, &cfg), nullptr, "frm_create");
  frm_parameters p;
  frm_parameters_default(&p);
  frm_parameters_update_aspect(&p, width, height);
  frm_parameters_update_camera(&p, pos, yaw, pitch);
  p.time = time;
  p.num_iterations = iters;
  p.scene_index = scene;
  check(frm_resize(ctx, width, height), ctx, "frm_resize");
  check(frm_set_parameters(ctx, &p), ctx, "frm_set_parameters");
  frm_stats st;
  check(frm_render(ctx, &st), ctx, "frm_render");
  std::vector<uint8_t> rgba((size_t)width * height * 4);
  check(frm_read_frame(ctx, rgba.data(), rgba.size()), ctx, "frm_read_frame");
  FILE* f = fopen(out, "wb");
  if (!f) { perror(out); return 1; }
  fprintf(f, "P6\n%u %u\n255\n", width, height);
  for (size_t i = 0; i < (size_t)width * height; ++i) fwrite(&rgba[4 * i], 1, 3, f);
  fclose(f);
  printf("{\"out\": \"%s\", \"width\": %u, \"height\": %u, \"kernel_ms\": %.3f, \"march_steps\": %llu, "
         "\"hit_pixels\": %llu, \"gsteps_per_s\": %.3f}\n",
         out, width, height, st.kernel_ms, (unsigned long long)st.march_steps,
         (unsigned long long)st.hit_pixels, st.march_steps / (st.kernel_ms * 1e-3) / 1e9);
  frm_destroy(ctx);
  return 0;
}
