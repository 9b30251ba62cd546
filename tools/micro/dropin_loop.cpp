// The drop-in binding's frame loop from a C host (no torch in the process, so libfrm runs on
// /opt/rocm's HIP runtime and its readback copies go to a DMA engine): one
// frame per frm_render with frames_in_flight 2, each frame read back asynchronously and the
// previous frame's pixels awaited, as INTEGRATION.md's Rust Graphics does. Parameters follow
// frm.frame_sequence: the 4K headline at pose P1, and for "fly" time += 1/60 plus a yaw-locked
// 0.5 rad/s orbit per frame (timing.rs:23-30, camera.rs:100-147). Prints one JSON line; with
// argv[3] it writes frame 0's RGBA bytes there (checked against the golden hash by the script).
//   dropin_loop fly|fixed [frames] [frame0.rgba]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "frm.h"

#define CK(x) do { int rc_ = (x); if (rc_) { fprintf(stderr, "%s: %d %s\n", #x, rc_, frm_last_error(ctx)); return 1; } } while (0)

int main(int argc, char** argv) {
  const bool fly = argc > 1 && !strcmp(argv[1], "fly");
  const int frames = argc > 2 ? atoi(argv[2]) : 20;
  const char* dump = argc > 3 ? argv[3] : nullptr;
  const uint32_t W = 3840, H = 2160;
  frm_ctx* ctx = nullptr;
  frm_config cfg = {0, 256, 0, 2};
  CK(frm_create(&ctx, &cfg));
  frm_parameters p;
  frm_parameters_default(&p);
  frm_parameters_update_aspect(&p, W, H);
  frm_camera cam;
  frm_camera_default(&cam);
  cam.position[0] = 0.0f, cam.position[1] = 0.0f, cam.position[2] = -1.6f;
  cam.yaw = 0.0f, cam.pitch = 0.0f;
  frm_parameters_update_camera_from(&p, &cam);
  p.time = 3.2175055f;
  p.num_iterations = 12;
  p.scene_index = 18;
  if (fly) {
    cam.orbit_angle_per_second = 0.5f;
    cam.lock_yaw_mode = FRM_LOCK_YAW_INWARDS;
  }
  frm_timing timing;
  frm_timing_init(&timing);
  const float dt = 1.0f / 60.0f;
  std::vector<frm_parameters> seq(frames + 2);
  for (int k = 0; k < frames + 2; ++k) {  // 2 warmup frames render frame 0
    seq[k] = p;
    if (fly && k >= 1) {
      frm_timing_update(&timing, &p, dt);
      frm_camera_update(&cam, 0, dt);
      frm_parameters_update_camera_from(&p, &cam);
    }
  }
  CK(frm_resize(ctx, W, H));
  uint64_t prev = 0;
  const uint8_t* px = nullptr;
  size_t nb = 0;
  for (int k = 0; k < 2; ++k) {  // warmup: scheduling history, streams, pinned images
    CK(frm_set_parameters(ctx, &seq[0]));
    CK(frm_render(ctx, nullptr));
    CK(frm_read_frame_async(ctx, &prev));
    CK(frm_frame_pixels(ctx, prev, &px, &nb));
  }
  prev = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < frames; ++k) {
    CK(frm_set_parameters(ctx, &seq[fly ? k : 0]));
    CK(frm_render(ctx, nullptr));
    uint64_t t = 0;
    CK(frm_read_frame_async(ctx, &t));
    if (prev) {
      CK(frm_frame_pixels(ctx, prev, &px, &nb));
      if (k == 1 && dump) {
        FILE* f = fopen(dump, "wb");
        if (!f || fwrite(px, 1, nb, f) != nb) return 1;
        fclose(f);
      }
    }
    prev = t;
  }
  CK(frm_frame_pixels(ctx, prev, &px, &nb));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"loop\": \"c_host_dropin\", \"workload\": \"%s\", \"frames_in_flight\": 2, \"present_latency_frames\": 1, "
         "\"frames\": %d, \"ms_per_frame\": %.4f}\n", fly ? "HEADLINE_FLY" : "HEADLINE", frames, ms / frames);
  frm_destroy(ctx);
  return 0;
}
