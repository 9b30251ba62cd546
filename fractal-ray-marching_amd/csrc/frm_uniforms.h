// frm_uniforms.h — host-side declarations of libfrm that need no HIP headers (the
// uniform precompute of frm_host.cpp and the device counter layout).
#pragma once
#include "frm.h"
#include "frm_scene.h"

namespace frm {


// Indices of the device work counters (FRM_NUM_COUNTERS uint64 words).
enum CounterIndex : uint32_t {
  kCntPixels = 0,
  kCntHits = 1,
  kCntPrimary = 2,
  kCntShadow = 3,
  kCntNormal = 4,
  kCntBodies = 5,
  kCntBailouts = 6,
  kCntReserved = 7,
};

// frm_host.cpp
void compute_scene_uniforms(const frm_parameters& p, uint32_t flags, SceneUniforms* u);
void compute_frame_uniforms(const frm_parameters& p, uint32_t width, uint32_t height,
                            uint32_t max_steps, FrameUniforms* f);
uint64_t wom_ops(const SceneUniforms& u, const uint64_t* counters);

}  // namespace frm
