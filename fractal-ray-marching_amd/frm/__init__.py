"""frm — MI355X-native offscreen fractal ray-marcher (host-side package).

Mirrors the reference's host interface (src/parameters.rs, src/camera.rs,
src/graphics.rs) over the C ABI of include/frm.h (libfrm.so, HIP kernels for gfx950).
"""
from ._lib import (FRM_DEFAULT_MAX_STEPS, FRM_FLAG_PERSISTENT_KERNEL, FRM_FLAG_SCENE_SPHERE, FRM_FLAG_SIMPLE_KERNEL,
                   FRM_FLAG_HW_MATH, FRM_FLAG_UNBOUNDED_ITERATIONS,
                   FRM_MAX_BATCH, FRM_MAX_FRAMES_IN_FLIGHT, FRM_MAX_NUM_ITERATIONS, FRM_NUM_COUNTERS, FRM_NUM_SCENES, FrmError, LIB_PATH,
                   load)
from .parameters import Camera, HeldKeys, Parameters, Timing
from .renderer import Renderer, device_count
from .workloads import FRAME_SECONDS, POSES, POWER8_TIME, WORKLOADS, Workload, frame_sequence, make_parameters

__all__ = [
    "Camera", "HeldKeys", "Parameters", "Renderer", "Timing", "FrmError", "device_count", "load", "LIB_PATH",
    "FRAME_SECONDS", "POSES", "POWER8_TIME", "WORKLOADS", "Workload", "frame_sequence", "make_parameters",
    "FRM_DEFAULT_MAX_STEPS", "FRM_FLAG_PERSISTENT_KERNEL", "FRM_FLAG_SCENE_SPHERE", "FRM_FLAG_SIMPLE_KERNEL",
    "FRM_FLAG_UNBOUNDED_ITERATIONS", "FRM_FLAG_HW_MATH",
    "FRM_MAX_BATCH", "FRM_MAX_FRAMES_IN_FLIGHT", "FRM_MAX_NUM_ITERATIONS", "FRM_NUM_COUNTERS", "FRM_NUM_SCENES",
]
