"""Render one frame of a BASELINE workload with the libfrm named by FRM_LIB (default: the
product build), as bench.py renders it (2 frames in flight, the second frame kept), and save
its RGBA8 bytes as .npy. Used for the FRM_HW_MATH measurement build's image comparison."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import numpy as np  # noqa: E402

import frm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="HEADLINE")
ap.add_argument("--pose", default="P1")
ap.add_argument("--out", required=True)
a = ap.parse_args()
w = frm.WORKLOADS[a.workload]
p = frm.make_parameters(w, pose=a.pose)
with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=2) as r:
    r.resize(w.width, w.height)
    r.update_parameters_buffer(p)
    r.render(stats=False)
    st = r.render(stats=True)
    img = r.read_frame()
np.save(a.out, img)
print(a.workload, a.pose, "march steps", st["march_steps"], "hits", st["hit_pixels"], "->", a.out)
