"""The FRM_HW_MATH measurement build's headline frame (tools/gpu_hw_math.sh ->
gpurun_out/hw/frame_hw_math.npy) against the oracle in both math modes: how far a frame
rendered with gfx950's hardware transcendentals (what a Vulkan driver emits for
fragment.wgsl's builtins) lies from the precise-builtin frame (MODE_LIBM), next to how far the
bit-exact frm frame (MODE_FRM, = the product's bytes) lies from it. Writes
profiles/round2/hw_math/compare.json."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import frm  # noqa: E402
from oracle import frm_oracle  # noqa: E402


def diff(a, b):
    d = np.abs(a[..., :3].astype(np.int16) - b[..., :3].astype(np.int16)).max(-1)
    bg_a, bg_b = np.all(a[..., :3] == 0, -1), np.all(b[..., :3] == 0, -1)
    return {"gt1_frac": float((d > 1).mean()), "any_frac": float((d > 0).mean()), "max_code_diff": int(d.max()),
            "mean_abs_code_diff": float(np.abs(a[..., :3].astype(np.int16) - b[..., :3].astype(np.int16)).mean()),
            "background_flip_frac": float((bg_a != bg_b).mean())}


w = frm.WORKLOADS["HEADLINE"]
p = frm.make_parameters(w, pose="P1")
hw = np.load(os.path.join(ROOT, "gpurun_out", "hw", "frame_hw_math.npy"))
prod = np.load(os.path.join(ROOT, "gpurun_out", "hw", "frame_product.npy"))
libm = frm_oracle.render(p, w.width, w.height, w.max_steps, mode=frm_oracle.MODE_LIBM)
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))["HEADLINE_P1"]
out = {
    "frame": "headline 3840x2160, pose P1, 12 iterations, 256 steps",
    "product_frame_is_oracle_frm": hashlib.sha256(prod.tobytes()).hexdigest() == gold["sha256"],
    "hw_math_vs_libm": diff(hw, libm["rgba"]),
    "frm_vs_libm": diff(prod, libm["rgba"]),
    "hw_math_vs_frm": diff(hw, prod),
}
path = os.path.join(ROOT, "profiles", "round2", "hw_math", "compare.json")
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(out))
