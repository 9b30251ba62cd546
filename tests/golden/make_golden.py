"""Generate the committed golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

The reference (Rust + WGSL) cannot be built or executed here and ships no fixtures or
golden images, so these vectors are produced by the CPU oracle (oracle/frm_oracle.c,
MODE_FRM) and pin it against regressions; its correctness is established separately by
closed-form known answers (tests/test_oracle_kat.py), the float64-libm cross-check
(tests/test_p1_semantic.py) and the independent host compile of the product source
(tests/test_host_replay.py). Contents:
  frames.json  — sha256 of the RGBA8 bytes + the 8 work counters of 64x36 frames for all
                 19 scenes x num_iterations {0,3,6} x time {0, 3.2175055} (pose P1,
                 128 max steps), plus the Parameters blob of each case;
  frames.npz   — full RGBA8 frames: the headline Mandelbulb at poses P0/P1/P2 (96x54,
                 256 steps) and config C1 (256x256 sphere, 64 steps);
  de.npz       — scene() distance + colour at 1000 seeded points (rng(0), U[-1.5,1.5]^3)
                 for scenes 0, 15, 16, 18 x N {0,3,8,12} at time 3.2175055;
  camera.json  — Parameters blobs (hex) for the poses P0/P1/P2 at 3840x2160.
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "fractal-ray-marching_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import frm  # noqa: E402
from helpers import params_for  # noqa: E402
from oracle import frm_oracle as fo  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
TIMES = (0.0, 3.2175055)
ITERS = (0, 3, 6)


def frame_cases():
    for scene in range(19):
        for n in ITERS:
            for t in TIMES:
                yield scene, n, t


def main():
    frames = []
    for scene, n, t in frame_cases():
        p = params_for(scene, n, t, 64, 36)
        r = fo.render(p, 64, 36, 128)
        frames.append({
            "scene": scene, "iters": n, "time": t, "width": 64, "height": 36, "max_steps": 128,
            "params": p.to_bytes().hex(),
            "sha256": hashlib.sha256(r["rgba"].tobytes()).hexdigest(),
            "counters": [int(c) for c in r["counters"]],
        })
    with open(os.path.join(HERE, "frames.json"), "w") as f:
        json.dump(frames, f, indent=0)

    full = {}
    for pose in ("P0", "P1", "P2"):
        p = params_for(18, 12, frm.POWER8_TIME, 96, 54, pose=pose)
        full[f"mandelbulb_{pose}"] = fo.render(p, 96, 54, 256)["rgba"]
        full[f"mandelbulb_{pose}_params"] = np.frombuffer(p.to_bytes(), np.uint8)
    p = params_for(0, 0, 0.0, 256, 256)
    full["sphere_c1"] = fo.render(p, 256, 256, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)["rgba"]
    full["sphere_c1_params"] = np.frombuffer(p.to_bytes(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **full)

    rng = np.random.default_rng(0)
    pts = rng.uniform(-1.5, 1.5, size=(1000, 3)).astype(np.float32)
    de = {"points": pts}
    for scene in (0, 15, 16, 18):
        for n in (0, 3, 8, 12):
            p = params_for(scene, n, 3.2175055, 64, 36)
            d, col, _ = fo.scene_de(p, pts)
            de[f"s{scene}_n{n}_d"] = d
            de[f"s{scene}_n{n}_c"] = col
    np.savez_compressed(os.path.join(HERE, "de.npz"), **de)

    cams = {}
    for pose in ("P0", "P1", "P2"):
        p = frm.make_parameters(frm.WORKLOADS["HEADLINE"], pose=pose)
        cams[pose] = p.to_bytes().hex()
    with open(os.path.join(HERE, "camera.json"), "w") as f:
        json.dump(cams, f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
