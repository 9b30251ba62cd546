"""Whole-frame golden hashes at BASELINE.json's full sizes (run from the repo root:
`nice python tests/golden/make_fullsize_golden.py [NAME ...]`; C5 takes hours of CPU).

The CPU oracle (oracle/frm_oracle.c, MODE_FRM) renders every pixel of each frame once, in
this container; the sha256 of the RGBA8 bytes and the 8 work counters are written to
tests/golden/fullsize.json together with the exact 96-byte Parameters of the frame, so the
GPU tests (tests/test_gpu_fullsize.py) and bench.py's frame check compare whole frames
without re-running the oracle on the box. Cases: the headline, C2 and C3 at pose P1, C4 at
P1 and C5 at P1 at its first two animation times (time and time + 1/60, as bench.py's
Timing::update advances it); the headline, C2, C3 and C4 at poses P0 and P2; frames 1 and 2 of
the headline fly-through (HEADLINE_FLY: time += 1/60 and a yaw-locked orbit per frame,
frm.frame_sequence; its frame 0 is HEADLINE_P1). The file is rewritten after each case, so an
interrupted run keeps what it finished."""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")):
    sys.path.insert(0, p)

import frm  # noqa: E402
from oracle import frm_oracle as fo  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize.json")


def cases():
    """(key, workload name, pose, Parameters) in the order they are rendered."""
    for name in ("HEADLINE", "C2", "C3", "C4"):
        w = frm.WORKLOADS[name]
        yield f"{name}_P1", name, "P1", frm.make_parameters(w, pose="P1")
    w = frm.WORKLOADS["C5"]
    p = frm.make_parameters(w, pose="P1")
    yield "C5_P1_t0", "C5", "P1", p
    p1 = frm.make_parameters(w, pose="P1")
    frm.Timing().update(p1, 1.0 / 60.0)  # the second frame bench.py renders
    yield "C5_P1_t1", "C5", "P1", p1
    for name in ("HEADLINE", "C2", "C3", "C4"):
        for pose in ("P0", "P2"):
            yield f"{name}_{pose}", name, pose, frm.make_parameters(frm.WORKLOADS[name], pose=pose)
    seq = frm.frame_sequence(frm.WORKLOADS["HEADLINE_FLY"], pose="P1")
    next(seq)  # frame 0 = HEADLINE_P1
    for k in (1, 2):
        yield f"HEADLINE_FLY_P1_f{k}", "HEADLINE_FLY", "P1", next(seq)


def main(only):
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    threads = os.cpu_count() or 1
    for key, name, pose, p in cases():
        if (only and key not in only and name not in only) or key in out:
            continue
        w = frm.WORKLOADS[name]
        flags = frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0
        t0 = time.time()
        r = fo.render(p, w.width, w.height, w.max_steps, flags=flags, threads=threads)
        out[key] = {
            "workload": name, "width": w.width, "height": w.height, "max_steps": w.max_steps,
            "flags": flags, "pose": pose, "time": float(np.float32(p.time)),
            "params": p.to_bytes().hex(),
            "sha256": hashlib.sha256(r["rgba"].tobytes()).hexdigest(),
            "counters": [int(c) for c in r["counters"]],
            "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": threads,
        }
        del r
        with open(OUT + ".tmp", "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
        os.replace(OUT + ".tmp", OUT)
        print(key, out[key]["sha256"], out[key]["oracle_seconds"], "s", flush=True)


if __name__ == "__main__":
    main(set(sys.argv[1:]))
