#!/usr/bin/env python3
"""Scheduling history of a moving frame loop ("history across a camera move").

For frames 0..F of a workload's frame sequence (frm.frame_sequence: HEADLINE_FLY = time + orbit,
HEADLINE_TIME = time only, HEADLINE_ORBIT = orbit only) one context (frames_in_flight = 1)
renders every frame twice through frm_render with stats:
  hist  the first render: fetched in the order of the previous frame's cost keys (projected into
        this frame's camera unless FRM_NO_REPROJECT=1), the drop-in loop's situation;
  own   the second render: fetched by this frame's own keys (the fixed-pose situation, the
        lower bound any history can reach).
Prints one JSON line per workload: median kernel ms of each, over frames 2..F.

    python tools/fly_probe.py [--frames 12] [--workloads HEADLINE_FLY,HEADLINE_TIME,HEADLINE_ORBIT]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--workloads", default="HEADLINE_FLY,HEADLINE_TIME,HEADLINE_ORBIT")
    ap.add_argument("--pose", default="P1")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: frm binds torch's)

    import frm

    for name in args.workloads.split(","):
        w = frm.WORKLOADS[name]
        seq = frm.frame_sequence(w, pose=args.pose)
        hist, own = [], []
        with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=1) as r:
            r.resize(w.width, w.height)
            for k in range(args.frames):
                r.update_parameters_buffer(next(seq))
                a = r.render(stats=True)["kernel_ms"]
                b = r.render(stats=True)["kernel_ms"]
                if k >= 2:
                    hist.append(a)
                    own.append(b)
        print(json.dumps({"workload": name, "reproject": os.environ.get("FRM_NO_REPROJECT") != "1",
                          "frames": len(hist), "hist_ms": statistics.median(hist), "own_ms": statistics.median(own),
                          "hist_all": [round(v, 3) for v in hist], "own_all": [round(v, 3) for v in own]}),
              flush=True)


if __name__ == "__main__":
    main()
