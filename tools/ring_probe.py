#!/usr/bin/env python3
"""Round 6: frame loops through the resident ring (frm_render without stats, frames in flight 2)
against the per-frame grids (FRM_RING=0 in a child process), on the 4K headline or HEADLINE_FLY:
  latency  - render k, read back k asynchronously, present k-1 (bench.py's dropin loop)
  noread   - render every frame, no readback, synchronize at the end
  wait     - render k, read back k, wait for it (render-and-wait through the ring)
One JSON line per (mode, loop) with ms/frame.
    python tools/ring_probe.py [--workload HEADLINE|HEADLINE_FLY] [--frames 30] [--fif 2]"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
    import torch  # noqa: F401  (one HIP runtime, as bench.py)
    import frm

    w = frm.WORKLOADS[args.workload]
    seq = frm.frame_sequence(w, pose="P1")
    frames = [next(seq) for _ in range(args.frames)] if w.moving else [next(seq)] * args.frames
    out = {}
    shas = set()
    with frm.Renderer(max_steps=w.max_steps, frames_in_flight=args.fif) as r:
        r.resize(w.width, w.height)
        r.update_parameters_buffer(frames[0])
        for _ in range(3):
            r.render(stats=False)
            r.frame_pixels(r.read_frame_async(), copy=False)
        for loop in args.loops.split(","):
            r.synchronize()
            t0 = time.perf_counter()
            held = []
            for p in frames:
                r.update_parameters_buffer(p)
                r.render(stats=False)
                if loop == "noread":
                    continue
                held.append(r.read_frame_async())
                lag = 1 if loop == "latency" else 0
                if len(held) > lag:
                    r.frame_pixels(held.pop(0), copy=False)
            for t in held:
                r.frame_pixels(t, copy=False)
            r.synchronize()
            out[loop] = (time.perf_counter() - t0) / len(frames) * 1e3
        if not w.moving:  # untimed: four more frames of the latency loop, each read back and hashed
            held = []
            for p in frames[:4]:
                r.update_parameters_buffer(p)
                r.render(stats=False)
                held.append(r.read_frame_async())
                if len(held) > 1:
                    shas.add(hashlib.sha256(r.frame_pixels(held.pop(0)).tobytes()).hexdigest())
            shas.add(hashlib.sha256(r.frame_pixels(held.pop(0)).tobytes()).hexdigest())
    res = {"mode": os.environ.get("FRM_RING", "1"), "service": os.environ.get("FRM_RING_SERVICE"),
           "workload": args.workload, **{k: round(v, 3) for k, v in out.items()}}
    if shas:  # a fixed workload: every frame read back must be the golden frame
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json"))).get(args.workload + "_P1")
        res["frames_ok"] = g is not None and shas == {g["sha256"]}
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="HEADLINE")
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--fif", type=int, default=2)
    ap.add_argument("--loops", default="latency,noread,wait")
    ap.add_argument("--modes", default="1,0", help="FRM_RING values to run (1: the ring, 0: per-frame grids, the default)")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    env = dict(os.environ)
    env.setdefault("GPU_MAX_HW_QUEUES", "16")
    for ring in args.modes.split(","):
        e = dict(env, FRM_RING=ring)
        p = subprocess.run([sys.executable, __file__, "--child"] + sys.argv[1:], env=e, capture_output=True, text=True,
                           timeout=300)
        sys.stdout.write(p.stdout)
        sys.stdout.write("".join(l + "\n" for l in p.stderr.splitlines() if l.startswith("frm ring")))
        if p.returncode:
            sys.stderr.write(p.stderr[-3000:])
            raise SystemExit(p.returncode)


if __name__ == "__main__":
    main()
