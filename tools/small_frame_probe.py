#!/usr/bin/env python3
"""Round 6: where a small frame's drop-in loop spends its time. The loop of
bench.py's dropin (frames in flight 2, frm_render, frm_read_frame_async, frm_frame_pixels of the
previous frame) on a BASELINE config, timing each call's host wall separately (median over the
frames, us), beside the loop's ms/frame and the render-and-wait loop's.
    python tools/small_frame_probe.py [--workload C1] [--frames 200]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2] * 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C1")
    ap.add_argument("--frames", type=int, default=200)
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    import torch  # noqa: F401
    import frm

    w = frm.WORKLOADS[args.workload]
    p = next(frm.frame_sequence(w, pose="P1"))
    flags = frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0
    out = {"workload": args.workload, "size": [w.width, w.height]}
    for fif, lag in ((2, 1), (1, 0)):
        with frm.Renderer(max_steps=w.max_steps, flags=flags, frames_in_flight=fif) as r:
            r.resize(w.width, w.height)
            r.update_parameters_buffer(p)
            for _ in range(10):
                r.render(stats=False)
                r.frame_pixels(r.read_frame_async(), copy=False)
            t_render, t_async, t_pixels, held = [], [], [], []
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                a = time.perf_counter()
                r.update_parameters_buffer(p)
                r.render(stats=False)
                b = time.perf_counter()
                held.append(r.read_frame_async())
                c = time.perf_counter()
                if len(held) > lag:
                    r.frame_pixels(held.pop(0), copy=False)
                d = time.perf_counter()
                t_render.append(b - a)
                t_async.append(c - b)
                t_pixels.append(d - c)
            for t in held:
                r.frame_pixels(t, copy=False)
            ms = (time.perf_counter() - t0) / args.frames * 1e3
        key = "dropin" if lag else "dropin_sync"
        out[key] = {"ms_per_frame": round(ms, 4), "render_us": med(t_render), "read_async_us": med(t_async),
                    "frame_pixels_us": med(t_pixels)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
