"""Frame intervals across resizes in the drop-in loop: one frame per frm_render, 2 in
flight, every frame read back with a frame of presentation latency (frm_read_frame_async), as the
drop-in binding drives it. The render texture steps by the reference's RenderTextureConfig factor
(+-1: 160f x 90f, render_texture_config.rs:7-13; 4K is f = 24) every `--every` frames, between
f = 24 and f = 23 / 25, with the aspect updated as the reference's resize does. The interval of
frame k is the host time between frame k-1's and frame k's pixels becoming available. Prints one
JSON line: the mean frame interval over the loop with its resizes and over the same loop at a fixed
4K size (the control), and the per-frame intervals. Completions come in pairs (two frames in flight
finish close together), so single intervals say little; the mean is the loop's frame rate.
    python tools/resize_loop_probe.py [--workload HEADLINE|HEADLINE_FLY] [--cycles 4] [--every 6]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="HEADLINE")
    ap.add_argument("--cycles", type=int, default=4)
    ap.add_argument("--every", type=int, default=6)
    args = ap.parse_args()
    import torch  # noqa: F401  (libfrm shares torch's HIP runtime)

    import frm

    w = frm.WORKLOADS[args.workload]
    out = {"workload": args.workload, "frames_in_flight": 2, "present_latency_frames": 1, "every": args.every}
    for name, cycle in (("resize", (25, 24, 23, 24)), ("fixed", (24, 24, 24, 24))):
        iv = run(frm, w, args, [24] + [f for _ in range(args.cycles) for f in cycle])
        body = [iv[k] for k in sorted(iv)][args.every - 1:]
        out[f"{name}_mean_ms"] = round(statistics.mean(body), 3)
        out[f"{name}_intervals_ms"] = [round(x, 2) for x in body]
    out["cost_per_resize_ms"] = round((out["resize_mean_ms"] - out["fixed_mean_ms"]) * args.every, 3)
    print(json.dumps(out))


def run(frm, w, args, factors):
    seq = frm.frame_sequence(w, pose="P1")
    frames = []  # (factor, Parameters)
    for f in factors:
        for _ in range(args.every):
            p = next(seq) if w.moving else frm.make_parameters(w, pose="P1")
            p.update_aspect(160 * f, 90 * f)
            frames.append((f, p))
    with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=2) as r:
        r.resize(160 * 24, 90 * 24)
        r.update_parameters_buffer(frames[0][1])
        for _ in range(3):  # history for the first size
            r.render(stats=False)
            r.frame_pixels(r.read_frame_async(), copy=False)
        held, done = [], []
        for k, (f, p) in enumerate(frames):
            if (160 * f, 90 * f) != (r.width, r.height):
                r.resize(160 * f, 90 * f)
            r.update_parameters_buffer(p)
            r.render(stats=False)
            held.append((k, r.read_frame_async()))
            if len(held) > 1:
                j, t = held.pop(0)
                r.frame_pixels(t, copy=False)
                done.append((j, time.perf_counter()))
        for j, t in held:
            r.frame_pixels(t, copy=False)
            done.append((j, time.perf_counter()))
    return {j: (t - done[i - 1][1]) * 1e3 for i, (j, t) in enumerate(done) if i > 0}


if __name__ == "__main__":
    main()
