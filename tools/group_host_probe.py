#!/usr/bin/env python3
"""Round 6: the host cost of frm_render on a group context, per frame, for
1/4/8 members (devices [0] * N on the one-GPU box: the copy transport). Each sample starts from an
idle context (frm_synchronize) and times the wall of `--calls` back-to-back frm_render(NULL) calls
whose slots are free (frames_in_flight = calls), so no call waits for the GPU: the time is the
host's enqueue work (per member: device switch, slot stream, scheduling and launch enqueues, event
records; then the gather and the reassembly on device 0). One JSON line per group size.
    python tools/group_host_probe.py [--sizes 1,4,8] [--samples 30] [--calls 3] [--workload HEADLINE]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,4,8")
    ap.add_argument("--samples", type=int, default=30)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--workload", default="HEADLINE")
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    import torch  # noqa: F401  (one HIP runtime, as bench.py)
    import frm

    w = frm.WORKLOADS[args.workload]
    p = next(frm.frame_sequence(w, pose="P1"))
    for n in (int(v) for v in args.sizes.split(",")):
        with frm.Renderer(max_steps=w.max_steps, frames_in_flight=args.calls, devices=[0] * n) as r:
            r.resize(w.width, w.height)
            r.update_parameters_buffer(p)
            for _ in range(2 * args.calls):  # warm: every slot's buffers and streams exist
                r.render(stats=False)
            per_call = []
            for _ in range(args.samples):
                r.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.calls):
                    r.render(stats=False)
                per_call.append((time.perf_counter() - t0) / args.calls * 1e6)
            r.synchronize()
        per_call.sort()
        print(json.dumps({"members": n, "workload": args.workload, "host_us_per_frame_median": round(per_call[len(per_call) // 2], 1),
                          "host_us_per_frame_min": round(per_call[0], 1), "samples": args.samples, "calls": args.calls}))


if __name__ == "__main__":
    main()
