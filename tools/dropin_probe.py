"""Drop-in frame loop probe (bench.py's dropin_loop in isolation, several forms side by side).

Every form renders one frame per frm_render with that frame's Parameters (frm.frame_sequence).
  sync       frames_in_flight 1, readback of every frame, wait for each frame
  latency    frames_in_flight F, frm_read_frame_async per frame, pixels of frame k-F+1 awaited
  noread     frames_in_flight F, no readback, no host wait until the end (frm_synchronize)
Prints one JSON line per form: ms per frame over --frames timed frames (after 2 warmup frames).

    python tools/dropin_probe.py --workload HEADLINE_FLY --frames 20 --forms sync,latency,latency3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fractal-ray-marching_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="HEADLINE_FLY")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--forms", default="sync,latency,latency3,noread")
    ap.add_argument("--hw-queues", type=int, default=0)
    args = ap.parse_args()
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch  # noqa: F401  (libfrm shares torch's HIP runtime)

    import frm

    w = frm.WORKLOADS[args.workload]
    seq = frm.frame_sequence(w, pose="P1")
    n = args.frames
    frames = [next(seq) for _ in range(n)] if w.moving else [next(seq)] * n
    for form in args.forms.split(","):
        fif = {"sync": 1, "latency": 2, "latency3": 3, "noread": 2, "noread3": 3}[form]
        lag = fif - 1
        with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=fif) as r:
            r.resize(w.width, w.height)
            r.update_parameters_buffer(frames[0])
            for _ in range(2):
                r.render(stats=False)
                r.frame_pixels(r.read_frame_async(), copy=False)
            held = []
            t0 = time.perf_counter()
            for k in range(n):
                r.update_parameters_buffer(frames[k])
                r.render(stats=False)
                if form.startswith("noread"):
                    continue  # every frame enqueued at once: the GPU's overlap alone
                held.append(r.read_frame_async())
                if len(held) > lag:
                    r.frame_pixels(held.pop(0), copy=False)
            if form.startswith("noread"):
                r.synchronize()
            else:
                for t in held:
                    r.frame_pixels(t, copy=False)
            dt = time.perf_counter() - t0
        print(json.dumps({"workload": args.workload, "form": form, "frames_in_flight": fif,
                          "ms_per_frame": dt / n * 1e3, "frames": n,
                          "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)


if __name__ == "__main__":
    main()
