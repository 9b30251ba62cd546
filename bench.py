#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X fractal ray-marcher.

Workload (BASELINE.json metric): 3840x2160 Mandelbulb (scene 18 at power 8), 12 DE
iterations, 256 march steps, fixed camera pose P1; one "step" = one whole frame of the
hot path (fragment_main for every pixel) with inputs resident on the GPU. Frames are
rendered several per launch (--batch; frm_render_bands_batch; by default on one GPU all timed
frames, up to 32, in one launch): every frame is computed in full, the frames' pixels share one
work queue so a launch's tail is paid once per batch. The moving HEADLINE_FLY batches too (its
frames differ in camera and in the Mandelbulb's time: each lane carries its frame's power).

N GPUs (one process each): launched by torch.distributed.run (the driver's multi-GPU runs),
or, when no launcher set WORLD_SIZE, bench.py starts `torch.distributed.run` itself as a child
process (before anything touches a GPU) and prints rank 0's line:
* --split rows (default): every frame is split into interleaved row bands across the
  ranks, gathered to rank 0 over RCCL (xGMI) and reassembled there (frm_unshuffle_bands):
  strong scaling of the fixed-pose workload, as BASELINE.json's north star describes. A
  rank's share of a frame is short next to the frame's longest pixel (a sequential march),
  so each rank keeps --inflight frames in flight (3 by default when split): frame k+1's
  bands render while frame k's slowest pixels finish and frame k-1 is gathered.
* --split frames: alternate-frame rendering. Frames are independent units, so each rank
  renders whole frames of the same workload, seen from the base pose rotated about +y by
  rank * pi/4 (an orbit fly-through; rank 0 = the base pose). There is no data-path
  collective and per-GPU work is fixed, so scaling is "weak".

Prints ONE JSON line on rank 0. `value` = G ray-march-steps/s of the whole job
(primary + shadow march() iterations, counted exactly by the kernel, / wall time).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload HEADLINE|HEADLINE_FLY|C2|C3|C4|C5]
                    [--pose P0|P1|P2] [--kernel persistent|simple] [--no-cpu-baseline]
"""
import argparse
import hashlib
import math
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "fractal-ray-marching_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# Peak VALU issue of MI355X: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz (f32 lane-ops/s;
# = 157.3 TFLOP/s counting an FMA as 2), /opt/skills/guides/MI355X_MICROARCH.md.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
METRIC = "Gray-march-steps/sec + frames/sec, 4K Mandelbulb 12-iter/256-step, 1 & 8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30,
                    help="timed frames; frames in flight fill and drain inside the timed region, so more "
                    "frames measure the steady state more closely (N=1: 10 -> 40 frames +0.4 %%)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="HEADLINE")
    ap.add_argument("--pose", default="P1")
    ap.add_argument("--kernel", default="auto", choices=["auto", "persistent", "simple"],
                    help="auto: libfrm's choice (simple below one resident persistent grid of pixels)")
    ap.add_argument("--band-rows", type=int, default=0)
    ap.add_argument("--split", default="rows", choices=["frames", "rows"],
                    help="N>1: 'rows' = every frame split into interleaved row bands + RCCL gather to "
                    "rank 0 (strong scaling); 'frames' = alternate-frame rendering, each rank renders "
                    "whole frames of an orbit fly-through (no data-path collective, weak scaling)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="launches in flight per GPU (frm_config.frames_in_flight): launch k+1 renders "
                    "while launch k's longest pixels finish; 0 = measured best (DESIGN.md): with several "
                    "frames per launch 2 for a rank's bands and frames below 4 M pixels, else 1; one frame "
                    "per launch 3 / 2")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (0: raise to 16 if lower). Frames in flight "
                    "overlap only on distinct hardware queues: HIP maps streams onto at most that many "
                    "queues per process (4, HIP's default), shared by the null stream, torch's, libfrm's "
                    "and RCCL's; with 4 the second render stream lands on the timing stream's queue and "
                    "two frames in flight never overlap (DESIGN.md section 5)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch (frm_render_bands_batch: the frames' pixels share one work "
                    "queue, so a launch's tail is paid once per batch); 0 = auto (DESIGN.md section 7); "
                    "animated workloads (a new time every frame) always 1")
    ap.add_argument("--math", default="exact", choices=["exact", "hw"],
                    help="exact: the bit-exact frm builtins (the product default, the headline); hw: "
                    "FRM_FLAG_HW_MATH, the Mandelbulb on hardware transcendentals (opt-in, not bit-exact, "
                    "gated by tests/test_gpu_hw_math.py; a separate line, never the headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in loop measurement (dropin_ms_per_frame)")
    ap.add_argument("--dropin-only", action="store_true",
                    help="internal: only the drop-in loop (2 in flight, a frame of latency), one JSON line; "
                    "bench.py runs it as a child at HIP's default 4 hardware queues (dropin_q4)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--reload", default=None, help="render with kernels recompiled at run time from this "
                    "copy of csrc/ (frm_reload, hiprtc)")
    ap.add_argument("--mode", default="ranks", choices=["ranks", "group"],
                    help="ranks: one process per GPU (torch.distributed.run, the driver's runs); group: ONE "
                    "process drives all --gpus devices through a group context (frm_config.device_count: "
                    "every frm_render row-tiles the frame over the devices, gathers the bands on device 0 "
                    "with RCCL and reassembles it), the path a C or Rust host binding include/frm.h takes "
                    "(INTEGRATION.md section 3); FRM_BENCH_GROUP_DEVICES=0,0,0 lists the devices explicitly "
                    "(a repeated device rehearses ranks on one GPU with device copies)")
    return ap.parse_args()


def cpu_baseline(params, w, seconds):
    """Oracle (C restatement, thread pool with a dynamic row queue) on a bounded, evenly
    spaced row sample of the same frame, sized to about `seconds` of CPU work; steps/s
    extrapolates per march step."""
    from oracle import frm_oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    flags = 1 if w.sphere else 0

    def sample(n, nthreads):
        stride = max(1, w.height // max(1, n))
        rows = list(range(stride // 2, w.height, stride))
        t0 = time.perf_counter()
        r = frm_oracle.render(params, w.width, w.height, w.max_steps, flags=flags, rows=rows, threads=nthreads)
        return rows, stride, r, time.perf_counter() - t0

    def timed(nthreads, target):
        # calibrate with >= 2 rows per thread (fewer rows than threads would time the slowest
        # row, not the pool), then size the sample to the target, twice at most
        n = min(w.height, 2 * nthreads)
        rows, stride, r, dt = sample(n, nthreads)
        for _ in range(2):
            if dt >= 0.6 * target or len(rows) >= w.height:
                break
            n = min(w.height, int(len(rows) * target / max(dt, 1e-3)))
            rows, stride, r, dt = sample(n, nthreads)
        steps = int(r["counters"][2]) + int(r["counters"][3])
        text = (f"{len(rows)} evenly spaced rows (one in {stride}) of the {w.width}x{w.height} frame, "
                f"{steps} march steps in {dt:.2f} s; oracle/frm_oracle.c, gcc -O3 -mfma -ffp-contract=off (oracle/Makefile), {nthreads} thread"
                f"{'s' if nthreads > 1 else ''}")
        return steps / dt / 1e9, text, (len(rows) / w.height) / dt

    value, text, fps = timed(threads, seconds)
    value1, text1, _ = timed(1, seconds / 3)  # also a 1-core timing
    return {
        "value": value,
        "unit": "Gray-march-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": text,
        "frames_per_s_extrapolated": fps,
        "single_core": {"value": value1, "unit": "Gray-march-steps/s", "cores": 1, "sample": text1},
    }


HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def pmc_summary(workload, world, math="exact"):
    """Hardware counters of the render kernels from the committed rocprofv3 --pmc passes of
    this workload (tools/pmc.sh + tools/pmc_summary.py: one counter group per pass; FETCH_SIZE
    doubled and KiB -> B per MI355X_MICROARCH.md): march_persistent (the dominant kernel:
    VALU busy, lane utilisation, HBM bytes) and shade_pass (HBM bytes). N > 1: the summary of
    one rank's share of the row split (pmc_<workload>_share<N>_*.json) when committed.
    PMC collection needs its own profiler passes (they serialise the kernels), so bench.py
    reports the committed measurement and names it, newest round first, and only when the
    summary's recorded source hash equals the hash of the kernel sources being run
    (frm.provenance): counters of an older kernel are reported as stale, never as current.
    --math hw runs another kernel (the FRM_FLAG_HW_MATH instantiation): its counters are keyed
    pmc_<workload>_hw_<...>.json and are null unless such a pass is committed."""
    from frm import provenance

    cur = provenance.source_sha256()
    stale = None
    tag = (workload if world == 1 else f"{workload}_share{world}") + ("_hw" if math == "hw" else "")
    for rnd in sorted((d for d in os.listdir(os.path.join(ROOT, "profiles")) if d.startswith("round")),
                      key=lambda d: int(d[5:]) if d[5:].isdigit() else -1, reverse=True):
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_{tag}_march.json")
        if not os.path.exists(path):
            continue
        with open(path) as fh:
            s = json.load(fh)
        if s.get("source_sha256") != cur:
            stale = stale or os.path.relpath(path, ROOT)
            continue
        B = s.get("frames_per_dispatch", 1)
        march = (s["hbm_read_bytes"] + s["hbm_write_bytes"]) / B
        shade = shade_src = None
        spath = path.replace("_march.json", "_shade.json")
        if os.path.exists(spath):
            with open(spath) as fh:
                sh = json.load(fh)
            if sh.get("source_sha256") == cur:
                shade = (sh["hbm_read_bytes"] + sh["hbm_write_bytes"]) / sh.get("frames_per_dispatch", 1)
                shade_src = os.path.relpath(spath, ROOT)
        # rank_pass (fused scheduling): once per launch, i.e. per B frames of the march's dispatch
        rank = None
        rpath = path.replace("_march.json", "_rank.json")
        if os.path.exists(rpath):
            with open(rpath) as fh:
                rk = json.load(fh)
            if rk.get("source_sha256") == cur and "hbm_read_bytes" in rk:
                rank = (rk["hbm_read_bytes"] + rk["hbm_write_bytes"]) / B
                shade_src = (shade_src + " + " if shade_src else "") + os.path.relpath(rpath, ROOT)
        return {
            # HBM bytes per frame (a dispatch renders B frames): march + shade + rank, and the split
            "traffic": march + (shade or 0.0) + (rank or 0.0),
            "traffic_split": {"march_persistent": march, "shade_pass": shade, "rank_pass": rank},
            "valu_busy": s["valu_busy"],
            "valu_lane_utilization": s["valu_lane_utilization"],
            "hbm_write_gbps": s["hbm_write_gbps"],
            "hbm_write_frac": s["hbm_write_gbps"] / HBM_PEAK_GBPS,
            "source": os.path.relpath(path, ROOT) + (f" + {shade_src}" if shade_src else ""),
            "source_sha256": cur,
        }
    return {"stale": stale, "source_sha256": cur} if stale else None


def dropin_loop(frm, torch, w, args, flags, local, camera, forms=(("dropin", 2, 1), ("dropin_sync", 1, 0))):
    """The drop-in binding's frame loop, measured in the same run: one
    frm_render per frame with that frame's Parameters (frm.frame_sequence, as bench's timed
    region), every frame read back to the host (the reference presents every frame,
    graphics.rs:91-110). Two forms:
    * dropin (the binding): frames_in_flight = 2 and presentation with a frame of latency, as the
      reference's surface has it (wgpu's default desired_maximum_frame_latency = 2,
      persistent_graphics.rs:158-162): render frame k, start its readback
      (frm_read_frame_async), then wait for frame k-1's pixels (frm_frame_pixels);
    * dropin_sync: frames_in_flight = 1 and a wait for every frame before the next.
    Untimed: 2 frames of frame 0. Timed: min(--steps, 30) frames, the bench's own frame count by
    default (the loop's fill and drain weigh 1/n: HEADLINE_FLY 12.2 ms/frame over 20 frames,
    12.04-12.05 over 30, profiles/round4/dropin_sm). The march steps come from a second, untimed
    pass over the same frames with stats."""
    seq = frm.frame_sequence(w, pose=args.pose, camera=camera)
    n = max(1, min(args.steps, 30))
    frames = [next(seq) for _ in range(n)] if w.moving else [next(seq)] * n
    out = {}
    steps = kernel_ms = 0  # the march steps of the frames (the dropin form's stats pass; same frames in both)
    for name, fif, lag in forms:
        with frm.Renderer(device=local, max_steps=w.max_steps, flags=flags, frames_in_flight=fif) as r:
            r.resize(w.width, w.height)
            r.update_parameters_buffer(frames[0])
            for _ in range(2):
                r.render(stats=False)
                r.frame_pixels(r.read_frame_async(), copy=False)
            held = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(n):
                r.update_parameters_buffer(frames[k])
                r.render(stats=False)
                held.append(r.read_frame_async())
                if len(held) > lag:
                    r.frame_pixels(held.pop(0), copy=False)  # present frame k - lag
            for t in held:
                r.frame_pixels(t, copy=False)
            dt = time.perf_counter() - t0
            if name == "dropin" and not args.dropin_only:
                for p in frames:
                    r.update_parameters_buffer(p)
                    st = r.render(stats=True)
                    steps += st["march_steps"]
                    kernel_ms += st["kernel_ms"]
        out[f"{name}_ms_per_frame"] = dt / n * 1e3
        out[name] = {"frames": n, "value": steps / dt / 1e9 if steps else None, "unit": "Gray-march-steps/s",
                     "frames_in_flight": fif, "frames_per_launch": 1, "present_latency_frames": lag,
                     "loop": ("frm_render + frm_read_frame_async per frame, frm_frame_pixels of the previous "
                              "frame (INTEGRATION.md section 3)" if lag else
                              "frm_render + readback per frame, host waits for each frame")}
        if name == "dropin" and steps:
            out[name]["kernel_ms_per_frame_alone"] = kernel_ms / n
    return out


def dropin_q4(args):
    """The drop-in loop at HIP's default GPU_MAX_HW_QUEUES=4 (a host that does not raise it, e.g. a
    Rust binding), in a child process: the queue count is fixed when HIP starts, and this process
    runs at 16. None when the child fails."""
    cmd = [sys.executable, os.path.abspath(__file__), "--dropin-only", "--hw-queues", "4", "--workload", args.workload,
           "--pose", args.pose, "--steps", str(args.steps), "--kernel", args.kernel, "--math", args.math]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        return json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else None
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return None


def dropin_only(args):
    import torch

    import frm

    w = frm.WORKLOADS[args.workload]
    flags = (frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0) | (
        {"auto": 0, "simple": frm.FRM_FLAG_SIMPLE_KERNEL, "persistent": frm.FRM_FLAG_PERSISTENT_KERNEL}[args.kernel]) | (
        frm.FRM_FLAG_HW_MATH if args.math == "hw" else 0)
    torch.cuda.set_device(0)
    out = dropin_loop(frm, torch, w, args, flags, 0, None, forms=(("dropin", 2, 1),))
    print(json.dumps({"dropin_ms_per_frame": out["dropin_ms_per_frame"],
                      "gpu_max_hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])}))


def launch_ranks(args):
    """--gpus N > 1 with no torch.distributed.run environment: run N ranks under a child
    `python -m torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1) and
    forward rank 0's JSON line. This process never initialises HIP, so nothing here execs
    over a GPU context; the child's exit status is ours."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    for ln in p.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if p.returncode != 0 or len(lines) != 1:
        raise SystemExit(f"bench.py: {args.gpus} ranks exited with {p.returncode}, {len(lines)} result lines")
    out = json.loads(lines[0])
    out["launcher"] = "bench.py -> torch.distributed.run (child process)"
    print(json.dumps(out))


GOLDEN = os.path.join(ROOT, "tests", "golden", "fullsize.json")


def motion(w):
    """What changes from frame to frame (frm.frame_sequence)."""
    parts = (["time += 1/60 s per frame (Timing::update)"] if w.animated else []) + (
        ["yaw-locked orbit at 0.5 rad/s (Camera::update)"] if w.fly else [])
    return " + ".join(parts) if parts else "fixed camera pose, fixed time"


def golden_key(workload, pose):
    """The golden frame that equals frame 0 of the timed sequence (frm.frame_sequence): the
    fixed frame itself; C5's first animation time; the fly-through's frame 0 is the headline."""
    if workload == "C5":
        return f"C5_{pose}_t0"
    if workload.startswith("HEADLINE_"):  # HEADLINE_FLY / _TIME / _ORBIT: frame 0 is the headline
        return f"HEADLINE_{pose}"
    return f"{workload}_{pose}"


def frame_check(frame, workload, pose):
    """sha256 of the first timed frame (for N>1: gathered and reassembled; kept by
    RowTiledFrame.run(capture=...)) against the oracle's whole-frame golden hash
    (tests/golden/fullsize.json, generated on the CPU by tests/golden/make_fullsize_golden.py):
    the output does not depend on how the frame was tiled over ranks or scheduled. Timed frame
    0 is frame 0 of the workload's frame sequence (animated workloads too: the warmup renders
    frame 0, the timed region frames 0..K-1). None when no golden frame exists."""
    sha = hashlib.sha256(frame.cpu().numpy().tobytes()).hexdigest()
    key = golden_key(workload, pose)
    gold = None
    if os.path.exists(GOLDEN):
        with open(GOLDEN) as fh:
            gold = json.load(fh).get(key)
    return {"frame_sha256": sha, "frame_sha_ok": None if gold is None else sha == gold["sha256"],
            "frame_golden": None if gold is None else f"tests/golden/fullsize.json[{key}]"}


COUNTER_NAMES = ("pixels", "hit_pixels", "primary_steps", "shadow_steps", "normal_evals", "fractal_bodies",
                 "fractal_bailouts")


def counters_check(counters, workload, pose, frames, golden_path=GOLDEN):
    """The kernel's summed work counters of the timed region against `frames` x the oracle's
    counters of the golden frame (tests/golden/fullsize.json). The roofline's algorithmic ops
    are derived from these counters (fractal bodies and bailouts are data dependent) and the
    frame hash cannot see them, so a wrong count must not reach the line. Applies when every
    timed frame is the golden frame (fixed workloads; all ranks of a row split together);
    returns None when it does not apply, else {"counters_ok": bool, ...}."""
    gold = None
    if os.path.exists(golden_path):
        with open(golden_path) as fh:
            gold = json.load(fh).get(f"{workload}_{pose}")
    if gold is None:
        return None
    want = [frames * int(v) for v in gold["counters"][:len(COUNTER_NAMES)]]
    got = [int(v) for v in counters[:len(COUNTER_NAMES)]]
    bad = {n: {"got": g, "want": e} for n, g, e in zip(COUNTER_NAMES, got, want) if g != e}
    return {"counters_ok": not bad, "counters_golden": f"{frames} x tests/golden/fullsize.json[{workload}_{pose}]",
            **({"counters_mismatch": bad} if bad else {})}


def group_bench(args):
    """--mode group: one process, one group context over --gpus devices (include/frm.h ABI 5). The
    timed region is --steps frm_render calls (frames_in_flight slots rotate; each frame's bands are
    rendered on every device, gathered on device 0 and reassembled there) bracketed by
    frm_synchronize; march steps come from an untimed pass with stats over the same frames."""
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"
    import torch  # noqa: F401  (one HIP runtime: libfrm binds to torch's)
    import frm

    w = frm.WORKLOADS[args.workload]
    env = os.environ.get("FRM_BENCH_GROUP_DEVICES")
    devices = [int(v) for v in env.split(",")] if env else list(range(args.gpus))
    if len(devices) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but FRM_BENCH_GROUP_DEVICES lists {len(devices)} devices")
    inflight = max(1, min(args.inflight or 3, frm.FRM_MAX_FRAMES_IN_FLIGHT))
    flags = (frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0) | (
        {"auto": 0, "simple": frm.FRM_FLAG_SIMPLE_KERNEL, "persistent": frm.FRM_FLAG_PERSISTENT_KERNEL}[args.kernel])
    seq = frm.frame_sequence(w, pose=args.pose)
    frames = [next(seq) for _ in range(args.steps)] if w.moving else [next(seq)] * args.steps
    with frm.Renderer(max_steps=w.max_steps, flags=flags, frames_in_flight=inflight, devices=devices) as r:
        r.resize(w.width, w.height)
        for _ in range(max(1, args.warmup)):
            r.update_parameters_buffer(frames[0])
            r.render(stats=False)
        r.synchronize()
        t0 = time.perf_counter()
        for p in frames:
            r.update_parameters_buffer(p)
            r.render(stats=False)
        r.synchronize()
        elapsed = time.perf_counter() - t0
        steps_total = 0
        counters = [0] * len(COUNTER_NAMES)
        for k, p in enumerate(frames):
            r.update_parameters_buffer(p)
            st = r.render(stats=True)
            steps_total += st["march_steps"]
            counters = [a + st[n] for a, n in zip(counters, COUNTER_NAMES)]
            if k == 0:
                import numpy as np
                sha = hashlib.sha256(np.ascontiguousarray(r.read_frame()).tobytes()).hexdigest()
                if w.moving:
                    break
        if w.moving:  # the stats pass rendered frame 0 only
            steps_total = None
    key = golden_key(args.workload, args.pose)
    gold = json.load(open(GOLDEN)).get(key) if os.path.exists(GOLDEN) else None
    out = {
        "metric": METRIC,
        "value": None if steps_total is None else steps_total / elapsed / 1e9,
        "unit": "Gray-march-steps/s",
        "n_gpus": len(devices),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: deterministic Parameters (" + motion(w) + "), no input data",
        "config": {"workload": w.name, "width": w.width, "height": w.height, "scene_index": w.scene,
                   "num_iterations": w.iters, "max_steps": w.max_steps, "pose": args.pose,
                   "frames_in_flight": inflight, "frames_per_launch": 1, "devices": devices,
                   "parallelism": f"group context over {len(devices)} devices: row bands + "
                                  + ("RCCL point-to-point gather" if len(set(devices)) == len(devices) > 1 else
                                     "device-copy gather" if len(devices) > 1 else "no gather (one device)")
                                  + " to device 0, reassembled there (one process)"},
        "launcher": "single process (--mode group, frm_config.device_count)",
        "frames_per_sec": args.steps / elapsed,
        "frame_sha256": sha,
        "frame_sha_ok": None if gold is None else sha == gold["sha256"],
        "frame_golden": None if gold is None else f"tests/golden/fullsize.json[{key}]",
    }
    if not w.moving:
        cc = counters_check(counters, args.workload, args.pose, args.steps)
        if cc is not None:
            out.update(cc)
    print(json.dumps(out))


def main():
    args = parse()
    if args.mode == "group":
        return group_bench(args)
    if args.dropin_only:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues or 4)
        return dropin_only(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    # before torch initialises HIP
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    elif int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"
    import torch
    import torch.distributed as dist

    import frm
    from frm import tiling
    from frm.distributed import RowTiledFrame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    backend = None
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torch.distributed.run)")
    # test hooks for a 1-GPU box: every rank on device 0, and gloo (RCCL refuses two ranks
    # on one GPU); the driver's multi-GPU runs use neither
    if os.environ.get("FRM_BENCH_SHARED_DEVICE"):
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if os.environ.get("FRM_BENCH_BACKEND") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        backend = dist.get_backend()
        comm_ranks = dist.get_world_size()

    w = frm.WORKLOADS[args.workload]
    afr = world > 1 and args.split == "frames"
    camera = None
    if afr and rank > 0:
        # alternate-frame rendering: rank r renders the view of the same workload from the
        # pose rotated about +y by r * pi/4 (an orbit fly-through, looking at the same
        # point as the base pose; rank 0 renders the base pose itself)
        (x, y, z), yaw, pitch = frm.POSES[args.pose]
        a = rank * math.pi / 4
        camera = ((math.cos(a) * x + math.sin(a) * z, y, -math.sin(a) * x + math.cos(a) * z), yaw + a, pitch)
    # Frame k of the timed region renders frame k of the workload's frame sequence
    # (frm.frame_sequence: the reference's InitializedApp::update, initialized_app.rs:43-48;
    # fixed workloads repeat frame 0, animated ones advance time by 1/60 s per frame, the
    # fly-through also orbits the camera). The warmup renders frame 0.
    seq = frm.frame_sequence(w, pose=args.pose, camera=camera)
    params = next(seq)
    frame0 = params
    flags = (frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0) | (
        {"auto": 0, "simple": frm.FRM_FLAG_SIMPLE_KERNEL, "persistent": frm.FRM_FLAG_PERSISTENT_KERNEL}[args.kernel]) | (
        frm.FRM_FLAG_HW_MATH if args.math == "hw" else 0)
    split = 1 if (world == 1 or afr) else world  # ranks sharing one frame
    band_rows = args.band_rows or (w.height if split == 1 else tiling.choose_band_rows(w.height, world))
    local_pixels = w.width * min(w.height, tiling.rank_rows(w.height, band_rows, 0 if split == 1 else rank, split))
    # frames in flight: a frame's costliest pixels set its tail, which weighs more the fewer
    # pixels a launch has (measured: 4K/8K whole frames best at 2, 1080p and a rank's share
    # of a split frame at 3)
    # frames per launch: the frames' pixels share one work queue, so a launch's tail (its
    # costliest pixels' sequential marches) is paid once per batch (measured, DESIGN.md sections
    # 6-7: 8-way rank share 1.67 ms/frame at 1 frame per launch and 3 in flight -> 1.38-1.44 at
    # 8 per launch and 2 in flight; whole 4K frame 11.20 -> 10.84 ms at 8 per launch, 1080p
    # 3.12 -> 2.80; 16 per launch: 10.42 -> 10.37 ms, 1080p 2.66 -> 2.63, 8-way share 1.416 ->
    # 1.385-1.402, profiles/round2/batch32/). Auto: the timed frames in equal launches of at
    # most 16 (20 frames: 2 x 10). Moving workloads batch too when their frames differ only in
    # camera and the Mandelbulb's time (frm_render_bands_batch: a per-lane power), i.e. scene 18;
    # other animated scenes change more scene constants per frame: one frame per launch.
    # (C5's 16384^2 frames: a launch's tail is ~1 % of a frame; 3 per launch measured 682 ms/frame
    # against 634 at one per launch, profiles/round4/final/configs)
    if w.moving and (w.scene != 18 or w.sphere or local_pixels > 64_000_000):
        batch = 1
    elif args.batch:
        batch = max(1, min(args.batch, frm.FRM_MAX_BATCH))
    else:
        # one GPU: up to FRM_MAX_BATCH per launch (30 frames in one launch against 2 x 15 after
        # fused scheduling: headline 10.11-10.18 -> 10.10-10.12 ms, C3 1.01-1.04 -> 0.99-1.00, C2
        # equal, fly-through 10.66-10.77 -> 10.57-10.58; profiles/round4/batch_sweep); a row split
        # keeps launches of at most 16 so one launch's gather overlaps the next launch's render
        cap = frm.FRM_MAX_BATCH if split == 1 else 16
        k = max(1, args.steps)
        batch = -(-k // -(-k // cap))
    if args.inflight:
        inflight = args.inflight
    elif batch > 1:
        inflight = 2 if split > 1 else 1
    else:
        # moving frames (a new time / camera every frame): the previous frame's cost keys do not
        # predict the costliest pixels, so frames overlap more of each
        # other's tail: 3 in flight (HEADLINE_FLY 11.61 / 11.37 / 11.51 ms at 2 / 3 / 4)
        inflight = 3 if split > 1 or local_pixels < 4_000_000 or w.moving else 2
    inflight = max(1, min(inflight, frm.FRM_MAX_FRAMES_IN_FLIGHT))
    # exactly --steps timed and --warmup untimed frames: launches of `batch` frames, the last one
    # of each run takes the remainder (RowTiledFrame.run)
    r = frm.Renderer(device=local, max_steps=w.max_steps, flags=flags, frames_in_flight=inflight)
    r.resize(w.width, w.height)
    r.update_parameters_buffer(params)
    if args.reload:
        r.reload(args.reload)

    kernel_used = r.kernel_for(local_pixels) + (" (auto)" if args.kernel == "auto" else "")
    dev = torch.device("cuda", local)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    # Frame k renders (and, split over ranks, is gathered and unshuffled) on streams[k % F]:
    # dedicated streams, so their handles are non-null and libfrm launches on them (a NULL
    # handle means "the context's own stream"), and the HIP events below see the kernels.
    streams = [torch.cuda.Stream(device=dev) for _ in range(inflight)]
    main_stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(main_stream)
    kev = []  # (start, stop) HIP events around every render launch of the timed region
    launch_params = []  # moving workloads in batches: the next launch's frames (before_frame)
    timing = {"on": False}

    def render_bands(buf, br, first, stride, slot, count):
        s = streams[slot]
        ev = None
        if timing["on"]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(s)
        if batch > 1:  # one launch, `count` frames, frame b at b * tf.nbytes
            ps = launch_params[:count] if launch_params else [params] * count  # warmup: frame 0
            del launch_params[:count]
            r.render_bands_batch(ps, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=tf.nbytes, band_rows=br, first_band=first, band_stride=stride,
                                 stream=s.cuda_stream, dev_counters=counters.data_ptr())
        else:
            r.render_bands(buf.data_ptr(), buf.numel(), br, first, stride, s.cuda_stream, counters.data_ptr())
        if ev is not None:
            ev[1].record(s)
            kev.append(ev)

    def unshuffle(gathered, rank_stride, frame, slot):
        r.unshuffle_bands(gathered.data_ptr(), rank_stride, frame.data_ptr(), frame.numel(),
                          band_rows, world, streams[slot].cuda_stream)

    tf = RowTiledFrame(w.width, w.height, 0 if split == 1 else rank, split, band_rows, dev, render_bands, unshuffle,
                       inflight=inflight, streams=streams, batch=batch)

    # Animated workloads (C5, HEADLINE_FLY): timed frame k renders frame k of the sequence (a
    # launch of `batch` frames takes the next `batch` of them)
    before_frame = None
    if w.moving:
        def before_frame(k):
            p = frame0 if k == 0 else next(seq)
            if batch > 1:
                launch_params.append(p)
            else:
                r.update_parameters_buffer(p)

    tf.run(args.warmup)
    torch.cuda.synchronize()
    counters.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timing["on"] = True
    # device span of the timed region on the render streams: every stream waits for `begin`,
    # `end` waits for every stream
    begin, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    begin.record(main_stream)
    for s in streams:
        s.wait_event(begin)
    # rank 0 keeps timed frame 0 (for the golden-frame check) with one device copy on its stream
    first = torch.empty(w.width * w.height * 4, dtype=torch.uint8, device=dev) if rank == 0 else None
    t0 = time.perf_counter()
    tf.run(args.steps, before_frame, capture=first)
    for s in streams:
        e = torch.cuda.Event()
        e.record(s)
        main_stream.wait_event(e)
    end.record(main_stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    span_ms = begin.elapsed_time(end)
    launch_ms = sum(a.elapsed_time(b) for a, b in kev) / max(1, len(kev))

    # the drop-in binding's one-frame-per-frm_render loop on the same workload (rank 0, N = 1)
    dropin = None
    if world == 1 and not args.no_dropin:
        dropin = dropin_loop(frm, torch, w, args, flags, local, camera)
        if int(os.environ["GPU_MAX_HW_QUEUES"]) != 4:
            q4 = dropin_q4(args)
            dropin["dropin_q4_ms_per_frame"] = q4["dropin_ms_per_frame"] if q4 else None
            dropin["dropin_q4"] = q4

    stats_vec = torch.tensor([elapsed, span_ms], dtype=torch.float64, device=dev)
    cnt = counters.clone()
    if world > 1:
        dist.all_reduce(stats_vec[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    elapsed = float(stats_vec[0])
    if world > 1:
        # the communicator the frames actually went through: every rank reports its size
        seen = torch.tensor([comm_ranks], dtype=torch.int64, device=dev)
        dist.all_reduce(seen, op=dist.ReduceOp.MIN)
        comm_ranks = int(seen)
    c = [int(v) for v in cnt.cpu().tolist()]
    st = r.stats_from_counters(c)
    steps_total = st["march_steps"]
    if rank == 0:
        # per-frame device time of the pipelined render (the HIP-event span of the timed
        # region / frames): with F frames in flight launches overlap, so a single launch's
        # start-to-end time (avg_launch_ms) also holds the previous frame's tail
        frame_s = span_ms / 1e3 / args.steps
        # WOM ops of one frame (the whole frame: all ranks' shares of a split frame; AFR: per
        # rank's frame) and the device time per frame
        wom_per_frame = st["wom_ops"] / args.steps / (world if split == 1 else 1)
        achieved = st["wom_ops"] / args.steps / world / frame_s / 1e12  # per GPU
        pmc = pmc_summary(args.workload, world, args.math) or {}
        out = {
            "metric": METRIC,
            "value": steps_total / elapsed / 1e9,
            "unit": "Gray-march-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if split > 1 else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: deterministic Parameters (" + motion(w) + "), no input data",
            "config": {
                "workload": w.name, "width": w.width, "height": w.height, "scene_index": w.scene,
                "num_iterations": w.iters, "max_steps": w.max_steps, "time": w.time,
                "pose": args.pose, "frames_in_flight": inflight, "frames_per_launch": batch,
                "math": ("exact (frm builtins, bit-exact with the oracle)" if args.math == "exact" else
                         "hw (FRM_FLAG_HW_MATH: hardware transcendentals, NOT bit-exact; P1-classified, "
                         "tests/test_gpu_hw_math.py)"),
                "gpu_max_hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]), "kernel": kernel_used + (" (runtime-compiled)" if args.reload else ""),
                "animated": motion(w) if w.moving else False,
                "parallelism": (f"row-bands x{world} (band_rows={band_rows}) + "
                                f"{'RCCL' if backend == 'nccl' else backend + ' (host-staged)'} gather" if split > 1 else
                                f"alternate-frame rendering x{world}: rank r renders the {args.pose} view "
                                f"rotated by r*pi/4 about +y, whole frames, no data-path collective"
                                if world > 1 else "single GPU"),
            },
            "frames_per_sec": args.steps * (world if split == 1 else 1) / elapsed,
            "normal_de_evals_per_sec": st["normal_evals"] / elapsed,  # the 4 taps per hit, apart from steps
            "march_steps_per_frame": steps_total / args.steps / (world if split == 1 else 1),
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": VALU_PEAK_TOPS,
                "unit": "Tlane-op/s",
                "frac": achieved / VALU_PEAK_TOPS,
                "traffic": pmc.get("traffic"),
                "traffic_source": pmc.get("source"),
                "pmc_source_sha256": pmc.get("source_sha256"),
                "pmc_stale": pmc.get("stale"),
                # rocprofv3 hardware view of the same kernel (committed PMC passes):
                # SQ VALU-busy, active-lane fraction, HBM write rate against the 8 TB/s peak
                "valu_busy": pmc.get("valu_busy"),
                "valu_lane_utilization": pmc.get("valu_lane_utilization"),
                "hbm_write_gbps": pmc.get("hbm_write_gbps"),
                "hbm_write_frac": pmc.get("hbm_write_frac"),
                "traffic_split": pmc.get("traffic_split"),
                "traffic_unit": "HBM bytes per frame (PMC FETCH_SIZE + WRITE_SIZE, march_persistent + shade_pass)",
                "kernel": "frm::march_persistent + sort + shade_pass (one frame's launches)",
                "device_ms_per_frame": frame_s * 1e3,
                "avg_launch_ms": launch_ms,
                "frames_per_launch": batch,
                "timing": "HIP events on the render streams: span of the timed region / frames",
                "algorithmic_ops_per_frame": wom_per_frame,
                "model": "WOM VALU lane-ops counted from fragment.wgsl (DESIGN.md §Roofline)",
            },
            "counters": st,
        }
        if world > 1:
            out["comm"] = {"backend": backend, "ranks": comm_ranks,
                           "data_path": "dist.gather of row bands to rank 0" if split > 1 else "none (timing only)"}
            out["rccl_ranks"] = comm_ranks if backend == "nccl" else None
        if args.math == "exact":
            out.update(frame_check(first, args.workload, args.pose))
        else:  # no golden: the hardware-math frame differs from the oracle's by design
            out.update({"frame_sha256": hashlib.sha256(first.cpu().numpy().tobytes()).hexdigest(),
                        "frame_sha_ok": None, "frame_golden": "none (FRM_FLAG_HW_MATH is not bit-exact)"})
        # every timed frame is frame 0 (fixed workloads; a row split's ranks sum to whole frames):
        # the summed counters must be steps x the golden frame's, or the roofline is not reported
        cc = None
        if args.math == "exact" and not w.moving and not afr:
            cc = counters_check(c, args.workload, args.pose, args.steps)
        if cc is not None:
            out.update(cc)
            if not cc["counters_ok"]:
                for k in ("achieved", "frac", "algorithmic_ops_per_frame"):
                    out["roofline"][k] = None
        if dropin:
            out.update(dropin)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(params, w, args.cpu_seconds)
        print(json.dumps(out))
        if cc is not None and not cc["counters_ok"]:
            print(f"bench.py: work counters differ from the oracle's: {cc['counters_mismatch']}", file=sys.stderr)
            r.close()
            raise SystemExit(3)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
