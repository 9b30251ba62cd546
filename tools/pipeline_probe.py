"""Probe: frames in flight on one GPU. F contexts (each with its own records and
scheduling arrays) render frames round-robin on F streams; prints ms/frame and G
march-steps/s for a whole frame and for one rank's bands of a P-way row split."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:  # see bench.py
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import torch  # noqa: E402

import frm  # noqa: E402
from frm import tiling  # noqa: E402


def cumask_stream(dev):
    """A stream on its own hardware queue: ROCclr never pools CU-masked queues."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value, device=dev)


def run(workload, ranks, rank, inflight, frames, warmup, mode="slots", events=False, cumask=False, gather=False,
        batch=1):
    """mode 'slots': one context with frames_in_flight = F; 'contexts': F contexts."""
    w = frm.WORKLOADS[workload]
    p = frm.make_parameters(w, pose="P1")
    dev = torch.device("cuda", 0)
    br = w.height if ranks == 1 else tiling.choose_band_rows(w.height, ranks)
    rows = tiling.rank_buffer_rows(w.height, br, ranks)
    rs, ss, bufs = [], [], []
    one = None
    if mode == "slots":
        one = frm.Renderer(device=0, max_steps=w.max_steps, flags=frm.FRM_FLAG_PERSISTENT_KERNEL,
                           frames_in_flight=inflight)
        one.resize(w.width, w.height)
        one.update_parameters_buffer(p)
    for _ in range(inflight):
        if one is None:
            r = frm.Renderer(device=0, max_steps=w.max_steps, flags=frm.FRM_FLAG_PERSISTENT_KERNEL)
            r.resize(w.width, w.height)
            r.update_parameters_buffer(p)
        else:
            r = one
        rs.append(r)
        ss.append(cumask_stream(dev) if cumask else torch.cuda.Stream(device=dev))
        bufs.append(torch.zeros(batch * rows * w.width * 4, dtype=torch.uint8, device=dev))
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    # gather: rank 0's extra work per frame of a real P-way run, on its render stream after its
    # bands: P - 1 rank buffers arriving (device-to-device copies of its own buffer stand in
    # for RCCL's receives over xGMI) and frm_unshuffle_bands into the row-major frame
    gbufs = frames_out = None
    if gather and ranks > 1:
        gbufs = [torch.zeros(ranks * bufs[0].numel(), dtype=torch.uint8, device=dev) for _ in range(inflight)]
        frames_out = [torch.zeros(batch * w.width * w.height * 4, dtype=torch.uint8, device=dev)
                      for _ in range(inflight)]
    fbytes = rows * w.width * 4

    def go(n):
        for k in range(n):
            i = k % inflight
            if events:
                torch.cuda.Event(enable_timing=True).record(ss[i])
            if batch > 1:
                rs[i].render_bands_batch([p] * batch, bufs[i].data_ptr(), dst_bytes=bufs[i].numel(), frame_stride=fbytes, band_rows=br, first_band=rank, band_stride=ranks,
                                         stream=ss[i].cuda_stream, dev_counters=counters.data_ptr())
            else:
                rs[i].render_bands(bufs[i].data_ptr(), bufs[i].numel(), br, rank, ranks, ss[i].cuda_stream,
                                   counters.data_ptr())
            if gbufs is not None:
                with torch.cuda.stream(ss[i]):
                    nb = bufs[i].numel()
                    gbufs[i][:nb].copy_(bufs[i])
                    for q in range(1, ranks):
                        gbufs[i][q * nb:(q + 1) * nb].copy_(bufs[i], non_blocking=True)
                fb = w.width * w.height * 4
                for b in range(batch):
                    rs[i].unshuffle_bands(gbufs[i].data_ptr() + b * fbytes, nb, frames_out[i].data_ptr() + b * fb, fb,
                                          br, ranks, ss[i].cuda_stream)
            if events:
                torch.cuda.Event(enable_timing=True).record(ss[i])

    go(warmup * inflight)
    torch.cuda.synchronize()
    counters.zero_()
    t0 = time.perf_counter()
    go(frames // batch)  # launches
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    frames = frames // batch * batch
    st = rs[0].stats_from_counters([int(v) for v in counters.cpu().tolist()])
    for r in set(rs):
        r.close()
    return {"workload": workload, "ranks": ranks, "rank": rank, "inflight": inflight, "mode": mode, "events": events, "cumask": cumask,
            "gather": bool(gbufs is not None), "batch": batch,
            "ms_per_frame": dt / frames * 1e3, "gsteps": st["march_steps"] / dt / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="HEADLINE,C2")
    ap.add_argument("--ranks", default="1,8")
    ap.add_argument("--inflight", default="1,2,3,4")
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--modes", default="slots")
    ap.add_argument("--events", default="0")
    ap.add_argument("--cumask", default="0")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--rank-ids", default="0", help="ranks whose share to time ('all' = every rank)")
    ap.add_argument("--gather", default="0", help="1: rank 0 also receives and unshuffles (see run())")
    ap.add_argument("--batch", default="1", help="frames per launch (frm_render_bands_batch)")
    args = ap.parse_args()
    for wl in args.workloads.split(","):
        for P in [int(x) for x in args.ranks.split(",")]:
            for F in [int(x) for x in args.inflight.split(",")]:
                for m in args.modes.split(","):
                    for ev in [bool(int(x)) for x in args.events.split(",")]:
                        for cm in [bool(int(x)) for x in args.cumask.split(",")]:
                            ids = range(P) if args.rank_ids == "all" else [int(x) for x in args.rank_ids.split(",") if int(x) < P]
                            for rk in ids:
                                for g in [bool(int(x)) for x in args.gather.split(",")]:
                                    if g and rk != 0:
                                        continue
                                    for B in [int(x) for x in args.batch.split(",")]:
                                        for _ in range(args.repeat):
                                            print(json.dumps(run(wl, P, rk, F, args.frames, 2, m, ev, cm, g, B)),
                                                  flush=True)


if __name__ == "__main__":
    main()
