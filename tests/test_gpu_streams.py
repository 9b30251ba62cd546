"""libfrm's render streams and a torch host: frames in
flight run on non-blocking slot streams by default (FRM_SLOT_STREAMS=cumask opts into CU-masked
streams, which HIP creates as blocking streams that synchronise with the legacy null stream,
torch's default stream). Work a torch host puts on its default stream while two frames are in
flight neither waits for them nor disturbs them. HIP maps streams onto at most GPU_MAX_HW_QUEUES
hardware queues per process (4 by default) and work on a shared queue runs in order, so this holds
only while libfrm's streams and the null stream fit: with frames in flight libfrm now uses one
stream per slot (the readback copies go on the render's own stream), 2 for 2 in flight. Asserted at
the default 4 queues and at 16, by ordering rather than a time bound: the null stream's event
completes while the in-flight frames are still running (it is not queued behind them)."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "fullsize.json")

CHILD = r"""
import hashlib, json, os, sys, time
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "fractal-ray-marching_amd")]
import torch
import frm
g = json.load(open(sys.argv[2]))["HEADLINE_P1"]
p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
x = torch.ones(1 << 20, device="cuda")
(x * 2).sum().item()
with frm.Renderer(max_steps=g["max_steps"], frames_in_flight=2) as r:
    r.resize(g["width"], g["height"])
    r.update_parameters_buffer(p)
    r.render(stats=False)
    r.synchronize()
    t0 = time.perf_counter()
    r.render(stats=False)
    r.render(stats=False)  # two frames in flight on the slot streams
    ev = torch.cuda.Event()
    ev.record(torch.cuda.default_stream())
    while not ev.query():  # the null stream's event, polled
        if time.perf_counter() - t0 > 10:
            break
    t_ev = (time.perf_counter() - t0) * 1e3
    y = float((x * 3).sum())
    r.synchronize()  # both frames
    t_frames = (time.perf_counter() - t0) * 1e3
    ok = hashlib.sha256(r.read_frame().tobytes()).hexdigest() == g["sha256"]
print(json.dumps({"t_event_ms": t_ev, "t_frames_ms": t_frames, "sum_ok": y == 3.0 * (1 << 20), "frame_ok": ok}))
"""


def _run(queues):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues))
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, GOLDEN], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("queues", [4, 16])
def test_torch_default_stream_independent_of_inflight_render(frm_lib, queues):
    r = _run(queues)
    assert r["sum_ok"] and r["frame_ok"], r
    # ordering: the null stream's event completed while the two frames were still rendering (queued
    # behind them it would complete with them, t_event ~ t_frames)
    assert r["t_event_ms"] < 0.5 * r["t_frames_ms"], r
    print(f"GPU_MAX_HW_QUEUES={queues}:", r)
