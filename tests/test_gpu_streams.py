"""libfrm's render streams and a torch host: frames in flight run on non-blocking
slot streams by default (FRM_SLOT_STREAMS=cumask opts into CU-masked streams, which HIP creates
as blocking streams that synchronise with the legacy null stream, torch's default stream). Work a
torch host puts on its default stream while a second frame is in flight neither waits for the
render nor disturbs it."""
import hashlib
import json
import os
import time

import pytest

import frm

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")


def test_torch_default_stream_independent_of_inflight_render(frm_lib):
    import torch
    g = json.load(open(GOLDEN))["HEADLINE_P1"]
    p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
    x = torch.ones(1 << 20, device="cuda")
    (x * 2).sum().item()  # warm torch's kernels up
    with frm.Renderer(max_steps=g["max_steps"], frames_in_flight=2) as r:
        r.resize(g["width"], g["height"])
        r.update_parameters_buffer(p)
        frame_ms = r.render(stats=True)["kernel_ms"]
        r.render(stats=False)  # slot 1
        r.render(stats=False)  # slot 0 again: two frames in flight on the slot streams
        t0 = time.perf_counter()
        y = (x * 3).sum()  # the default (null) stream
        torch.cuda.current_stream().synchronize()
        dt_ms = (time.perf_counter() - t0) * 1e3
        assert float(y) == 3.0 * (1 << 20)
        r.synchronize()
        assert hashlib.sha256(r.read_frame().tobytes()).hexdigest() == g["sha256"]
    # a blocking stream would have held the torch op behind both frames (about 2 x frame_ms)
    assert dt_ms < 0.5 * frame_ms, (dt_ms, frame_ms)
