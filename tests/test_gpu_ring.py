"""The resident frame ring (frm_api.hip ring_render, march_persistent<..., RES>): single-frame
frm_render calls without stats on a context with frames in flight are served by one persistent grid
that marches the posted frames in order and shades each as its last pixel finishes. Every frame of
every loop form below must equal the oracle's render of its own Parameters, as the reference's
draw renders each frame from the uniform of that frame (initialized_app.rs:37-48, graphics.rs:91-110):
fixed and moving loops, 2 and 4 slots, a frame of readback latency or none, scene and size changes
in the middle of a loop (a new ring generation), frames outside the ring in between (stats, a band
launch), the synchronous readbacks, and the headline frame at 4K against its golden hash."""
import hashlib
import json
import os

import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _ring_on(monkeypatch):
    """The ring is opt-in (FRM_RING=1, read when a context is created)."""
    monkeypatch.setenv("FRM_RING", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = 160, 90
PERSISTENT = frm.FRM_FLAG_PERSISTENT_KERNEL


def _moving(n, scene=18, iters=8, w=W, h=H):
    # time (the Mandelbulb power) and pose change every frame
    return [params_for(scene, iters, frm.POWER8_TIME + 0.37 * k, w, h, pose=("P0", "P1", "P2")[k % 3])
            for k in range(n)]


def _loop(r, frames, lag):
    """frm_render + frm_read_frame_async per frame, the pixels of frame k - lag after frame k."""
    held, got = [], []
    for p in frames:
        r.update_parameters_buffer(p)
        r.render(stats=False)
        held.append(r.read_frame_async())
        if len(held) > lag:
            got.append(r.frame_pixels(held.pop(0)))
    got += [r.frame_pixels(t) for t in held]
    return got


def _check(oracle, frames, got, w=W, h=H, steps=256):
    assert len(got) == len(frames)
    for k, (p, g) in enumerate(zip(frames, got)):
        ref = oracle.render(p, w, h, steps)["rgba"]
        bad = int(np.any(g.reshape(h, w, 4) != ref, axis=-1).sum())
        assert bad == 0, f"frame {k}: {bad} pixels differ from the oracle"


@pytest.mark.parametrize("fif", [2, 3])
@pytest.mark.parametrize("lag", [0, 1])
def test_ring_moving_loop_bit_exact(frm_lib, oracle, fif, lag):
    frames = _moving(9)
    with frm.Renderer(device=0, max_steps=256, flags=PERSISTENT, frames_in_flight=fif) as r:
        r.resize(W, H)
        got = _loop(r, frames, lag)
    _check(oracle, frames, got)


@pytest.mark.parametrize("scene,iters", [(0, 4), (15, 5), (16, 3), (13, 3), (18, 0)])
def test_ring_families_bit_exact(frm_lib, oracle, scene, iters):
    # fixed pose, the other families (animated Menger scene 13 at a fixed time), N = 0 Mandelbulb
    frames = [params_for(scene, iters, 1.25, W, H, pose=pose) for pose in ("P1", "P1", "P2", "P0")]
    with frm.Renderer(device=0, max_steps=256, flags=PERSISTENT, frames_in_flight=2) as r:
        r.resize(W, H)
        got = _loop(r, frames, 1)
    _check(oracle, frames, got)


def test_ring_sphere_extension(frm_lib, oracle):
    p = params_for(18, 3, frm.POWER8_TIME, W, H)
    with frm.Renderer(device=0, max_steps=64, flags=PERSISTENT | frm.FRM_FLAG_SCENE_SPHERE,
                      frames_in_flight=2) as r:
        r.resize(W, H)
        got = _loop(r, [p] * 3, 1)
    ref = oracle.render(p, W, H, 64, flags=1)["rgba"]
    for g in got:
        assert np.array_equal(g.reshape(H, W, 4), ref)


def test_ring_generation_changes_mid_loop(frm_lib, oracle):
    """Scene, iteration count and size change inside a running loop: each change starts a new
    ring generation (the earlier frames finish first), every frame stays the oracle's."""
    seq = [(W, H, p) for p in _moving(3)]
    seq += [(W, H, p) for p in (params_for(0, 4, 0.0, W, H), params_for(0, 4, 0.0, W, H, pose="P2"))]
    seq += [(W, H, p) for p in _moving(2, iters=6)]
    w2, h2 = 128, 72
    seq += [(w2, h2, p) for p in _moving(3, w=w2, h=h2)]
    seq += [(W, H, p) for p in _moving(2)]
    got = []
    with frm.Renderer(device=0, max_steps=256, flags=PERSISTENT, frames_in_flight=2) as r:
        held = []
        size = None
        for w, h, p in seq:
            if (w, h) != size:
                r.resize(w, h)
                size = (w, h)
            r.update_parameters_buffer(p)
            r.render(stats=False)
            held.append((w, h, r.read_frame_async()))
            if len(held) > 1:
                hw, hh, t = held.pop(0)
                got.append(r.frame_pixels(t).reshape(hh, hw, 4))
        for hw, hh, t in held:
            got.append(r.frame_pixels(t).reshape(hh, hw, 4))
    for k, ((w, h, p), g) in enumerate(zip(seq, got)):
        assert np.array_equal(g, oracle.render(p, w, h, 256)["rgba"]), f"frame {k}"


def test_ring_mixed_with_stats_bands_and_sync_readback(frm_lib, oracle):
    """Ring frames, then a stats frame (outside the ring), a band launch and the synchronous
    readbacks of a ring frame; the counters of the stats frame are the oracle's."""
    import torch

    frames = _moving(4)
    with frm.Renderer(device=0, max_steps=256, flags=PERSISTENT, frames_in_flight=2) as r:
        r.resize(W, H)
        for p in frames[:2]:
            r.update_parameters_buffer(p)
            r.render(stats=False)
        # synchronous readback of the last ring frame, and its presentation at its own size
        assert np.array_equal(r.read_frame(), oracle.render(frames[1], W, H, 256)["rgba"])
        assert np.array_equal(r.present(W, H), oracle.render(frames[1], W, H, 256)["rgba"])
        r.update_parameters_buffer(frames[2])
        st = r.render(stats=True)
        ref = oracle.render(frames[2], W, H, 256)
        assert np.array_equal(r.read_frame(), ref["rgba"])
        assert st["march_steps"] == int(ref["counters"][2]) + int(ref["counters"][3])
        buf = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
        r.render_bands(buf.data_ptr(), buf.numel(), H, 0, 1)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy().reshape(H, W, 4), ref["rgba"])
        r.update_parameters_buffer(frames[3])
        r.render(stats=False)
        t = r.read_frame_async()
        assert np.array_equal(r.frame_pixels(t).reshape(H, W, 4), oracle.render(frames[3], W, H, 256)["rgba"])
        r.synchronize()


def test_ring_headline_4k_golden(frm_lib):
    """The 4K headline frame through the ring, frames in flight 2, read back zero-copy: the golden
    hash of tests/golden/fullsize.json (bench.py's frame check)."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))["HEADLINE_P1"]
    p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
    with frm.Renderer(max_steps=g["max_steps"], frames_in_flight=2) as r:
        r.resize(g["width"], g["height"])
        got = _loop(r, [p] * 4, 1)
    for k, img in enumerate(got):
        assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == g["sha256"], f"frame {k}"
