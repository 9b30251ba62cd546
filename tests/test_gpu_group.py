"""Group contexts (frm_config.device_count, include/frm.h ABI 5): one context row-tiles every frame
over a device list and gathers the bands on devices[0] (RCCL point-to-point for distinct devices,
device-to-device copies for a repeated device), so a C or Rust host selects N GPUs by config alone
(graphics.rs:25-37 Graphics::init). On the one-GPU test box a group of
one device runs the whole group path (bands, gather buffer, reassembly) and a device listed three
times rehearses three ranks with the copy transport. Every frame equals the oracle's render, or the
golden whole-frame hash at BASELINE size."""
import hashlib
import json
import os

import numpy as np
import pytest

import frm
from frm import _lib
from helpers import params_for

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("w,h", [(96, 54), (130, 9), (64, 100)])
def test_group_frame_bit_exact(frm_lib, oracle, devices, w, h):
    p = params_for(18, 8, frm.POWER8_TIME, w, h, pose="P1")
    ref = oracle.render(p, w, h, 256)
    with frm.Renderer(max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, devices=devices) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        for _ in range(2):  # the second frame runs in the scheduled order
            st = r.render(stats=True)
            assert np.array_equal(r.read_frame(), ref["rgba"])
            got = [st[k] for k in ("pixels", "hit_pixels", "primary_steps", "shadow_steps", "normal_evals",
                                   "fractal_bodies", "fractal_bailouts")]
            assert got == [int(v) for v in ref["counters"][:7]]


@pytest.mark.parametrize("fif", [1, 2, 3])
def test_group_moving_loop_with_latency(frm_lib, oracle, fif):
    """The drop-in loop (frames in flight, a frame of presentation latency) on a three-rank group:
    every frame read back is the oracle's render of its own Parameters."""
    W, H = 96, 54
    frames = [params_for((18, 0, 15)[k % 3], 6, frm.POWER8_TIME + 0.3 * k, W, H, pose=("P0", "P1", "P2")[k % 3])
              for k in range(6)]
    refs = [oracle.render(p, W, H, 256)["rgba"] for p in frames]
    with frm.Renderer(max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=fif,
                      devices=[0, 0, 0]) as r:
        r.resize(W, H)
        held, got = [], []
        for p in frames:
            r.update_parameters_buffer(p)
            r.render(stats=False)
            held.append(r.read_frame_async())
            if len(held) > fif - 1:
                got.append(r.frame_pixels(held.pop(0)))
        got += [r.frame_pixels(t) for t in held]
    for k, (g, ref) in enumerate(zip(got, refs)):
        assert np.array_equal(g, ref), f"frame {k}"


def test_group_resize_and_present(frm_lib, oracle):
    p = params_for(18, 6, frm.POWER8_TIME, 160, 90)
    with frm.Renderer(max_steps=128, frames_in_flight=2, devices=[0, 0]) as r, \
            frm.Renderer(max_steps=128, frames_in_flight=2) as one:
        for w, h in ((160, 90), (97, 61), (160, 90)):
            q = params_for(18, 6, frm.POWER8_TIME, w, h)
            for x in (r, one):
                x.resize(w, h)
                x.update_parameters_buffer(q)
                x.render(stats=False)
            assert np.array_equal(r.read_frame(), one.read_frame())
            assert np.array_equal(r.present(64, 40, srgb=False, bgra=True), one.present(64, 40, srgb=False, bgra=True))
            assert np.array_equal(r.read_frame(), oracle.render(q, w, h, 128)["rgba"])


def test_group_refuses_per_rank_entry_points(frm_lib):
    import torch
    with frm.Renderer(max_steps=64, devices=[0, 0]) as r:
        r.resize(32, 32)
        r.update_parameters_buffer(params_for(18, 4, frm.POWER8_TIME, 32, 32))
        buf = torch.empty(32 * 32 * 4, dtype=torch.uint8, device="cuda")
        with pytest.raises(frm.FrmError) as e:
            r.render_bands(buf.data_ptr(), buf.numel(), 16, 0, 1)
        assert e.value.code == _lib.FRM_ERR_UNSUPPORTED
        with pytest.raises(frm.FrmError) as e:
            r.trace()
        assert e.value.code == _lib.FRM_ERR_UNSUPPORTED


@pytest.mark.parametrize("case", ["HEADLINE_P1", "C4_P1"])
def test_group_full_size_golden(frm_lib, case):
    """BASELINE's headline and C4 frames through a group context: a one-device group (the group path
    with every band on device 0) and a four-rank rehearsal (C4's 8K frame over the copy transport)
    equal the oracle's golden hash and work counters."""
    g = json.load(open(GOLDEN))[case]
    p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
    devices = [0] if case == "HEADLINE_P1" else [0, 0, 0, 0]
    with frm.Renderer(max_steps=g["max_steps"], frames_in_flight=2, devices=devices) as r:
        r.resize(g["width"], g["height"])
        r.update_parameters_buffer(p)
        for k in range(2):
            st = r.render(stats=True)
            got = [st[k] for k in ("pixels", "hit_pixels", "primary_steps", "shadow_steps", "normal_evals",
                                   "fractal_bodies", "fractal_bailouts")]
            assert got == g["counters"][:7]
            assert hashlib.sha256(r.read_frame().tobytes()).hexdigest() == g["sha256"]
