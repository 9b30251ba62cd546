"""Asynchronous readback (frm_read_frame_async / frm_present_async / frm_frame_pixels): the
drop-in binding's frame loop with a frame of presentation latency, as the reference's surface
(wgpu's default desired_maximum_frame_latency = 2, persistent_graphics.rs:158-162) runs it.
Every frame read back this way equals the oracle's render of that frame's own Parameters."""
import numpy as np
import pytest

import frm
from frm import _lib
from helpers import params_for

pytestmark = pytest.mark.gpu

W, H = 96, 54


def _frames(n):
    # a moving loop: the time (the Mandelbulb power) and the camera change every frame
    out = []
    for k in range(n):
        p = params_for(18, 8, frm.POWER8_TIME + 0.4 * k, W, H, pose=("P0", "P1", "P2")[k % 3])
        out.append(p)
    return out


@pytest.mark.parametrize("fif", [1, 2, 3])
def test_latency_one_loop_every_frame_bit_exact(frm_lib, oracle, fif):
    frames = _frames(6)
    refs = [oracle.render(p, W, H, 256)["rgba"] for p in frames]
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=fif) as r:
        r.resize(W, H)
        held, got = [], []
        lag = fif - 1  # a slot's image lives until frames_in_flight further renders
        for p in frames:
            r.update_parameters_buffer(p)
            r.render(stats=False)
            held.append(r.read_frame_async())
            if len(held) > lag:
                got.append(r.frame_pixels(held.pop(0)))
        got += [r.frame_pixels(t) for t in held]
    for k, (g, ref) in enumerate(zip(got, refs)):
        assert np.array_equal(g, ref), f"frame {k}"


def test_present_async_matches_present(frm_lib):
    p = params_for(18, 6, 3.2175055, 160, 90)
    with frm.Renderer(device=0, max_steps=128, frames_in_flight=2) as r:
        r.resize(160, 90)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        sync = r.present(97, 61, srgb=False, bgra=True)
        t = r.present_async(97, 61, srgb=False, bgra=True)
        assert np.array_equal(r.frame_pixels(t, shape=(61, 97, 4)), sync)
        # the same-size sRGB present is the frame itself
        t = r.present_async(160, 90)
        assert np.array_equal(r.frame_pixels(t), r.read_frame())


def test_ticket_expires_with_its_slot(frm_lib):
    p = params_for(18, 4, 3.2175055, 32, 18)
    with frm.Renderer(device=0, max_steps=64, frames_in_flight=2) as r:
        r.resize(32, 18)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        t0 = r.read_frame_async()
        r.render(stats=False)
        t1 = r.read_frame_async()
        r.frame_pixels(t0)  # still held: its slot has not been read back again
        r.render(stats=False)           # slot of t0 again
        t2 = r.read_frame_async()
        with pytest.raises(frm.FrmError) as e:
            r.frame_pixels(t0)
        assert e.value.code == _lib.FRM_ERR_INVALID_ARGUMENT
        r.frame_pixels(t1)
        r.frame_pixels(t2)
        with pytest.raises(frm.FrmError):
            r.frame_pixels(0)


def test_readback_before_render_refused(frm_lib):
    with frm.Renderer(device=0, max_steps=64) as r:
        r.resize(16, 16)
        with pytest.raises(frm.FrmError) as e:
            r.read_frame_async()
        assert e.value.code == _lib.FRM_ERR_NOT_READY


def test_debug_trace_refused_after_slot_reuse(frm_lib):
    """frm_debug_trace reads the records of the last frm_render: a later band launch that takes
    the same slot makes it refuse instead of returning another launch's records."""
    import torch

    w, h = 64, 36
    p = params_for(18, 6, frm.POWER8_TIME, w, h)
    with frm.Renderer(device=0, max_steps=128, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        tr = r.trace()
        assert tr.shape == (h, w, 10)
        buf = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
        r.render_bands(buf.data_ptr(), buf.numel(), h, 0, 1)  # one slot: reuses the render's
        torch.cuda.synchronize()
        with pytest.raises(frm.FrmError) as e:
            r.trace()
        assert e.value.code == _lib.FRM_ERR_NOT_READY
