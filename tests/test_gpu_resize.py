"""Resizing keeps the pixel-scheduling history: the first frame of a new whole-frame size
fetches its pixels in the order of the previous size's cost keys, resampled (frm_sched.hip
rescale_keys), instead of row-major. Order never changes bytes: every frame of a resize
sequence (up, down, odd sizes; one and two frames in flight) equals the oracle's. Also:
num_iterations above the old 4096 cap renders the reference's semantics (Sierpinski's
i32(N) loop runs no fold for N >= 2^31)."""
import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("inflight", [1, 2])
def test_resize_sequence_bit_exact(frm_lib, oracle, inflight):
    sizes = [(96, 54), (160, 90), (64, 36), (130, 9), (160, 90)]
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=inflight) as r:
        for w, h in sizes:
            p = params_for(18, 12, frm.POWER8_TIME, w, h)
            r.resize(w, h)
            r.update_parameters_buffer(p)
            ref = oracle.render(p, w, h, 256)
            for k in range(inflight + 1):  # the first frame(s) of the size, then a scheduled one
                st = r.render(stats=True)
                img = r.read_frame()
                assert np.array_equal(img, ref["rgba"]), f"{w}x{h} frame {k}"
                assert st["march_steps"] == int(ref["counters"][2] + ref["counters"][3])


@pytest.mark.parametrize("inflight", [2, 3])
def test_resize_in_flight_loop_bit_exact(frm_lib, oracle, inflight):
    """frm_resize does not drain: the drop-in loop (frame k rendered, its readback started, frame
    k - inflight + 1's pixels awaited) resizes between frames while earlier frames of the old size
    are still rendering and being read back. Every frame, before and after each size change (up
    past the framebuffer headroom, down, the reference's +-1 factor steps), equals the oracle's."""
    sizes = [(160, 90), (168, 94), (160, 90), (320, 180), (96, 54), (152, 86), (160, 90)]
    frames, want = [], {}
    for w, h in sizes:
        p = params_for(18, 12, frm.POWER8_TIME, w, h)
        want[(w, h)] = oracle.render(p, w, h, 256)["rgba"]
        frames += [(w, h, p)] * 3
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=inflight) as r:
        held = []
        for k, (w, h, p) in enumerate(frames):
            if (w, h) != (r.width, r.height):
                r.resize(w, h)
            r.update_parameters_buffer(p)
            r.render(stats=False)
            held.append((k, w, h, r.read_frame_async()))
            while len(held) > inflight - 1:
                j, fw, fh, t = held.pop(0)
                assert np.array_equal(r.frame_pixels(t), want[(fw, fh)]), f"frame {j} ({fw}x{fh})"
        for j, fw, fh, t in held:
            assert np.array_equal(r.frame_pixels(t), want[(fw, fh)]), f"frame {j} ({fw}x{fh})"


@pytest.mark.parametrize("scene,iters", [(15, 2 ** 31 + 5), (15, 0xFFFFFFFF), (18, 5000), (0, 4100)])
def test_num_iterations_above_old_cap(frm_lib, oracle, scene, iters):
    w, h = 32, 18
    p = params_for(scene, iters, frm.POWER8_TIME, w, h)
    with frm.Renderer(device=0, max_steps=64) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        img = r.read_frame()
    ref = oracle.render(p, w, h, 64)
    assert np.array_equal(img, ref["rgba"])


def test_unbounded_num_iterations_are_refused_not_rendered(frm_lib, oracle):
    """Parameters whose fractal loop never ends (Mandelbulb N = 0xffffffff: `i <= N` wraps,
    fragment.wgsl:245) are refused even with FRM_FLAG_UNBOUNDED_ITERATIONS; loops above
    FRM_MAX_NUM_ITERATIONS trips are refused unless the context opted out. A refused update keeps
    the previous parameters (the next frame renders them); the opt-out renders the reference's
    semantics bit-exact."""
    from frm import _lib

    w, h = 16, 9
    good = params_for(18, 12, frm.POWER8_TIME, w, h)
    with frm.Renderer(device=0, max_steps=64) as r:
        r.resize(w, h)
        r.update_parameters_buffer(good)
        for scene, iters in ((18, 0xFFFFFFFF), (18, frm.FRM_MAX_NUM_ITERATIONS + 1), (0, 0xFFFFFFFE),
                             (16, frm.FRM_MAX_NUM_ITERATIONS + 1), (15, 2 ** 31 - 1)):
            with pytest.raises(frm.FrmError) as e:
                r.update_parameters_buffer(params_for(scene, iters, frm.POWER8_TIME, w, h))
            assert e.value.code == _lib.FRM_ERR_UNSUPPORTED
        r.update_parameters_buffer(params_for(0, frm.FRM_MAX_NUM_ITERATIONS, 0.0, w, h))  # the cap itself
        r.update_parameters_buffer(good)
        with pytest.raises(frm.FrmError):
            r.update_parameters_buffer(params_for(18, 0xFFFFFFFF, frm.POWER8_TIME, w, h))
        r.render(stats=False)
        assert np.array_equal(r.read_frame(), oracle.render(good, w, h, 64)["rgba"])
    with frm.Renderer(device=0, max_steps=8, flags=frm.FRM_FLAG_UNBOUNDED_ITERATIONS) as r:
        r.resize(w, h)
        with pytest.raises(frm.FrmError):
            r.update_parameters_buffer(params_for(18, 0xFFFFFFFF, frm.POWER8_TIME, w, h))
        p = params_for(0, frm.FRM_MAX_NUM_ITERATIONS + 7, 0.0, w, h)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        assert np.array_equal(r.read_frame(), oracle.render(p, w, h, 8)["rgba"])


def test_pixel_keys_roundtrip_and_injected_orders_keep_bytes(frm_lib, oracle):
    """The scheduling diagnostics (frm_debug_pixel_keys / frm_debug_set_pixel_keys): the keys the
    persistent kernel records are 16 log2(bodies + 1) per pixel (0 only where a pixel ran no
    body); any injected order (reversed, all equal = row-major, random) renders the oracle's bytes
    and counters; a key map of the wrong size is refused."""
    w, h = 160, 90
    p = params_for(18, 12, frm.POWER8_TIME, w, h)
    ref = oracle.render(p, w, h, 256)
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        r.render(stats=True)
        keys = r.pixel_keys()
        assert keys.shape == (w * h,) and keys.max() > 100
        rng = np.random.default_rng(3)
        for inj in (255 - keys, np.zeros_like(keys), rng.integers(0, 256, keys.size).astype(np.uint8)):
            r.set_pixel_keys(inj)
            st = r.render(stats=True)
            assert np.array_equal(r.read_frame(), ref["rgba"])
            assert st["march_steps"] == int(ref["counters"][2] + ref["counters"][3])
            assert np.array_equal(r.pixel_keys(), keys)  # the keys a frame records are its own costs
        with pytest.raises(frm.FrmError):
            r.set_pixel_keys(keys[:-1])
