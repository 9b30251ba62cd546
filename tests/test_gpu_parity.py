"""GPU parity (gate P0): the gfx950 kernel's RGBA8 bytes and work counters equal the
CPU oracle's (oracle/frm_oracle.c, MODE_FRM) bit for bit."""
import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu

W, H = 96, 54
SCENES = list(range(19))


def gpu_render(make, p, width, height, max_steps, flags=0):
    with make(max_steps=max_steps, flags=flags) as r:
        r.resize(width, height)
        r.update_parameters_buffer(p)
        st = r.render(stats=True)
        return r.read_frame(), st


def counters_of(st):
    return [st["pixels"], st["hit_pixels"], st["primary_steps"], st["shadow_steps"],
            st["normal_evals"], st["fractal_bodies"], st["fractal_bailouts"], 0]


@pytest.mark.parametrize("kernel_flags", [frm.FRM_FLAG_PERSISTENT_KERNEL, frm.FRM_FLAG_SIMPLE_KERNEL], ids=["persistent", "simple"])
@pytest.mark.parametrize("scene", SCENES)
def test_all_scenes_bit_exact(gpu_renderer_factory, oracle, scene, kernel_flags):
    for iters, time in ((0, 0.0), (3, 3.2175055), (6, 1.0)):
        p = params_for(scene, iters, time, W, H)
        img, st = gpu_render(gpu_renderer_factory, p, W, H, 128, kernel_flags)
        ref = oracle.render(p, W, H, 128)
        diff = np.any(img != ref["rgba"], axis=-1)
        assert not diff.any(), f"scene {scene} N={iters} t={time}: {diff.sum()} pixels differ"
        assert counters_of(st) == [int(c) for c in ref["counters"]]


@pytest.mark.parametrize("kernel_flags", [frm.FRM_FLAG_PERSISTENT_KERNEL, frm.FRM_FLAG_SIMPLE_KERNEL], ids=["persistent", "simple"])
def test_headline_mandelbulb_bit_exact(gpu_renderer_factory, oracle, kernel_flags):
    for pose in ("P0", "P1", "P2"):
        p = params_for(18, 12, frm.POWER8_TIME, 192, 108, pose=pose)
        img, st = gpu_render(gpu_renderer_factory, p, 192, 108, 256, kernel_flags)
        ref = oracle.render(p, 192, 108, 256)
        assert np.array_equal(img, ref["rgba"]), pose
        assert counters_of(st) == [int(c) for c in ref["counters"]]


@pytest.mark.parametrize("kernel_flags", [0, frm.FRM_FLAG_PERSISTENT_KERNEL], ids=["auto", "persistent"])
def test_sphere_extension_c1(gpu_renderer_factory, oracle, kernel_flags):
    p = params_for(0, 0, 0.0, 256, 256)
    img, st = gpu_render(gpu_renderer_factory, p, 256, 256, 64, frm.FRM_FLAG_SCENE_SPHERE | kernel_flags)
    ref = oracle.render(p, 256, 256, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)
    assert np.array_equal(img, ref["rgba"])
    assert counters_of(st) == [int(c) for c in ref["counters"]]


@pytest.mark.parametrize("kernel_flags", [frm.FRM_FLAG_PERSISTENT_KERNEL, 0], ids=["persistent", "auto"])
def test_ragged_sizes_and_edge_params(gpu_renderer_factory, oracle, kernel_flags):
    cases = [(1, 1, 18, 12), (7, 5, 0, 4), (33, 17, 15, 5), (130, 9, 16, 3), (9, 130, 18, 8)]
    for w, h, scene, iters in cases:
        p = params_for(scene, iters, 3.2175055, w, h)
        img, st = gpu_render(gpu_renderer_factory, p, w, h, 200, kernel_flags)
        ref = oracle.render(p, w, h, 200)
        assert np.array_equal(img, ref["rgba"]), (w, h, scene)
    # out-of-range scene index -> scene 0 (`case 0, default`); huge Sierpinski N wraps
    for scene, iters in ((19, 3), (1000, 2), (15, 33), (15, 31)):
        p = params_for(scene, iters, 0.5, 40, 24)
        img, _ = gpu_render(gpu_renderer_factory, p, 40, 24, 100, kernel_flags)
        ref = oracle.render(p, 40, 24, 100)
        assert np.array_equal(img, ref["rgba"]), (scene, iters)


def test_camera_inside_geometry(gpu_renderer_factory, oracle):
    # default reference pose (0,0,-1) lies inside the Mandelbulb: step 0 hits at t = 0
    p = params_for(18, 12, frm.POWER8_TIME, 64, 36)
    p.update_camera(frm.Camera((0.0, 0.0, -1.0), 0.0, 0.0))
    p2 = params_for(0, 3, 0.0, 64, 36)
    p2.update_camera(frm.Camera((0.1, 0.1, 0.1), 0.3, -0.2))
    for q in (p, p2):
        img, _ = gpu_render(gpu_renderer_factory, q, 64, 36, 64, frm.FRM_FLAG_PERSISTENT_KERNEL)
        ref = oracle.render(q, 64, 36, 64)
        assert np.array_equal(img, ref["rgba"])


def test_scheduling_history_does_not_change_bytes(gpu_renderer_factory, oracle):
    """Frames after the first fetch tiles most-expensive-first (previous frame's costs);
    the bytes and counters must not change, also after a parameter change (stale order)."""
    p = params_for(18, 12, frm.POWER8_TIME, 200, 120)
    q = params_for(18, 8, 1.0, 200, 120, pose="P2")
    ref_p = oracle.render(p, 200, 120, 256)
    ref_q = oracle.render(q, 200, 120, 256)
    with gpu_renderer_factory(max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(200, 120)
        for params, ref in ((p, ref_p), (p, ref_p), (q, ref_q), (q, ref_q), (p, ref_p)):
            r.update_parameters_buffer(params)
            st = r.render()
            assert np.array_equal(r.read_frame(), ref["rgba"])
            assert counters_of(st) == [int(c) for c in ref["counters"]]


def test_kernel_choice(gpu_renderer_factory):
    """Without a kernel flag a launch below one resident persistent grid of pixels runs the
    simple kernel (frm_kernel_for_pixels); the flags force either; both flags or an unknown
    flag are refused at create."""
    with gpu_renderer_factory() as r:
        assert r.kernel_for(256 * 256) == "simple"
        assert r.kernel_for(1920 * 1080) == "persistent"
        assert r.kernel_for(3840 * 2160) == "persistent"
    with gpu_renderer_factory(flags=frm.FRM_FLAG_SIMPLE_KERNEL) as r:
        assert r.kernel_for(3840 * 2160) == "simple"
    with gpu_renderer_factory(flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        assert r.kernel_for(1) == "persistent"
    for bad in (frm.FRM_FLAG_SIMPLE_KERNEL | frm.FRM_FLAG_PERSISTENT_KERNEL, 0x80):
        with pytest.raises(frm.FrmError):
            gpu_renderer_factory(flags=bad)


@pytest.mark.parametrize("scene,iters,time", [(18, 12, frm.POWER8_TIME), (0, 3, 0.0)], ids=["mandelbulb", "menger"])
def test_step0_once_per_frame_edge_cases(gpu_renderer_factory, oracle, scene, iters, time):
    """Step 0 of the primary rays is evaluated once per frame on the host (frm_kernels.hip
    first_steps) and skipped per pixel only when it neither hits nor ends the march and the
    origin has no -0 component. Each case below takes the other branch or an edge of it; bytes
    and counters equal the oracle's either way."""
    cases = [
        ((-0.0, 0.0, -1.6), 0.0, 0.0, 64),    # -0 component: 0 * d would follow d's sign, no skip
        ((0.0, -0.0, -1.6), 0.2, 0.1, 64),
        ((0.0, 0.0, -1.6), 0.0, 0.0, 1),      # one step: step 0 ends the march, no skip
        ((0.0, 0.0, -1.6), 0.0, 0.0, 2),      # two steps: skip, then the last step
        ((0.0, 0.0, -1500.0), 0.0, 0.0, 64),  # step 0's distance beyond MAX_TOTAL_DISTANCE: no skip
        ((0.3, -0.2, -2.5), 0.4, -0.3, 64),   # no zero component
    ]
    for pos, yaw, pitch, steps in cases:
        p = params_for(scene, iters, time, 48, 27)
        p.update_camera(frm.Camera(pos, yaw, pitch))
        img, st = gpu_render(gpu_renderer_factory, p, 48, 27, steps, frm.FRM_FLAG_PERSISTENT_KERNEL)
        ref = oracle.render(p, 48, 27, steps)
        assert np.array_equal(img, ref["rgba"]), (pos, steps)
        assert counters_of(st) == [int(c) for c in ref["counters"]], (pos, steps)
