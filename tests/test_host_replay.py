"""The product's per-pixel source (csrc/frm_scene.h + frm_math.h + frm_host.cpp), compiled
for the CPU, equals the independent oracle bit for bit: frames, counters, DEs, builtins.
(The GPU tests then check that the gfx950 build of the same source does too.)"""
import ctypes

import numpy as np
import pytest

import frm
from helpers import hr_render, hr_scene_de, params_for, same_bits


@pytest.mark.parametrize("scene", range(19))
def test_frames_and_counters(host_replay, oracle, scene):
    for iters, time in ((0, 0.0), (3, 3.2175055), (6, 1.0)):
        p = params_for(scene, iters, time, 72, 40)
        img, c = hr_render(host_replay, p, 72, 40, 128)
        ref = oracle.render(p, 72, 40, 128)
        assert np.array_equal(img, ref["rgba"]), (scene, iters, time)
        assert np.array_equal(c, ref["counters"]), (scene, iters, time)


def test_sphere_and_rows_subset(host_replay, oracle):
    p = params_for(0, 0, 0.0, 64, 64)
    img, c = hr_render(host_replay, p, 64, 64, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)
    ref = oracle.render(p, 64, 64, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)
    assert np.array_equal(img, ref["rgba"]) and np.array_equal(c, ref["counters"])
    p = params_for(18, 12, frm.POWER8_TIME, 384, 216)
    rows = [0, 50, 107, 108, 215]
    img, c = hr_render(host_replay, p, 384, 216, 256, rows=rows)
    ref = oracle.render(p, 384, 216, 256, rows=rows)
    assert np.array_equal(img, ref["rgba"]) and np.array_equal(c, ref["counters"])


@pytest.mark.parametrize("scene", [0, 4, 9, 12, 14, 15, 16, 17, 18])
def test_scene_de(host_replay, oracle, scene):
    pts = np.random.default_rng(scene).uniform(-1.6, 1.6, (5000, 3)).astype(np.float32)
    for iters in (0, 2, 5, 9):
        p = params_for(scene, iters, 2.5, 8, 8)
        d, col = hr_scene_de(host_replay, p, pts)
        rd, rcol, _ = oracle.scene_de(p, pts)
        assert same_bits(d, rd) and same_bits(col, rcol), (scene, iters)


@pytest.mark.parametrize("fn,name", [(0, "sin"), (1, "cos"), (2, "acos"), (3, "atan2"), (4, "log"),
                                     (5, "log2"), (6, "exp2"), (7, "pow")])
def test_builtins(host_replay, oracle, fn, name):
    rng = np.random.default_rng(fn)
    a = np.concatenate([rng.uniform(-40, 40, 50000), np.exp(rng.uniform(-87, 87, 50000)),
                        [0, -0.0, np.inf, -np.inf, np.nan, 1, -1, 1e-45]]).astype(np.float32)
    b = rng.uniform(-5, 20, a.size).astype(np.float32)
    out = np.zeros_like(a)
    host_replay.hr_math(fn, ctypes.c_void_p(a.ctypes.data), ctypes.c_void_p(b.ctypes.data), a.size,
                        ctypes.c_void_p(out.ctypes.data))
    ref = oracle.math_fn(name, a, b)
    assert same_bits(out, ref)
