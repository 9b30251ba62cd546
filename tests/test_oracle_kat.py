"""Closed-form known answers for the CPU oracle (what pins it, since the reference has
no tests or golden outputs). Each case cites the fragment.wgsl lines it exercises."""
import math
import os
import sys

import numpy as np
import pytest

import frm
from helpers import params_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f32 = np.float32


def de(oracle, scene, iters, pts, time=0.0, flags=0):
    p = params_for(scene, iters, time, 8, 8)
    return oracle.scene_de(p, np.asarray(pts, np.float32), flags=flags)


def test_box_closed_form(oracle):  # Menger N=0 == box(p, 0.5), fragment.wgsl:138-141,204
    d, col, _ = de(oracle, 0, 0, [[1, 0, 0], [0, 0, 0], [1, 1, 1], [0.25, 0.1, -0.3], [0, 2, 0]])
    assert d[0] == f32(0.5) and d[1] == f32(-0.5) and d[4] == f32(1.5)
    assert abs(d[2] - math.sqrt(0.75)) < 1e-7
    assert d[3] == f32(abs(f32(-0.3))) - f32(0.5)  # interior: max component of |p| - 0.5
    assert np.allclose(col[1], [0.5, 0.5, 0.5])  # colorize(p) = min(1, p + 0.5)


def test_menger_center_is_hollow(oracle):  # first cross removes the cube centre
    d, _, _ = de(oracle, 0, 1, [[0, 0, 0]])
    assert d[0] == f32(1.0 / 6.0)  # max(-0.5, -(0 - 1/6)/1)


def test_sphere_extension(oracle):
    pts = np.random.default_rng(3).uniform(-2, 2, (1000, 3)).astype(np.float32)
    d, _, _ = de(oracle, 0, 0, pts, flags=frm.FRM_FLAG_SCENE_SPHERE)
    ref = np.linalg.norm(pts.astype(np.float64), axis=1) - 0.5
    assert np.max(np.abs(d - ref)) < 3e-7


def test_sierpinski_n0_is_one_tetrahedron(oracle):  # fragment.wgsl:151-157,164-188 with N=0
    h = 4 / math.sqrt(6)
    top = np.array([0, h * 0.5, 0])
    s = 0.5
    a = top + s * np.array([-1, -h, -1 / math.sqrt(3)])
    b = top + s * np.array([1, -h, -1 / math.sqrt(3)])
    c = top + s * np.array([0, -h, 2 / math.sqrt(3)])

    def pn(a, b, c):
        n = np.cross(c - a, b - a)
        return n / np.linalg.norm(n)

    planes = [(top, pn(top, a, b)), (top, pn(top, b, c)), (top, pn(top, c, a)), (a, pn(a, c, b))]
    pts = np.random.default_rng(5).uniform(-1, 1, (2000, 3))
    q = pts + np.array([0, h * 0.25, 0])
    ref = np.max([(q - an) @ n for an, n in planes], axis=0)
    d, _, _ = de(oracle, 15, 0, pts.astype(np.float32))
    assert np.max(np.abs(d - ref)) < 2e-6


def test_mandelbulb_far_point_bails_out_immediately(oracle):  # fragment.wgsl:245-249,269
    d, _, cnt = de(oracle, 18, 12, [[200, 0, 0], [0, -150, 0]], time=frm.POWER8_TIME)
    assert cnt[0] == 0 and cnt[1] == 2  # no bodies, two bailouts
    assert abs(d[0] - 0.5 * math.log(200) * 200) < 2e-4
    assert abs(d[1] - 0.5 * math.log(150) * 150) < 2e-4


def test_animate_between_and_scene_table(oracle):  # fragment.wgsl:18-82
    info = oracle.frame_info(params_for(18, 12, frm.POWER8_TIME, 8, 8))
    assert info["family"] == 3 and info["mb_power"] == 8.0  # power 8 exactly
    assert oracle.frame_info(params_for(18, 12, 0.0, 8, 8))["mb_power"] == 6.5  # 4 + 5*0.5
    assert oracle.frame_info(params_for(4, 3, 0.0, 8, 8))["menger_cross"] == f32(1 / 5)
    assert oracle.frame_info(params_for(12, 3, 0.0, 8, 8))["menger_scale"] == 4.0
    for s in (19, 20, 1000, 2**32 - 1):  # `case 0, default`
        i = oracle.frame_info(params_for(s, 3, 0.0, 8, 8))
        assert i["family"] == 0 and i["menger_cross"] == f32(1 / 6) and i["menger_scale"] == 3.0
    assert oracle.frame_info(params_for(16, 3, 0.0, 8, 8))["koch_normal_z"] == f32(math.sqrt(3))


def test_camera_origin_is_translation(oracle):  # transform_position(Position(0)), :319-331
    for pose in ("P0", "P1", "P2"):
        p = params_for(18, 12, 0.0, 8, 8, pose=pose)
        pos = frm.POSES[pose][0]
        assert oracle.frame_info(p)["origin"] == tuple(float(f32(v)) for v in pos)


def test_background_pixels(oracle):  # miss -> BACKGROUND_COLOR (0,0,0), alpha 1
    p = params_for(18, 12, frm.POWER8_TIME, 32, 18, pose="P0")
    p.update_camera(frm.Camera((0, 0, -2.5), math.pi, 0))  # looking away from the fractal
    r = oracle.render(p, 32, 18, 256)
    assert (r["rgba"][..., :3] == 0).all() and (r["rgba"][..., 3] == 255).all()
    assert r["counters"][1] == 0 and r["counters"][3] == 0  # no hits, no shadow rays


def test_camera_inside_geometry_hits_at_step_zero(oracle):  # :289-297 with distance <= 0
    p = params_for(0, 0, 0.0, 16, 16)
    p.update_camera(frm.Camera((0, 0, 0), 0, 0))  # inside the unit box
    r = oracle.render(p, 16, 16, 64, info=True)
    assert r["counters"][1] == 256 and r["counters"][2] == 256  # every pixel hits at step 0
    assert ((r["info"] >> 8) == 0).all()


def test_nan_shadow_class_renders_zero(oracle):  # 0 * 32 * -inf = NaN, :292,344,346
    p = params_for(18, 12, frm.POWER8_TIME, 160, 90)
    r = oracle.render(p, 160, 90, 256, info=True, linear=True)
    nan = (r["info"] & oracle.INFO_NAN) != 0
    hits = (r["info"] & oracle.INFO_HIT) != 0
    assert 0.01 < nan.sum() / hits.sum() < 0.08  # survey: ~4.3% of Mandelbulb hit pixels
    assert (r["rgba"][nan][:, :3] == 0).all()


def test_srgb_thresholds_match_mpmath_generator(oracle):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_srgb_table
    ref = np.array(gen_srgb_table.thresholds()[1:], np.float32)
    assert np.array_equal(oracle.srgb_thresholds()[1:], ref)


def test_srgb_known_codes(oracle):
    c = np.array([0, 1, 0.5, 0.0031308, np.nan, -1, 2, 0.2, 1e-30], np.float32)
    assert list(oracle.encode_srgb(c)) == [0, 255, 188, 10, 0, 0, 255, 124, 0]
    x = np.random.default_rng(1).uniform(0, 1, 200000).astype(np.float32)
    xd = x.astype(np.float64)
    s = np.where(xd <= 0.0031308, 12.92 * xd, 1.055 * xd ** (1 / 2.4) - 0.055) * 255
    ok = np.abs(s - np.round(s)) < 0.5 - 1e-9  # away from exact ties
    assert np.array_equal(oracle.encode_srgb(x)[ok], np.floor(s[ok] + 0.5).astype(np.uint8))
