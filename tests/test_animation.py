"""§8(f) row 2 — the animation driver: libfrm's host restatement of src/camera.rs and
src/timing.rs (frm_camera_* / frm_timing_*), checked step by step against an independent
numpy-float32 restatement of the same Rust code written here, plus the properties the
reference's lock modes and orbit guarantee. Host code only: runs without a GPU."""
import ctypes
import math

import numpy as np
import pytest

import frm
from frm import HeldKeys

f32 = np.float32
FULL_TURN = f32(2 * math.pi)
MAX_PITCH = f32(math.pi / 2)


def lqd(current, delta):  # utils.rs:62-69
    current, delta = f32(current), f32(delta)
    factor = f32(0.025) if current == 0 else f32(min(max(abs(current), f32(0.0001)), f32(0.1)))
    return f32(f32(f32(0.2) * delta) * factor)


def mag(keys, pos, neg):  # held_keys.rs:32-34
    return f32(int(bool(keys & pos)) - int(bool(keys & neg)))


def ref_step(state, keys, seconds):
    """camera.rs:100-147 in float32, cgmath operation order."""
    px, py, pz, pitch, yaw, mps, orbit, lock_yaw, lock_pitch = state
    seconds = f32(seconds)
    sy, cy = f32(np.sin(yaw)), f32(np.cos(yaw))
    fm = mag(keys, HeldKeys.MOVE_FORWARD, HeldKeys.MOVE_BACKWARD)
    rm = mag(keys, HeldKeys.MOVE_RIGHT, HeldKeys.MOVE_LEFT)
    um = mag(keys, HeldKeys.MOVE_UP, HeldKeys.MOVE_DOWN)
    mv = [f32(f32(sy * fm + cy * rm) + f32(0) * um), f32(f32(f32(0) * fm + f32(0) * rm) + um),
          f32(f32(cy * fm + f32(-sy) * rm) + f32(0) * um)]
    if any(v != 0 for v in mv):
        length = f32(np.sqrt(f32(f32(mv[0] * mv[0] + mv[1] * mv[1]) + mv[2] * mv[2])))
        s = f32(f32(mps * seconds) / length)
        px, py, pz = f32(px + mv[0] * s), f32(py + mv[1] * s), f32(pz + mv[2] * s)
    rot = f32(f32(0.5) * seconds)
    pitch = f32(min(max(f32(pitch + f32(rot * mag(keys, HeldKeys.PITCH_DOWN, HeldKeys.PITCH_UP))), -MAX_PITCH),
                    MAX_PITCH))
    yaw = f32(np.fmod(f32(yaw + f32(rot * mag(keys, HeldKeys.YAW_RIGHT, HeldKeys.YAW_LEFT))), FULL_TURN))
    a = f32(orbit * seconds)
    so, co = f32(np.sin(a)), f32(np.cos(a))
    px, py, pz = (f32(f32(co * px + f32(0) * py) + so * pz), f32(f32(f32(0) * px + py) + f32(0) * pz),
                  f32(f32(f32(-so) * px + f32(0) * py) + co * pz))
    if lock_yaw:
        offset = {1: -FULL_TURN / f32(2), 2: -FULL_TURN / f32(4), 3: f32(0), 4: FULL_TURN / f32(4)}[lock_yaw]
        yaw = f32(f32(np.arctan2(px, pz)) + f32(offset))
    if lock_pitch:
        pitch = f32(np.arctan2(py, f32(np.sqrt(f32(px * px + pz * pz)))))
    return [px, py, pz, pitch, yaw, mps, orbit, lock_yaw, lock_pitch]


def state_of(cam):
    r = cam.raw
    return [f32(r.position[0]), f32(r.position[1]), f32(r.position[2]), f32(r.pitch), f32(r.yaw),
            f32(r.movement_per_second), f32(r.orbit_angle_per_second), r.lock_yaw_mode, r.lock_pitch]


def test_default_camera_and_timing():
    c = frm.Camera()
    assert c.position == (0.0, 0.0, -1.0) and c.yaw == 0.0 and c.pitch == 0.0  # camera.rs:176-188
    assert c.movement_per_second == 1.0 and c.orbit_angle_per_second == 0.0
    assert c.lock_yaw_mode == "None" and not c.lock_pitch
    assert frm.Timing().time_factor == 1.0  # timing.rs:13-21


def test_update_matches_restatement_step_by_step():
    rng = np.random.default_rng(3)
    cam = frm.Camera(position=(0.3, -0.2, -1.7), yaw=0.4, pitch=-0.1)
    for step in range(2000):
        if step % 97 == 0:
            cam.cycle_lock_yaw_mode(backwards=bool(rng.integers(2)))
        if step % 131 == 0:
            cam.toggle_lock_pitch()
        if step % 53 == 0:
            cam.update_orbit_speed(float(rng.normal(0, 20)))
        if step % 71 == 0:
            cam.update_speed(float(rng.normal(0, 5)))
        keys = int(rng.integers(0, 1 << 10))
        seconds = float(rng.uniform(0, 0.05))
        before = state_of(cam)
        want = ref_step(before, keys, seconds)
        cam.update(keys, seconds)
        got = state_of(cam)
        np.testing.assert_allclose(np.array(got[:5], np.float64), np.array(want[:5], np.float64),
                                   rtol=2e-6, atol=2e-6, err_msg=f"step {step}")
        assert got[5:] == want[5:]


def test_lock_modes_and_orbit_properties():
    cam = frm.Camera(position=(1.5, 0.9, -1.5))
    cam.cycle_lock_yaw_mode()  # None -> Inwards
    assert cam.lock_yaw_mode == "Inwards"
    cam.toggle_lock_pitch()
    cam.update_orbit_speed(30.0)
    r0 = math.hypot(cam.position[0], cam.position[2])
    for _ in range(200):
        cam.update(0, 1 / 60)
        x, y, z = cam.position
        # orbit: rotation about +y keeps height and radius
        assert y == pytest.approx(0.9, abs=1e-6)
        assert math.hypot(x, z) == pytest.approx(r0, rel=1e-5)
        # inwards lock: the forward vector points at the y axis
        fx, _, fz = cam.forward()
        assert fx * x + fz * z == pytest.approx(-r0, rel=1e-5)
        # pitch lock: pitch = atan2(y, radius)
        assert cam.pitch == pytest.approx(math.atan2(y, math.hypot(x, z)), abs=1e-6)
    assert cam.orbit_angle_per_second != 0.0
    cam.reset_orbit_speed()
    assert cam.orbit_angle_per_second == 0.0


def test_cycle_order_clamp_and_cursor():
    cam = frm.Camera()
    order = [cam.lock_yaw_mode]
    for _ in range(5):
        cam.cycle_lock_yaw_mode()
        order.append(cam.lock_yaw_mode)
    assert order == ["None", "Inwards", "Right", "Outwards", "Left", "None"]  # camera.rs:90-96
    cam.cycle_lock_yaw_mode(backwards=True)
    assert cam.lock_yaw_mode == "Left"  # camera.rs:82-88
    cam.cycle_lock_yaw_mode()  # back to None
    cam.rotate_from_cursor_movement(0.0, 1e6)  # 0.0003 rad per pixel, clamped to pi/2
    assert cam.pitch == pytest.approx(float(MAX_PITCH))
    cam.rotate_from_cursor_movement(1000.0, 0.0)
    assert cam.yaw == pytest.approx(0.3, abs=1e-6)
    cam.update(HeldKeys.YAW_RIGHT, 100.0)  # +50 rad, kept in (-2pi, 2pi) by fmod
    assert abs(cam.yaw) < float(FULL_TURN)
    assert cam.yaw == pytest.approx(math.fmod(0.3 + 50.0, 2 * math.pi), abs=1e-5)


def test_movement_speed_and_direction():
    cam = frm.Camera(yaw=math.pi / 2)  # forward = +x
    cam.update(HeldKeys.MOVE_FORWARD | HeldKeys.MOVE_BACKWARD, 1.0)  # cancels: no move
    assert cam.position == (0.0, 0.0, -1.0)
    cam.update(HeldKeys.MOVE_FORWARD, 0.5)
    assert cam.position[0] == pytest.approx(0.5, abs=1e-6)
    cam.update_speed(10.0)  # x exp(1)
    assert cam.movement_per_second == pytest.approx(math.e, rel=1e-6)
    before = cam.position
    cam.update(HeldKeys.MOVE_FORWARD | HeldKeys.MOVE_UP, 1.0)  # diagonal, length = speed
    d = np.subtract(cam.position, before)
    assert np.linalg.norm(d) == pytest.approx(math.e, rel=1e-5)
    assert d[1] == pytest.approx(math.e / math.sqrt(2), rel=1e-5)


def test_timing_drives_parameters_time():
    p = frm.Parameters()
    t = frm.Timing()
    assert t.update(p, 0.25) == pytest.approx(0.25)
    assert p.time == pytest.approx(0.25)
    t.update_time_factor(10.0)  # += 0.2 * 10 * clamp(1, 1e-4, 0.1) = 0.2
    assert t.time_factor == pytest.approx(1.2)
    t.update(p, 0.5)
    assert p.time == pytest.approx(0.25 + 0.6)
    t.stop_time()
    t.update(p, 1.0)
    assert p.time == pytest.approx(0.85)
    t.update_time_factor(1.0)  # from 0: 0.2 * 1 * 0.025
    assert t.time_factor == pytest.approx(0.005)


def test_parameters_follow_the_camera():
    cam = frm.Camera(position=(1.5, 0.9, -1.5), yaw=-math.pi / 4, pitch=0.4)
    a, b = frm.Parameters(), frm.Parameters()
    a.update_camera(cam)
    frm.load().frm_parameters_update_camera_from(ctypes.byref(b.raw), ctypes.byref(cam.raw))
    assert a.to_bytes() == b.to_bytes()
