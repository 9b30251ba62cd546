"""Host-side mirror of src/parameters.rs and Camera::to_matrix (src/camera.rs:26-44)."""
import math

import numpy as np
import pytest

import frm


def test_default_is_zeroed():
    p = frm.Parameters()
    assert p.to_bytes() == bytes(96)  # #[derive(Default)]


@pytest.mark.parametrize("w,h", [(1920, 1080), (1080, 1920), (256, 256), (160, 90), (7, 3)])
def test_update_aspect(w, h):  # parameters.rs:18-21
    p = frm.Parameters()
    p.update_aspect(w, h)
    m = np.float32(min(w, h))
    assert p.aspect_scale == (float(np.float32(w) / m), float(np.float32(h) / m))


def test_update_num_iterations_saturates():  # u32::saturating_add_signed
    p = frm.Parameters()
    p.update_num_iterations(-1)
    assert p.num_iterations == 0
    p.update_num_iterations(5)
    assert p.num_iterations == 5
    p.num_iterations = 2**32 - 2
    p.update_num_iterations(10)
    assert p.num_iterations == 2**32 - 1


@pytest.mark.parametrize("start,delta,expect", [(0, -1, 18), (18, 1, 0), (5, 40, 7), (3, -22, 0), (0, -19 * 5 - 1, 18)])
def test_update_scene_index_rem_euclid(start, delta, expect):  # parameters.rs:37-40
    p = frm.Parameters()
    p.scene_index = start
    p.update_scene_index(delta)
    assert p.scene_index == expect


def test_update_time_accumulates_in_f32():
    p = frm.Parameters()
    for _ in range(10):
        p.update_time(0.1)
    t = np.float32(0)
    for _ in range(10):
        t = np.float32(t + np.float32(0.1))
    assert p.time == float(t)


def cgmath_matrix(pos, yaw, pitch):
    """Independent restatement: T(pos) * Ry(yaw) * Rx(pitch) (cgmath, column vectors)."""
    sy, cy, sx, cx = (np.float32(math.sin(yaw)), np.float32(math.cos(yaw)),
                      np.float32(math.sin(pitch)), np.float32(math.cos(pitch)))
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = pos
    Ry = np.array([[cy, 0, sy, 0], [0, 1, 0, 0], [-sy, 0, cy, 0], [0, 0, 0, 1]], np.float32)
    Rx = np.array([[1, 0, 0, 0], [0, cx, -sx, 0], [0, sx, cx, 0], [0, 0, 0, 1]], np.float32)
    return (T @ Ry @ Rx).astype(np.float32)


@pytest.mark.parametrize("pose", ["P0", "P1", "P2"])
def test_update_camera_matches_cgmath(pose):  # parameters.rs:23-25
    pos, yaw, pitch = frm.POSES[pose]
    p = frm.Parameters()
    p.update_camera(frm.Camera(pos, yaw, pitch))
    C = cgmath_matrix(pos, yaw, pitch)
    # uploaded transposed, column-major: camera_matrix[4*row + col] = C[row][col]
    got = np.array(p.camera_matrix, np.float32).reshape(4, 4)
    np.testing.assert_allclose(got, C, rtol=0, atol=2e-7)


def test_default_camera_pose():
    p = frm.Parameters()
    p.update_camera(frm.Camera())  # camera.rs: position (0,0,-1), yaw = pitch = 0
    assert p.camera_matrix == [1, 0, 0, 0, 0, 1, -0.0, 0, -0.0, 0, 1, -1, 0, 0, 0, 1]


def test_forward_vector_convention():
    cam = frm.Camera((0, 0, 0), math.pi / 2, 0)  # yaw_matrix().z = (sin yaw, 0, cos yaw)
    f = cam.forward()  # yaw is an f32 (camera.rs:13): cos(f32(pi/2)) = -4.37e-8
    assert abs(f[0] - 1) < 1e-12 and abs(f[2]) < 1e-7


def test_parameters_blob_roundtrip():
    p = frm.make_parameters(frm.WORKLOADS["C2"])
    q = frm.Parameters.from_bytes(p.to_bytes())
    assert q.to_bytes() == p.to_bytes()
    assert q.scene_index == 18 and q.num_iterations == 12
