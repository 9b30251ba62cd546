"""Host-side mirror of src/parameters.rs (the drop-in uniform) and src/camera.rs's
Camera::to_matrix, driven through libfrm's C helpers so the Python host and a C/C++
host share one implementation."""
import ctypes
import math

from . import _lib


class Parameters:
    """`Parameters` (parameters.rs:6-15) with the reference's mutators (18-40)."""

    NUM_SCENES = _lib.FRM_NUM_SCENES

    def __init__(self):
        self.raw = _lib.FrmParameters()
        _lib.load().frm_parameters_default(ctypes.byref(self.raw))

    # parameters.rs:18-21
    def update_aspect(self, width, height):
        _lib.load().frm_parameters_update_aspect(ctypes.byref(self.raw), width, height)

    # parameters.rs:23-25 (camera.rs:26-44 for the matrix)
    def update_camera(self, camera):
        pos = (ctypes.c_float * 3)(*camera.position)
        _lib.load().frm_parameters_update_camera(ctypes.byref(self.raw), pos, camera.yaw, camera.pitch)

    # parameters.rs:27-29
    def update_time(self, delta):
        _lib.load().frm_parameters_update_time(ctypes.byref(self.raw), delta)

    # parameters.rs:31-33
    def update_num_iterations(self, delta):
        _lib.load().frm_parameters_update_num_iterations(ctypes.byref(self.raw), delta)

    # parameters.rs:37-40
    def update_scene_index(self, delta):
        _lib.load().frm_parameters_update_scene_index(ctypes.byref(self.raw), delta)

    @property
    def time(self):
        return self.raw.time

    @time.setter
    def time(self, v):
        self.raw.time = v

    @property
    def num_iterations(self):
        return self.raw.num_iterations

    @num_iterations.setter
    def num_iterations(self, v):
        self.raw.num_iterations = v

    @property
    def scene_index(self):
        return self.raw.scene_index

    @scene_index.setter
    def scene_index(self, v):
        self.raw.scene_index = v

    @property
    def camera_matrix(self):
        return list(self.raw.camera_matrix)

    @property
    def aspect_scale(self):
        return tuple(self.raw.aspect_scale)

    def to_bytes(self):
        return bytes(ctypes.string_at(ctypes.addressof(self.raw), 96))

    @classmethod
    def from_bytes(cls, b):
        assert len(b) == 96
        p = cls()
        ctypes.memmove(ctypes.addressof(p.raw), bytes(b), 96)
        return p


class Camera:
    """Camera pose of src/camera.rs (position, yaw, pitch); default pose (0,0,-1)."""

    def __init__(self, position=(0.0, 0.0, -1.0), yaw=0.0, pitch=0.0):
        self.position = tuple(float(v) for v in position)
        self.yaw = float(yaw)
        self.pitch = float(pitch)

    def forward(self):  # camera.rs:48-50 (yaw_matrix().z)
        return (math.sin(self.yaw), 0.0, math.cos(self.yaw))

    def __repr__(self):
        return f"Camera(position={self.position}, yaw={self.yaw}, pitch={self.pitch})"
