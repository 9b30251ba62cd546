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


class HeldKeys:
    """Held-key bits of src/held_keys.rs:3-19 (FRM_KEY_* in include/frm.h)."""

    MOVE_FORWARD = 1 << 0
    MOVE_BACKWARD = 1 << 1
    MOVE_RIGHT = 1 << 2
    MOVE_LEFT = 1 << 3
    MOVE_UP = 1 << 4
    MOVE_DOWN = 1 << 5
    PITCH_UP = 1 << 6
    PITCH_DOWN = 1 << 7
    YAW_RIGHT = 1 << 8
    YAW_LEFT = 1 << 9


class Camera:
    """`Camera` of src/camera.rs over libfrm's host restatement (frm_camera_*): the pose
    (position, yaw, pitch) and the movement / orbit / lock-mode controller. Keyboard and
    mouse input become explicit arguments (held-key bits, seconds, cursor pixels)."""

    LOCK_YAW_MODES = ("None", "Inwards", "Right", "Outwards", "Left")  # camera.rs:16-23

    def __init__(self, position=(0.0, 0.0, -1.0), yaw=0.0, pitch=0.0):
        self.raw = _lib.FrmCamera()
        _lib.load().frm_camera_default(ctypes.byref(self.raw))  # camera.rs:176-188
        self.position = position
        self.yaw = yaw
        self.pitch = pitch

    @property
    def position(self):
        return tuple(self.raw.position)

    @position.setter
    def position(self, v):
        self.raw.position = (ctypes.c_float * 3)(*(float(x) for x in v))

    @property
    def yaw(self):
        return self.raw.yaw

    @yaw.setter
    def yaw(self, v):
        self.raw.yaw = float(v)

    @property
    def pitch(self):
        return self.raw.pitch

    @pitch.setter
    def pitch(self, v):
        self.raw.pitch = float(v)

    @property
    def movement_per_second(self):
        return self.raw.movement_per_second

    @property
    def orbit_angle_per_second(self):
        return self.raw.orbit_angle_per_second

    @property
    def lock_yaw_mode(self):
        return self.LOCK_YAW_MODES[self.raw.lock_yaw_mode]

    @property
    def lock_pitch(self):
        return bool(self.raw.lock_pitch)

    def forward(self):  # camera.rs:48-50 (yaw_matrix().z)
        return (math.sin(self.yaw), 0.0, math.cos(self.yaw))

    # camera.rs:100-105
    def update(self, held_keys, seconds):
        _lib.load().frm_camera_update(ctypes.byref(self.raw), int(held_keys), float(seconds))

    # camera.rs:60-62
    def update_speed(self, delta):
        _lib.load().frm_camera_update_speed(ctypes.byref(self.raw), float(delta))

    # camera.rs:64-69
    def update_orbit_speed(self, delta):
        _lib.load().frm_camera_update_orbit_speed(ctypes.byref(self.raw), float(delta))

    # camera.rs:71-73
    def reset_orbit_speed(self):
        _lib.load().frm_camera_reset_orbit_speed(ctypes.byref(self.raw))

    # camera.rs:75-77
    def toggle_lock_pitch(self):
        _lib.load().frm_camera_toggle_lock_pitch(ctypes.byref(self.raw))

    # camera.rs:79-98
    def cycle_lock_yaw_mode(self, backwards=False):
        _lib.load().frm_camera_cycle_lock_yaw_mode(ctypes.byref(self.raw), 1 if backwards else 0)

    # camera.rs:151-154
    def rotate_from_cursor_movement(self, yaw_pixels, pitch_pixels):
        _lib.load().frm_camera_rotate_from_cursor(ctypes.byref(self.raw), float(yaw_pixels), float(pitch_pixels))

    def __repr__(self):
        return (f"Camera(position={self.position}, yaw={self.yaw}, pitch={self.pitch}, "
                f"lock_yaw={self.lock_yaw_mode}, lock_pitch={self.lock_pitch})")


class Timing:
    """`Timing` of src/timing.rs with the frame time passed in (no wall clock, no FPS log)."""

    def __init__(self):
        self.raw = _lib.FrmTiming()
        _lib.load().frm_timing_init(ctypes.byref(self.raw))  # timing.rs:13-21

    @property
    def time_factor(self):
        return self.raw.time_factor

    # timing.rs:23-30: parameters.time += time_factor * delta; returns delta
    def update(self, parameters, delta_seconds):
        return _lib.load().frm_timing_update(ctypes.byref(self.raw), ctypes.byref(parameters.raw),
                                             float(delta_seconds))

    # timing.rs:32-34
    def update_time_factor(self, delta):
        _lib.load().frm_timing_update_time_factor(ctypes.byref(self.raw), float(delta))

    # timing.rs:36-38
    def stop_time(self):
        _lib.load().frm_timing_stop_time(ctypes.byref(self.raw))
