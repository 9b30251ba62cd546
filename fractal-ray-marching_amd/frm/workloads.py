"""Fixed benchmark poses and the BASELINE.json configurations."""
import math
from dataclasses import dataclass

from .parameters import Camera, Parameters, Timing

# asin(0.6)/0.2: animate_between(4, 9) == 8.0 exactly in f32 -> Mandelbulb power 8.
POWER8_TIME = 3.2175055

POSES = {
    # name: (position, yaw, pitch)
    "P0": ((0.0, 0.0, -2.5), 0.0, 0.0),
    "P1": ((0.0, 0.0, -1.6), 0.0, 0.0),
    # yaw-lock "inwards" + pitch-lock (camera.rs:129-147) at (1.5, 0.9, -1.5)
    "P2": ((1.5, 0.9, -1.5), -math.pi / 4, 0.4),
}


@dataclass(frozen=True)
class Workload:
    name: str
    width: int
    height: int
    scene: int
    iters: int
    max_steps: int
    time: float
    sphere: bool = False
    note: str = ""
    animated: bool = False  # frame k renders at time + k/60
    fly: bool = False  # frame k orbits the camera (frame_sequence)

    @property
    def moving(self):
        """Frames differ (time or camera): one frame per launch, history from another frame."""
        return self.animated or self.fly


WORKLOADS = {
    "C1": Workload("C1-sphere-256", 256, 256, 0, 0, 64, 0.0, sphere=True,
                   note="256x256 single-sphere SDF (build extension), 64 steps"),
    "C2": Workload("C2-mandelbulb-1080p", 1920, 1080, 18, 12, 256, POWER8_TIME,
                   note="1920x1080 Mandelbulb power 8, 12 iters, 256 steps"),
    "C3": Workload("C3-menger-4k", 3840, 2160, 0, 8, 512, 0.0,
                   note="3840x2160 Menger sponge, 8 iters, 512 steps"),
    "C4": Workload("C4-mandelbulb-8k", 7680, 4320, 18, 16, 512, POWER8_TIME,
                   note="7680x4320 Mandelbulb, 16 iters, 512 steps"),
    "C5": Workload("C5-mandelbulb-16k", 16384, 16384, 18, 20, 1024, POWER8_TIME,
                   note="16384x16384 animated Mandelbulb, 20 iters, 1024 steps", animated=True),
    "HEADLINE": Workload("headline-mandelbulb-4k", 3840, 2160, 18, 12, 256, POWER8_TIME,
                         note="3840x2160 Mandelbulb power 8, 12 iters, 256 steps"),
    # the reference's own frame loop on the headline scene: every frame Timing::update advances
    # the time (so the Mandelbulb power moves, fragment.wgsl:75,80-82) and Camera::update orbits
    # the camera about +y with the yaw locked inwards (camera.rs:100-147); frame 0 is the
    # headline frame itself
    "HEADLINE_FLY": Workload("headline-fly-4k", 3840, 2160, 18, 12, 256, POWER8_TIME,
                             note="3840x2160 Mandelbulb from power 8, 12 iters, 256 steps; time += 1/60 and "
                             "a 0.5 rad/s yaw-locked orbit per frame", animated=True, fly=True),
    # its two halves (scheduling diagnostics, tools/fly_probe.py): the time alone, the orbit alone
    "HEADLINE_TIME": Workload("headline-time-4k", 3840, 2160, 18, 12, 256, POWER8_TIME,
                              note="HEADLINE_FLY without the orbit (time += 1/60 per frame)", animated=True),
    "HEADLINE_ORBIT": Workload("headline-orbit-4k", 3840, 2160, 18, 12, 256, POWER8_TIME,
                               note="HEADLINE_FLY at a fixed time (the orbit alone)", fly=True),
}

FLY_ORBIT_RAD_PER_S = 0.5  # = camera.rs:46's rotation speed; 0.48 degrees of orbit per 60 Hz frame
FRAME_SECONDS = 1.0 / 60.0


def frame_sequence(w, pose="P1", dt=FRAME_SECONDS, camera=None):
    """Parameters of frames 0, 1, 2, ... of workload `w` as the reference's frame loop
    produces them (InitializedApp::update, initialized_app.rs:43-48: Timing::update, then
    Camera::update and Parameters::update_camera). Frame 0 is make_parameters(w, pose). Fixed
    workloads repeat frame 0; animated ones advance time by dt per frame (timing.rs:23-30); fly
    workloads also orbit the camera at FLY_ORBIT_RAD_PER_S about +y with the yaw locked
    inwards (camera.rs:119-147). camera = (position, yaw, pitch) replaces the pose's camera.
    Yields a fresh Parameters object per frame."""
    p = make_parameters(w, pose=pose)
    pos, yaw, pitch = POSES[pose] if camera is None else camera
    cam = Camera(pos, yaw, pitch)
    p.update_camera(cam)
    if w.fly:
        cam.raw.orbit_angle_per_second = FLY_ORBIT_RAD_PER_S
        cam.raw.lock_yaw_mode = 1  # LockYawMode::Inwards
    clock = Timing()
    while True:
        yield Parameters.from_bytes(p.to_bytes())
        if w.animated:
            clock.update(p, dt)
        if w.fly:
            cam.update(0, dt)
            p.update_camera(cam)


def make_parameters(w, pose="P1", time=None, width=None, height=None):
    """Parameters for workload `w` at a fixed pose (aspect from the frame size)."""
    pos, yaw, pitch = POSES[pose]
    p = Parameters()
    p.update_aspect(width or w.width, height or w.height)
    p.update_camera(Camera(pos, yaw, pitch))
    p.time = w.time if time is None else time
    p.num_iterations = w.iters
    p.scene_index = w.scene
    return p
