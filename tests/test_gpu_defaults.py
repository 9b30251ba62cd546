"""GPU parity at the reference's own defaults: 5000 march steps (MAX_ITERATIONS,
fragment.wgsl:4; it also scales the ambient occlusion, fragment.wgsl:289, 342), 1920x1080
(render_texture_config.rs:16-21), and the drop-in binding's context (INTEGRATION.md section 3:
max_steps = 0 = FRM_DEFAULT_MAX_STEPS). Every frame of tests/golden/defaults.json
(tests/golden/make_defaults_golden.py: Parameters::default() seen from Camera::default(); scenes
0, 4, 12, 14, 15, 16, 17, 18 at num_iterations 3, 8, 12 and two times at pose P1; the 4K
headline at 5000 steps) is rendered whole by both kernels and compared with the oracle's
sha256 and work counters. Long shadow marches (up to 5000 steps) and AO at /5000 run here."""
import hashlib
import json
import os

import pytest

import frm

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "defaults.json")


def _golden():
    with open(GOLDEN) as fh:
        return json.load(fh)


def counters_of(st):
    return [st["pixels"], st["hit_pixels"], st["primary_steps"], st["shadow_steps"],
            st["normal_evals"], st["fractal_bodies"], st["fractal_bailouts"], 0]


KEYS = sorted(k for k in _golden() if k != "HEADLINE_5000")


@pytest.mark.parametrize("kernel", ["persistent", "simple"])
def test_defaults_whole_frames(frm_lib, kernel):
    """All 1920x1080 default-step frames through one context per kernel (a resize-free run of
    scene and iteration changes, as the reference's `n`/`+` keys produce); the persistent
    kernel renders every frame twice, the second time in the scheduled order of the first."""
    g = _golden()
    flag = frm.FRM_FLAG_PERSISTENT_KERNEL if kernel == "persistent" else frm.FRM_FLAG_SIMPLE_KERNEL
    bad = []
    with frm.Renderer(device=0, max_steps=0, flags=flag) as r:
        r.resize(1920, 1080)
        for key in KEYS:
            e = g[key]
            assert e["max_steps"] == frm.FRM_DEFAULT_MAX_STEPS and (e["width"], e["height"]) == (1920, 1080)
            r.update_parameters_buffer(frm.Parameters.from_bytes(bytes.fromhex(e["params"])))
            if kernel == "persistent":
                r.render(stats=False)
            st = r.render(stats=True)
            sha = hashlib.sha256(r.read_frame().tobytes()).hexdigest()
            if sha != e["sha256"] or counters_of(st) != e["counters"]:
                bad.append((key, counters_of(st), e["counters"]))
    assert not bad, f"{len(bad)} of {len(KEYS)} frames differ: {bad[:3]}"


def test_headline_at_5000_steps(frm_lib):
    """The 4K headline frame (scene 18, N = 12, power 8, P1) at the reference's 5000 steps,
    rendered as bench.py renders (two frames in flight, scheduled second frame)."""
    e = _golden()["HEADLINE_5000"]
    with frm.Renderer(device=0, max_steps=0, frames_in_flight=2) as r:
        r.resize(e["width"], e["height"])
        r.update_parameters_buffer(frm.Parameters.from_bytes(bytes.fromhex(e["params"])))
        r.render(stats=False)
        st = r.render(stats=True)
        img = r.read_frame()
    assert counters_of(st) == e["counters"]
    assert hashlib.sha256(img.tobytes()).hexdigest() == e["sha256"]
