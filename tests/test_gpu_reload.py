"""§8(f) row 3 on the GPU: runtime kernel reload (frm_reload, hiprtc), the reference's
shader hot reload (graphics.rs:39-48, reloadable_graphics.rs:15-52).
* Recompiled from an unmodified copy of csrc/, both kernels produce the oracle's bytes.
* An edited copy takes effect (the sphere extension's radius), and reload(None) returns
  to the built-in kernels.
* A broken copy raises FRM_ERR_COMPILE with the compiler's message, and the previous
  kernels keep rendering (the reference prints the error and keeps its pipeline)."""
import os
import shutil

import numpy as np
import pytest

import frm
from frm import _lib
from helpers import params_for

pytestmark = pytest.mark.gpu

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fractal-ray-marching_amd", "csrc")


def copy_sources(tmp_path, name):
    d = tmp_path / name
    shutil.copytree(CSRC, d)
    return d


def edit(path, old, new):
    s = path.read_text()
    assert old in s
    path.write_text(s.replace(old, new))


@pytest.mark.parametrize("kernel_flags", [frm.FRM_FLAG_PERSISTENT_KERNEL, frm.FRM_FLAG_SIMPLE_KERNEL], ids=["persistent", "simple"])
def test_reload_unmodified_sources_is_bit_exact(gpu_renderer_factory, oracle, tmp_path, kernel_flags):
    src = copy_sources(tmp_path, "csrc")
    with gpu_renderer_factory(max_steps=256, flags=kernel_flags) as r:
        r.reload(str(src))
        for scene, iters, time in ((18, 6, frm.POWER8_TIME), (0, 3, 0.0), (15, 3, 1.0)):
            p = params_for(scene, iters, time, 96, 54)
            r.resize(96, 54)
            r.update_parameters_buffer(p)
            st = r.render()
            ref = oracle.render(p, 96, 54, 256)
            assert np.array_equal(r.read_frame(), ref["rgba"]), f"scene {scene}"
            assert st["march_steps"] == int(ref["counters"][2]) + int(ref["counters"][3])


def test_reload_edit_takes_effect_and_revert(gpu_renderer_factory, oracle, tmp_path):
    src = copy_sources(tmp_path, "csrc_edit")
    edit(src / "frm_scene.h", "FRM_HD float de_sphere(v3 p) { return length(p) - 0.5f; }",
         "FRM_HD float de_sphere(v3 p) { return length(p) - 0.25f; }")
    p = params_for(0, 0, 0.0, 64, 64, pose="P0")
    ref = oracle.render(p, 64, 64, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)
    with gpu_renderer_factory(max_steps=64, flags=frm.FRM_FLAG_SCENE_SPHERE) as r:
        r.resize(64, 64)
        r.update_parameters_buffer(p)
        base = r.render()
        assert np.array_equal(r.read_frame(), ref["rgba"])
        r.reload(str(src))
        small = r.render()
        assert 0 < small["hit_pixels"] < base["hit_pixels"]  # half the radius: fewer hits
        assert not np.array_equal(r.read_frame(), ref["rgba"])
        r.reload(None)
        r.render()
        assert np.array_equal(r.read_frame(), ref["rgba"])


def test_reload_error_keeps_previous_kernels(gpu_renderer_factory, oracle, tmp_path):
    good = copy_sources(tmp_path, "csrc_good")
    bad = copy_sources(tmp_path, "csrc_bad")
    edit(bad / "frm_scene.h", "FRM_HD float de_sphere(v3 p) { return length(p) - 0.5f; }",
         "FRM_HD float de_sphere(v3 p) { return length(p) - ; }")
    p = params_for(18, 6, frm.POWER8_TIME, 96, 54)
    ref = oracle.render(p, 96, 54, 128)
    with gpu_renderer_factory(max_steps=128) as r:
        r.reload(str(good))
        with pytest.raises(frm.FrmError) as e:
            r.reload(str(bad))
        assert e.value.code == _lib.FRM_ERR_COMPILE
        assert "frm_scene.h" in str(e.value) and "error" in str(e.value)
        assert r.try_reload(str(bad)) is False
        with pytest.raises(frm.FrmError):
            r.reload(str(tmp_path / "does_not_exist"))
        r.resize(96, 54)
        r.update_parameters_buffer(p)
        r.render()
        assert np.array_equal(r.read_frame(), ref["rgba"])


def test_reload_with_frames_in_flight(frm_lib, oracle, tmp_path):
    """Reloaded kernels with 3 frames in flight: consecutive frames with their own parameters
    render on rotating slots through hipModuleLaunchKernel; every frame equals the oracle's
    (frm_render with stats waits for every slot, so each frame is read back alone)."""
    src = copy_sources(tmp_path, "csrc")
    frames = [params_for(18, 6, frm.POWER8_TIME, 96, 54, pose=pose) for pose in ("P0", "P1", "P2")]
    frames += [params_for(0, 3, 0.0, 96, 54), params_for(18, 4, 1.5, 96, 54)]
    refs = [oracle.render(p, 96, 54, 256)["rgba"] for p in frames]
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=3) as r:
        r.resize(96, 54)
        r.reload(str(src))
        for rounds in range(2):
            for p, ref in zip(frames, refs):
                r.update_parameters_buffer(p)
                r.render(stats=False)
                r.render(stats=False)  # a second frame in flight of the same parameters
                assert np.array_equal(r.read_frame(), ref)
