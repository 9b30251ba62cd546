"""FRM_FLAG_HW_MATH (opt-in, never the default): the Mandelbulb on the GPU's hardware
transcendentals, as a Vulkan driver lowers fragment.wgsl's builtins (WGSL leaves their precision
to the implementation). Not bit-exact with the oracle by design, so it is gated like the oracle's
own builtins are against precise ones (P1): at BASELINE's sizes (the 4K
headline, C2), against the MODE_LIBM oracle (float64 libm builtins rounded once),
* the GPU frame's own geometry (frm_debug_trace) re-shaded with the exact frm shading reproduces
  its bytes: the hardware math changes the march only, never the shading or the sRGB store;
* every pixel more than one code off is in a named geometric class, 0 unexplained;
* the fraction of such pixels stays at the level of the bit-exact frm builtins' (3.5 %).
Scenes without a transcendental in their DE (Menger, Sierpinski, Koch) render bit-exact."""
import os

import numpy as np
import pytest

import frm
from helpers import params_for
from p1_classify import classify_frame

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


@pytest.mark.parametrize("name", ["C2", "HEADLINE"])
def test_hw_math_differences_classified(frm_lib, oracle, name):
    w = frm.WORKLOADS[name]
    p = frm.make_parameters(w, pose="P1")
    with frm.Renderer(device=0, max_steps=w.max_steps, flags=frm.FRM_FLAG_HW_MATH | frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w.width, w.height)
        r.update_parameters_buffer(p)
        r.render(stats=False)
        r.render(stats=True)
        img = r.read_frame()
        tr = r.trace()
    res = classify_frame(oracle, p, w.width, w.height, w.max_steps, img, tr, threads=THREADS)
    print(name, res)
    assert res["trace_mismatch_pixels"] == 0
    assert res["unexplained"] == 0
    assert res["differ_gt1_frac"] < 0.06
    assert res["differ_any"] > 0  # it is not the bit-exact path


@pytest.mark.parametrize("scene,iters", [(0, 4), (15, 5), (16, 4)])
def test_hw_math_leaves_other_scenes_bit_exact(frm_lib, oracle, scene, iters):
    w, h = 96, 54
    p = params_for(scene, iters, 0.0, w, h)
    ref = oracle.render(p, w, h, 256)
    for kernel in (frm.FRM_FLAG_PERSISTENT_KERNEL, frm.FRM_FLAG_SIMPLE_KERNEL):
        with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_HW_MATH | kernel) as r:
            r.resize(w, h)
            r.update_parameters_buffer(p)
            r.render(stats=False)
            assert np.array_equal(r.read_frame(), ref["rgba"])


def test_trace_of_exact_frame_matches_oracle_trace(frm_lib, oracle):
    """frm_debug_trace on the bit-exact path equals the oracle's own trace on hit pixels (the
    entry the HW-math gate relies on)."""
    w, h = 160, 90
    p = params_for(18, 12, frm.POWER8_TIME, w, h)
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        r.render(stats=True)
        tr = r.trace()
    ref = oracle.render(p, w, h, 256, trace=True)["trace"].reshape(h, w, 10)
    hit = ref[..., 0] != 0
    assert np.array_equal(tr[..., 0] != 0, hit)
    a, b = tr[hit], ref[hit]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all()
