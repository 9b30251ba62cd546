"""§8(f) row 4 on the GPU: frm_present (the blit pass + present) equals the oracle's
restatement (om_blit) of the rendered frame bit for bit, for magnification, minification,
mixed aspect, sRGB or linear surfaces and both byte orders."""
import numpy as np
import pytest

from helpers import params_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("out_w,out_h", [(160, 90), (400, 225), (80, 45), (320, 90), (97, 61), (1, 1)])
@pytest.mark.parametrize("flags", [1, 0, 2, 3])
def test_present_matches_oracle(gpu_renderer_factory, oracle, out_w, out_h, flags):
    p = params_for(18, 6, 3.2175055, 160, 90)
    with gpu_renderer_factory(max_steps=128) as r:
        r.resize(160, 90)
        r.update_parameters_buffer(p)
        r.render()
        src = r.read_frame()
        got = r.present(out_w, out_h, srgb=bool(flags & 1), bgra=bool(flags & 2))
    want = oracle.blit(src, out_w, out_h, flags)
    assert np.array_equal(got, want)
    if (out_w, out_h) == (160, 90) and flags == 1:
        assert np.array_equal(got, src)
