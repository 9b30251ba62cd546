"""GPU parity at BASELINE.json's full sizes: the frames bench.py measures, rendered as the bench
renders them (persistent kernel, two frames in flight, the second frame fetched in the
scheduled order of the first's costs), equal the oracle's bytes bit for bit.

C2 (1920x1080), the headline and C3 (3840x2160) are compared whole, with their work counters;
C4 (7680x4320) and C5 (16384x16384) on an evenly spaced row sample of the full frame (the
oracle would need minutes for all of it), C5 at two consecutive animation times."""
import os

import numpy as np
import pytest

import frm

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share


def counters_of(st):
    return [st["pixels"], st["hit_pixels"], st["primary_steps"], st["shadow_steps"],
            st["normal_evals"], st["fractal_bodies"], st["fractal_bailouts"], 0]


def render_like_bench(w, params, frames=2):
    """frames consecutive renders of one context with 2 frames in flight; returns the last
    frame's bytes and counters (frm_render with stats waits for every slot first)."""
    flags = frm.FRM_FLAG_SCENE_SPHERE if w.sphere else 0
    with frm.Renderer(device=0, max_steps=w.max_steps, flags=flags, frames_in_flight=2) as r:
        r.resize(w.width, w.height)
        r.update_parameters_buffer(params)
        for _ in range(frames - 1):
            r.render(stats=False)
        st = r.render(stats=True)
        return r.read_frame(), st


@pytest.mark.parametrize("name", ["C2", "HEADLINE", "C3"])
def test_full_frame_bit_exact(frm_lib, oracle, name):
    w = frm.WORKLOADS[name]
    p = frm.make_parameters(w, pose="P1")
    img, st = render_like_bench(w, p)
    ref = oracle.render(p, w.width, w.height, w.max_steps, threads=THREADS)
    diff = np.any(img != ref["rgba"], axis=-1)
    assert not diff.any(), f"{name}: {int(diff.sum())} of {w.width * w.height} pixels differ"
    assert counters_of(st) == [int(c) for c in ref["counters"]]
    assert st["march_steps"] == int(ref["counters"][2]) + int(ref["counters"][3])


@pytest.mark.parametrize("name,stride", [("C4", 36), ("C5", 256)])
def test_full_size_row_sample_bit_exact(frm_lib, oracle, name, stride):
    w = frm.WORKLOADS[name]
    p = frm.make_parameters(w, pose="P1")
    times = [w.time, w.time + 1.0 / 60.0] if w.animated else [w.time]
    rows = list(range(stride // 2, w.height, stride))
    for t in times:
        p.time = t
        img, st = render_like_bench(w, p)
        assert st["pixels"] == w.width * w.height
        ref = oracle.render(p, w.width, w.height, w.max_steps, rows=rows, threads=THREADS)
        got = img[rows]
        diff = np.any(got != ref["rgba"], axis=-1)
        assert not diff.any(), f"{name} t={t}: {int(diff.sum())} of {diff.size} sampled pixels differ"
