"""GPU parity at BASELINE.json's full sizes: the frames bench.py measures, rendered as the bench
renders them (persistent kernel, two frames in flight, the second frame fetched in the
scheduled order of the first's costs), equal the oracle's bytes bit for bit.

C2 (1920x1080), the headline and C3 (3840x2160) are compared whole against the oracle run
here, with their work counters; every config, C4 (7680x4320) and C5 (16384x16384, two
consecutive animation times) included, is compared whole against the oracle's golden frame
hash and counters (tests/golden/fullsize.json)."""
import os

import numpy as np
import pytest

import frm

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share
_ORACLE = {}  # whole-frame oracle renders, shared by the tests of this module


def oracle_frame(oracle, name):
    if name not in _ORACLE:
        w = frm.WORKLOADS[name]
        p = frm.make_parameters(w, pose="P1")
        _ORACLE[name] = oracle.render(p, w.width, w.height, w.max_steps, threads=THREADS)
    return _ORACLE[name]


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
    ref = oracle_frame(oracle, name)
    diff = np.any(img != ref["rgba"], axis=-1)
    assert not diff.any(), f"{name}: {int(diff.sum())} of {w.width * w.height} pixels differ"
    assert counters_of(st) == [int(c) for c in ref["counters"]]
    assert st["march_steps"] == int(ref["counters"][2]) + int(ref["counters"][3])


def _golden():
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("key", ["HEADLINE_P1", "C2_P1", "C3_P1", "C4_P1", "C5_P1_t0", "C5_P1_t1",
                                 "HEADLINE_P0", "HEADLINE_P2", "C2_P0", "C2_P2", "C3_P0", "C3_P2",
                                 "C4_P0", "C4_P2"])
def test_full_frame_matches_golden_hash(frm_lib, key):
    """Every BASELINE GPU config as a whole frame: the sha256 of the RGBA8 bytes and the work
    counters equal the oracle's, rendered once on the CPU into tests/golden/fullsize.json
    (tests/golden/make_fullsize_golden.py; C5 took hours of CPU there, so the box compares
    hashes). C4 = 7680x4320, N=16, 512 steps; C5 = 16384x16384, N=20, 1024 steps at its
    first two animation times (time, time + 1/60: the frames bench.py renders first); the
    headline, C2, C3 and C4 also at the other fixed poses P0 and P2."""
    import hashlib

    g = _golden().get(key)
    if g is None:
        pytest.fail(f"no golden frame {key}: run tests/golden/make_fullsize_golden.py")
    w = frm.WORKLOADS[g["workload"]]
    p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
    img, st = render_like_bench(w, p)
    assert st["pixels"] == w.width * w.height
    assert counters_of(st) == g["counters"], key
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["sha256"], key


def test_headline_row_split_8_ranks(frm_lib, oracle):
    """bench.py's default 8-GPU data path, simulated on one device: 8 contexts render their
    interleaved 18-row bands of the 4K headline (three frames in flight each, so the
    scheduled order runs), frm_unshuffle_bands reassembles rank-major buffers into the frame,
    which equals the oracle's; the summed counters equal the whole frame's."""
    import torch

    from frm import tiling

    w = frm.WORKLOADS["HEADLINE"]
    ranks = 8
    p = frm.make_parameters(w, pose="P1")
    band_rows = tiling.choose_band_rows(w.height, ranks)
    rows = tiling.rank_buffer_rows(w.height, band_rows, ranks)
    rank_stride = rows * w.width * 4
    dev = torch.device("cuda", 0)
    gathered = torch.zeros(ranks * rank_stride, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    rds = [frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=3) for _ in range(ranks)]
    try:
        for rd in rds:
            rd.resize(w.width, w.height)
            rd.update_parameters_buffer(p)
        for frame in range(3):
            counters.zero_()
            for r, rd in enumerate(rds):
                view = gathered[r * rank_stride:(r + 1) * rank_stride]
                rd.render_bands(view.data_ptr(), rank_stride, band_rows, r, ranks, 0, counters.data_ptr())
            torch.cuda.synchronize()
        out = torch.zeros(w.width * w.height * 4, dtype=torch.uint8, device=dev)
        rds[0].unshuffle_bands(gathered.data_ptr(), rank_stride, out.data_ptr(), out.numel(), band_rows, ranks)
        torch.cuda.synchronize()
        img = out.cpu().numpy().reshape(w.height, w.width, 4)
        ref = oracle_frame(oracle, "HEADLINE")
        diff = np.any(img != ref["rgba"], axis=-1)
        assert not diff.any(), f"{int(diff.sum())} pixels differ"
        assert [int(v) for v in counters.cpu().tolist()][:7] == [int(v) for v in ref["counters"][:7]]
    finally:
        for rd in rds:
            rd.close()


def test_fly_through_sequence_matches_golden(frm_lib):
    """bench.py's HEADLINE_FLY workload as it renders it: one context, one frame per launch, two
    in flight, Parameters from frm.frame_sequence (time += 1/60, yaw-locked orbit per frame), so
    every frame after the first is fetched in the order of the previous (different) frame's
    costs. Frames 0, 1, 2 equal the oracle's (frame 0 = HEADLINE_P1; tests/golden/fullsize.json,
    make_fullsize_golden.py)."""
    import hashlib

    g = _golden()
    w = frm.WORKLOADS["HEADLINE_FLY"]
    seq = frm.frame_sequence(w, pose="P1")
    with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=2) as r:
        r.resize(w.width, w.height)
        for k, key in enumerate(("HEADLINE_P1", "HEADLINE_FLY_P1_f1", "HEADLINE_FLY_P1_f2")):
            p = next(seq)
            assert p.to_bytes().hex() == g[key]["params"], key
            r.update_parameters_buffer(p)
            st = r.render(stats=True)
            assert counters_of(st) == g[key]["counters"], key
            assert hashlib.sha256(r.read_frame().tobytes()).hexdigest() == g[key]["sha256"], key


def test_fly_through_batched_matches_golden(frm_lib):
    """The same frames 0, 1, 2 of HEADLINE_FLY in ONE multi-frame launch (the time, hence the
    Mandelbulb's power, and the camera differ per frame; bench.py renders the fly-through so), on a
    context whose previous launch was the same batch (scheduled order): every frame matches its
    golden hash and the launch's counters are the three frames' sums."""
    import hashlib

    import torch

    g = _golden()
    w = frm.WORKLOADS["HEADLINE_FLY"]
    seq = frm.frame_sequence(w, pose="P1")
    keys = ("HEADLINE_P1", "HEADLINE_FLY_P1_f1", "HEADLINE_FLY_P1_f2")
    ps = [next(seq) for _ in keys]
    nb = w.width * w.height * 4
    buf = torch.zeros(len(keys) * nb, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    with frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=1) as r:
        r.resize(w.width, w.height)
        for rep in range(2):
            counters.zero_()
            r.render_bands_batch(ps, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=nb, band_rows=w.height, first_band=0, band_stride=1, stream=0, dev_counters=counters.data_ptr())
            r.synchronize()
            host = buf.cpu().numpy()
            for b, key in enumerate(keys):
                assert hashlib.sha256(host[b * nb:(b + 1) * nb].tobytes()).hexdigest() == g[key]["sha256"], (rep, key)
            want = [sum(g[k]["counters"][i] for k in keys) for i in range(7)]
            assert counters.cpu().tolist()[:7] == want, rep


def _split_frames(name, ranks, params_list, batch, inflight):
    """bench.py's --split rows data path for `ranks` ranks, simulated on one device: one context
    per rank (frames_in_flight = inflight); the frames of params_list in launches of `batch`
    (frm_render_bands_batch for batch > 1, as bench.py batches fixed workloads; one
    frm_render_bands per frame otherwise, as for animated ones), each rank's interleaved bands
    into its rank-major slice of the gathered buffer (what dist.gather delivers to rank 0),
    frm_unshuffle_bands per frame. Yields (frame bytes, summed counters of its launch) per
    launch's frames."""
    import torch

    from frm import tiling

    w = frm.WORKLOADS[name]
    band_rows = tiling.choose_band_rows(w.height, ranks)
    nbytes = tiling.rank_buffer_rows(w.height, band_rows, ranks) * w.width * 4  # one frame's bands
    dev = torch.device("cuda", 0)
    gathered = torch.zeros(ranks * batch * nbytes, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    frame = torch.zeros(w.width * w.height * 4, dtype=torch.uint8, device=dev)
    rds = [frm.Renderer(device=0, max_steps=w.max_steps, frames_in_flight=inflight) for _ in range(ranks)]
    try:
        for rd in rds:
            rd.resize(w.width, w.height)
            rd.update_parameters_buffer(params_list[0])
        for k0 in range(0, len(params_list), batch):
            ps = params_list[k0:k0 + batch]
            n = len(ps) * nbytes
            counters.zero_()
            for r, rd in enumerate(rds):
                buf = gathered[r * n:(r + 1) * n]
                if batch > 1:
                    rd.render_bands_batch(ps, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=nbytes, band_rows=band_rows, first_band=r, band_stride=ranks, stream=0,
                                          dev_counters=counters.data_ptr())
                else:
                    rd.update_parameters_buffer(ps[0])
                    rd.render_bands(buf.data_ptr(), n, band_rows, r, ranks, 0, counters.data_ptr())
            torch.cuda.synchronize()
            cnt = [int(v) for v in counters.cpu().tolist()]
            for b in range(len(ps)):
                src = gathered[b * nbytes:]
                rds[0].unshuffle_bands(src.data_ptr(), n, frame.data_ptr(), frame.numel(), band_rows, ranks)
                torch.cuda.synchronize()
                yield frame.cpu().numpy(), cnt
    finally:
        for rd in rds:
            rd.close()


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_c4_row_split_matches_golden(frm_lib, ranks):
    """BASELINE config 4 (7680x4320, N = 16, 512 steps) row-tiled across 2/4/8 ranks as bench.py
    runs it (2 launches in flight per rank, 2 frames per launch, 2 launches so the second is
    scheduled by the first's costs): every reassembled frame equals the oracle's C4 frame and the
    summed counters of a launch equal 2 x the whole frame's."""
    import hashlib

    g = _golden()["C4_P1"]
    p = frm.Parameters.from_bytes(bytes.fromhex(g["params"]))
    frames = 0
    for img, cnt in _split_frames("C4", ranks, [p] * 4, batch=2, inflight=2):
        assert hashlib.sha256(img.tobytes()).hexdigest() == g["sha256"], (ranks, frames)
        assert cnt[:7] == [2 * c for c in g["counters"][:7]]
        frames += 1
    assert frames == 4


def test_c5_row_split_8_ranks_matches_golden(frm_lib):
    """BASELINE config 5 (16384x16384, N = 20, 1024 steps, animated) row-tiled across 8 ranks as
    bench.py runs it (one frame per launch, 3 in flight per rank): its first two animation times
    (frm.frame_sequence: time, time + 1/60), the second scheduled by the first's costs, equal the
    oracle's golden frames; the summed counters equal each frame's."""
    import hashlib

    g = _golden()
    seq = frm.frame_sequence(frm.WORKLOADS["C5"], pose="P1")
    ps = [next(seq), next(seq)]
    keys = ("C5_P1_t0", "C5_P1_t1")
    for p, key in zip(ps, keys):
        assert p.to_bytes().hex() == g[key]["params"], key
    for k, (img, cnt) in enumerate(_split_frames("C5", 8, ps, batch=1, inflight=3)):
        assert cnt[:7] == g[keys[k]]["counters"][:7], keys[k]
        assert hashlib.sha256(img.tobytes()).hexdigest() == g[keys[k]]["sha256"], keys[k]
