"""Multi-frame launches (frm_render_bands_batch): several frames of one scene whose cameras
differ render in one persistent launch (one work queue, frames interleaved chunk by chunk),
each frame byte-identical to the oracle's render of its own Parameters; counters are the
frames' sums. Whole frames and a simulated 2-rank band split, several consecutive batches
(the scheduled order of the previous batch's last frame), 1 and 2 frames in flight."""
import numpy as np
import pytest

import frm
from frm import _lib, tiling
from helpers import params_for

pytestmark = pytest.mark.gpu


def _poses(scene, iters, time, w, h):
    return [params_for(scene, iters, time, w, h, pose=pz) for pz in ("P0", "P1", "P2", "P1")]


@pytest.mark.parametrize("scene,iters,steps", [(18, 12, 256), (0, 5, 128), (16, 4, 128)])
@pytest.mark.parametrize("inflight", [1, 2])
def test_batch_whole_frames_bit_exact(frm_lib, oracle, scene, iters, steps, inflight):
    import torch

    w, h = 96, 54
    ps = _poses(scene, iters, frm.POWER8_TIME, w, h)
    refs = [oracle.render(p, w, h, steps) for p in ps]
    fb = w * h * 4
    dev = torch.device("cuda", 0)
    out = torch.zeros(len(ps) * fb, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    with frm.Renderer(device=0, max_steps=steps, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=inflight) as r:
        r.resize(w, h)
        for rep in range(3):  # the second and third batches fetch in the scheduled order
            counters.zero_()
            out.zero_()
            r.render_bands_batch(ps, out.data_ptr(), dst_bytes=out.numel(), frame_stride=fb, band_rows=h, first_band=0, band_stride=1, stream=0, dev_counters=counters.data_ptr())
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(len(ps), h, w, 4)
            for k, ref in enumerate(refs):
                assert np.array_equal(img[k], ref["rgba"]), f"batch {rep} frame {k}"
            got = [int(v) for v in counters.cpu().tolist()][:7]
            assert got == [sum(int(ref["counters"][i]) for ref in refs) for i in range(7)]


def test_batch_band_split_bit_exact(frm_lib, oracle):
    """Two simulated ranks, each rendering its interleaved bands of 3 frames in one launch;
    frame b reassembled from the rank-major buffers (rank stride = batch x bands)."""
    import torch

    w, h, ranks, br = 80, 45, 2, 8
    ps = _poses(18, 12, frm.POWER8_TIME, w, h)[:3]
    B = len(ps)
    nb = tiling.rank_buffer_rows(h, br, ranks) * w * 4
    dev = torch.device("cuda", 0)
    gathered = torch.zeros(ranks * B * nb, dtype=torch.uint8, device=dev)
    rds = [frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) for _ in range(ranks)]
    try:
        for rep in range(2):
            for rk, rd in enumerate(rds):
                rd.resize(w, h)
                rd.render_bands_batch(ps, gathered.data_ptr() + rk * B * nb, dst_bytes=B * nb, frame_stride=nb, band_rows=br, first_band=rk, band_stride=ranks)
            torch.cuda.synchronize()
            for b, p in enumerate(ps):
                frame = torch.zeros(w * h * 4, dtype=torch.uint8, device=dev)
                rds[0].unshuffle_bands(gathered.data_ptr() + b * nb, B * nb, frame.data_ptr(), frame.numel(), br, ranks)
                torch.cuda.synchronize()
                ref = oracle.render(p, w, h, 256)
                assert np.array_equal(frame.cpu().numpy().reshape(h, w, 4), ref["rgba"]), f"rep {rep} frame {b}"
    finally:
        for rd in rds:
            rd.close()


def test_batch_rejects_frames_that_differ_beyond_the_camera(frm_lib):
    """A batch's frames share the scene uniforms, except the Mandelbulb's power (its only
    time-derived constant): another iteration count, another scene, or another time of an
    animated Menger scene is refused."""
    import torch

    w, h = 32, 18
    a = params_for(18, 12, frm.POWER8_TIME, w, h)
    c = params_for(18, 11, frm.POWER8_TIME, w, h)  # other iteration count
    m0 = params_for(4, 3, 0.5, w, h)               # animated Menger: the time moves its cross size
    m1 = params_for(4, 3, 1.5, w, h)
    d = params_for(0, 12, frm.POWER8_TIME, w, h)   # another scene
    buf = torch.zeros(2 * w * h * 4, dtype=torch.uint8, device="cuda")
    with frm.Renderer(device=0, max_steps=64) as r:
        r.resize(w, h)
        for first, other in ((a, c), (m0, m1), (a, d)):
            with pytest.raises(frm.FrmError) as e:
                r.render_bands_batch([first, other], buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=w * h * 4, band_rows=h, first_band=0, band_stride=1)
            assert e.value.code == _lib.FRM_ERR_INVALID_ARGUMENT
        with pytest.raises(frm.FrmError):
            r.render_bands_batch([a] * (frm.FRM_MAX_BATCH + 1), buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=w * h * 4, band_rows=h, first_band=0, band_stride=1)
        # the destination must hold every frame: (count - 1) strides + one frame
        for n, stride in ((2, w * h * 4 + 4), (3, w * h * 4)):
            with pytest.raises(frm.FrmError) as e:
                r.render_bands_batch([a] * n, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=stride, band_rows=h, first_band=0, band_stride=1)
            assert e.value.code == _lib.FRM_ERR_BUFFER_TOO_SMALL
        with pytest.raises(frm.FrmError) as e:  # strides of 16 GiB and more do not fit the kernel's word stride
            r.render_bands_batch([a] * 2, buf.data_ptr(), dst_bytes=1 << 35, frame_stride=1 << 34, band_rows=h, first_band=0, band_stride=1)
        assert e.value.code == _lib.FRM_ERR_INVALID_ARGUMENT
        r.render_bands_batch([a] * 2, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=w * h * 4, band_rows=h, first_band=0, band_stride=1)


def test_batch_of_max_frames_two_slots(frm_lib, oracle):
    """FRM_MAX_BATCH frames per launch (the cameras cycling over four poses), two frames in
    flight: the second slot's first launch fetches by the keys the first slot recorded
    (history shared between slots); every frame of both launches equals the oracle's."""
    import torch

    w, h = 64, 36
    poses = _poses(18, 12, frm.POWER8_TIME, w, h)
    refs = [oracle.render(p, w, h, 256) for p in poses]
    B = frm.FRM_MAX_BATCH
    ps = [poses[k % len(poses)] for k in range(B)]
    fb = w * h * 4
    dev = torch.device("cuda", 0)
    outs = [torch.zeros(B * fb, dtype=torch.uint8, device=dev) for _ in range(2)]
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=2) as r:
        r.resize(w, h)
        for rep in range(3):
            for o in outs:
                r.render_bands_batch(ps, o.data_ptr(), dst_bytes=o.numel(), frame_stride=fb, band_rows=h, first_band=0, band_stride=1, stream=0, dev_counters=counters.data_ptr())
            torch.cuda.synchronize()
            for j, o in enumerate(outs):
                img = o.cpu().numpy().reshape(B, h, w, 4)
                for k in range(B):
                    assert np.array_equal(img[k], refs[k % len(refs)]["rgba"]), f"rep {rep} launch {j} frame {k}"


def test_batch_rank_without_bands(frm_lib):
    """A rank that holds no band of the frame (rows == 0) renders nothing and succeeds, also
    with a zero frame stride and a zero-byte destination (no division by the stride)."""
    import torch

    w, h, br, ranks = 32, 8, 8, 2  # one band: rank 1 has none
    a = params_for(18, 12, frm.POWER8_TIME, w, h)
    buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    with frm.Renderer(device=0, max_steps=64) as r:
        r.resize(w, h)
        for stride, nbytes in ((0, 0), (4, buf.numel())):
            r.render_bands_batch([a] * 3, buf.data_ptr(), dst_bytes=nbytes, frame_stride=stride, band_rows=br, first_band=1, band_stride=ranks, stream=0, dev_counters=counters.data_ptr())
        torch.cuda.synchronize()
        assert int(counters.sum()) == 0 and int(buf.sum()) == 0


@pytest.mark.parametrize("kernel", ["persistent", "simple"])
def test_batch_animated_mandelbulb_bit_exact(frm_lib, oracle, kernel):
    """Frames of a fly-through whose time advances (frm.frame_sequence sped up 20x: the Mandelbulb's
    power moves every frame) in multi-frame launches of 3, two launches in flight: each lane
    carries its frame's power (the ANIM instantiation; the simple kernel renders frame by frame).
    Every frame equals the oracle's render of its own Parameters; a launch's counters are the sum
    of its frames'."""
    import torch

    w = frm.WORKLOADS["HEADLINE_FLY"]
    width, height, B = 160, 90, 3
    seq = frm.frame_sequence(w, pose="P1", dt=20 * frm.FRAME_SECONDS)
    frames = [next(seq) for _ in range(3 * B)]
    assert len({p.time for p in frames}) == len(frames)
    for p in frames:
        p.update_aspect(width, height)
    refs = [oracle.render(p, width, height, 256) for p in frames]
    nb = width * height * 4
    flags = frm.FRM_FLAG_PERSISTENT_KERNEL if kernel == "persistent" else frm.FRM_FLAG_SIMPLE_KERNEL
    bufs = [torch.zeros(B * nb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    with frm.Renderer(device=0, max_steps=256, flags=flags, frames_in_flight=2) as r:
        r.resize(width, height)
        for launch in range(3):
            ps = frames[launch * B:(launch + 1) * B]
            buf = bufs[launch % 2]
            counters.zero_()
            r.render_bands_batch(ps, buf.data_ptr(), dst_bytes=buf.numel(), frame_stride=nb, band_rows=height, first_band=0, band_stride=1, stream=0, dev_counters=counters.data_ptr())
            r.synchronize()
            got = buf.cpu().numpy()
            for b in range(B):
                k = launch * B + b
                assert np.array_equal(got[b * nb:(b + 1) * nb].reshape(height, width, 4), refs[k]["rgba"]), f"frame {k}"
            want = sum(np.asarray(refs[launch * B + b]["counters"], dtype=np.int64) for b in range(B))
            assert np.array_equal(counters.cpu().numpy()[:7], want[:7]), f"launch {launch}"
