"""GPU parity with several frames in flight (frm_config.frames_in_flight): consecutive
frames overlap on the GPU, each with its own slot of device scratch (pixel records,
scheduling arrays, work queue) and, for frm_render, its own framebuffer and stream. Every
frame below has different Parameters (pose, time), so a frame computed from another
frame's scratch, schedule or buffer would show; each must equal the oracle's render of its
own Parameters byte for byte, with its own work counters."""
import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu

W, H = 160, 96
FRAMES = [("P1", frm.POWER8_TIME), ("P0", frm.POWER8_TIME), ("P2", frm.POWER8_TIME + 1.0),
          ("P1", frm.POWER8_TIME + 2.0), ("P2", frm.POWER8_TIME), ("P1", frm.POWER8_TIME)]


def frame_params(k):
    pose, t = FRAMES[k % len(FRAMES)]
    return params_for(18, 12, t, W, H, pose=pose)


@pytest.fixture(scope="module")
def refs(oracle):
    return [oracle.render(frame_params(k), W, H, 256) for k in range(len(FRAMES))]


@pytest.mark.parametrize("inflight", [2, 3, frm.FRM_MAX_FRAMES_IN_FLIGHT])
def test_render_bands_rotating_streams(frm_lib, refs, inflight):
    """The multi-GPU / bench path: frame k renders into its own buffer on stream k % F."""
    import torch

    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(inflight)]
    n = 2 * len(FRAMES)  # every slot is reused, with a stale schedule from another pose
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device=dev) for _ in range(n)]
    counters = torch.zeros((n, 8), dtype=torch.int64, device=dev)
    with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL,
                      frames_in_flight=inflight) as r:
        r.resize(W, H)
        for k in range(n):
            r.update_parameters_buffer(frame_params(k))  # copied at the call: frames differ
            s = streams[k % inflight]
            r.render_bands(bufs[k].data_ptr(), bufs[k].numel(), H, 0, 1, s.cuda_stream,
                           counters[k].data_ptr())
        torch.cuda.synchronize()
        for k in range(n):
            ref = refs[k % len(FRAMES)]
            img = bufs[k].cpu().numpy().reshape(H, W, 4)
            assert np.array_equal(img, ref["rgba"]), f"frame {k}"
            c = [int(v) for v in counters[k].cpu().tolist()]
            assert c[:7] == [int(v) for v in ref["counters"][:7]], f"frame {k}"


@pytest.mark.parametrize("flags", [frm.FRM_FLAG_PERSISTENT_KERNEL, frm.FRM_FLAG_SIMPLE_KERNEL])
def test_render_read_frame_sees_last_frame(frm_lib, oracle, refs, flags):
    """frm_render rotates slots (own streams and framebuffers); read_frame and present see
    the last frame; a stats render waits for the frames in flight and counts only itself."""
    with frm.Renderer(device=0, max_steps=256, flags=flags, frames_in_flight=3) as r:
        r.resize(W, H)
        for k in range(5):
            r.update_parameters_buffer(frame_params(k))
            r.render(stats=False)
        assert np.array_equal(r.read_frame(), refs[4]["rgba"])
        assert np.array_equal(r.present(W, H), refs[4]["rgba"])
        r.update_parameters_buffer(frame_params(2))
        r.render(stats=False)
        r.update_parameters_buffer(frame_params(1))
        st = r.render(stats=True)
        assert np.array_equal(r.read_frame(), refs[1]["rgba"])
        got = [st["pixels"], st["hit_pixels"], st["primary_steps"], st["shadow_steps"], st["normal_evals"],
               st["fractal_bodies"], st["fractal_bailouts"]]
        assert got == [int(v) for v in refs[1]["counters"][:7]]
        r.synchronize()
        r.resize(W // 2, H)  # waits for every slot, then frees the framebuffers
        p = frame_params(0)
        p.update_aspect(W // 2, H)
        r.update_parameters_buffer(p)
        for _ in range(4):
            r.render(stats=False)
        assert np.array_equal(r.read_frame(), oracle.render(p, W // 2, H, 256)["rgba"])


def test_rccl_gather_pipeline_one_rank(frm_lib, refs):
    """bench.py's N>1 data path on real RCCL, with the one rank a single GPU allows (RCCL
    refuses two ranks on one device): RowTiledFrame renders on 3 rotating streams, gathers
    through ProcessGroupNCCL (async, stream-ordered waits) and unshuffles on the GPU. Every
    frame has its own Parameters; the last assembled frame must equal the oracle's."""
    import socket

    import torch
    import torch.distributed as dist

    from frm.distributed import RowTiledFrame

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    try:
        F, band_rows = 3, 16
        streams = [torch.cuda.Stream(device=dev) for _ in range(F)]
        counters = torch.zeros(8, dtype=torch.int64, device=dev)
        with frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL,
                          frames_in_flight=F) as r:
            r.resize(W, H)

            def render_bands(buf, br, first, stride, slot, count):
                assert count == 1
                r.render_bands(buf.data_ptr(), buf.numel(), br, first, stride, streams[slot].cuda_stream,
                               counters.data_ptr())

            def unshuffle(gathered, rank_stride, frame, slot):
                r.unshuffle_bands(gathered.data_ptr(), rank_stride, frame.data_ptr(), frame.numel(),
                                  band_rows, 1, streams[slot].cuda_stream)

            tf = RowTiledFrame(W, H, 0, 1, band_rows, dev, render_bands, unshuffle, inflight=F, streams=streams,
                               collective=True)
            n = 7
            tf.run(n, lambda k: r.update_parameters_buffer(frame_params(k)))
            torch.cuda.synchronize()
            img = tf.output().cpu().numpy().reshape(H, W, 4)
            assert np.array_equal(img, refs[(n - 1) % len(FRAMES)]["rgba"])
            c = [int(v) for v in counters.cpu().tolist()]
            assert c[2] == sum(int(refs[k % len(FRAMES)]["counters"][2]) for k in range(n))
    finally:
        dist.destroy_process_group()
