"""GPU parity of the multi-GPU data path on one device: each simulated rank renders its
interleaved row bands (frm_render_bands, first_band = rank, band_stride = ranks) into its
own device buffer, repeatedly (the persistent kernel's pixel scheduling then runs from
history), and frm_unshuffle_bands reassembles the frame. Bytes and summed counters must
equal the oracle's whole-frame render; ragged last bands included."""
import ctypes

import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu


def local_rows(height, band_rows, first, stride):
    out = ctypes.c_uint32(0)
    assert frm.load().frm_band_rows_for(height, band_rows, first, stride, ctypes.byref(out)) == 0
    return out.value


@pytest.mark.parametrize("width,height,band_rows,ranks,kernel_flags", [
    (200, 118, 8, 3, frm.FRM_FLAG_PERSISTENT_KERNEL),  # 15 bands, the last one 6 rows
    (131, 77, 5, 2, frm.FRM_FLAG_PERSISTENT_KERNEL),   # odd width, last band 2 rows
    (96, 54, 54, 2, frm.FRM_FLAG_PERSISTENT_KERNEL),   # one band: rank 1 renders nothing
    (200, 118, 8, 3, frm.FRM_FLAG_SIMPLE_KERNEL),
])
def test_bands_reassemble_to_oracle_frame(gpu_renderer_factory, oracle, width, height, band_rows, ranks,
                                          kernel_flags):
    import torch

    p = params_for(18, 12, frm.POWER8_TIME, width, height)
    ref = oracle.render(p, width, height, 256)
    dev = torch.device("cuda", 0)
    stride_rows = max(local_rows(height, band_rows, r, ranks) for r in range(ranks))
    rank_stride = stride_rows * width * 4
    gathered = torch.zeros(ranks * max(rank_stride, 4), dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    renderers = [gpu_renderer_factory(max_steps=256, flags=kernel_flags) for _ in range(ranks)]
    try:
        first_frame = None
        for frame in range(3):  # frames 2 and 3 fetch pixels in the scheduled order
            counters.zero_()
            for r, rd in enumerate(renderers):
                if frame == 0:
                    rd.resize(width, height)
                    rd.update_parameters_buffer(p)
                rows = local_rows(height, band_rows, r, ranks)
                if rows == 0:
                    continue
                view = gathered[r * rank_stride:(r + 1) * rank_stride]
                rd.render_bands(view.data_ptr(), rows * width * 4, band_rows, r, ranks, 0, counters.data_ptr())
            torch.cuda.synchronize()
            out = torch.zeros(width * height * 4, dtype=torch.uint8, device=dev)
            renderers[0].unshuffle_bands(gathered.data_ptr(), rank_stride, out.data_ptr(), out.numel(), band_rows,
                                         ranks)
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(height, width, 4)
            assert np.array_equal(img, ref["rgba"]), f"frame {frame}"
            c = [int(v) for v in counters.cpu().tolist()]
            assert c[:7] == [int(v) for v in ref["counters"][:7]], f"frame {frame}"
            if first_frame is None:
                first_frame = gathered.clone()
            else:
                assert torch.equal(gathered, first_frame)
    finally:
        for rd in renderers:
            rd.close()


@pytest.mark.parametrize("ranks,inflight", [(1, 1), (1, 2), (3, 2)])
def test_moving_camera_history_bit_exact(gpu_renderer_factory, oracle, ranks, inflight):
    """A camera and a time that move every frame (frm.frame_sequence's fly-through, sped up 20x)
    so every launch fetches its pixels in the order of another frame's cost keys; whole frames
    (ranks = 1) and interleaved bands of 3 ranks reassembled: every frame equals the oracle's
    render of its own Parameters."""
    import torch

    w = frm.WORKLOADS["HEADLINE_FLY"]
    width, height, band_rows = 192, 108, 8
    seq = frm.frame_sequence(w, pose="P1", dt=20 * frm.FRAME_SECONDS)
    dev = torch.device("cuda", 0)
    stride_rows = max(local_rows(height, band_rows, r, ranks) for r in range(ranks))
    rank_stride = stride_rows * width * 4
    gathered = torch.zeros(ranks * rank_stride, dtype=torch.uint8, device=dev)
    out = torch.zeros(width * height * 4, dtype=torch.uint8, device=dev)
    rds = [frm.Renderer(device=0, max_steps=256, flags=frm.FRM_FLAG_PERSISTENT_KERNEL, frames_in_flight=inflight)
           for _ in range(ranks)]
    try:
        for frame in range(5):
            p = next(seq)
            for r, rd in enumerate(rds):
                if frame == 0:
                    rd.resize(width, height)
                rd.update_parameters_buffer(p)
                view = gathered[r * rank_stride:(r + 1) * rank_stride]
                rd.render_bands(view.data_ptr(), rank_stride, band_rows if ranks > 1 else height, r, ranks, 0)
            torch.cuda.synchronize()  # the ranks' context streams, before the reassembly reads them
            if ranks > 1:
                rds[0].unshuffle_bands(gathered.data_ptr(), rank_stride, out.data_ptr(), out.numel(), band_rows, ranks)
            else:
                out.copy_(gathered[:out.numel()])
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(height, width, 4)
            assert np.array_equal(img, oracle.render(p, width, height, 256)["rgba"]), f"frame {frame}"
    finally:
        for rd in rds:
            rd.close()
