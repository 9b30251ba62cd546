"""The persistent kernel's XCD-aware work queue (frm_internal.h kQueue*): the head of the fetch order
from a shared counter, the rest over 8 per-XCD partitions with stealing. Every chunk of 64 fetch
positions must be claimed exactly once whatever the chunk count (fewer chunks than partitions, a head
of zero chunks, counts around multiples of 8 and 64), single frames and multi-frame launches: the
bytes and all work counters equal the oracle's."""
import numpy as np
import pytest

import frm
from helpers import params_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunks", [1, 3, 7, 8, 9, 15, 16, 17, 63, 64, 65, 129])
def test_every_chunk_claimed_once(frm_lib, oracle, chunks):
    import torch

    w, h = 64, chunks  # one 64-pixel chunk per row (the launch's fetch order covers w * h positions)
    p = params_for(18, 6, frm.POWER8_TIME, w, h, pose="P1")
    ref = oracle.render(p, w, h, 128)
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    buf = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
    with frm.Renderer(device=0, max_steps=128, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w, h)
        r.update_parameters_buffer(p)
        for rep in range(2):  # the second launch fetches in the scheduled order
            counters.zero_()
            r.render_bands(buf.data_ptr(), buf.numel(), h, 0, 1, 0, counters.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(buf.cpu().numpy().reshape(h, w, 4), ref["rgba"]), f"launch {rep}"
            assert [int(v) for v in counters.cpu().tolist()][:7] == [int(c) for c in ref["counters"][:7]]


@pytest.mark.parametrize("chunks,batch", [(1, 2), (3, 3), (5, 2), (9, 7), (33, 4)])
def test_multi_frame_launch_claims_every_chunk_once(frm_lib, oracle, chunks, batch):
    import torch

    w, h = 64, chunks
    poses = ("P0", "P1", "P2")
    ps = [params_for(18, 6, frm.POWER8_TIME, w, h, pose=poses[k % 3]) for k in range(batch)]
    refs = [oracle.render(p, w, h, 128) for p in ps]
    fb = w * h * 4
    out = torch.zeros(batch * fb, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    with frm.Renderer(device=0, max_steps=128, flags=frm.FRM_FLAG_PERSISTENT_KERNEL) as r:
        r.resize(w, h)
        for rep in range(2):
            counters.zero_()
            r.render_bands_batch(ps, out.data_ptr(), dst_bytes=out.numel(), frame_stride=fb, band_rows=h, first_band=0, band_stride=1, stream=0, dev_counters=counters.data_ptr())
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(batch, h, w, 4)
            for k, ref in enumerate(refs):
                assert np.array_equal(img[k], ref["rgba"]), f"launch {rep} frame {k}"
            want = [sum(int(ref["counters"][i]) for ref in refs) for i in range(7)]
            assert [int(v) for v in counters.cpu().tolist()][:7] == want
