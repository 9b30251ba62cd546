"""Which device-to-host copies run as blit kernels inside a libfrm process: one case
per run (argv[1]), counted under rocprofv3 --kernel-trace --memory-copy-trace (tools/gpu_d2h_frm.sh).
  torch      a pinned-host torch copy, nothing else
  cumask     the same after a CU-masked stream exists (libfrm's slot streams > 0)
  frm        libfrm's readback (frm_read_frame_async), slot streams CU-masked (the default)
  frmplain   the same with FRM_SLOT_STREAMS=plain (pooled plain streams)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
case = sys.argv[1]
if case == "frmplain":
    os.environ["FRM_SLOT_STREAMS"] = "plain"
import torch  # noqa: E402

import frm  # noqa: E402

n = 3840 * 2160 * 4
if case in ("torch", "cumask"):
    if case == "cumask":
        r = frm.Renderer(device=0, max_steps=64, frames_in_flight=2)
        r.resize(64, 36)
        r.update_parameters_buffer(frm.make_parameters(frm.WORKLOADS["HEADLINE"], width=64, height=36))
        for _ in range(3):
            r.render(stats=False)
        r.synchronize()
    x = torch.ones(n, dtype=torch.uint8, device="cuda")
    y = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            y.copy_(x, non_blocking=True)
    torch.cuda.synchronize()
    print(case, int(y[:16].sum()))
else:
    w = frm.WORKLOADS["HEADLINE"]
    with frm.Renderer(device=0, max_steps=8, frames_in_flight=2) as r:
        r.resize(w.width, w.height)
        r.update_parameters_buffer(frm.make_parameters(w))
        for _ in range(3):
            r.render(stats=False)
            t = r.read_frame_async()
        r.frame_pixels(t, copy=False)
    print(case, "ok")
