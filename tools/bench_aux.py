"""The §8(f) / multi-GPU helper kernels measured: run under
`rocprofv3 --kernel-trace --stats` and summarised by tools/aux_summary.py, which divides each
kernel's algorithmic bytes by its average dispatch time. Workload, REPS dispatches each:

  shade     the headline frame (3840x2160, P1) rendered REPS times: shade_pass reads the 8-B
            tail of every pixel + the 16-B geometry of hit pixels, writes RGBA8 + the 1-B key
  present   frm_present of that frame to 1920x1080 (nearest minification), 3840x2160 (linear,
            same size) and 7680x4320 (linear magnification): blit_kernel
  unshuffle the 8-rank row-band reassembly of a 4K frame (frm_unshuffle_bands, 16-B copies)

Prints the byte model as JSON (stdout) for aux_summary.py."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import torch  # noqa: E402

import frm  # noqa: E402
from frm import tiling  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
w = frm.WORKLOADS["HEADLINE"]
W, H = w.width, w.height
model = {}
with frm.Renderer(device=0, max_steps=w.max_steps) as r:
    r.resize(W, H)
    r.update_parameters_buffer(frm.make_parameters(w, pose="P1"))
    hits = 0
    for _ in range(REPS):
        hits = r.render(stats=True)["hit_pixels"]
    model["shade_pass"] = {"bytes": W * H * (8 + 4 + 1) + hits * 16, "dispatches": REPS}
    for ow, oh in ((1920, 1080), (3840, 2160), (7680, 4320)):
        for _ in range(REPS):
            r.present(ow, oh)
    # blit bytes: every output pixel written; source texels read once (cached) when every texel
    # is sampled (same size / magnification), one texel per output pixel when minifying
    model["blit_kernel"] = {
        "bytes_per_dispatch": {"1920x1080": 1920 * 1080 * 8, "3840x2160": W * H * 8,
                               "7680x4320": W * H * 4 + 7680 * 4320 * 4},
        "dispatches": 3 * REPS}
    ranks = 8
    band_rows = tiling.choose_band_rows(H, ranks)
    rows = tiling.rank_buffer_rows(H, band_rows, ranks)
    stride = rows * W * 4
    src = torch.zeros(ranks * stride, dtype=torch.uint8, device="cuda")
    dst = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    for _ in range(REPS):
        r.unshuffle_bands(src.data_ptr(), stride, dst.data_ptr(), dst.numel(), band_rows, ranks)
    torch.cuda.synchronize()
    model["unshuffle_bands"] = {"bytes": 2 * W * H * 4, "dispatches": REPS}
print(json.dumps(model))
