"""Diagnostic (FRM_POOL_STAMPS build, FRM_POOL=1): where march_pool's wave cycles go. Renders
the headline a few times (scheduling history), then FRAMES frames, and prints the share of wave
cycles in service passes, swaps and body loops, with their counts."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import frm  # noqa: E402

w = frm.WORKLOADS[os.environ.get("WL", "HEADLINE")]
lib = frm.load()
lib.frm_debug_pool.argtypes = [ctypes.c_void_p]
out = np.zeros(8, np.uint64)
with frm.Renderer(max_steps=w.max_steps) as r:
    r.resize(w.width, w.height)
    r.update_parameters_buffer(frm.make_parameters(w, pose="P1"))
    for _ in range(3):
        r.render(stats=True)
    lib.frm_debug_pool(out.ctypes.data)
    sts = [r.render(stats=True) for _ in range(int(os.environ.get("FRAMES", "4")))]
    ms = [st["kernel_ms"] for st in sts]
    bodies = sum(st["fractal_bodies"] for st in sts)
    lib.frm_debug_pool(out.ctypes.data)
tot, sv, sw, bd, ns, nf, nw, nl = [float(x) for x in out]
print(f"frame ms {[round(m, 2) for m in ms]}")
print(f"wave cycles: service {sv / tot:.3f}, swap {sw / tot:.3f}, body loop {bd / tot:.3f}, other {(tot - sv - sw - bd) / tot:.3f}")
print(f"services {ns:.0f} (full {nf / ns:.3f}), swaps {nw:.0f}, body iterations {nl:.0f}; "
      f"cycles per service {sv / ns:.0f}, per swap {sw / nw:.0f}, per body iteration {bd / nl:.0f}; "
      f"body-loop lane utilisation {bodies / (64 * nl):.3f}")
