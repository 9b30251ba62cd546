"""Diagnostic (FRM_STAMPS build): fraction of wave time spent in service passes."""
import ctypes, os, sys, time
sys.path.insert(0, "."); sys.path.insert(0, "fractal-ray-marching_amd")
import torch
import frm
w = frm.WORKLOADS[os.environ.get("WL", "HEADLINE")]
p = frm.make_parameters(w, pose="P1")
r = frm.Renderer(max_steps=w.max_steps)
r.resize(w.width, w.height); r.update_parameters_buffer(p)
buf = torch.empty(w.width * w.height * 4, dtype=torch.uint8, device="cuda")
cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
for k in range(3):
    cnt.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    r.render_bands(buf.data_ptr(), buf.numel(), w.height, 0, 1, s.cuda_stream, cnt.data_ptr())
    e1.record(s); torch.cuda.synchronize()
    c = cnt.cpu().tolist()
    print(f"frame {k}: {e0.elapsed_time(e1):.2f} ms, service wave-cycles {c[7]:.4g}")
try:
    import numpy as np
    lib = frm.load()
    out = np.zeros(5, np.uint64)
    lib.frm_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.frm_debug_read(r.ctx, out.ctypes.data)
    start, exhaust, end = int(out[3]), int(out[2]), int(out[4])
    print(f"waves {int(out[1])} services; realtime: queue exhausted at {(exhaust-start)/100:.0f} us, last wave ends at {(end-start)/100:.0f} us")
except AttributeError:
    pass
try:
    npix = w.width * w.height
    keys = np.zeros(npix, np.uint8)
    lib.frm_debug_pixel_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    n = lib.frm_debug_pixel_keys(r.ctx, keys.ctypes.data, npix)
    bodies = np.sort(np.exp2(keys[:n] / 16.0) - 1.0)[::-1]  # key -> approx. bodies per pixel
    print("per-pixel bodies (from keys): max", int(bodies[0]), "p99.9", int(bodies[int(n * 0.001)]),
          "p99", int(bodies[int(n * 0.01)]), "p90", int(bodies[int(n * 0.1)]), "median", int(bodies[n // 2]))
    print("share of all bodies in the top 1% of pixels:", round(float(bodies[: n // 100].sum() / bodies.sum()), 3))
except AttributeError:
    pass
