"""Diagnostic (FRM_STAMPS build, FRM_LIB=variants/stamps.so): per-wave records of the last
persistent launch -> body-loop lane utilisation, service share, and the frame's tail
(how many waves are still running over time)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "fractal-ray-marching_amd")
import torch  # noqa: E402

import frm  # noqa: E402

w = frm.WORKLOADS[os.environ.get("WL", "HEADLINE")]
p = frm.make_parameters(w, pose=os.environ.get("POSE", "P1"))
r = frm.Renderer(max_steps=w.max_steps)
r.resize(w.width, w.height)
r.update_parameters_buffer(p)
buf = torch.empty(w.width * w.height * 4, dtype=torch.uint8, device="cuda")
cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
for k in range(3):
    cnt.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    r.render_bands(buf.data_ptr(), buf.numel(), w.height, 0, 1, s.cuda_stream, cnt.data_ptr())
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
lib = frm.load()
lib.frm_debug_waves.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
raw = np.zeros((16384, 16), np.uint64)
n = lib.frm_debug_waves(raw.ctypes.data, 16384)
rec = raw[:n]
rec = rec[rec[:, 4] > 0]
loops, bodies, nserv, scyc, tcyc, start, exh, endw = (rec[:, i].astype(np.float64) for i in range(8))
end_rel = (rec[:, 7] & 0xFFFFFFFF).astype(np.float64) / 100.0  # us after the wave's start
t0 = start.min()
st = (start - t0) / 100.0
en = st + end_rel
ex = np.where(exh > 0, (exh - t0) / 100.0, np.nan)
print(f"{w.name}: frame {ms:.2f} ms (kernel+shade), waves {len(rec)}")
print(f"body-loop lane utilisation {bodies.sum() / (64 * loops.sum()):.3f}; "
      f"bodies per wave-iteration {bodies.sum() / loops.sum():.1f}")
print(f"service share of wave cycles {scyc.sum() / tcyc.sum():.3f}; service passes per wave {nserv.mean():.0f}; "
      f"body iterations per service pass {loops.sum() / nserv.sum():.2f}; cycles per pass {scyc.sum() / nserv.sum():.0f}; "
      f"cycles per body iteration {(tcyc.sum() - scyc.sum()) / loops.sum():.0f}")
cons, refl, nfetch = (rec[:, i].astype(np.float64) for i in (8, 9, 10))
print(f"service pass cycles: consume {cons.sum() / nserv.sum():.0f}, refill {refl.sum() / nserv.sum():.0f}, "
      f"start-DE+counters {(scyc.sum() - cons.sum() - refl.sum()) / nserv.sum():.0f}; "
      f"fetches per wave {nfetch.mean():.1f}")
sub = [rec[:, 11 + k].astype(np.float64).sum() / nserv.sum() for k in range(4)]
print("sub-stamps, cycles per pass: [0] %.0f, [1] %.0f, [2] %.0f, [3] %.0f" % tuple(sub))
print(f"wave start spread {st.max():.0f} us; first exhaust {np.nanmin(ex):.0f} us, median exhaust {np.nanmedian(ex):.0f} us")
q = np.percentile(en, [0, 10, 50, 90, 99, 100])
print("wave end percentiles (us): " + " ".join(f"p{p_}={v:.0f}" for p_, v in zip([0, 10, 50, 90, 99, 100], q)))
T = en.max()
line = []
for f_ in np.linspace(0.5, 1.0, 11):
    line.append(f"{f_ * T:.0f}us:{int(((st <= f_ * T) & (en > f_ * T)).sum())}")
print("running waves over time: " + " ".join(line))
# mean lanes busy: integrate wave cycle time vs pixel work
print(f"mean wave lifetime {np.mean(en - st):.0f} us of {T:.0f} us ({np.mean(en - st) / T:.3f})")
