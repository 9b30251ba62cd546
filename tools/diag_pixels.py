"""Diagnostic: compare one GPU frame with the oracle and print differing pixels."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "fractal-ray-marching_amd"); sys.path.insert(0, "tests")
import frm
from oracle import frm_oracle as fo
from helpers import params_for

scene, iters, time, W, H, ms = [float(v) for v in sys.argv[1:7]] if len(sys.argv) > 6 else (15, 0, 0.0, 96, 54, 128)
scene, iters, W, H, ms = int(scene), int(iters), int(W), int(H), int(ms)
p = params_for(scene, iters, time, W, H)
with frm.Renderer(max_steps=ms) as r:
    r.resize(W, H)
    r.update_parameters_buffer(p)
    st = r.render()
    img = r.read_frame()
ref = fo.render(p, W, H, ms, linear=True, info=True)
print("gpu counters", [st[k] for k in ("pixels", "hit_pixels", "primary_steps", "shadow_steps", "normal_evals")])
print("cpu counters", ref["counters"][:5])
d = np.argwhere(np.any(img != ref["rgba"], axis=-1))
print("differing", len(d))
for y, x in d[:12]:
    print((x, y), "gpu", img[y, x], "cpu", ref["rgba"][y, x], "lin", ref["linear"][y, x], "info", hex(ref["info"][y, x]))
