"""Classified P1 report (tests/p1_classify.py) for the bench's frames at BASELINE size and
the fixed poses at 320x180: writes profiles/round2/p1_classes.json (quoted in DESIGN §3)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd"), os.path.join(ROOT, "tests")]
import frm  # noqa: E402
import p1_classify  # noqa: E402
from helpers import params_for  # noqa: E402
from oracle import frm_oracle  # noqa: E402

out = {}
for name in ("HEADLINE", "C2"):
    w = frm.WORKLOADS[name]
    t0 = time.time()
    out[f"{name}_P1"] = p1_classify.classify(frm_oracle, frm.make_parameters(w, pose="P1"), w.width, w.height,
                                             w.max_steps, threads=os.cpu_count())
    out[f"{name}_P1"]["seconds"] = round(time.time() - t0, 1)
    print(name, json.dumps(out[f"{name}_P1"]), flush=True)
for pose in ("P0", "P1", "P2"):
    out[f"mandelbulb_320x180_{pose}"] = p1_classify.classify(
        frm_oracle, params_for(18, 12, frm.POWER8_TIME, 320, 180, pose=pose), 320, 180, 256)
path = os.path.join(ROOT, "profiles", "round2", "p1_classes.json")
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
print("wrote", path)
