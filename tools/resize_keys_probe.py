"""Scheduling history across a resize, measured: a 4K headline frame (pose P1) is
rendered one at a time with the pixel order sorted by different cost-key maps injected through
frm_debug_set_pixel_keys, interleaved over ROUNDS rounds:

  exact     the 4K frame's own keys (the steady state)
  rowmajor  all keys equal (the stable sort keeps row-major order: no history)
  <name>    a map predicted from the keys of a 1920x1080 frame of the same view, by each
            resampler of RESAMPLERS below (max1 = the library's rescale_keys_kernel)

Prints one JSON line (ms per candidate, per round) and saves the key maps to OUT/keys.npz."""
import json
import os
import sys

import numpy as np
from scipy.ndimage import maximum_filter, uniform_filter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import frm  # noqa: E402

OUT = os.environ.get("OUT", "gpurun_out/resize")
ROUNDS = int(os.environ.get("ROUNDS", "3"))
os.makedirs(OUT, exist_ok=True)
w = frm.WORKLOADS["HEADLINE"]
W, H = w.width, w.height
p4k = frm.make_parameters(w, pose="P1")
p1080 = frm.make_parameters(w, pose="P1", width=1920, height=1080)


def upsample(src, pad):
    """max over the source pixels within `pad` of the one each destination pixel maps to"""
    sh, sw = src.shape
    m = maximum_filter(src, size=2 * pad + 1, mode="nearest") if pad else src
    ys = (np.arange(H) * sh) // H
    xs = (np.arange(W) * sw) // W
    return m[ys][:, xs]


def spikes(src, thr, pad, boost=255):
    """max1, raised to `boost` wherever a source pixel of key >= thr lies within `pad`"""
    hi = upsample((src >= thr).astype(np.uint8), pad) > 0
    return np.where(hi, np.maximum(upsample(src, 1), boost), upsample(src, 1))


def local_sd(src, size=9):
    """standard deviation of the source keys over a size x size window (noisy regions)"""
    f = src.astype(np.float32)
    m = uniform_filter(f, size)
    return np.sqrt(np.maximum(uniform_filter(f * f, size) - m * m, 0.0))


def noisy(src, pad, alpha, size=9):
    """max over +-pad, raised by alpha x the local standard deviation of the source keys"""
    up = upsample(src, pad).astype(np.float32)
    sd = upsample(local_sd(src, size), 0)
    return np.clip(up + alpha * sd, 0, 255)


RESAMPLERS = {
    "max1": lambda s: upsample(s, 1),
    "max4": lambda s: upsample(s, 4),
    "max8": lambda s: upsample(s, 8),
    "max16": lambda s: upsample(s, 16),
    "spk190p16": lambda s: spikes(s, 190, 16),
    "spk185p8": lambda s: spikes(s, 185, 8),
    "max4sd1": lambda s: noisy(s, 4, 1.0),
    "max4sd2": lambda s: noisy(s, 4, 2.0),
    "max8sd2": lambda s: noisy(s, 8, 2.0),
    "max8sd4": lambda s: noisy(s, 8, 4.0),
    "max1sd3": lambda s: noisy(s, 1, 3.0),
}
if os.environ.get("RESAMPLERS"):
    RESAMPLERS = {k: RESAMPLERS[k] for k in os.environ["RESAMPLERS"].split(",")}

res = {"ms": {}}
with frm.Renderer(device=0, max_steps=w.max_steps) as r:
    r.resize(1920, 1080)
    r.update_parameters_buffer(p1080)
    for _ in range(3):
        r.render(stats=True)
    k1080 = r.pixel_keys().reshape(1080, 1920)
    r.resize(W, H)
    r.update_parameters_buffer(p4k)
    res["ms_4k_first_frames"] = [r.render(stats=True)["kernel_ms"] for _ in range(6)]
    k4k = r.pixel_keys()
    cands = {"exact": k4k, "rowmajor": np.zeros_like(k4k)}
    for name, fn in RESAMPLERS.items():
        cands[name] = fn(k1080).astype(np.uint8).ravel()
    for rnd in range(ROUNDS):
        for name, keys in cands.items():
            r.render(stats=True)  # a steady frame in between (clocks)
            r.set_pixel_keys(keys)
            res["ms"].setdefault(name, []).append(round(r.render(stats=True)["kernel_ms"], 3))
        print(json.dumps({k: v[-1] for k, v in res["ms"].items()}), file=sys.stderr, flush=True)
np.savez_compressed(os.path.join(OUT, "keys.npz"), k1080=k1080, k4k=k4k)
print(json.dumps(res))
