#!/usr/bin/env python3
"""Summary of tools/keys_dump.py maps (moving frames): how well frame k's
per-pixel cost keys predict frame k+1's costliest pixels, and the frame end a list schedule by
each candidate key map would reach (model: a pixel starts when the work fetched before it is
done, T = 11 ms of work, and then runs its bodies at 0.55 us each, a lone lane's rate).

    python tools/keys_analysis.py keys_time.npz [keys_orbit.npz ...] > summary.json
"""
import json
import sys

import numpy as np
from scipy.ndimage import maximum_filter, uniform_filter


def cost(k):
    return 2.0 ** (k / 16.0) - 1.0  # bodies from the key 16 log2(bodies + 1)


def frame_end(order_keys, cb, T=11.0, us=0.55e-3):
    order = np.argsort(-order_keys.ravel(), kind="stable")
    c = cb[order]
    start = (np.cumsum(c) - c) / c.sum() * T
    e = start + c * us
    i = int(np.argmax(e))
    return {"end_ms": round(float(e[i]), 3), "worst_pixel_bodies": round(float(c[i])), "its_start_ms": round(float(start[i]), 3)}


def main(paths):
    out = {}
    for p in paths:
        K = np.load(p)["keys"].astype(np.int32)
        a, b = K[1], K[2]
        cb = cost(b.ravel())
        spike = b >= 190
        top = np.argsort(-cb)[:10]
        res = {
            "frames": int(K.shape[0]), "size": [int(K.shape[2]), int(K.shape[1])],
            "same_key_frac": float((a == b).mean()), "corr": float(np.corrcoef(a.ravel(), b.ravel())[0, 1]),
            "spikes_ge190": int(spike.sum()),
            "prev_key_at_spikes_p10_p50_p90": [float(v) for v in np.percentile(a[spike], [10, 50, 90])],
            "top10_bodies": [round(float(v)) for v in cb[top]],
            "top10_prev_keys": [int(v) for v in a.ravel()[top]],
            "model_own_keys": frame_end(b, cb),
            "model_prev_keys": frame_end(a, cb),
        }
        for r in (1, 2, 4, 8, 16):
            res[f"model_prev_max_r{r}"] = frame_end(maximum_filter(a, size=2 * r + 1), cb)
        res["model_prev_mean_r2"] = frame_end(uniform_filter(a.astype(float), size=5), cb)
        out[p.rsplit("/", 1)[-1]] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
