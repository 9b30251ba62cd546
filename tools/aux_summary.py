"""Summarise tools/bench_aux.py: `python tools/aux_summary.py MODEL.json KERNEL_TRACE.csv` ->
per kernel (and per blit output size) the average dispatch time from the rocprofv3 kernel
trace and the algorithmic HBM rate against MI355X's 8 TB/s (MI355X_MICROARCH.md). Prints JSON."""
import csv
import json
import sys

PEAK = 8.0e12
model = json.load(open(sys.argv[1]))
rows = list(csv.DictReader(open(sys.argv[2])))


def durations(name):
    out = []
    for r in rows:
        if name in r["Kernel_Name"]:
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r))
    return [d for _, d, _ in sorted(out)], [r for _, _, r in sorted(out)]


res = {}
for k in ("shade_pass", "unshuffle_bands"):
    d, _ = durations(k)
    d = d[1:]  # the first dispatch pays for cold caches / first touch
    ns = sum(d) / len(d)
    res[k] = {"avg_us": round(ns / 1e3, 2), "bytes": model[k]["bytes"],
              "GBps": round(model[k]["bytes"] / ns, 1), "frac_of_8TBps": round(model[k]["bytes"] / ns * 1e9 / PEAK, 3)}
d, rr = durations("blit_kernel")
reps = len(d) // 3
for i, (size, b) in enumerate(model["blit_kernel"]["bytes_per_dispatch"].items()):
    part = d[i * reps + 1:(i + 1) * reps]
    ns = sum(part) / len(part)
    res[f"blit_kernel {size}"] = {"avg_us": round(ns / 1e3, 2), "bytes": b, "GBps": round(b / ns, 1),
                                  "frac_of_8TBps": round(b / ns * 1e9 / PEAK, 3)}
print(json.dumps(res, indent=1))
