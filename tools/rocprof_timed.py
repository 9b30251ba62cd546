"""Per-frame device time of the LAST k launches of a rocprofv3 kernel trace (the bench's timed
region: `bench.py --steps k` runs warmup frames first), to compare with bench.py's live
HIP-event roofline.avg_kernel_ms. With B frames per launch (bench --batch; argv[3]) the
times are divided by B: per frame.

With frames in flight (bench.py --inflight F > 1) the frames' kernels overlap, so the
per-frame time is the SPAN of the last k frames' dispatches (first start to last end) / k,
which is what bench.py's events measure; the per-kernel average durations are printed too
(a persistent march dispatch then also holds the time it shares the GPU with its
neighbours)."""
import collections
import csv
import sys


def kind(n):
    return ("march_persistent" if "march_persistent" in n else "shade_pass" if "shade_pass" in n
            else "rank_pass" if "rank_pass" in n else "radix_sort" if "radix_sort" in n else None)


def main(trace, k, batch=1):
    rows = []
    for r in csv.DictReader(open(trace)):
        name = kind(r["Kernel_Name"])
        if name:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    per = collections.defaultdict(list)
    for s, e, name in rows:
        per[name].append((e - s) / 1e6)
    calls = len(per["march_persistent"])
    total = 0.0
    for name in ("march_persistent", "radix_sort", "shade_pass", "rank_pass"):
        d = per.get(name, [])
        per_frame = len(d) // max(calls, 1) if calls else 1  # radix sort: several dispatches per frame
        last = d[-k * max(per_frame, 1):]
        avg = sum(last) / k / batch if last else 0.0
        total += avg
        print(f"{name:18s} last {k} launches: {avg:.3f} ms per frame ({len(d)} dispatches in the trace, "
              f"{batch} frames per launch)")
    print(f"{'sum':18s} {total:.3f} ms per frame (sum of dispatch durations)")
    # span: from the first dispatch of the first timed frame's march (minus its sort) to the
    # end of the last dispatch
    marches = [(s, e) for s, e, n in rows if n == "march_persistent"]
    if len(marches) >= k:
        first = marches[-k][0]
        sorts_before = [s for s, e, n in rows if n == "radix_sort" and s <= first]
        t0 = sorts_before[-1] if sorts_before else first
        t0 = min([t0] + [s for s, e, n in rows if s >= t0])
        t1 = max(e for s, e, n in rows if s >= t0)
        print(f"{'span':18s} {(t1 - t0) / 1e6 / k / batch:.3f} ms per frame (first start to last end of the last "
              f"{k} launches)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5, int(sys.argv[3]) if len(sys.argv) > 3 else 1)
