"""Per-kernel average duration over the LAST k dispatches of a rocprofv3 kernel trace (the
bench's timed region: `bench.py --steps k` runs warmup frames first), to compare with
bench.py's live HIP-event roofline.avg_kernel_ms (which brackets sort + march + shade)."""
import collections
import csv
import sys


def main(trace, k):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        n = r["Kernel_Name"]
        name = ("march_persistent" if "march_persistent" in n else "shade_pass" if "shade_pass" in n
                else "radix_sort" if "radix_sort" in n else None)
        if name:
            per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    total = 0.0
    for name in ("march_persistent", "radix_sort", "shade_pass"):
        d = per.get(name, [])
        calls = len(per["march_persistent"])
        # radix sort: several dispatches per frame; take the frames' share
        per_frame = len(d) // max(calls, 1) if calls else 1
        last = d[-k * max(per_frame, 1):]
        avg = sum(last) / k if last else 0.0
        total += avg
        print(f"{name:18s} last {k} frames: {avg:.3f} ms per frame ({len(d)} dispatches in the trace)")
    print(f"{'sum':18s} {total:.3f} ms per frame")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
