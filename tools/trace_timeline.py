"""Timeline of the last dispatches of a rocprofv3 kernel trace: one line per dispatch with
start / end relative to the first printed dispatch (ms), duration and queue id, to see how
frames in flight overlap (sort -> march -> shade of consecutive frames)."""
import csv
import sys


def main(trace, n):
    rows = []
    for r in csv.DictReader(open(trace)):
        name = r["Kernel_Name"]
        short = ("march" if "march_persistent" in name else "shade" if "shade_pass" in name
                 else "sort" if "radix_sort" in name or "Radix" in name else name.split("(")[0][-30:])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short,
                     r.get("Queue_Id", r.get("Stream_Id", "?")), r.get("Grid_Size", r.get("Grid_Size_X", "?"))))
    rows.sort()
    rows = rows[-n:]
    t0 = rows[0][0]
    for s, e, name, q, g in rows:
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  q{q:>3s} {name} grid={g}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
