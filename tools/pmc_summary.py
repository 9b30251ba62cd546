"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output) for the render kernel.

Derived values follow MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8 XCDs;
VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64); VALU busy =
SQ_ACTIVE_INST_VALU * 2 cycles (wave64 on SIMD32) / (1024 SIMDs * GRBM_GUI_ACTIVE / 8);
WRITE_SIZE/FETCH_SIZE are in KiB (FETCH_SIZE doubled for gfx950's half-counted reads)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fractal-ray-marching_amd"))
from frm import provenance  # noqa: E402


KERNEL = "march_persistent"
# dispatches skipped at the start: the first launch of each frames-in-flight slot has no
# scheduling history (row-major fetch order) and is not the steady state bench.py times
SKIP = 2


def load(d, name):
    files = glob.glob(f"{d}/{name}/**/*counter_collection.csv", recursive=True)
    if not files:
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(files[0])):
        if KERNEL in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    # average over the steady-state dispatches of the render kernel
    keep = sorted(agg)[SKIP:] or sorted(agg)
    out = collections.defaultdict(float)
    for i in keep:
        for k, v in agg[i].items():
            out[k] += v / len(keep)
    return dict(out)


def frames_per_dispatch(d):
    """bench.py's frames per launch in the profiled run (its JSON line, written by pmc.sh)."""
    for n in ("sq", "wr", "rd", "sq2"):
        try:
            with open(f"{d}/{n}.json") as fh:
                line = json.loads(fh.read().strip().splitlines()[-1])
                if "config" in line:  # a bench.py line
                    return int(line["config"].get("frames_per_launch", 1))
                return int(line.get("batch", 1))  # a tools/pipeline_probe.py line
        except (OSError, ValueError, KeyError, IndexError):
            continue
    return 1


def main(d):
    c = {}
    c3 = load(d, "sq3")  # where the wave cycles go (SQ_WAVE_CYCLES of that pass)
    for n in ("sq", "sq2", "wr", "rd"):
        c.update(load(d, n))
    trace = glob.glob(f"{d}/sq/**/*kernel_trace.csv", recursive=True)
    dur = []
    for r in csv.DictReader(open(trace[0])):
        if KERNEL in r["Kernel_Name"]:
            dur.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    dur = [d for _, d in sorted(dur)]
    dur = dur[SKIP:] or dur
    t = sum(dur) / len(dur)
    grbm_xcd = c["GRBM_GUI_ACTIVE"] / 8
    B = frames_per_dispatch(d)
    s = {
        "frames_per_dispatch": B,
        "kernel_s_profiled": t,
        "clock_ghz": grbm_xcd / t / 1e9,
        "valu_wave_insts": c["SQ_INSTS_VALU"],
        "valu_lane_utilization": c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64),
        "valu_busy": c["SQ_ACTIVE_INST_VALU"] * 2 / (1024 * grbm_xcd),
        "salu_insts": c.get("SQ_INSTS_SALU"),
        "waves": c["SQ_WAVES"],
        "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"],
        "active_inst_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"],
        "smem_insts": c.get("SQ_INSTS_SMEM"),
        "vmem_insts": c.get("SQ_INSTS_VMEM"),
        # pass sq3 (its own SQ_WAVE_CYCLES): wave-parked (s_waitcnt / barrier) cycles, scalar /
        # misc / LDS issue, SALU and SMEM instruction cycles, branches (quad-cycle units cancel)
        "sq3": ({
            "wait_any_frac": c3["SQ_WAIT_ANY"] / c3["SQ_WAVE_CYCLES"],
            "active_inst_sca_frac": c3["SQ_ACTIVE_INST_SCA"] / c3["SQ_WAVE_CYCLES"],
            "active_inst_misc_frac": c3["SQ_ACTIVE_INST_MISC"] / c3["SQ_WAVE_CYCLES"],
            "active_inst_lds_frac": c3["SQ_ACTIVE_INST_LDS"] / c3["SQ_WAVE_CYCLES"],
            "inst_cycles_salu_frac": c3["SQ_INST_CYCLES_SALU"] / c3["SQ_WAVE_CYCLES"],
            "inst_cycles_smem_frac": c3["SQ_INST_CYCLES_SMEM"] / c3["SQ_WAVE_CYCLES"],
            "branch_insts": c3["SQ_INSTS_BRANCH"],
        } if c3 else None),
        "hbm_write_bytes": c.get("WRITE_SIZE", 0) * 1024,
        "hbm_read_bytes": 2 * c.get("FETCH_SIZE", 0) * 1024,
        "hbm_write_gbps": c.get("WRITE_SIZE", 0) * 1024 / t / 1e9,
        # per frame of the dispatch (a multi-frame launch renders B frames per dispatch)
        "hbm_write_bytes_per_frame": c.get("WRITE_SIZE", 0) * 1024 / B,
        "hbm_read_bytes_per_frame": 2 * c.get("FETCH_SIZE", 0) * 1024 / B,
        "kernel_s_per_frame_profiled": t / B,
        "dispatches_averaged": len(dur),
        # the kernel sources these counters were measured on (bench.py cites only a match)
        "source_sha256": provenance.source_sha256(),
    }
    print(json.dumps(s, indent=1))
    return s


if __name__ == "__main__":
    if len(sys.argv) > 2:
        KERNEL = sys.argv[2]
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
