#!/bin/bash
# PMC passes of the drop-in loop (one frame per frm_render, 2 in flight, every frame read back a
# frame late; tools/dropin_probe.py) on the moving and the fixed headline: VALU busy of the
# single-frame march dispatches the binding runs.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_dropin}
mkdir -p "$OUT"
for wl in HEADLINE_FLY HEADLINE; do
  OUT="$OUT/pmc_raw/${wl}_dropin" PROG=tools/dropin_probe.py ARGS="--workload $wl --forms latency --frames 30" bash tools/pmc.sh > /dev/null || { echo "pmc $wl failed"; exit 1; }
  python tools/pmc_summary.py "$OUT/pmc_raw/${wl}_dropin" > "$OUT/pmc_${wl}_dropin_march.json" || exit 1
  python -c "import json;s=json.load(open('$OUT/pmc_${wl}_dropin_march.json'));print('$wl dropin', 'valu_busy', round(s['valu_busy'],3), 'lane_util', round(s['valu_lane_utilization'],3), 'kernel ms', round(s['kernel_s_per_frame_profiled']*1e3,3))"
done
