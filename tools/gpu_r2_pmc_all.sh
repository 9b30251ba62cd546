#!/bin/bash
# PMC passes (tools/pmc.sh: one counter group per rocprofv3 run) for every BASELINE GPU
# config at bench.py's defaults, summarised per kernel with the source hash
# (tools/pmc_summary.py). Every pass time-limited inside pmc.sh; stops at a failure.
set -o pipefail
OUT=${OUT:-gpurun_out/r2pmc}
mkdir -p "$OUT"
for spec in "HEADLINE:--batch 16 --steps 32 --warmup 32" "C2:--batch 16 --steps 32 --warmup 32" "C3:--batch 16 --steps 32 --warmup 32" "C4:--batch 16 --steps 32 --warmup 32" "C5:--steps 3 --warmup 2"; do
  wl=${spec%%:*}; a=${spec#*:}
  OUT=$OUT/$wl ARGS="--workload $wl $a --no-cpu-baseline" bash tools/pmc.sh > /dev/null || { echo "pmc $wl failed"; exit 1; }
  python tools/pmc_summary.py $OUT/$wl march_persistent > $OUT/pmc_${wl}_march.json || exit 1
  python tools/pmc_summary.py $OUT/$wl shade_pass > $OUT/pmc_${wl}_shade.json || exit 1
  python -c "import json;s=json.load(open('$OUT/pmc_${wl}_march.json'));print('$wl march valu_busy', round(s['valu_busy'],3), 'lane_util', round(s['valu_lane_utilization'],3), 'wr MB/frame', round(s['hbm_write_bytes_per_frame']/1e6,1), 'rd MB/frame', round(s['hbm_read_bytes_per_frame']/1e6,1), 'GB/s wr', round(s['hbm_write_gbps'],1), 'B', s['frames_per_dispatch'])"
done
