#!/bin/bash
# The headline rendered the ways a host can drive libfrm: one frame per
# frm_render with 1 or 2 frames in flight and 4 or 16 hardware queues, and bench's default of
# 8 frames per launch. 2 interleaved rounds; every run time-limited; stops at a failure.
set -o pipefail
OUT=${OUT:-gpurun_out/dropin}
mkdir -p "$OUT"
for r in 1 2; do
  for m in "b1f1q4:--batch 1 --inflight 1 --hw-queues 4" "b1f2q4:--batch 1 --inflight 2 --hw-queues 4" "b1f1q16:--batch 1 --inflight 1 --hw-queues 16" "b1f2q16:--batch 1 --inflight 2 --hw-queues 16" "b8:"; do
    n=${m%%:*}; a=${m#*:}
    timeout -k 10 200 python bench.py --no-cpu-baseline $a > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err" || { echo "$n failed"; tail -5 "$OUT/${n}_$r.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${n}_$r.json'));c=d['config'];print('r$r $n', round(d['ms_per_step'],3), 'ms', round(d['value'],2), 'G/s', 'batch', c.get('frames_per_launch'), 'inflight', c.get('frames_in_flight'), 'queues', c.get('gpu_max_hw_queues'))"
  done
done
