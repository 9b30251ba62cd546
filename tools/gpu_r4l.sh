#!/bin/bash
# service_min on the drop-in loops (one frame per frm_render, 2 in flight), 2 interleaved rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/r4l}
mkdir -p "$OUT"
for round in 1 2; do
  for sm in 16 20 24; do
    FRM_SERVICE_MIN=$sm timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency --frames 30 > "$OUT/fly_${sm}_$round.jsonl" 2> "$OUT/fly_${sm}_$round.err" || { tail -3 "$OUT/fly_${sm}_$round.err"; exit 1; }
    FRM_SERVICE_MIN=$sm timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency --frames 30 > "$OUT/fix_${sm}_$round.jsonl" 2> "$OUT/fix_${sm}_$round.err" || { tail -3 "$OUT/fix_${sm}_$round.err"; exit 1; }
    python3 -c "import json;a=json.loads(open('$OUT/fly_${sm}_$round.jsonl').read().splitlines()[-1]);b=json.loads(open('$OUT/fix_${sm}_$round.jsonl').read().splitlines()[-1]);print('r$round service_min $sm: fly', round(a['ms_per_frame'],3), 'fixed', round(b['ms_per_frame'],3))"
  done
done
