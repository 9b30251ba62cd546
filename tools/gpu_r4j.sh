#!/bin/bash
# Round 4: frames per launch / frames in flight for the fixed workloads after fused scheduling
# (30 timed frames, the driver's default count).
set -o pipefail
OUT=${OUT:-gpurun_out/r4j}
mkdir -p "$OUT"
for round in 1 2 3; do
  for wl in HEADLINE C2 C3; do
    for spec in "15:1" "15:2" "30:1" "10:2"; do
      b=${spec%%:*}; f=${spec#*:}
      timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 10 --batch $b --inflight $f --no-cpu-baseline --no-dropin > "$OUT/${wl}_${b}_${f}_$round.json" 2> "$OUT/${wl}_${b}_${f}_$round.err" || { tail -5 "$OUT/${wl}_${b}_${f}_$round.err"; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/${wl}_${b}_${f}_$round.json'));print('r$round $wl batch $b inflight $f:', round(d['ms_per_step'],4), 'ms sha', d.get('frame_sha_ok'), 'cnt', d.get('counters_ok'))"
    done
  done
done
