#!/bin/bash
# Round 4: the batched fly-through's frame check after the capture fix, and a frames-per-launch /
# frames-in-flight sweep of the batched HEADLINE_FLY line (30 timed frames).
set -o pipefail
OUT=${OUT:-gpurun_out/r4i}
mkdir -p "$OUT"
for round in 1 2; do
  for spec in "15:1" "15:2" "10:2" "8:2" "5:3" "30:1"; do
    b=${spec%%:*}; f=${spec#*:}
    timeout -k 10 200 python bench.py --workload HEADLINE_FLY --steps 30 --warmup 10 --batch $b --inflight $f --no-cpu-baseline --no-dropin > "$OUT/fly_${b}_${f}_$round.json" 2> "$OUT/fly_${b}_${f}_$round.err" || { tail -5 "$OUT/fly_${b}_${f}_$round.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/fly_${b}_${f}_$round.json'));c=d['config'];print('r$round fly batch $b inflight $f:', round(d['ms_per_step'],3), 'ms', c.get('frames_per_launch'), c.get('frames_in_flight'), 'sha', d.get('frame_sha_ok'))"
  done
done
