#!/bin/bash
# Round 4 closing extras: the D2H copy-path probe, then service_min on the closing kernel (the
# driver's bench command, one launch of 30 frames), 2 interleaved rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/r4k}
mkdir -p "$OUT"
bash tools/gpu_d2h_modes.sh || exit 1
for round in 1 2; do
  for sm in 20 24 28; do
    FRM_SERVICE_MIN=$sm timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/sm_${sm}_$round.json" 2> "$OUT/sm_${sm}_$round.err" || { tail -5 "$OUT/sm_${sm}_$round.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/sm_${sm}_$round.json'));print('r$round service_min $sm:', round(d['ms_per_step'],4), 'ms sha', d.get('frame_sha_ok'), 'cnt', d.get('counters_ok'))"
  done
done
