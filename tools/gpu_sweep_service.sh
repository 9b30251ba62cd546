#!/bin/bash
# FRM_SERVICE_MIN sweep (lanes waiting before a Mandelbulb wave's service pass) on bench.py's
# headline and C2 lines, ROUNDS interleaved rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/svc}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-2}); do
  for sm in ${SMS:-16 20 24 28}; do
    for wl in ${WORKLOADS:-HEADLINE C2}; do
      FRM_SERVICE_MIN=$sm timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > "$OUT/${wl}_${sm}_$round.json" 2> "$OUT/${wl}_${sm}_$round.err" || { tail -3 "$OUT/${wl}_${sm}_$round.err"; exit 1; }
    done
    python -c "import json;print('round $round service_min $sm', ' '.join('%s %.3f' % (w, json.load(open('$OUT/%s_${sm}_$round.json' % w))['ms_per_step']) for w in '${WORKLOADS:-HEADLINE C2}'.split()))"
  done
done
