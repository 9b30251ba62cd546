#!/bin/bash
# Interleaved A/B of libfrm builds (ab/NAME.so) on the drop-in loop alone (tools/dropin_probe.py, 2 in
# flight, a frame of readback latency): HEADLINE_FLY and the fixed headline, ROUNDS rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/ab_dropin_only}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-3}); do
  for n in $VARIANTS; do
    for wl in HEADLINE_FLY HEADLINE; do
      FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 200 python tools/dropin_probe.py --workload $wl --forms ${FORMS:-latency} > "$OUT/${wl}_${n}_$round.jsonl" 2> "$OUT/${wl}_${n}_$round.err" || { tail -5 "$OUT/${wl}_${n}_$round.err"; exit 1; }
    done
    python -c "import json;print('round $round $n', ' '.join('%s %s %.3f' % (w, d['form'], d['ms_per_frame']) for w in ('HEADLINE_FLY','HEADLINE') for d in map(json.loads, open('$OUT/%s_${n}_$round.jsonl' % w))))"
  done
done
