#!/bin/bash
# FRM_SERVICE_MIN sweep on the headline and C2 (bench defaults, 2 interleaved rounds)
mkdir -p gpurun_out/svcmin
for round in 1 2; do
  for wl in HEADLINE C2; do
    for m in ${MS:-16 20 24 28 32 40}; do
      FRM_SERVICE_MIN=$m timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-dropin > gpurun_out/svcmin/${wl}_${m}_$round.json 2> gpurun_out/svcmin/${wl}_${m}_$round.err || { tail -5 gpurun_out/svcmin/${wl}_${m}_$round.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/svcmin/${wl}_${m}_$round.json'));print('round $round $wl service_min $m', round(d['ms_per_step'],3), 'ms', d.get('counters_ok'))"
    done
  done
done
