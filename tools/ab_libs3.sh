#!/bin/bash
# A/B of alternative libfrm builds (fractal-ray-marching_amd/variants/*.so): ROUNDS interleaved
# rounds of the default bench (30 timed frames) per build, then a summary per build.
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
WL=${WL:-HEADLINE}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-3}); do
  for lib in fractal-ray-marching_amd/variants/*.so; do
    n=$(basename $lib .so)
    FRM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline $ARGS > "$OUT/ab_${WL}_${n}_$round.json" 2>"$OUT/ab_${WL}_${n}_$round.err" || { echo "bench $n failed"; tail -5 "$OUT/ab_${WL}_${n}_$round.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_${WL}_${n}_$round.json'));print('round $round $n', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],3), 'ms', 'sha_ok', d.get('frame_sha_ok'))"
  done
done
