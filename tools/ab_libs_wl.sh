#!/bin/bash
# A/B of libfrm builds (fractal-ray-marching_amd/variants/*.so) on several workloads,
# interleaved rounds. WLS: workloads (default HEADLINE).
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for round in 1 2; do
  for wl in ${WLS:-HEADLINE}; do
    for lib in fractal-ray-marching_amd/variants/*.so; do
      n=$(basename $lib .so)
      FRM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_$n.json" 2>"$OUT/ab_$n.err" || { echo "bench $n failed"; tail -5 "$OUT/ab_$n.err"; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab_$n.json'));print('r$round $wl $n', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],3), 'ms')"
    done
  done
done
