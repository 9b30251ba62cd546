#!/bin/bash
# A/B benchmark of alternative libfrm builds (lib/variants/*.so), interleaved rounds.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for round in 1 2; do
  for lib in fractal-ray-marching_amd/variants/*.so; do
    n=$(basename $lib .so)
    FRM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_$n.json" 2>"$OUT/ab_$n.err" || { echo "bench $n failed"; tail -5 "$OUT/ab_$n.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$n.json'));print('round $round $n', round(d['value'],3), 'Gsteps/s', round(d['roofline']['avg_kernel_ms'],2), 'ms')"
  done
done
