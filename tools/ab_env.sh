#!/bin/bash
# interleaved A/B of environment settings on several workloads.
# CFGS: space-separated list of "base" or VAR=value tokens; WLS: workloads.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for round in 1 2; do
  for wl in ${WLS:-C2 HEADLINE}; do
    for cfg in ${CFGS:-base}; do
      if [ "$cfg" = base ]; then envset=""; else envset="$cfg"; fi
      env $envset timeout -k 10 200 python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/abenv.json" 2>"$OUT/abenv.err" || { echo "bench failed"; tail -5 "$OUT/abenv.err"; exit 1; }
      python -c "import json;d=json.load(open('$OUT/abenv.json'));print('r$round', '$wl', '$cfg', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],2), 'ms')"
    done
  done
done
