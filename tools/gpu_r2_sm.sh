#!/bin/bash
# service_min re-sweep with multi-frame launches (bench defaults), headline / C2 / C4.
set -o pipefail
OUT=${OUT:-gpurun_out/r2h}
mkdir -p "$OUT"
for wl in HEADLINE C2 C4; do for sm in 20 24 28 32; do
  st=32; [ $wl = C4 ] && st=8
  FRM_SERVICE_MIN=$sm timeout -k 10 200 python bench.py --workload $wl --steps $st --no-cpu-baseline > "$OUT/sm_${wl}_$sm.json" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sm_${wl}_$sm.json'));print('$wl service_min $sm', round(d['ms_per_step'],3), 'ms', round(d['value'],2), 'G/s')"
done; done
