#!/bin/bash
# A/B sweep of FRM_SERVICE_MIN on the headline bench (one process per setting)
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > "$OUT/pytest_parity.log" 2>&1 || { echo "parity failed"; tail -20 "$OUT/pytest_parity.log"; exit 1; }
tail -1 "$OUT/pytest_parity.log"
for m in ${MS:-1 8 16 24 32 40 48}; do
  FRM_SERVICE_MIN=$m timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/sweep_$m.json" 2>"$OUT/sweep_$m.err" || { echo "bench $m failed"; tail -5 "$OUT/sweep_$m.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sweep_$m.json'));print('service_min $m', round(d['value'],3), 'Gsteps/s', round(d['roofline']['avg_kernel_ms'],2), 'ms')"
done
