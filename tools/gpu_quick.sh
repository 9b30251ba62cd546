#!/bin/bash
# parity tests then bench both kernels; every GPU step time-limited, chain stops on failure
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for k in persistent simple; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --kernel $k --no-cpu-baseline > "$OUT/bench_$k.json" 2> "$OUT/bench_$k.err" || { echo "bench $k failed"; tail -20 "$OUT/bench_$k.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$k.json'));print('$k', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],2), 'ms', 'kernel', round(d['roofline']['avg_kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],4))"
done
