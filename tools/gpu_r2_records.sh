#!/bin/bash
# Round 2: GPU suite after the record split / resize history / iteration-cap changes; the
# resize probe; bench with 1 or 2 frames in flight at 4 and 16 hardware queues (INTEGRATION
# §3); PMC passes of the headline (march + shade kernels). Every GPU step time-limited.
set -o pipefail
OUT=${OUT:-gpurun_out/r2d}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python tools/resize_probe.py > "$OUT/resize_probe.json" 2> "$OUT/resize.err" || { tail "$OUT/resize.err"; exit 1; }
cat "$OUT/resize_probe.json"
for q in 4 16; do for f in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --hw-queues $q --inflight $f > "$OUT/bench_q${q}_f${f}.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_q${q}_f${f}.json'));print('queues $q inflight $f', round(d['ms_per_step'],3), 'ms', round(d['value'],2), 'G/s')"
done; done
OUT=$OUT/pmc ARGS="--steps 6 --warmup 2 --no-cpu-baseline" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py $OUT/pmc march_persistent > $OUT/pmc_HEADLINE_march.json && python tools/pmc_summary.py $OUT/pmc shade_pass > $OUT/pmc_HEADLINE_shade.json && cat $OUT/pmc_HEADLINE_march.json $OUT/pmc_HEADLINE_shade.json
