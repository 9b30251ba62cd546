#!/bin/bash
# Round 2: full GPU suite, the default bench line, bench.py --gpus 2 self-launched (two gloo
# ranks sharing device 0, both N>1 modes). Every GPU step time-limited; stops at a failure.
set -o pipefail
OUT=${OUT:-gpurun_out/r2a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
for split in rows frames; do
  FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --split $split --no-cpu-baseline > "$OUT/bench2_$split.json" 2> "$OUT/bench2_$split.err" || { echo "bench2 $split failed"; tail -30 "$OUT/bench2_$split.err"; exit 1; }
  cat "$OUT/bench2_$split.json"
done
echo ALL_OK
