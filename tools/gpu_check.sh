#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace. Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
(lscpu | head -20; nproc; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS") > "$OUT/host.txt" 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name "*stats*" | head
echo ALL_OK
