#!/bin/bash
# One GPU session: parity tests, the default bench line (+ CPU baseline), a rocprofv3 kernel
# trace of the same command, every BASELINE config. GPU steps are time-limited; the chain
# stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
(lscpu | head -20; nproc; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS") > "$OUT/host.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 1; }
python tools/rocprof_timed.py $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) 10 | tee "$OUT/rocprof_timed.txt"
[ -n "$NO_ALL" ] || OUT=$OUT/all bash tools/bench_all.sh
echo ALL_OK
