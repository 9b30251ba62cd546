#!/bin/bash
# Round 2: the default bench line (+ CPU baseline), its rocprofv3 kernel trace, C4 frames per
# launch, bench.py --gpus 2 (self-launched gloo ranks sharing device 0). Time-limited steps.
set -o pipefail
OUT=${OUT:-gpurun_out/r2g}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 1; }
python tools/rocprof_timed.py $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) 10 > "$OUT/rocprof_timed.txt" && cat "$OUT/rocprof_timed.txt"
for b in 1 2 4; do
  timeout -k 10 300 python bench.py --workload C4 --batch $b --steps 8 --warmup 4 --no-cpu-baseline > "$OUT/C4_b$b.json" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/C4_b$b.json'));print('C4 batch $b', round(d['ms_per_step'],2), 'ms', round(d['value'],2), 'G/s inflight', d['config']['frames_in_flight'], 'sha', d['frame_sha_ok'])"
done
FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { tail -30 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
