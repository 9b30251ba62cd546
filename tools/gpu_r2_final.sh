#!/bin/bash
# Round-2 closing session on one GPU: the GPU test suite, the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace of it, and every BASELINE config at bench defaults.
# Every GPU step time-limited; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/final}
mkdir -p "$OUT/configs"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py > "$OUT/bench_HEADLINE.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_HEADLINE.json'));print('HEADLINE', round(d['value'],3), 'G/s', round(d['ms_per_step'],3), 'ms frac', round(d['roofline']['frac'],4), 'valu_busy', d['roofline'].get('valu_busy'), 'sha_ok', d['frame_sha_ok'], 'cpu', d['cpu_baseline']['value'])"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 1; }
# the profiled run's timed launches: steps / frames_per_launch of them, that many frames each
read K B < <(python -c "import json;d=json.load(open('$OUT/prof_bench.json'));b=d['config']['frames_per_launch'];print(-(-d['steps']//b), b)")
python tools/rocprof_timed.py $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) $K $B > "$OUT/rocprof_timed_HEADLINE.txt" && tail -n 3 "$OUT/rocprof_timed_HEADLINE.txt"
cp $(find "$OUT/prof" -name "*kernel_stats.csv" | head -1) "$OUT/rocprof_kernel_stats_HEADLINE.csv"
for spec in "C1:" "C2:" "C3:" "C4:" "C5:--steps 2 --warmup 1"; do
  wl=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python bench.py --workload $wl $a --no-cpu-baseline > "$OUT/configs/$wl.json" 2> "$OUT/configs/$wl.err" || { echo "bench $wl failed"; tail -5 "$OUT/configs/$wl.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/configs/$wl.json'));print('$wl', round(d['value'],3), 'G/s', round(d['ms_per_step'],3), 'ms/frame', 'frac', round(d['roofline']['frac'],4), 'valu_busy', d['roofline'].get('valu_busy'), 'sha_ok', d.get('frame_sha_ok'))"
done
echo FINAL_OK
