#!/bin/bash
# Round 4: GPU tests on the fused-scheduling tree (rank pass, copy-stream readback, pool, no-drain
# resize), a drop-in kernel trace, then the A/B base (HEAD) vs r1 on the moving-frame loops.
set -o pipefail
OUT=${OUT:-gpurun_out/r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
d="$OUT/trace_HEADLINE_latency"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 tools/dropin_probe.py --workload HEADLINE --forms latency --frames 16 > "$d.jsonl" 2> "$d.err" || { tail "$d.err"; exit 1; }
python3 tools/trace_timeline.py $(ls "$d"/*/*kernel_trace.csv "$d"/*kernel_trace.csv 2>/dev/null | head -1) 40 > "$d.timeline.txt" || exit 1
VARIANTS="base r1" ROUNDS=2 OUT=gpurun_out/ab_r1 bash tools/gpu_ab_dropin.sh
for n in base r1; do
  FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 200 python tools/resize_loop_probe.py --workload HEADLINE > "$OUT/resize_loop_$n.json" 2> "$OUT/resize_loop_$n.err" || { tail -5 "$OUT/resize_loop_$n.err"; exit 1; }
  echo "$n $(cat $OUT/resize_loop_$n.json)"
done
