#!/bin/bash
# Kernel trace of the drop-in loop (2 in flight, a frame of readback latency) on HEADLINE_FLY and on
# the fixed headline: per-frame march spans and overlap (tools/trace_timeline.py-style summary).
set -o pipefail
OUT=${OUT:-gpurun_out/dropin_trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in HEADLINE_FLY HEADLINE; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$wl" -o run --output-format csv -- python3 tools/dropin_probe.py --workload $wl --forms latency --frames 16 > "$OUT/$wl.jsonl" 2> "$OUT/$wl.err" || { tail "$OUT/$wl.err"; exit 1; }
  cat "$OUT/$wl.jsonl"
done
