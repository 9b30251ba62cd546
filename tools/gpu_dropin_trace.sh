#!/bin/bash
# The drop-in loop's forms (tools/dropin_probe.py: sync, latency 2/3 in flight, no readback) on the
# fixed headline and HEADLINE_FLY, then a kernel trace of the latency form (2 in flight, a frame of
# readback latency) with its dispatch timeline (tools/trace_timeline.py): where frames overlap and
# where the frame boundary's short kernels wait.
set -o pipefail
OUT=${OUT:-gpurun_out/dropin_trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in HEADLINE HEADLINE_FLY; do
  timeout -k 10 300 python3 tools/dropin_probe.py --workload $wl --forms sync,latency,latency3,noread,noread3 --frames 20 \
    > "$OUT/${wl}_forms.jsonl" 2> "$OUT/${wl}_forms.err" || { tail "$OUT/${wl}_forms.err"; exit 1; }
  cat "$OUT/${wl}_forms.jsonl"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$wl" -o run --output-format csv -- python3 tools/dropin_probe.py --workload $wl --forms latency --frames 16 > "$OUT/$wl.jsonl" 2> "$OUT/$wl.err" || { tail "$OUT/$wl.err"; exit 1; }
  python3 tools/trace_timeline.py "$(find "$OUT/$wl" -name '*kernel_trace.csv' | head -1)" 60 > "$OUT/${wl}_timeline.txt"
done
echo DROPIN_TRACE_OK
