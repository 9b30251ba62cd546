#!/bin/bash
# Round 4, re-entry session: smoke on the rebuilt tree, then a kernel trace of the drop-in loop
# (one frame per frm_render, 2 in flight, a frame of readback latency) on the moving headline and
# the fixed one, with a per-dispatch timeline of the last frames (where the frame boundary goes).
set -o pipefail
OUT=${OUT:-gpurun_out/r4d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
for wl in HEADLINE_FLY HEADLINE; do
  for form in latency noread; do
    d="$OUT/trace_${wl}_${form}"
    timeout -k 10 300 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 tools/dropin_probe.py --workload $wl --forms $form --frames 16 > "$d.jsonl" 2> "$d.err" || { tail "$d.err"; exit 1; }
    cat "$d.jsonl"
    csv=$(ls "$d"/*/*kernel_trace.csv "$d"/*kernel_trace.csv 2>/dev/null | head -1)
    python3 tools/trace_timeline.py "$csv" 60 > "$d.timeline.txt" || exit 1
  done
done
