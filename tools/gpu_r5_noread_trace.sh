#!/bin/bash
# kernel trace of the drop-in loop without readback (noread: 2 frames in flight, no host waits)
OUT=gpurun_out/noread_trace${FRM_BLOCKS_PER_CU:+_bpc$FRM_BLOCKS_PER_CU}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/HEADLINE" -o run --output-format csv -- python3 tools/dropin_probe.py --workload HEADLINE --forms noread --frames 16 --hw-queues 16 > "$OUT/HEADLINE.jsonl" 2> "$OUT/HEADLINE.err" || { tail "$OUT/HEADLINE.err"; exit 1; }
python3 tools/trace_timeline.py "$(find "$OUT/HEADLINE" -name '*kernel_trace.csv' | head -1)" 48 > "$OUT/HEADLINE_timeline.txt"
cat "$OUT/HEADLINE.jsonl"
