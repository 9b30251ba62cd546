#!/bin/bash
# Drop-in loop forms (tools/dropin_probe.py) with libfrm's slot streams on own (CU-masked) queues
# and on pooled plain streams (FRM_SLOT_STREAMS=plain), + a kernel trace of the noread form.
set -o pipefail
OUT=${OUT:-gpurun_out/dropin}
mkdir -p "$OUT"
export TMPDIR=/tmp
for kind in cumask plain; do
  FRM_SLOT_STREAMS=$kind timeout -k 10 300 python tools/dropin_probe.py --workload HEADLINE_FLY --forms sync,latency,noread,noread3 > "$OUT/fly_$kind.jsonl" 2> "$OUT/fly_$kind.err" || { tail "$OUT/fly_$kind.err"; exit 1; }
  sed "s/^/$kind /" "$OUT/fly_$kind.jsonl"
done
FRM_SLOT_STREAMS=plain timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_plain" -o run --output-format csv -- python3 tools/dropin_probe.py --workload HEADLINE_FLY --forms noread --frames 6 > "$OUT/prof.jsonl" 2> "$OUT/prof.err" || { tail "$OUT/prof.err"; exit 1; }
echo DONE
