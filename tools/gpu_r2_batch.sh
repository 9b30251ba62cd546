#!/bin/bash
# Round 2: multi-frame launches. GPU suite, then one rank's share of an 8/4/2-way split with
# 1, 2, 4 frames per launch (3 or 2 launches in flight), rank 0 with gather, the whole frame
# with 1/2/4 per launch; bench row split on one GPU... Every GPU step time-limited.
set -o pipefail
OUT=${OUT:-gpurun_out/r2f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-not nothing}" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 3,2 --batch 1,2,4 --frames 48 > "$OUT/probe_8way_batch.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
timeout -k 10 400 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch 4,8 --frames 48 --rank-ids all > "$OUT/probe_8way_all.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
timeout -k 10 400 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8,4,2 --inflight 2 --batch 4 --frames 48 --gather 1 > "$OUT/probe_gather_batch.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
timeout -k 10 400 python tools/pipeline_probe.py --workloads HEADLINE,C2 --ranks 1 --inflight 1,2 --batch 1,2,4 --frames 32 > "$OUT/probe_whole_batch.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
cat "$OUT"/probe_*.jsonl | python tools/pipe_summary.py
