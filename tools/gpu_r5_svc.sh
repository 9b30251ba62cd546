#!/bin/bash
# drop-in loop forms with the frame's shade/rank passes on the slot stream (off), on a service
# stream at default priority (normal) or at the device's greatest priority (high; also the copy
# streams): FRM_SVC_STREAM
mkdir -p gpurun_out/svc
for round in 1 2; do
for mode in off normal high; do
  for wl in HEADLINE HEADLINE_FLY; do
    if [ $mode = off ]; then unset FRM_SVC_STREAM; else export FRM_SVC_STREAM=$mode; fi
    timeout -k 10 300 python3 tools/dropin_probe.py --workload $wl --forms latency,noread,latency3 --frames 20 --hw-queues 16 > gpurun_out/svc/${wl}_${mode}_$round.jsonl 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/svc/${wl}_${mode}_$round.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('round $round svc $mode', d['workload'], d['form'], round(d['ms_per_frame'],3))"
  done
done
done
