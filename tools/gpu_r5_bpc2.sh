#!/bin/bash
# persistent-grid size for frames in flight: the drop-in forms at 11/13/14 blocks per CU, and one
# rank's share of the 8-way row split (bench.py's N = 8 launches: 10 frames per launch, 2 in
# flight) at the default grid and at 12/14
mkdir -p gpurun_out/bpc2
for round in 1 2; do
for bpc in 0 11 12 13 14; do
  if [ $bpc = 0 ]; then unset FRM_BLOCKS_PER_CU; else export FRM_BLOCKS_PER_CU=$bpc; fi
  for wl in HEADLINE HEADLINE_FLY; do
    timeout -k 10 300 python3 tools/dropin_probe.py --workload $wl --forms latency,noread --frames 20 --hw-queues 16 > gpurun_out/bpc2/${wl}_${bpc}_$round.jsonl 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/bpc2/${wl}_${bpc}_$round.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('round $round bpc $bpc', d['workload'], d['form'], round(d['ms_per_frame'],3))"
  done
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch 10 --frames 40 > gpurun_out/bpc2/share8_${bpc}_$round.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/bpc2/share8_${bpc}_$round.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('round $round bpc $bpc share8', {k: v for k, v in d.items() if 'ms' in k})"
done
done
