#!/bin/bash
# drop-in loop forms (tools/dropin_probe.py) at several persistent-grid sizes (FRM_BLOCKS_PER_CU:
# one-wave workgroups per CU; 0 = the occupancy limit): frames in flight share the GPU when each
# grid leaves room for the other frame's grid and the frames' shading passes
mkdir -p gpurun_out/bpc
for round in 1 2; do
for bpc in ${BPCS:-0 16 12 10}; do
  for wl in HEADLINE HEADLINE_FLY; do
    if [ $bpc = 0 ]; then unset FRM_BLOCKS_PER_CU; else export FRM_BLOCKS_PER_CU=$bpc; fi
    timeout -k 10 300 python3 tools/dropin_probe.py --workload $wl --forms ${FORMS:-latency,noread,latency3,noread3} --frames 20 --hw-queues 16 > gpurun_out/bpc/${wl}_${bpc}_$round.jsonl 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/bpc/${wl}_${bpc}_$round.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('round $round bpc $bpc', d['workload'], d['form'], round(d['ms_per_frame'],3))"
  done
done
done
