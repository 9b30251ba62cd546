#!/bin/bash
# bench.py --mode group on the one-GPU box (a one-device group, and 4 ranks rehearsed on device 0
# with the copy gather), and one rank's share of an 8-way split in single-frame launches (2 in
# flight) at the in-flight grid cap (12 per CU) and at the full grid (FRM_BLOCKS_PER_CU=28)
mkdir -p gpurun_out/group
timeout -k 10 300 python bench.py --gpus 1 --mode group --steps 20 > gpurun_out/group/g1.json 2> gpurun_out/group/g1.err || { tail gpurun_out/group/g1.err; exit 1; }
FRM_BENCH_GROUP_DEVICES=0,0,0,0 timeout -k 10 300 python bench.py --gpus 4 --mode group --steps 20 > gpurun_out/group/g4.json 2> gpurun_out/group/g4.err || { tail gpurun_out/group/g4.err; exit 1; }
for f in g1 g4; do python3 -c "import json;d=json.load(open('gpurun_out/group/$f.json'));print('$f', round(d['ms_per_step'],3), 'ms', d['frame_sha_ok'], d.get('counters_ok'), d['config']['parallelism'])"; done
for round in 1 2; do
for bpc in 0 28; do
  if [ $bpc = 0 ]; then unset FRM_BLOCKS_PER_CU; else export FRM_BLOCKS_PER_CU=$bpc; fi
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch 1 --frames 40 > gpurun_out/group/share8_b1_${bpc}_$round.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/group/share8_b1_${bpc}_$round.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('round $round bpc $bpc share8 batch1', round(d['ms_per_frame'],4))"
done
done
