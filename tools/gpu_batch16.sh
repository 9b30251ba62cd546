#!/bin/bash
# frames per launch 8 / 16 / 32 (a build with FRM_MAX_BATCH=32): whole headline and C2 frames
# and rank 0's share of an 8-way headline split with its simulated gather; interleaved rounds
set -o pipefail
OUT=gpurun_out/batch32
mkdir -p $OUT
LIB=$PWD/fractal-ray-marching_amd/variants/b32.so
for round in 1 2 3; do
  for B in 8 16 32; do
    FRM_LIB=$LIB timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE,C2 --ranks 1 --inflight 1 --batch $B --frames 192 > $OUT/whole_${B}_${round}.jsonl 2>> $OUT/err || { tail $OUT/err; exit 1; }
    FRM_LIB=$LIB timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch $B --frames 384 --gather 1 > $OUT/share_${B}_${round}.jsonl 2>> $OUT/err || { tail $OUT/err; exit 1; }
    python - <<PY
import json
w=[json.loads(l) for l in open("$OUT/whole_${B}_${round}.jsonl")]
s=[json.loads(l) for l in open("$OUT/share_${B}_${round}.jsonl")]
print("round $round batch $B", " ".join(f"{d['workload']} {d['ms_per_frame']:.4f}" for d in w), "share8", f"{s[-1]['ms_per_frame']:.4f}")
PY
  done
done
