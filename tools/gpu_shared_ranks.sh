#!/bin/bash
# The row split at world sizes 4 and 8 on ONE GPU (ranks share device 0 over gloo, host-staged
# gather; bench.py's test hooks): checks the band geometry, rank-major gather and unshuffle of
# the headline frame at the driver's world sizes (frame_sha_ok against the golden hash).
# Timing is meaningless here (the ranks share one GPU).
set -o pipefail
OUT=gpurun_out/shared_ranks
mkdir -p $OUT
for n in 4 8; do
  FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --no-cpu-baseline > $OUT/gpus$n.json 2> $OUT/gpus$n.err || { echo "gpus $n failed"; tail -20 $OUT/gpus$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/gpus$n.json'));print($n, d['comm'], 'sha_ok', d['frame_sha_ok'], d['config'].get('frames_per_launch'), d['config'].get('parallelism'))"
done
