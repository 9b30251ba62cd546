#!/bin/bash
# after the batch-32 / slot-history / exact-step-count change: GPU tests, the driver's bench
# command at N=1, the default bench, the row split over 2 gloo ranks on the one GPU with the
# driver's step counts, and the 8-way share probe at 10 and 16 frames per launch
set -o pipefail
OUT=gpurun_out/s5batch
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
show() { python -c "import json;d=json.load(open('$1'));print('$1', 'steps', d['steps'], 'warmup', d['warmup'], round(d['ms_per_step'],4), 'ms', round(d['value'],3), 'G/s', 'B', d['config'].get('frames_per_launch'), 'F', d['config'].get('frames_in_flight'), 'sha_ok', d.get('frame_sha_ok'))"; }
for rnd in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drv_$rnd.json 2> $OUT/drv.err || { tail -20 $OUT/drv.err; exit 1; }
show $OUT/drv_$rnd.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/def_$rnd.json 2> $OUT/def.err || { tail -20 $OUT/def.err; exit 1; }
show $OUT/def_$rnd.json
done
FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/g2.json 2> $OUT/g2.err || { tail -20 $OUT/g2.err; exit 1; }
show $OUT/g2.json
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch 10,16 --frames 320 --gather 1 --repeat 2 > $OUT/share.jsonl 2> $OUT/share.err || { tail $OUT/share.err; exit 1; }
python -c "
import json
for l in open('$OUT/share.jsonl'): d=json.loads(l); print('share8 batch', d['batch'], round(d['ms_per_frame'],4))"
