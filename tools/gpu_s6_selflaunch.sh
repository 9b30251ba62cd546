#!/bin/bash
# bench.py --gpus N started WITHOUT a launcher (bench starts torch.distributed.run itself),
# N ranks sharing the one GPU over gloo (test hooks): the driver's N>1 invocation, rehearsed.
set -o pipefail
O=gpurun_out/selflaunch
mkdir -p $O
for n in 2 4 8; do
  FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus $n --steps 8 --warmup 2 --no-cpu-baseline > $O/gpus$n.json 2> $O/gpus$n.err || { tail -20 $O/gpus$n.err; exit 1; }
  tail -1 $O/gpus$n.json > $O/gpus$n.line && python3 -c "import json;d=json.load(open('$O/gpus$n.line'));print('$n', d['n_gpus'], round(d['value'],2), round(d['ms_per_step'],3), d['config']['parallelism'], d.get('comm'), 'sha_ok', d.get('frame_sha_ok'))"
done
