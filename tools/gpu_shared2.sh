# 2 ranks sharing one GPU over gloo (test hooks): the N>1 bench paths end to end
set -o pipefail
O=gpurun_out/shared2
mkdir -p $O
for split in rows frames; do
  FRM_BENCH_SHARED_DEVICE=1 FRM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --split $split --steps 6 --warmup 3 > $O/$split.json 2> $O/$split.err || { tail -20 $O/$split.err; exit 1; }
  tail -1 $O/$split.json > $O/$split.line && python -c "import json;d=json.load(open('$O/$split.line'));print('$split', round(d['value'],2), round(d['ms_per_step'],3), d['config']['parallelism'], d['config']['frames_in_flight'], d['scaling'])"
done
