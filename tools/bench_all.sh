#!/bin/bash
# bench every BASELINE configuration on one GPU, both kernels (C5 persistent only)
set -o pipefail
OUT=${OUT:-gpurun_out/all}
mkdir -p "$OUT"
run() {  # workload kernel steps
  timeout -k 10 400 python bench.py --workload $1 --kernel $2 --steps $3 --warmup 2 --no-cpu-baseline > "$OUT/$1_$2.json" 2> "$OUT/$1_$2.err" || { echo "bench $1 $2 failed"; tail -5 "$OUT/$1_$2.err"; return 1; }
  python -c "import json;d=json.load(open('$OUT/$1_$2.json'));print('$1', '$2', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],2), 'ms/frame', round(d['frames_per_sec'],2), 'fps', 'steps/frame', int(d['march_steps_per_frame']))"
}
for w in C1 C2 C3 HEADLINE C4; do  # persistent first: as the bench contract (--steps 5 --warmup 2)
  for k in persistent simple; do run $w $k 5 || exit 1; done
done
run C5 persistent 1 || exit 1
echo ALL_DONE
