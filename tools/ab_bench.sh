#!/bin/bash
# Interleaved A/B of libfrm builds (fractal-ray-marching_amd/ab/NAME.so, made by
# tools/build_variant.sh) on one box: ROUNDS rounds of `bench.py ARGS` per variant.
# Usage: VARIANTS="base new" ROUNDS=3 ARGS="--steps 20 --warmup 5" OUT=gpurun_out/ab bash tools/ab_bench.sh
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
ARGS=${ARGS:---steps 20 --warmup 5}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-3}); do
  for n in $VARIANTS; do
    FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-dropin \
      > "$OUT/${n}_$round.json" 2> "$OUT/${n}_$round.err" || { echo "bench $n failed"; tail -5 "$OUT/${n}_$round.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${n}_$round.json'));print('round $round $n', round(d['ms_per_step'],3), 'ms', d['frame_sha_ok'])"
  done
done
