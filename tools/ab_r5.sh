#!/bin/bash
# Interleaved A/B of libfrm builds (fractal-ray-marching_amd/ab/NAME.so) on one box, tolerant of
# builds whose frames differ from the current goldens (bench.py exit 3 = counters differ): the
# ms/frame of each round is printed either way.
# Usage: VARIANTS="v1 w5 w6" ROUNDS=3 ARGS="--steps 30" OUT=gpurun_out/ab bash tools/ab_r5.sh
OUT=${OUT:-gpurun_out/ab}
ARGS=${ARGS:---steps 30 --warmup 3}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-3}); do
  for n in $VARIANTS; do
    FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-dropin \
      > "$OUT/${n}_$round.json" 2> "$OUT/${n}_$round.err"
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $n rc=$rc"; tail -5 "$OUT/${n}_$round.err"; exit $rc; fi
    python -c "import json;d=json.load(open('$OUT/${n}_$round.json'));print('round $round $n', round(d['ms_per_step'],3), 'ms sha_ok', d.get('frame_sha_ok'), 'counters_ok', d.get('counters_ok'))"
  done
done
