#!/bin/bash
# C5 (one frame per launch, 3 in flight) on the capped in-flight grid (12 one-wave workgroups per
# CU, the default for single-frame launches with frames in flight) against the full grid
# (FRM_BLOCKS_PER_CU=28: 7 waves/SIMD), interleaved.
OUT=${OUT:-gpurun_out/c5cap}
mkdir -p "$OUT"
for round in 1 2; do
  for bpc in 0 28; do
    FRM_BLOCKS_PER_CU=$bpc timeout -k 10 300 python bench.py --workload C5 --steps 8 --warmup 2 --no-cpu-baseline --no-dropin \
      > "$OUT/bpc${bpc}_$round.json" 2> "$OUT/bpc${bpc}_$round.err"
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -5 "$OUT/bpc${bpc}_$round.err"; exit $rc; fi
    python -c "import json;d=json.load(open('$OUT/bpc${bpc}_$round.json'));print('round $round bpc $bpc', round(d['ms_per_step'],2), 'ms')"
  done
done
