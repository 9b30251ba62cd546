#!/bin/bash
# The drop-in loop (bench.py's dropin_ms_per_frame: single-frame launches, 2 in flight) at 8K (C4)
# and 4K (HEADLINE) on the occupancy-limit grid (the default above two 4K frames of pixels) and on
# the in-flight cap (FRM_BLOCKS_PER_CU=12), interleaved; FRM_BLOCKS_PER_CU also resizes the batched
# launches, so only the drop-in numbers compare.
OUT=${OUT:-gpurun_out/c4cap}
mkdir -p "$OUT"
for wl in C4 HEADLINE; do
  for bpc in 0 12 28; do
    FRM_BLOCKS_PER_CU=$bpc timeout -k 10 200 python bench.py --workload $wl --steps 12 --warmup 2 --no-cpu-baseline \
      > "$OUT/${wl}_bpc${bpc}.json" 2> "$OUT/${wl}_bpc${bpc}.err"
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -5 "$OUT/${wl}_bpc${bpc}.err"; exit $rc; fi
    python -c "import json;d=json.load(open('$OUT/${wl}_bpc${bpc}.json'));print('$wl bpc $bpc dropin', round(d['dropin_ms_per_frame'],3), 'ms', 'batched', round(d['ms_per_step'],3))"
  done
done
