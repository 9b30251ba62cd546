#!/bin/bash
# Interleaved A/B of libfrm builds (ab/NAME.so) on bench.py's drop-in loop measurement
# (dropin_ms_per_frame: one frm_render per frame, 2 in flight, a frame of presentation latency)
# and the batched line, for WORKLOADS (default HEADLINE HEADLINE_FLY).
# Usage: VARIANTS="n5 n6" ROUNDS=2 OUT=gpurun_out/abd bash tools/ab_r5_dropin.sh
OUT=${OUT:-gpurun_out/abd}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-2}); do
  for wl in ${WORKLOADS:-HEADLINE HEADLINE_FLY}; do
    for n in $VARIANTS; do
      FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline \
        > "$OUT/${n}_${wl}_$round.json" 2> "$OUT/${n}_${wl}_$round.err"
      rc=$?
      if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $n $wl rc=$rc"; tail -5 "$OUT/${n}_${wl}_$round.err"; exit $rc; fi
      python -c "import json;d=json.load(open('$OUT/${n}_${wl}_$round.json'));print('round $round $wl $n', round(d['ms_per_step'],3), 'ms; dropin', round(d['dropin_ms_per_frame'],3), 'sync', round(d['dropin_sync_ms_per_frame'],3), 'sha_ok', d.get('frame_sha_ok'))"
    done
  done
done
