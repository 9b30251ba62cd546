#!/bin/bash
# Interleaved A/B of libfrm builds (fractal-ray-marching_amd/ab/NAME.so) on bench.py's config lines
# (WORKLOADS, default C2 C3 HEADLINE) and one rank's share of the 8-way headline split as bench.py
# runs it (tools/pipeline_probe.py: 2 in flight, 10 frames per launch, gather + unshuffle on rank 0).
set -o pipefail
OUT=${OUT:-gpurun_out/ab_cfg}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-2}); do
  for n in $VARIANTS; do
    export FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so
    line="round $round $n:"
    for wl in ${WORKLOADS:-C2 C3 HEADLINE}; do
      timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > "$OUT/${wl}_${n}_$round.json" 2> "$OUT/${wl}_${n}_$round.err" || { echo "$wl $n failed"; tail -5 "$OUT/${wl}_${n}_$round.err"; exit 1; }
      line="$line $wl $(python -c "import json;d=json.load(open('$OUT/${wl}_${n}_$round.json'));print(round(d['ms_per_step'],3), d['frame_sha_ok'])")"
    done
    timeout -k 10 200 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 2 --batch 10 --frames 40 --gather 1 > "$OUT/share8_${n}_$round.jsonl" 2> "$OUT/share8_${n}_$round.err" || { echo "share8 $n failed"; tail -5 "$OUT/share8_${n}_$round.err"; exit 1; }
    line="$line share8 $(python -c "import json;d=[json.loads(l) for l in open('$OUT/share8_${n}_$round.jsonl') if l.startswith('{')][-1];print(round(d['ms_per_frame'],3))")"
    echo "$line"
  done
done
