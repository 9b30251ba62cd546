#!/bin/bash
# FRM_BLOCKS_PER_CU sweep of one libfrm build (FRM_LIB) on the drop-in loop (HEADLINE_FLY and the
# fixed headline, 2 in flight, a frame of readback latency) and bench.py's batched headline.
set -o pipefail
OUT=${OUT:-gpurun_out/bpc}
mkdir -p "$OUT"
for round in 1 2; do
for bpc in $BPCS; do
  export FRM_BLOCKS_PER_CU=$bpc
  [ "$bpc" = "0" ] && unset FRM_BLOCKS_PER_CU
  timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency > "$OUT/fly_${bpc}_$round.jsonl" 2> "$OUT/fly_$bpc.err" || { tail -5 "$OUT/fly_$bpc.err"; exit 1; }
  timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency > "$OUT/fixed_${bpc}_$round.jsonl" 2> "$OUT/fixed_$bpc.err" || { tail -5 "$OUT/fixed_$bpc.err"; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/headline_${bpc}_$round.json" 2> "$OUT/headline_$bpc.err" || { tail -5 "$OUT/headline_$bpc.err"; exit 1; }
  python - "$OUT" "$bpc" "$round" <<'PY'
import json, sys
o, b, r = sys.argv[1:]
f = json.loads(open(f"{o}/fly_{b}_{r}.jsonl").read().splitlines()[-1])
x = json.loads(open(f"{o}/fixed_{b}_{r}.jsonl").read().splitlines()[-1])
h = json.load(open(f"{o}/headline_{b}_{r}.json"))
print(f"round {r} bpc {b}: dropin fly {f['ms_per_frame']:.3f} fixed {x['ms_per_frame']:.3f} | batched headline {h['ms_per_step']:.3f} sha_ok {h['frame_sha_ok']}")
PY
done
done
