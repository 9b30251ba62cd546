#!/bin/bash
# Interleaved A/B of libfrm builds (fractal-ray-marching_amd/ab/NAME.so) on the moving-frame loops:
# the drop-in loop (tools/dropin_probe.py, 2 and 3 in flight with a frame of readback latency) and
# bench.py's HEADLINE_FLY line (3 in flight), ROUNDS rounds; the fixed headline once per variant.
set -o pipefail
OUT=${OUT:-gpurun_out/ab_dropin}
mkdir -p "$OUT"
for round in $(seq 1 ${ROUNDS:-2}); do
  for n in $VARIANTS; do
    export FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency,latency3 > "$OUT/dropin_${n}_$round.jsonl" 2> "$OUT/dropin_${n}_$round.err" || { echo "dropin $n failed"; tail -5 "$OUT/dropin_${n}_$round.err"; exit 1; }
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency > "$OUT/dropinfix_${n}_$round.jsonl" 2> "$OUT/dropinfix_${n}_$round.err" || { echo "dropin fixed $n failed"; tail -5 "$OUT/dropinfix_${n}_$round.err"; exit 1; }
    timeout -k 10 200 python bench.py --workload HEADLINE_FLY --no-cpu-baseline --no-dropin > "$OUT/fly_${n}_$round.json" 2> "$OUT/fly_${n}_$round.err" || { echo "fly $n failed"; tail -5 "$OUT/fly_${n}_$round.err"; exit 1; }
    python - "$OUT" "$n" "$round" <<'PY'
import json, sys
out, n, r = sys.argv[1:]
d = [json.loads(l) for l in open(f"{out}/dropin_{n}_{r}.jsonl")]
f = json.load(open(f"{out}/fly_{n}_{r}.json"))
x = json.loads(open(f"{out}/dropinfix_{n}_{r}.jsonl").read().splitlines()[-1])
print(f"round {r} {n}: dropin fly " + " ".join(f"{x['form']} {x['ms_per_frame']:.3f}" for x in d) + f" | fixed {x['ms_per_frame']:.3f} | fly bench {f['ms_per_step']:.3f} ms sha_ok {f['frame_sha_ok']}")
PY
  done
done
for n in $VARIANTS; do
  FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/headline_$n.json" 2> "$OUT/headline_$n.err" || { echo "headline $n failed"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/headline_$n.json'));print('headline $n', round(d['ms_per_step'],3), d['frame_sha_ok'], d['counters_ok'])"
done
