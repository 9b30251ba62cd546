#!/bin/bash
# The drop-in loop from a C host (tools/micro/dropin_loop.cpp: DMA readback copies) against the
# Python one (tools/dropin_probe.py: blit-kernel copies inside a torch process), 2 rounds, with
# timed frame 0 of the C loop checked against the headline's golden hash.
set -o pipefail
OUT=${OUT:-gpurun_out/dropin_c}
mkdir -p "$OUT"
for round in 1 2; do
  for wl in fly fixed; do
    timeout -k 10 120 ./tools/micro/dropin_loop $wl 20 "$OUT/frame0_$wl.rgba" > "$OUT/c_${wl}_$round.json" 2> "$OUT/c_${wl}_$round.err" || { tail -3 "$OUT/c_${wl}_$round.err"; exit 1; }
    cat "$OUT/c_${wl}_$round.json"
  done
  timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency > "$OUT/py_fly_$round.jsonl" 2> "$OUT/py_fly_$round.err" || { tail -3 "$OUT/py_fly_$round.err"; exit 1; }
  timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency > "$OUT/py_fixed_$round.jsonl" 2> "$OUT/py_fixed_$round.err" || { tail -3 "$OUT/py_fixed_$round.err"; exit 1; }
  cat "$OUT/py_fly_$round.jsonl" "$OUT/py_fixed_$round.jsonl"
done
python3 - "$OUT" <<'PY'
import hashlib, json, sys
out = sys.argv[1]
g = json.load(open("tests/golden/fullsize.json"))["HEADLINE_P1"]["sha256"]
for wl in ("fly", "fixed"):
    h = hashlib.sha256(open(f"{out}/frame0_{wl}.rgba", "rb").read()).hexdigest()
    print(wl, "timed frame 0 == golden HEADLINE_P1:", h == g)
PY
