#!/bin/bash
# Round 4: animated multi-frame launches (per-lane Mandelbulb power). GPU tests, then the batched
# HEADLINE_FLY bench line (default: frames per launch) vs one frame per launch (--batch 1, the old
# default), the headline, and C5 (animated, now batched).
set -o pipefail
OUT=${OUT:-gpurun_out/r4h}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for round in 1 2; do
  timeout -k 10 200 python bench.py --workload HEADLINE_FLY --no-cpu-baseline --no-dropin > "$OUT/fly_batched_$round.json" 2> "$OUT/fly_batched_$round.err" || { tail -5 "$OUT/fly_batched_$round.err"; exit 1; }
  timeout -k 10 200 python bench.py --workload HEADLINE_FLY --batch 1 --no-cpu-baseline --no-dropin > "$OUT/fly_single_$round.json" 2> "$OUT/fly_single_$round.err" || { tail -5 "$OUT/fly_single_$round.err"; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/headline_$round.json" 2> "$OUT/headline_$round.err" || { tail -5 "$OUT/headline_$round.err"; exit 1; }
  python3 - "$OUT" "$round" <<'PY'
import json, sys
out, r = sys.argv[1:]
for n in ("fly_batched", "fly_single", "headline"):
    d = json.load(open(f"{out}/{n}_{r}.json"))
    c = d["config"]
    print(f"r{r} {n}: {d['ms_per_step']:.3f} ms/frame, {c.get('frames_per_launch')} per launch, {c.get('frames_in_flight')} in flight, sha {d.get('frame_sha_ok')} cnt {d.get('counters_ok')}")
PY
done
timeout -k 10 300 python bench.py --workload C5 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/c5.json" 2> "$OUT/c5.err" || { tail -5 "$OUT/c5.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('C5', round(d['ms_per_step'],2), d['config'].get('frames_per_launch'), d.get('frame_sha_ok'))"
