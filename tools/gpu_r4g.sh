#!/bin/bash
# Round 4: fused scheduling with 4096-pixel shade/rank blocks and double-buffered framebuffers.
# GPU tests, then resize-loop and drop-in A/B: base (HEAD) vs r2, and r2 with FRM_SCHED=sort.
set -o pipefail
OUT=${OUT:-gpurun_out/r4g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
d="$OUT/trace_resize"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 tools/resize_loop_probe.py --cycles 1 > "$d.json" 2> "$d.err" || { tail "$d.err"; exit 1; }
python3 tools/trace_timeline.py $(ls "$d"/*/*kernel_trace.csv "$d"/*kernel_trace.csv 2>/dev/null | head -1) 150 > "$d.timeline.txt" || exit 1
cat "$d.json"
for round in 1 2; do
  for v in base r2 r2sort; do
    n=${v%sort}; export FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so
    if [ "$v" = r2sort ]; then export FRM_SCHED=sort; else unset FRM_SCHED; fi
    timeout -k 10 200 python tools/resize_loop_probe.py > "$OUT/resize_${v}_$round.json" 2> "$OUT/resize_${v}_$round.err" || { tail -5 "$OUT/resize_${v}_$round.err"; exit 1; }
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency,noread > "$OUT/fix_${v}_$round.jsonl" 2> "$OUT/fix_${v}_$round.err" || { tail -5 "$OUT/fix_${v}_$round.err"; exit 1; }
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency,latency3 > "$OUT/fly_${v}_$round.jsonl" 2> "$OUT/fly_${v}_$round.err" || { tail -5 "$OUT/fly_${v}_$round.err"; exit 1; }
    timeout -k 10 200 python bench.py --workload HEADLINE_FLY --no-cpu-baseline --no-dropin > "$OUT/flyb_${v}_$round.json" 2> "$OUT/flyb_${v}_$round.err" || { tail -5 "$OUT/flyb_${v}_$round.err"; exit 1; }
    python3 - "$OUT" "$v" "$round" <<'PY'
import json, sys
out, v, r = sys.argv[1:]
rs = json.load(open(f"{out}/resize_{v}_{r}.json"))
fx = [json.loads(l) for l in open(f"{out}/fix_{v}_{r}.jsonl")]
fl = [json.loads(l) for l in open(f"{out}/fly_{v}_{r}.jsonl")]
fb = json.load(open(f"{out}/flyb_{v}_{r}.json"))
print(f"r{r} {v}: resize steady {rs['steady_median_ms']:.2f} first max {rs['first_after_resize_max_ms']:.2f} second {rs['second_after_resize_mean_ms']:.2f} | fixed " +
      " ".join(f"{x['form']} {x['ms_per_frame']:.3f}" for x in fx) + " | fly " + " ".join(f"{x['form']} {x['ms_per_frame']:.3f}" for x in fl) +
      f" | fly bench {fb['ms_per_step']:.3f} sha {fb['frame_sha_ok']}")
PY
  done
done
unset FRM_SCHED
for n in base r2; do
  FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/headline_$n.json" 2> "$OUT/headline_$n.err" || { echo "headline $n failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/headline_$n.json'));print('headline $n', round(d['ms_per_step'],3), d['frame_sha_ok'], d['counters_ok'])"
done
