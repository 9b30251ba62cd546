#!/bin/bash
# Round 4: (1) the resize / readback GPU tests on the non-draining resize; (2) persistent grid size
# sweep (FRM_BLOCKS_PER_CU, one-wave workgroups: 24 = 6 waves/SIMD = every slot) on the drop-in
# loops (one frame per frm_render) and the batched headline: does leaving slots free let the next
# frame's sort / shade / readback run during a frame's march instead of at its tail?
set -o pipefail
OUT=${OUT:-gpurun_out/r4e}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resize.py tests/test_gpu_readback.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for round in 1 2; do
  for bpc in ${BPCS:-24 23 22 20}; do
    export FRM_BLOCKS_PER_CU=$bpc
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE --forms latency,noread > "$OUT/fix_${bpc}_$round.jsonl" 2> "$OUT/fix_${bpc}_$round.err" || { tail -5 "$OUT/fix_${bpc}_$round.err"; exit 1; }
    timeout -k 10 200 python tools/dropin_probe.py --workload HEADLINE_FLY --forms latency,noread > "$OUT/fly_${bpc}_$round.jsonl" 2> "$OUT/fly_${bpc}_$round.err" || { tail -5 "$OUT/fly_${bpc}_$round.err"; exit 1; }
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin > "$OUT/head_${bpc}_$round.json" 2> "$OUT/head_${bpc}_$round.err" || { tail -5 "$OUT/head_${bpc}_$round.err"; exit 1; }
    python3 - "$OUT" "$bpc" "$round" <<'PY'
import json, sys
out, b, r = sys.argv[1:]
fx = [json.loads(l) for l in open(f"{out}/fix_{b}_{r}.jsonl")]
fl = [json.loads(l) for l in open(f"{out}/fly_{b}_{r}.jsonl")]
h = json.load(open(f"{out}/head_{b}_{r}.json"))
print(f"r{r} bpc {b}: fixed " + " ".join(f"{x['form']} {x['ms_per_frame']:.3f}" for x in fx) +
      " | fly " + " ".join(f"{x['form']} {x['ms_per_frame']:.3f}" for x in fl) +
      f" | headline batched {h['ms_per_step']:.3f} sha {h['frame_sha_ok']} cnt {h['counters_ok']}")
PY
  done
done
