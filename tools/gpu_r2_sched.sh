#!/bin/bash
# Round 2: resize history (max-filter resample) tests + probe; service_min re-sweep on the
# round-2 kernel; one rank's share of an 8-way row split (every rank, 3 in flight) and rank 0
# with its gather + unshuffle. Every GPU step time-limited; stops at a failure.
set -o pipefail
OUT=${OUT:-gpurun_out/r2e}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resize.py tests/test_gpu_parity.py tests/test_gpu_bands.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python tools/resize_probe.py > "$OUT/resize_probe.json" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
cat "$OUT/resize_probe.json"
for wl in HEADLINE C2; do for sm in 16 20 24 28; do
  FRM_SERVICE_MIN=$sm timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > "$OUT/sm_${wl}_$sm.json" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sm_${wl}_$sm.json'));print('$wl service_min $sm', round(d['ms_per_step'],3), 'ms', round(d['value'],2), 'G/s')"
done; done
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 1 --inflight 1,2 --frames 30 > "$OUT/probe_whole.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
timeout -k 10 400 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 3 --frames 48 --rank-ids all > "$OUT/probe_8way.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8,4,2 --inflight 3 --frames 48 --rank-ids 0 --gather 0,1 > "$OUT/probe_gather.jsonl" 2> "$OUT/err" || { tail "$OUT/err"; exit 1; }
cat "$OUT"/probe_*.jsonl | python tools/pipe_summary.py
