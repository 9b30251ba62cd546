#!/bin/bash
# Every BASELINE config at bench defaults (one bench line each, PMC counters cited when the
# committed summary matches the kernel sources). Every GPU step time-limited; stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/configs}
mkdir -p "$OUT"
for spec in "HEADLINE:" "C1:" "C2:" "C3:" "C4:" "C5:--steps 2 --warmup 1"; do
  wl=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python bench.py --workload $wl $a --no-cpu-baseline > "$OUT/$wl.json" 2> "$OUT/$wl.err" || { echo "bench $wl failed"; tail -5 "$OUT/$wl.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$wl.json'));r=d['roofline'];print('$wl', round(d['value'],3), 'G/s', round(d['ms_per_step'],3), 'ms/frame', 'frac', round(r['frac'],4), 'valu_busy', r.get('valu_busy'), 'stale', r.get('pmc_stale'), 'sha_ok', d.get('frame_sha_ok'))"
done
echo CONFIGS_OK
