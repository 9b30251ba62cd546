#!/bin/bash
# march_pool experiment (FRM_POOL=1): parity on the GPU first, then an interleaved A/B of the
# default bench against march_persistent. Every GPU step time-limited; stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/pool}
mkdir -p "$OUT"
FRM_POOL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -n 2 "$OUT/pytest.log"
for round in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${CFGS:-FRM_POOL=0 FRM_POOL=1}; do
    env ${cfg//,/ } timeout -k 10 200 python bench.py --workload ${WL:-HEADLINE} --no-cpu-baseline > "$OUT/b_${cfg}_$round.json" 2> "$OUT/b_${cfg}_$round.err" || { echo "bench $cfg failed"; tail -5 "$OUT/b_${cfg}_$round.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${cfg}_$round.json'));print('r$round', '$cfg', round(d['value'],3), 'Gsteps/s', round(d['ms_per_step'],3), 'ms sha_ok', d.get('frame_sha_ok'))"
  done
done
