#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) on a short bench.
# Usage: OUT=gpurun_out/pmc ARGS="--steps 2 --warmup 1" bash tools/pmc.sh
# PROG replaces bench.py (e.g. PROG=tools/pipeline_probe.py ARGS="--ranks 8 ..." for one rank's
# share of a row split: the N > 1 counters bench.py cites)
set -o pipefail
OUT=${OUT:-gpurun_out/pmc}
ARGS=${ARGS:---steps 4 --warmup 2 --no-cpu-baseline --no-dropin}
PROG=${PROG:-bench.py}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 $PROG $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_COUNT && \
run sq3 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS && \
run wr WRITE_SIZE && \
run rd FETCH_SIZE && echo PMC_OK
