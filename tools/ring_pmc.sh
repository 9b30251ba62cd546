#!/bin/bash
# Round 6: PMC passes (tools/pmc.sh groups) of the resident ring's march (tools/ring_probe.py child,
# noread loop of the 4K headline) and of the per-frame grids for comparison. Summary: tools/pmc_summary.py.
set -o pipefail
OUT=${OUT:-gpurun_out/ring_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
for mode in 1 0; do
  for grp in "sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "sq3 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
             "sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_COUNT" \
             "sq4 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_INSTS_FLAT"; do
    set -- $grp; name=$1; shift
    lib=""; [ "$mode" = 1 ] && lib=${LIB1:-}
    FRM_LIB=$lib FRM_RING=$mode timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/${name}_m$mode" -o run --output-format csv \
      -- python3 tools/ring_probe.py --child --loops noread --frames 12 > "$OUT/${name}_m$mode.json" 2> "$OUT/${name}_m$mode.err" || exit 1
  done
done
echo RING_PMC_OK
