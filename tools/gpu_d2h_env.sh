#!/bin/bash
# tools/d2h_frm_probe.py (torch and frm cases) under runtime settings that may steer ROCclr's copy
# engine choice; then, for a setting that gives DMA copies, the drop-in loops with it.
set -o pipefail
OUT=${OUT:-gpurun_out/d2h_env}
mkdir -p "$OUT"
export TMPDIR=/tmp
for e in "NONE=1" "GPU_BLIT_ENGINE_TYPE=1" "GPU_BLIT_ENGINE_TYPE=2" "HSA_ENABLE_SDMA=1" "ROC_ENABLE_LARGE_BAR=0" "GPU_FORCE_BLIT_COPY_SIZE=0"; do
  tag=$(echo $e | tr '=' '_')
  d="$OUT/$tag"
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$d" -o run --output-format csv -- python3 tools/d2h_frm_probe.py frm > "$d.txt" 2>&1 || { echo "$e failed"; tail -3 "$d.txt"; continue; }
  python3 - "$d" "$e" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1:]
k = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
mc = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
kc = collections.Counter(r['Kernel_Name'][:30] for r in csv.DictReader(open(k[0]))) if k else {}
cc = collections.Counter(r.get('Direction', '?') for r in csv.DictReader(open(mc[0]))) if mc else {}
print(c, '| blit copy kernels', kc.get('__amd_rocclr_copyBuffer', 0), '| dma', dict(cc))
PY
done
