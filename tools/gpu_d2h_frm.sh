#!/bin/bash
# tools/d2h_frm_probe.py cases under the kernel and memory-copy traces: blit kernels vs DMA copies.
set -o pipefail
OUT=${OUT:-gpurun_out/d2h_frm}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in torch cumask frm frmplain; do
  d="$OUT/$c"
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$d" -o run --output-format csv -- python3 tools/d2h_frm_probe.py $c > "$d.txt" 2>&1 || { tail -3 "$d.txt"; exit 1; }
  python3 - "$d" "$c" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1:]
k = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
mc = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
kc = collections.Counter(r['Kernel_Name'][:30] for r in csv.DictReader(open(k[0]))) if k else {}
cc = collections.Counter(r.get('Direction', '?') for r in csv.DictReader(open(mc[0]))) if mc else {}
print(c, '| blit copy kernels', kc.get('__amd_rocclr_copyBuffer', 0), '| dma', dict(cc))
PY
done
