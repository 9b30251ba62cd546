#!/bin/bash
# Which pinned-host allocation makes hipMemcpyAsync device->host a DMA copy instead of a blit
# kernel (a kernel needs CU slots, which a running persistent grid holds)?
set -o pipefail
OUT=${OUT:-gpurun_out/d2h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/d2h_alloc_probe > "$OUT/plain.txt" 2>&1 || { cat "$OUT/plain.txt"; exit 1; }
cat "$OUT/plain.txt"
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/prof" -o run --output-format csv -- ./tools/micro/d2h_alloc_probe > "$OUT/prof.txt" 2>&1 || { tail "$OUT/prof.txt"; exit 1; }
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
k = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
m = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
kc = collections.Counter(r['Kernel_Name'][:40] for r in csv.DictReader(open(k[0]))) if k else {}
mc = collections.Counter(r.get('Direction', '?') for r in csv.DictReader(open(m[0]))) if m else {}
print('kernels', dict(kc))
print('dma copies', dict(mc))
PY
