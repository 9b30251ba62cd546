#!/bin/bash
# The D2H probe under torch's bundled HIP runtime (the one libfrm binds to inside bench.py and the
# tests): blit kernel or DMA engine? Then the drop-in loop's readback copies in a kernel trace.
set -o pipefail
OUT=${OUT:-gpurun_out/d2h_torch}
mkdir -p "$OUT"
export TMPDIR=/tmp
TL=$(python3 -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
LD_LIBRARY_PATH=$TL timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/prof" -o run --output-format csv -- ./tools/micro/d2h_alloc_probe > "$OUT/prof.txt" 2>&1 || { tail "$OUT/prof.txt"; exit 1; }
cat "$OUT/prof.txt" | grep -v "^W\|^E" | tail -8
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/dropin" -o run --output-format csv -- python3 tools/dropin_probe.py --workload HEADLINE_FLY --forms latency --frames 8 > "$OUT/dropin.jsonl" 2> "$OUT/dropin.err" || { tail "$OUT/dropin.err"; exit 1; }
for d in prof dropin; do
python3 - "$OUT/$d" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
k = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
m = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
kc = collections.Counter(r['Kernel_Name'][:40] for r in csv.DictReader(open(k[0]))) if k else {}
mc = collections.Counter(r.get('Direction', '?') for r in csv.DictReader(open(m[0]))) if m else {}
print(d, 'kernels', {a: b for a, b in kc.items() if 'rocclr' in a})
print(d, 'dma copies', dict(mc))
PY
done
