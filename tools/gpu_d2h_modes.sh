#!/bin/bash
# tools/micro/d2h_mode_probe.hip, one run per copy path under the kernel and memory-copy traces,
# with /opt/rocm's runtime and with torch's bundled one (libfrm's inside bench.py and the tests).
set -o pipefail
OUT=${OUT:-gpurun_out/d2h_modes}
mkdir -p "$OUT"
export TMPDIR=/tmp
TL=$(python3 -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
for rt in rocm torch; do
  for m in plain after evwait nocu; do
    d="$OUT/${rt}_$m"
    if [ $rt = torch ]; then export LD_LIBRARY_PATH=$TL; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 60 rocprofv3 --kernel-trace --memory-copy-trace -d "$d" -o run --output-format csv -- ./tools/micro/d2h_mode_probe $m > "$d.txt" 2>&1 || { tail -3 "$d.txt"; exit 1; }
    python3 - "$d" "$rt" "$m" "$(grep -E 'ms  bytes' $d.txt)" <<'PY'
import csv, glob, sys, collections
d, rt, m, line = sys.argv[1:]
k = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
mc = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
kc = collections.Counter(r['Kernel_Name'][:30] for r in csv.DictReader(open(k[0]))) if k else {}
cc = collections.Counter(r.get('Direction', '?') for r in csv.DictReader(open(mc[0]))) if mc else {}
print(rt, line, '| blit kernels', kc.get('__amd_rocclr_copyBuffer', 0), '| dma', dict(cc))
PY
  done
done
