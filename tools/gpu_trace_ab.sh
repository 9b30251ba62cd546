# kernel durations (F=1, whole headline frame) of the worktree base vs the working tree
set -o pipefail
O=gpurun_out/trace_ab
mkdir -p $O
export TMPDIR=/tmp
for side in base new; do
  dir=.; [ $side = base ] && dir=_abbase
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$side -o run --output-format csv -- python3 $dir/tools/pipeline_probe.py --workloads HEADLINE --ranks 1 --inflight 1 --frames 8 > $O/$side.log 2> $O/$side.err || { tail $O/$side.err; exit 1; }
  echo "== $side"; python - $O/$side <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "march" in n or "shade" in n or "Radix" in n or "radix" in n:
        print(n[:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
done
