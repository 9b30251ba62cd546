# VALU lane utilisation of the march kernel: whole frame vs one rank's share of an 8-way split
set -o pipefail
O=gpurun_out/pmc_share
mkdir -p $O
export TMPDIR=/tmp
for P in 1 8; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p$P -o run --output-format csv -- python3 tools/pipeline_probe.py --workloads HEADLINE --ranks $P --inflight 1 --frames 6 > $O/p$P.log 2> $O/p$P.err || { tail $O/p$P.err; exit 1; }
  python - $O/p$P <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "march_persistent" in r["Kernel_Name"]:
        agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(agg)[1:]
for i in ids:
    c = agg[i]
    print(sys.argv[1], i, "insts %.3g" % c["SQ_INSTS_VALU"], "lane_util %.3f" % (c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)),
          "valu_busy %.3f" % (c["SQ_ACTIVE_INST_VALU"] * 2 / (1024 * c["GRBM_GUI_ACTIVE"] / 8)))
PY
done
