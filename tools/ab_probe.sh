# A/B of libfrm variants (fractal-ray-marching_amd/variants/*.so) on pipeline_probe:
# one rank's share of an 8-way split (F=3) and the whole headline frame (F=2), 2 rounds.
set -o pipefail
O=${OUT:-gpurun_out/ab_probe}
mkdir -p $O
for round in 1 2; do
  for lib in fractal-ray-marching_amd/variants/*.so; do
    n=$(basename $lib .so)
    FRM_LIB=$PWD/$lib timeout -k 10 200 python tools/pipeline_probe.py --workloads ${WL:-HEADLINE} --ranks ${RANKS:-8,1} --inflight ${F:-3} --frames ${FRAMES:-24} > $O/$n.log 2> $O/$n.err || { tail $O/$n.err; exit 1; }
    echo "round $round $n"; python tools/pipe_summary.py < $O/$n.log
  done
done
