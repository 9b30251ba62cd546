# A/B of the working tree against a git worktree of another commit (checked out and built
# in ./_abbase): pipeline_probe from each tree, interleaved rounds.
set -o pipefail
O=${OUT:-gpurun_out/ab_wt}
mkdir -p $O
for round in 1 2; do
  for side in base new; do
    dir=.; [ $side = base ] && dir=_abbase
    timeout -k 10 300 python $dir/tools/pipeline_probe.py --workloads ${WL:-HEADLINE} --ranks ${RANKS:-1} --inflight ${F:-2} --frames ${FRAMES:-24} > $O/$side.log 2> $O/$side.err || { tail $O/$side.err; exit 1; }
    echo "round $round $side"; python tools/pipe_summary.py < $O/$side.log
  done
done
