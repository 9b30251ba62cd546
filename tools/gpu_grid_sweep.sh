# persistent grid size (FRM_BLOCKS_PER_CU) x frames in flight, whole frame and 8-way rank share
set -o pipefail
O=gpurun_out/grid_sweep
mkdir -p $O
for B in 2 3 4 6; do
  FRM_BLOCKS_PER_CU=$B timeout -k 10 200 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 3,4,6,8 --frames 48 > $O/p8_b$B.log 2> $O/p8_b$B.err || { tail $O/p8_b$B.err; exit 1; }
  echo "B=$B"; python tools/pipe_summary.py < $O/p8_b$B.log
  FRM_BLOCKS_PER_CU=$B timeout -k 10 200 python tools/pipeline_probe.py --workloads HEADLINE --ranks 1 --inflight 2,3,4 --frames 12 > $O/p1_b$B.log 2> $O/p1_b$B.err || { tail $O/p1_b$B.err; exit 1; }
  python tools/pipe_summary.py < $O/p1_b$B.log
done
