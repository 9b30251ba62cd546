# pipeline_probe under several settings of one environment variable
# usage: VAR=FRM_SERVICE_STREAMS VALS="0 1 2" P8F="3,4,6" P1F="2,3" bash tools/gpu_env_sweep.sh
set -o pipefail
O=gpurun_out/env_sweep
mkdir -p $O
for v in $VALS; do
  echo "$VAR=$v"
  env $VAR=$v timeout -k 10 200 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight ${P8F:-3,6} --frames 48 > $O/p8_$v.log 2> $O/p8_$v.err || { tail $O/p8_$v.err; exit 1; }
  python tools/pipe_summary.py < $O/p8_$v.log
  if [ -n "$P1F" ]; then
  env $VAR=$v timeout -k 10 200 python tools/pipeline_probe.py --workloads HEADLINE --ranks 1 --inflight $P1F --frames 12 > $O/p1_$v.log 2> $O/p1_$v.err || { tail $O/p1_$v.err; exit 1; }
  python tools/pipe_summary.py < $O/p1_$v.log
  fi
done
