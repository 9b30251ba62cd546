# frames in flight up to 8 and all 8 ranks' shares of an 8-way split (pipeline_probe)
set -o pipefail
O=gpurun_out/inflight8
mkdir -p $O
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 4,8 --inflight 3,4,5,6,8 --frames 48 > $O/probe_f.log 2> $O/probe_f.err || { tail $O/probe_f.err; exit 1; }
python tools/pipe_summary.py < $O/probe_f.log
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight 6 --frames 48 --rank-ids all > $O/probe_ranks.log 2> $O/probe_ranks.err || { tail $O/probe_ranks.err; exit 1; }
python tools/pipe_summary.py < $O/probe_ranks.log
timeout -k 10 300 python tools/pipeline_probe.py --workloads C4 --ranks 8 --inflight 3,6 --frames 24 > $O/probe_c4.log 2> $O/probe_c4.err || { tail $O/probe_c4.err; exit 1; }
python tools/pipe_summary.py < $O/probe_c4.log
