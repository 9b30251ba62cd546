# frames-in-flight sweep on one GPU: bench.py (whole frames) + pipeline_probe (rank shares)
set -o pipefail
O=gpurun_out/inflight
mkdir -p $O
for F in 1 2 3; do
  timeout -k 10 200 python bench.py --inflight $F --no-cpu-baseline > $O/bench_f$F.json 2> $O/bench_f$F.err || { tail $O/bench_f$F.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_f$F.json'));print('HEADLINE F=$F', round(d['value'],2), round(d['ms_per_step'],3), 'span', round(d['roofline']['avg_kernel_ms'],3), 'launch', round(d['roofline']['avg_launch_ms'],3))"
done
for F in 1 3; do
  timeout -k 10 200 python bench.py --workload C2 --inflight $F --no-cpu-baseline > $O/c2_f$F.json 2> $O/c2_f$F.err || { tail $O/c2_f$F.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_f$F.json'));print('C2 F=$F', round(d['value'],2), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python tools/pipeline_probe.py --workloads HEADLINE,C4 --ranks 1,2,4,8 --inflight 1,3 --repeat 2 > $O/probe.log 2> $O/probe.err || { tail $O/probe.err; exit 1; }
python tools/pipe_summary.py < $O/probe.log
