# kernel-trace timeline of one rank's share of an 8-way row split with F frames in flight
# usage: B=<blocks per CU> FS="3 1" bash tools/gpu_trace_share.sh
set -o pipefail
O=gpurun_out/trace_share
mkdir -p $O
export TMPDIR=/tmp
[ -n "$B" ] && export FRM_BLOCKS_PER_CU=$B
for F in ${FS:-3 1}; do
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/b${B}f$F -o run --output-format csv -- python3 tools/pipeline_probe.py --workloads HEADLINE --ranks 8 --inflight $F --frames 24 > $O/b${B}f$F.log 2> $O/b${B}f$F.err || { tail $O/b${B}f$F.err; exit 1; }
python tools/trace_timeline.py $(find $O/b${B}f$F -name "*kernel_trace.csv" | head -1) 120 | grep -v fillBuffer > $O/timeline_b${B}f$F.txt
tail -40 $O/timeline_b${B}f$F.txt
done
