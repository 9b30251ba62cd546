set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sdma
for e in "NONE=1" "HSA_ENABLE_SDMA=1" "GPU_FORCE_BLIT_COPY_SIZE=0" "HSA_ENABLE_SDMA=1 HSA_ENABLE_PEER_SDMA=1"; do
  tag=$(echo $e | tr ' =' '__')
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/sdma/$tag -o run --output-format csv -- python3 tools/dropin_probe.py --workload HEADLINE --forms latency --frames 6 > gpurun_out/sdma/$tag.jsonl 2> gpurun_out/sdma/$tag.err || { tail -3 gpurun_out/sdma/$tag.err; exit 1; }
  python3 - gpurun_out/sdma/$tag "$e" <<'PY'
import csv, glob, sys, collections, json
d, e = sys.argv[1:]
k = collections.Counter(r['Kernel_Name'][:28] for r in csv.DictReader(open(glob.glob(d + '/*kernel_trace.csv')[0])))
m = glob.glob(d + '/*memory_copy_trace.csv')
mc = collections.Counter(r['Direction'] for r in csv.DictReader(open(m[0]))) if m else {}
print(e, 'copyBuffer kernels', k.get('__amd_rocclr_copyBuffer', 0), 'dma copies', dict(mc))
PY
  cat gpurun_out/sdma/$tag.jsonl
done
