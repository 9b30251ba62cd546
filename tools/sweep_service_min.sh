set -o pipefail
mkdir -p gpurun_out/sm
for r in 1 2; do for sm in 24 20 22 26 28 32; do
  FRM_SERVICE_MIN=$sm timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sm/sm_${sm}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sm/sm_${sm}_$r.json'));print('r$r sm $sm', round(d['value'],3), round(d['ms_per_step'],3))"
done; done
