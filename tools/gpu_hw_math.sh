#!/bin/bash
# FRM_HW_MATH measurement build (variants/hw_math.so) vs the product build: interleaved
# bench rounds on the headline, and the headline frame of each saved for the CPU-side
# comparison with the oracle (tools/hw_math_compare.py). Every GPU step time-limited.
set -o pipefail
OUT=${OUT:-gpurun_out/hw}
mkdir -p "$OUT"
V=fractal-ray-marching_amd/variants/hw_math.so
timeout -k 10 120 python tools/render_frame.py --out $OUT/frame_product.npy || exit 1
FRM_LIB=$PWD/$V timeout -k 10 120 python tools/render_frame.py --out $OUT/frame_hw_math.npy || exit 1
for round in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_product_$round.json 2> $OUT/err || { tail $OUT/err; exit 1; }
  FRM_LIB=$PWD/$V timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_hw_math_$round.json 2> $OUT/err || { tail $OUT/err; exit 1; }
  python -c "import json;a=json.load(open('$OUT/bench_product_$round.json'));b=json.load(open('$OUT/bench_hw_math_$round.json'));print('round $round product', round(a['ms_per_step'],3), 'ms', round(a['value'],2), 'G/s; hw_math', round(b['ms_per_step'],3), 'ms', round(b['value'],2), 'G/s steps/frame', int(b['march_steps_per_frame']))"
done
export TMPDIR=/tmp
FRM_LIB=$PWD/$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
echo HW_OK
