set -o pipefail
OUT=gpurun_out/ab_vcut2; mkdir -p $OUT
for round in 1 2; do
for v in base vt vm vcut vcut6; do
  lib=$v; extra=""
  if [ $v = vcut6 ]; then lib=vcut; export FRM_BLOCKS_PER_CU=24; else unset FRM_BLOCKS_PER_CU; fi
  FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $OUT/h_${v}_$round.json 2> $OUT/h_${v}_$round.err || { tail -3 $OUT/h_${v}_$round.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/h_${v}_$round.json'));print('round $round $v HEADLINE', round(d['ms_per_step'],3), d['frame_sha_ok'], d.get('counters_ok'))"
done
done
