#!/bin/bash
# A/B of the record layout (profiles/round5/ab_records/pos.patch: records indexed by fetch position,
# shade_pass gathering through the order) against the product's pixel-indexed records: headline
# time (2 interleaved rounds) and PMC HBM bytes of march, shade and rank passes
mkdir -p gpurun_out/records
VARIANTS="base pos" ROUNDS=2 OUT=gpurun_out/records/ab bash tools/ab_r5.sh || exit 1
for n in base pos; do
  FRM_LIB=$PWD/fractal-ray-marching_amd/ab/$n.so OUT=gpurun_out/records/pmc_$n ARGS="--steps 48 --warmup 16 --batch 16 --no-cpu-baseline --no-dropin" bash tools/pmc.sh > /dev/null || { echo "pmc $n failed"; exit 1; }
  for k in march_persistent shade_pass rank_pass; do
    python3 tools/pmc_summary.py gpurun_out/records/pmc_$n $k > gpurun_out/records/pmc_${n}_$k.json || exit 1
    python3 -c "import json;s=json.load(open('gpurun_out/records/pmc_${n}_$k.json'));B=s['frames_per_dispatch'];print('$n $k MB/frame read', round(s['hbm_read_bytes']/B/1e6,1), 'write', round(s['hbm_write_bytes']/B/1e6,1))"
  done
done
