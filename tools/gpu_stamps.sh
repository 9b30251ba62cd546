#!/bin/bash
# FRM_STAMPS diagnostic build (fractal-ray-marching_amd/ab/stamps.so): per-wave cycle breakdown of
# the persistent kernel (tools/diag_waves.py) for the workloads in WLS.
set -o pipefail
OUT=${OUT:-gpurun_out/stamps}
mkdir -p "$OUT"
for wl in ${WLS:-C3 HEADLINE}; do
  WL=$wl FRM_LIB=$PWD/fractal-ray-marching_amd/ab/stamps.so timeout -k 10 200 python tools/diag_waves.py > "$OUT/$wl.txt" 2> "$OUT/$wl.err" || { tail -5 "$OUT/$wl.err"; exit 1; }
  cat "$OUT/$wl.txt"
done
