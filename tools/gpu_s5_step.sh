#!/bin/bash
# step-loop experiment: GPU test suite on the default build, then C3 A/B of the variants
set -o pipefail
OUT=gpurun_out/s5step
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
OUT=$OUT/ab WL=C3 ROUNDS=3 bash tools/ab_libs3.sh
