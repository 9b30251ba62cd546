set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_de.py -q -rf > gpurun_out/pytest_de.log 2>&1; echo rc=$?
tail -40 gpurun_out/pytest_de.log
