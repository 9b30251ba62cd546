# Everything a round's profiles/ need, in one GPU session: parity tests, the default bench
# line, a rocprofv3 kernel trace of it, every BASELINE config, PMC passes, the micro-
# benchmarks. GPU steps are time-limited; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/full}
mkdir -p "$OUT"
OUT=$OUT bash tools/profile_round.sh || exit 1
OUT=$OUT/pmc bash tools/pmc.sh > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; tail "$OUT/pmc.log"; exit 1; }
python tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_march.json" && python tools/pmc_summary.py "$OUT/pmc" shade_pass > "$OUT/pmc_shade.json" || exit 1
cat "$OUT/pmc_march.json"
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/isa_rate.hip -o /tmp/isa_rate 2>/dev/null || exit 1
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I fractal-ray-marching_amd/csrc tools/micro/ilp_bench.hip -o /tmp/ilp_bench 2>/dev/null || exit 1
timeout -k 5 120 /tmp/isa_rate > "$OUT/isa_rate.txt" && timeout -k 5 120 /tmp/ilp_bench > "$OUT/ilp_bench.txt" || exit 1
echo FULL_OK
