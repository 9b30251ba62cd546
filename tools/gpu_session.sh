#!/bin/bash
# Profile session (one gpurun call per PART; every GPU step has its own time limit and
# the chain stops at the first failure). Outputs under $OUT, copied into profiles/roundN/.
#   PART=tests   pytest -m gpu, the default bench line (+ CPU baseline), its rocprofv3 kernel
#                trace (--kernel-trace --stats) and per-frame span (rocprof_timed.py)
#   PART=configs every BASELINE config + HEADLINE_FLY + the FRM_FLAG_HW_MATH line, one bench line each
#   PART=pmc     PMC passes (tools/pmc.sh, one counter group per run) of the headline, C2-C5 and one
#                rank's share of the 8-way headline split; summaries for march_persistent and shade_pass
set -o pipefail
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$PART" in
tests)
  (lscpu | head -20; nproc) > "$OUT/host.txt" 2>&1
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  # the driver's command (defaults: 30 timed frames, one launch of 30 on one GPU)
  timeout -k 10 400 python bench.py > "$OUT/bench_HEADLINE.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-dropin > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail "$OUT/prof.err"; exit 1; }
  B=$(python3 -c "import json;print(json.load(open('$OUT/prof_bench.json'))['config']['frames_per_launch'])")
  python tools/rocprof_timed.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 1 "$B" > "$OUT/rocprof_timed_HEADLINE.txt"
  cp "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" "$OUT/rocprof_kernel_stats_HEADLINE.csv"
  echo TESTS_OK ;;
configs)
  for spec in "HEADLINE:" "HEADLINE_FLY:" "C1:" "C2:" "C3:" "C4:" "C5:--steps 3 --warmup 1" "HEADLINE:--math hw"; do
    wl=${spec%%:*}; a=${spec#*:}; tag=$wl; [ "$a" = "--math hw" ] && tag=${wl}_hw_math
    timeout -k 10 400 python bench.py --workload $wl $a --no-cpu-baseline > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "bench $tag failed"; tail -5 "$OUT/$tag.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$tag.json'));r=d['roofline'];print('$tag', round(d['value'],3), 'G/s', round(d['ms_per_step'],3), 'ms', 'dropin', round(d.get('dropin_ms_per_frame') or 0,3), 'frac', round(r['frac'],4), 'sha_ok', d.get('frame_sha_ok'))"
  done
  echo CONFIGS_OK ;;
pmc)
  # PMC_SPECS: "WORKLOAD:bench args" entries separated by '|' (default: every config and the batched
  # fly-through); SHARE8=1 adds one rank's share of the 8-way split. tools/pmc_summary.py averages the
  # dispatches after the first two: the defaults give every averaged dispatch the same frames per
  # launch (16 or 4 per launch, 2 averaged; C5, animated: 1 per launch, 4 averaged)
  IFS='|' read -r -a specs <<< "${PMC_SPECS:-HEADLINE:--steps 48 --warmup 16 --batch 16|HEADLINE_FLY:--steps 48 --warmup 16 --batch 16|C2:--steps 48 --warmup 16 --batch 16|C3:--steps 48 --warmup 16 --batch 16|C4:--steps 12 --warmup 4 --batch 4|C5:--steps 4 --warmup 2}"
  for spec in "${specs[@]}"; do
    wl=${spec%%:*}; a=${spec#*:}
    OUT="$OUT/pmc_raw/$wl" ARGS="--workload $wl $a --no-cpu-baseline --no-dropin" bash tools/pmc.sh > /dev/null || { echo "pmc $wl failed"; exit 1; }
    python tools/pmc_summary.py "$OUT/pmc_raw/$wl" > "$OUT/pmc_${wl}_march.json" && python tools/pmc_summary.py "$OUT/pmc_raw/$wl" shade_pass > "$OUT/pmc_${wl}_shade.json" && python tools/pmc_summary.py "$OUT/pmc_raw/$wl" rank_pass > "$OUT/pmc_${wl}_rank.json" || exit 1
    python -c "import json;s=json.load(open('$OUT/pmc_${wl}_march.json'));print('$wl', 'valu_busy', round(s['valu_busy'],3), 'lane_util', round(s['valu_lane_utilization'],3), 'valu_insts/frame %.3g' % (s['valu_wave_insts']/s['frames_per_dispatch']), 'sq3', s.get('sq3'))"
  done
  if [ -n "$SHARE8" ]; then
    # one rank's share of bench.py's 8-way row split (rank 0, 2 launches in flight, 10 frames per launch)
    OUT="$OUT/pmc_raw/HEADLINE_share8" PROG=tools/pipeline_probe.py ARGS="--workloads HEADLINE --ranks 8 --inflight 2 --batch 10 --frames 40" bash tools/pmc.sh > /dev/null || { echo "pmc share8 failed"; exit 1; }
    python tools/pmc_summary.py "$OUT/pmc_raw/HEADLINE_share8" > "$OUT/pmc_HEADLINE_share8_march.json" && python tools/pmc_summary.py "$OUT/pmc_raw/HEADLINE_share8" shade_pass > "$OUT/pmc_HEADLINE_share8_shade.json" && python tools/pmc_summary.py "$OUT/pmc_raw/HEADLINE_share8" rank_pass > "$OUT/pmc_HEADLINE_share8_rank.json" || exit 1
  fi
  echo PMC_OK ;;
*) echo "PART=tests|configs|pmc"; exit 2 ;;
esac
