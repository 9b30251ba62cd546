#!/bin/bash
# The C-host drop-in loop under /opt/rocm's HIP runtime and under torch's bundled one (same binary,
# LD_LIBRARY_PATH), 2 interleaved rounds: is the runtime what makes it slower than the Python loop?
set -o pipefail
OUT=${OUT:-gpurun_out/dropin_c2}
mkdir -p "$OUT"
TL=$(python3 -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
for round in 1 2; do
  for rt in rocm torch; do
    for wl in fly fixed; do
      if [ $rt = torch ]; then
        LD_LIBRARY_PATH=$TL timeout -k 10 120 ./tools/micro/dropin_loop $wl 20 > "$OUT/${rt}_${wl}_$round.json" 2> "$OUT/${rt}_${wl}_$round.err" || { tail -3 "$OUT/${rt}_${wl}_$round.err"; exit 1; }
      else
        timeout -k 10 120 ./tools/micro/dropin_loop $wl 20 > "$OUT/${rt}_${wl}_$round.json" 2> "$OUT/${rt}_${wl}_$round.err" || { tail -3 "$OUT/${rt}_${wl}_$round.err"; exit 1; }
      fi
      echo "r$round $rt $(cat $OUT/${rt}_${wl}_$round.json)"
    done
  done
done
