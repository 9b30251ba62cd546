#!/bin/bash
# GPU session steps: run the given steps in order, each under its own time limit; stop at the
# first step that ends in anything but success or ordinary test failures (rc 0/1/3).
# usage: tools/gpu_step.sh 'SECONDS|NAME|COMMAND' ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ]; then echo "stopping after $name"; exit $rc; fi
done
