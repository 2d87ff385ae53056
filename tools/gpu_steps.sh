#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop after a fault, abort, segfault,
# time limit or hang (exit >= 2 other than pytest's "tests failed" = 1).
# usage: tools/gpu_steps.sh "<secs>|<out>|<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; out=${rest%%|*}; cmd=${rest#*|}
  echo "[step] $cmd  (limit ${secs}s) -> $out"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$out" 2>&1
  rc=$?
  echo "[step] rc=$rc"
  tail -3 "gpurun_out/$out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[stop] rc=$rc"; exit $rc; fi
done
