#!/bin/bash
# Run GPU steps in order; each step has its own time limit.  A test failure (rc 1)
# does not stop the sequence, a fault / abort / timeout (rc >= 124 or signal) does.
# usage: scripts/gpu_run.sh <outdir> <name>:<seconds>:<command> ...
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd" | tee -a "$out/steps.log"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc $(( $(date +%s) - start ))s" | tee -a "$out/steps.log"
  tail -3 "$out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping after $name (rc=$rc)" | tee -a "$out/steps.log"; exit $rc
  fi
done
