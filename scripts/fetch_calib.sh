#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration at known byte counts (scripts/fetch_calib.hip):
# one plain run for the timings, then one rocprofv3 --pmc pass per counter (kernel trace
# only, no other trace domains).  Summarise with scripts/fetch_calib_summary.py <out>.
# usage: scripts/fetch_calib.sh <outdir>
out=${1:-gpurun_out/fcal}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/_fetch_calib 3 > "$out/timing.log" 2>&1 || exit $?
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  echo "=== pass $i: $p"
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- ./scripts/_fetch_calib 2 > "$out/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
