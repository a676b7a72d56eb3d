#!/bin/bash
# Latency / instruction-fetch PMC passes (one counter group per run, kernel trace only) over
# a command (default: the C5 corridor-dominated run).  usage: scripts/pmc_lat.sh <outdir> [cmd...]
out=${1:-gpurun_out/lat}; shift
cmd=${*:-"python scripts/run_phase.py C5 --only"}
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS"
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES"
  "SQC_DCACHE_HITS SQC_DCACHE_MISSES"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  echo "=== pass $i: $p"
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- $cmd > "$out/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
