#!/bin/bash
# rocprofv3 PMC passes over the C2 bench workload (counters in separate passes, kernel
# trace only; no sys/runtime trace).  usage: scripts/pmc.sh <outdir>
# Summarise with: python scripts/pmc_summary.py <outdir>
out=${1:-gpurun_out/pmc}
mkdir -p "$out"
export TMPDIR=/tmp
cmd=${PMC_CMD:-"python bench.py --steps 2 --warmup 0 --no-cpu --no-extras"}
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  echo "=== pass $i: $p"
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- $cmd > "$out/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
