#!/bin/bash
# round-6 GPU step 3: the second drop-in probe, plain and under rocprofv3 --kernel-trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dropin_kernel_probe2.py 6 > gpurun_out/probe2.log 2>&1 || { cat gpurun_out/probe2.log; exit 1; }
cat gpurun_out/probe2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe2_trace -o run --output-format csv -- python -u scripts/dropin_kernel_probe2.py 3 \
  > gpurun_out/probe2_trace.log 2>&1 || { tail -20 gpurun_out/probe2_trace.log; exit 1; }
grep '"none"' gpurun_out/probe2_trace.log
f=$(find gpurun_out/probe2_trace -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rl_optimize_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print("rocprof rl_optimize_kernel durations ms:", [round(x, 3) for x in d])
PY
