#!/bin/bash
# A/B of the overlapped download's polling (round 6): the product library and two variant
# builds, reused outputs, two alternations; prints call / kernel / ABI ms per library
V=practice_path_planning_for_formula_student_driverless_amd/_lib/variants
mkdir -p gpurun_out
for r in 1 2; do
for lib in base evq200 evq200s20; do
  if [ $lib = base ]; then L=practice_path_planning_for_formula_student_driverless_amd/_lib/librl.so; else L=$V/librl_$lib.so; fi
  PCIE_REUSE=1 PCIE_LIB=$L timeout -k 10 120 python -u scripts/pcie_overlap.py cmap1_n2000 1024 5 > gpurun_out/poll_$lib.log 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/poll_$lib.log').readline()); print('$lib', d['call_ms'], d['kernel_ms'], d['abi_ms'])"
done; done
