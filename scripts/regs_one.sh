#!/bin/bash
# Fast static register report of the C2/C3 kernel shape only (-DRL_ANALYZE_ONE): VGPRs,
# SGPRs, scratch and occupancy of rl_optimize_kernel<8,256,closed,*,*>; the assembly
# goes to /tmp/rl_one.s.  Extra hipcc flags pass through.
cd "$(dirname "$0")/../practice_path_planning_for_formula_student_driverless_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I../../include \
  --cuda-device-only -DRL_ANALYZE_ONE=${RL_ONE:-1} -S rl_kernels.hip -o /tmp/rl_one.s -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -E "Function Name|VGPRs:|TotalSGPRs|ScratchSize|Occupancy" | sed -E 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  paste - - - - - | sed -E 's/Function Name: _ZN2rl[0-9]*//; s/\t/ | /g'
