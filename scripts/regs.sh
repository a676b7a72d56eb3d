#!/bin/bash
# Per-kernel VGPR / scratch / occupancy report of the gfx950 kernels (static, no GPU).
# One line per kernel: <K,T,closed,mintime,ragged> (or the streaming kernel's <closed,mintime>).
cd "$(dirname "$0")/../practice_path_planning_for_formula_student_driverless_amd/csrc" || exit 1
for f in rl_kernels.hip rl_kernels_lat.hip rl_kernels_mid.hip rl_stream.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I../../include \
    --cuda-device-only -c "$f" -o /tmp/_regs.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
    grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
    paste - - - - | sed -E 's/Function Name: _ZN2rl[0-9]*//; s/EEEvNS_7KParams.*\t *VGPRs/ VGPRs/; s/ILi([0-9]+)ELi([0-9]+)ELb([01])ELb([01])ELb([01])/<\1,\2,\3,\4,\5>/; s/ILb([01])ELb([01])/<\1,\2>/; s/\t */ | /g'
done
