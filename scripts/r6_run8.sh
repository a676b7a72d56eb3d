set -o pipefail
mkdir -p gpurun_out/grp3
timeout -k 10 400 python -u scripts/ab_variants.py 7 > gpurun_out/grp3/ab2.log 2>&1 || { tail -20 gpurun_out/grp3/ab2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp3/ab2.log
timeout -k 10 200 python -u scripts/c4_group.py 7 > gpurun_out/grp3/c4.log 2>&1 || { tail -20 gpurun_out/grp3/c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp3/c4.log
