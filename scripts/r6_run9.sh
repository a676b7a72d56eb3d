set -o pipefail
mkdir -p gpurun_out/grp4
timeout -k 10 200 python -u scripts/c4_group.py 9 > gpurun_out/grp4/c4.log 2>&1 || { tail -20 gpurun_out/grp4/c4.log; exit 1; }
timeout -k 10 200 python -u scripts/c4_group.py 9 >> gpurun_out/grp4/c4.log 2>&1 || { tail -20 gpurun_out/grp4/c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp4/c4.log
