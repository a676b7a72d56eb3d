set -o pipefail
mkdir -p gpurun_out/grp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "run_group" > gpurun_out/grp/t.log 2>&1 || { tail -30 gpurun_out/grp/t.log; exit 1; }
tail -4 gpurun_out/grp/t.log
timeout -k 10 200 python -u scripts/c4_group.py 7 > gpurun_out/grp/c4.log 2>&1 || { tail -20 gpurun_out/grp/c4.log; exit 1; }
cat gpurun_out/grp/c4.log | grep -v amdgpu.ids
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u scripts/c4_group.py 7 >> gpurun_out/grp/c4.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py 5 > gpurun_out/grp/ab.log 2>&1 || { tail -20 gpurun_out/grp/ab.log; exit 1; }
cat gpurun_out/grp/ab.log | grep -v amdgpu.ids
