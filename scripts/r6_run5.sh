set -o pipefail
mkdir -p gpurun_out/grp
timeout -k 10 300 python -u scripts/ab_variants.py 6 > gpurun_out/grp/ab.log 2>&1 || { tail -20 gpurun_out/grp/ab.log; exit 1; }
cat gpurun_out/grp/ab.log | grep -v amdgpu.ids
