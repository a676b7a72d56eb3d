set -o pipefail
mkdir -p gpurun_out/prio
timeout -k 10 400 python -u scripts/ab_variants.py 7 > gpurun_out/prio/ab.log 2>&1 || { tail -20 gpurun_out/prio/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/prio/ab.log
