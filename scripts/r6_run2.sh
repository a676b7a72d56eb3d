#!/bin/bash
# round-6 GPU step 2: the drop-in kernel probe, the 2-rank same-device rehearsal of the
# result gather, and the N=1 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dropin_kernel_probe.py > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
RL_BENCH_SAME_DEVICE=1 RL_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-extras \
  > gpurun_out/rehearsal.log 2>&1 || { tail -30 gpurun_out/rehearsal.log; exit 1; }
grep '"metric"' gpurun_out/rehearsal.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('n_gpus','value','ms_per_step','result_gather','parity')}))"
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
tail -c 3000 gpurun_out/bench.log
