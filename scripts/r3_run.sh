#!/bin/bash
# round-3 measurement bundle: tests, bench, phase stamps (C2/C3 and C5) in one GPU call
out=${1:-gpurun_out/r3}
shift
steps=${*:-"tests bench stamps"}
specs=()
for s in $steps; do
  case $s in
    tests)  specs+=("tests:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    bench)  specs+=("bench:600:python bench.py > $out/bench.json") ;;
    benchq) specs+=("benchq:300:python bench.py --no-cpu > $out/bench.json") ;;
    stamps) specs+=("stamps:200:python scripts/stamps.py && python scripts/stamps_c5.py") ;;
    ab)     specs+=("ab:400:python scripts/ab_variants.py 5 > $out/ab.log") ;;
    rehearse) specs+=("rehearse:400:RL_BENCH_SAME_DEVICE=1 RL_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-extras > $out/rehearse.json") ;;
  esac
done
bash scripts/gpu_run.sh "$out" "${specs[@]}"
