#!/bin/bash
# One GPU-box measurement of the current tree (run through gpurun), every step under its
# own time limit, stopping at the first fault/abort/timeout (scripts/gpu_run.sh):
#   tests   pytest -m gpu
#   bench   python bench.py (default run, CPU leg included)          -> bench.json
#   stats   rocprofv3 --kernel-trace --stats of the C2 bench (no CPU leg, no extras)
#   stats5  the same for C5 alone (scripts/run_c5.py)
#   pmc2/5  PMC passes (scripts/pmc.sh) for C2 and C5, summarised with source_sha
# usage: scripts/measure.sh <outdir> [steps...]   (default: all steps)
out=${1:-gpurun_out/m}; shift
steps=${*:-"tests bench stats stats5 pmc2 pmc5"}
specs=()
for s in $steps; do
  case $s in
    tests)  specs+=("tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    bench)  specs+=("bench:600:python bench.py > $out/bench.json") ;;
    stats)  specs+=("stats:300:rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-extras") ;;
    stats5) specs+=("stats5:300:rocprofv3 --kernel-trace --stats -d $out/stats5 -o run --output-format csv -- python scripts/run_c5.py") ;;
    pmc2)   specs+=("pmc2:900:bash scripts/pmc.sh $out/pmc2 && python scripts/pmc_summary.py $out/pmc2 --commit --key c2_mincurv --profile profiles/${RND:-r03}/c2_pmc_summary.json") ;;
    pmc5)   specs+=("pmc5:900:PMC_CMD='python scripts/run_c5.py' bash scripts/pmc.sh $out/pmc5 && python scripts/pmc_summary.py $out/pmc5 --commit --key c5_mincurv --profile profiles/${RND:-r03}/c5_pmc_summary.json") ;;
  esac
done
bash scripts/gpu_run.sh "$out" "${specs[@]}"
rc=$?
cp profiles/pmc_traffic.json "$out/pmc_traffic.json" 2>/dev/null
exit $rc
