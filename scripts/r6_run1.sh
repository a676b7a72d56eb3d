#!/bin/bash
# round-6 GPU step 1: overlapped-download tests and timing, the idle-gap sweep, C5 corridor
# counters per pass, and the (2, 256) latency-shape A/B for the five-wave tracks
set -o pipefail
mkdir -p gpurun_out
L=practice_path_planning_for_formula_student_driverless_amd/_lib/variants
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "overlapped or plan_cache or dropin or lap_eval" > gpurun_out/t_ovl.log 2>&1 || { tail -30 gpurun_out/t_ovl.log; exit 1; }
tail -3 gpurun_out/t_ovl.log
timeout -k 10 200 python -u scripts/pcie_overlap.py > gpurun_out/ovl.log 2>&1 || { cat gpurun_out/ovl.log; exit 1; }
cat gpurun_out/ovl.log
PCIE_LIB=$L/librl_ovltrace.so timeout -k 10 200 python -u scripts/pcie_overlap.py cmap1_n2000 1024 4 \
  > gpurun_out/ovl_trace.log 2> gpurun_out/ovl_trace.err || { tail gpurun_out/ovl_trace.err; exit 1; }
grep ovl_trace gpurun_out/ovl_trace.err | tail -2
timeout -k 10 200 python -u scripts/gap_sweep.py > gpurun_out/gap.log 2>&1 || { cat gpurun_out/gap.log; exit 1; }
cat gpurun_out/gap.log
timeout -k 10 200 python -u scripts/counts_c5_outer.py > gpurun_out/counts_outer.log 2>&1 || { cat gpurun_out/counts_outer.log; exit 1; }
cat gpurun_out/counts_outer.log
bash scripts/fetch_calib.sh gpurun_out/fcal6 > gpurun_out/fcal6.log 2>&1 || { cat gpurun_out/fcal6.log; exit 1; }
python scripts/fetch_calib_summary.py gpurun_out/fcal6 > /dev/null && grep -A1 '"fetch_factor"\|read8' gpurun_out/fcal6/fetch_calib.json | head -30
AB_LAT_CASES=track_competition_map_testday1,track_competition_map_testday3,track_competition_map2 \
  timeout -k 10 300 python -u scripts/ab_lat.py 7 > gpurun_out/ab_lat_s5.log 2>&1 || { cat gpurun_out/ab_lat_s5.log; exit 1; }
cat gpurun_out/ab_lat_s5.log
