set -o pipefail
mkdir -p gpurun_out/grp3
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "run_group or latency_shape or ragged" > gpurun_out/grp3/t.log 2>&1 || { tail -30 gpurun_out/grp3/t.log; exit 1; }
tail -2 gpurun_out/grp3/t.log
AB_LAT_CASES=track_training_map,track_competition_map1,track_competition_map2,track_competition_map3,track_competition_map_testday1,track_competition_map_testday2,track_competition_map_testday3,cmap1_n2000 timeout -k 10 400 python -u scripts/ab_lat.py 7 > gpurun_out/grp3/lat.log 2>&1 || { tail -20 gpurun_out/grp3/lat.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp3/lat.log
timeout -k 10 300 python -u scripts/ab_variants.py 5 > gpurun_out/grp3/ab.log 2>&1 || { tail -20 gpurun_out/grp3/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp3/ab.log
