set -o pipefail
mkdir -p gpurun_out/grp2
timeout -k 10 200 python -u scripts/c4_group.py 7 > gpurun_out/grp2/c4.log 2>&1 || { tail -20 gpurun_out/grp2/c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp2/c4.log
AB_LAT_CASES=track_training_map,track_competition_map1,track_competition_map2,track_competition_map3,track_competition_map_testday1,track_competition_map_testday2,track_competition_map_testday3,cmap1_n2000 timeout -k 10 400 python -u scripts/ab_lat.py 7 > gpurun_out/grp2/lat.log 2>&1 || { tail -20 gpurun_out/grp2/lat.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grp2/lat.log
