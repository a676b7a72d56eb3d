"""C4 schedule timing (bench.run_c4 without the oracle): 7 tracks x 512 sweep points, one
plan per track (both modes), every plan on its own torch stream; prints ms per launch round.
Run under different GPU_MAX_HW_QUEUES settings to see the hardware-queue limit."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
import torch
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline
from practice_path_planning_for_formula_student_driverless_amd import distributed as D

base = O.case_cfg(O.load_case("track_training_map"))
cfgs = D.c4_cfgs(base)
plans = []
for t in D.C4_TRACKS:
    prob = O.case_problem(O.load_case("track_" + t))
    plans.append(raceline.Plan(prob, cfgs, B=512, modes=abi.RL_MODE_MINCURV | abi.RL_MODE_MINTIME))
streams = [torch.cuda.Stream() for _ in plans]

def launch():
    for pl, st in zip(plans, streams):
        pl.run(st.cuda_stream)
    for st in streams:
        st.synchronize()

launch(); launch()
ts = []
for _ in range(5):
    t0 = time.perf_counter(); launch(); ts.append(time.perf_counter() - t0)
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '(default)')}: C4 {1e3*np.median(ts):.3f} ms "
      f"(min {1e3*min(ts):.3f}); per-plan mc/mt kernel ms "
      + " ".join(f"{pl.kernel_ms(1):.2f}/{pl.kernel_ms(2):.2f}" for pl in plans), flush=True)
