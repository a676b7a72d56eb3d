#!/usr/bin/env python3
"""C4 as the bench runs it (7 bundled tracks x 512 sweep points x 2 modes = 14 single-mode
plans, shape batch 7168) under two schedules, interleaved rounds, wall ms of the whole sweep:
  s14    every plan on its own HIP stream (bench.run_c4 before rl_plan_run_group)
  group  rl_plan_run_group over the 14 plans: per mode one launch per K (the ragged form
         for a launch with any N % K != 0; profiles/r06/c4_group.log also holds the earlier
         split by N % K as `group` against this merged form as `group_mix`, and the merged
         form in plan order as `group` against longest-first as `group_sorted`, now the default)
and a bit-for-bit check of every plan's laps and counters between the two.
usage: python scripts/c4_group.py [rounds]   (GPU_MAX_HW_QUEUES as the environment sets it)"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import distributed as D  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
B = 512
cfgs = D.c4_cfgs(O.case_cfg(O.load_case("track_training_map")))
plans = []
for t in D.C4_TRACKS:
    prob = O.case_problem(O.load_case("track_" + t))
    for mode in (abi.RL_MODE_MINCURV, abi.RL_MODE_MINTIME):
        pl = raceline.Plan(prob, cfgs, B=B, modes=mode, device=0)
        pl.set_shape_batch(2 * len(D.C4_TRACKS) * B)
        plans.append(pl)
streams = [torch.cuda.Stream() for _ in plans]
main = torch.cuda.Stream()


def s14():
    for pl, st in zip(plans, streams):
        pl.run(st.cuda_stream)
    for st in streams:
        st.synchronize()


def group():
    raceline.Plan.run_group(plans, main.cuda_stream)
    main.synchronize()


def snapshot():
    out = []
    for pl in plans:
        mc, mt = pl.fetch()
        o = mc if mc is not None else mt
        out.append([o.evals.copy(), o.accepts.copy(), o.kappa.copy()] + ([mt.lap.copy()] if mt is not None else []))
    return out


s14()
ref = snapshot()
same = {}
for name, f in (("group", group),):
    f()
    got = snapshot()
    same[name] = all(all(np.array_equal(a, b) for a, b in zip(r, g)) for r, g in zip(ref, got))
res = {"s14": [], "group": []}
for _ in range(rounds):
    for name, f in (("s14", s14), ("group", group)):
        t0 = time.perf_counter()
        f()
        res[name].append((time.perf_counter() - t0) * 1e3)
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}; bit-exact vs s14: {same}")
for k, v in res.items():
    print(f"C4 {k:6s} wall ms: median {np.median(v):7.2f} min {np.min(v):7.2f}", flush=True)
for pl in plans:
    pl.close()
