"""C4 schedules over the product library (A/B, no oracle): the bench's 14 single-mode plans
(7 bundled tracks x 512 sweep points x 2 modes, shape batch = 3584), each schedule timed in
interleaved rounds:
  s14      every plan on its own stream, plans in track order (bench.run_c4 today);
  lptS     S streams, plans sorted by their own measured kernel time (longest first) and
           dealt to the least-loaded stream (longest-processing-time first).
usage: python scripts/c4_sched3.py [rounds]"""
import os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import raceline
from practice_path_planning_for_formula_student_driverless_amd import abi
from practice_path_planning_for_formula_student_driverless_amd import distributed as D

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
B = 512
cfgs = D.c4_cfgs(O.case_cfg(O.load_case("track_training_map")))
plans = []
for t in D.C4_TRACKS:
    prob = O.case_problem(O.load_case("track_" + t))
    for mode in (abi.RL_MODE_MINCURV, abi.RL_MODE_MINTIME):
        pl = raceline.Plan(prob, cfgs, B=B, modes=mode, device=0)
        pl.set_shape_batch(len(D.C4_TRACKS) * B)
        plans.append(pl)
# each plan alone (its kernel time, min of 3)
alone = []
for pl in plans:
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter(); pl.run(0); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
    alone.append(best)
order = sorted(range(len(plans)), key=lambda i: -alone[i])


def lpt(S):
    load = [0.0] * S
    assign = [[] for _ in range(S)]
    for i in order:
        s = min(range(S), key=lambda j: load[j])
        assign[s].append(i); load[s] += alone[i]
    return assign


scheds = {"s14": [[i] for i in range(len(plans))]}
for S in (4, 7, 8):
    scheds[f"lpt{S}"] = lpt(S)
streams = {k: [torch.cuda.Stream() for _ in v] for k, v in scheds.items()}


def run(k):
    for grp, st in zip(scheds[k], streams[k]):
        for i in grp:
            plans[i].run(st.cuda_stream)
    for st in streams[k]:
        st.synchronize()


res = {k: [] for k in scheds}
for r in range(rounds + 1):
    for k in scheds:
        t0 = time.perf_counter(); run(k); res[k].append((time.perf_counter() - t0) * 1e3)
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}; plans alone (ms): " +
      " ".join(f"{a * 1e3:.2f}" for a in alone))
for k in scheds:
    print(f"C4 schedule {k:6s} wall ms: median {np.median(res[k][1:]):7.2f} min {min(res[k][1:]):7.2f}", flush=True)
