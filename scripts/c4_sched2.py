"""C4 schedules at this process's GPU_MAX_HW_QUEUES (A/B, no oracle): 7 tracks x 512 sweep
points, both optimisers.
  both7   one plan per track with both modes (the plan runs min-time on its own second
          stream), every plan on its own torch stream (the round-3 bench)
  lptQ    one plan per (track, mode), the 14 kernels dealt onto Q streams (Q = the hardware
          queue count) longest-first by their measured solo time, each stream in order
  all14   one plan per (track, mode), each on its own stream
Prints the median ms per launch round of each schedule."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
import torch  # noqa: E402

from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import distributed as D  # noqa: E402

Q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
base = O.case_cfg(O.load_case("track_training_map"))
cfgs = D.c4_cfgs(base)
probs = [O.case_problem(O.load_case("track_" + t)) for t in D.C4_TRACKS]
MC, MT = abi.RL_MODE_MINCURV, abi.RL_MODE_MINTIME


def timed(launch, reps=5):
    launch()
    launch()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        launch()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


def run_lists(lists, streams):
    for pls, st in zip(lists, streams):
        for pl in pls:
            pl.run(st.cuda_stream)
    for st in streams:
        st.synchronize()


both = [raceline.Plan(p, cfgs, B=512, modes=MC | MT) for p in probs]
single = [(raceline.Plan(p, cfgs, B=512, modes=m), m) for p in probs for m in (MC, MT)]
res = {}
st7 = [torch.cuda.Stream() for _ in both]
res["both7"] = timed(lambda: run_lists([[pl] for pl in both], st7))
# solo times of the single-mode kernels (one at a time)
solo = []
s0 = torch.cuda.Stream()
for pl, m in single:
    pl.run(s0.cuda_stream)
    s0.synchronize()
    pl.run(s0.cuda_stream)
    s0.synchronize()
    solo.append(pl.kernel_ms(1 if m == MC else 2))
order = np.argsort(solo)[::-1]
for q in sorted({Q, 2, 4, 8}):
    lists, load = [[] for _ in range(q)], [0.0] * q
    for i in order:
        j = int(np.argmin(load))
        lists[j].append(single[i][0])
        load[j] += solo[i]
    sts = [torch.cuda.Stream() for _ in range(q)]
    res[f"lpt{q}"] = timed(lambda: run_lists(lists, sts))
st14 = [torch.cuda.Stream() for _ in single]
res["all14"] = timed(lambda: run_lists([[pl] for pl, _ in single], st14))
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}: " +
      " ".join(f"{k} {v:.3f}" for k, v in res.items()) +
      "  solo ms " + " ".join(f"{s:.2f}" for s in solo), flush=True)
for pl in both:
    pl.close()
for pl, _ in single:
    pl.close()
