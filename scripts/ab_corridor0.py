#!/usr/bin/env python3
"""A/B of the batch-wide first corridor (KParams::lo0/hi0, rl_plan_run): the same plans run
with RL_CORRIDOR0=1 (outer iteration 0's corridor cast once per batch by rl_corridor_kernel)
and RL_CORRIDOR0=0 (every instance casts it), interleaved; kernel ms of the mode's own events
plus the run bracket, and the outputs compared bit for bit.
usage: python scripts/ab_corridor0.py [rounds]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402

CASES = [("C2", "cmap1_n2000", 1024, abi.RL_MODE_MINCURV), ("C3mt", "cmap1_n2000_vp20", 4096, abi.RL_MODE_MINTIME),
         ("C5", "oval_n10000", 1024, abi.RL_MODE_MINCURV), ("C5mt", "oval_n10000", 1024, abi.RL_MODE_MINTIME),
         ("C4t3", "track_competition_map_testday3", 512, abi.RL_MODE_MINTIME),
         ("C4tm", "track_training_map", 512, abi.RL_MODE_MINCURV)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    sel = os.environ.get("AB_CASES")
    res = {}
    for name, cname, B, mode in CASES:
        if sel and name not in sel.split(","):
            continue
        case = O.load_case(cname)
        prob, cfg = O.case_problem(case), O.case_cfg(case)
        plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B, modes=mode)
        idx = 1 if mode == abi.RL_MODE_MINCURV else 2
        outs, times, runs = {}, {"1": [], "0": []}, {"1": [], "0": []}
        for r in range(rounds + 1):
            for v in ("1", "0"):
                os.environ["RL_CORRIDOR0"] = v
                plan.run()
                k = plan.kernel_ms(idx)
                w = plan.kernel_ms(0)
                if r == 0:
                    mc, mt = plan.fetch()
                    outs[v] = mc if mode == abi.RL_MODE_MINCURV else mt
                else:
                    times[v].append(k)
                    runs[v].append(w)
        plan.close()
        same = all(np.array_equal(getattr(outs["1"], f), getattr(outs["0"], f)) for f in abi.OUT_F64 + ("evals", "accepts"))
        res[name] = {"bitexact": bool(same),
                     "on_kernel_ms": round(float(np.median(times["1"])), 3), "off_kernel_ms": round(float(np.median(times["0"])), 3),
                     "on_run_ms": round(float(np.median(runs["1"])), 3), "off_run_ms": round(float(np.median(runs["0"])), 3)}
        print(json.dumps({name: res[name]}), flush=True)
    os.environ.pop("RL_CORRIDOR0", None)


if __name__ == "__main__":
    main()
