#!/usr/bin/env python3
"""Third drop-in probe (round 6): C2's kernel time (its own HIP events) in the drop-in call
pattern, separating the download mode from the caller's buffers, interleaved over rounds:
  reuse_ovl     rl_optimize into the same host arrays, overlapped download
  reuse_noovl   the same, RL_OVERLAP_DOWNLOAD=0 (one download after the kernel)
  fresh_ovl     fresh numpy arrays every call (freed after it), overlapped download
  fresh_noovl   fresh arrays, one download after the kernel
  plan_fetch    rl_plan_run + rl_plan_fetch into preallocated (pageable) arrays
  plan_idle     rl_plan_run after 1.5 ms of host spin (the drop-in call's GPU idle gap alone)
Each case runs twice in a row per round; the second call's kernel is reported."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    lib = abi.load_library()
    case = O.load_case("cmap1_n2000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    B, N, MO = 1024, prob.N, int(cfg.max_outer_iters)
    seeds = np.arange(B, dtype=np.uint64)
    outs = abi.Outputs.alloc(B, N, MO, False)
    oc = outs.as_c()
    p = prob.as_c()
    arr, n = abi.cfg_array(cfg)
    sd = abi.u64ptr(seeds)
    plan = raceline.Plan(prob, cfg, seeds=seeds, B=B, modes=abi.RL_MODE_MINCURV)
    pre = abi.Outputs.alloc(B, N, MO, False)
    pre_c = pre.as_c()

    def kmc():
        run, k, call = C.c_float(), C.c_float(), C.c_float()
        lib.rl_last_call_times(C.byref(run), C.byref(k), None, C.byref(call))
        return k.value

    def with_env(v, f):
        os.environ["RL_OVERLAP_DOWNLOAD"] = v
        try:
            return f()
        finally:
            os.environ.pop("RL_OVERLAP_DOWNLOAD", None)

    def reuse():
        assert lib.rl_optimize(C.byref(p), arr, n, sd, B, C.byref(oc), None) == 0
        return kmc()

    def fresh():
        o, _ = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
        del o
        return kmc()

    def plan_fetch():
        plan.run()
        k = plan.kernel_ms(1)
        assert lib.rl_plan_fetch(plan._h, C.byref(pre_c), None) == 0
        return k

    def plan_idle():
        t = time.perf_counter() + 1.5e-3
        while time.perf_counter() < t:
            pass
        plan.run()
        return plan.kernel_ms(1)

    cases = {"reuse_ovl": lambda: with_env("1", reuse), "reuse_noovl": lambda: with_env("0", reuse),
             "fresh_ovl": lambda: with_env("1", fresh), "fresh_noovl": lambda: with_env("0", fresh),
             "plan_fetch": plan_fetch, "plan_idle": plan_idle}
    res = {k: [] for k in cases}
    for f in cases.values():
        f()
    for _ in range(rounds):
        for k, f in cases.items():
            f()
            res[k].append(f())
    plan.close()
    print(json.dumps({k: {"median": round(float(np.median(v)), 3), "min": round(float(np.min(v)), 3),
                          "max": round(float(np.max(v)), 3)} for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
