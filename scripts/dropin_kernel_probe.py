#!/usr/bin/env python3
"""Why is C2's kernel ~1.4 ms slower inside rl_optimize than on the plan path (round 6)?
The optimiser kernel alone (HIP events), C2 (B=1024, min-curv), in interleaved rounds:
  plan_b2b        rl_plan_run back to back
  plan_fetch      rl_plan_run + rl_plan_fetch into preallocated host arrays
  opt_x_only      rl_optimize asking for x only (8 MB: below the overlap threshold)
  opt_reuse       rl_optimize into the same host arrays every call (pages already present)
  opt_fresh       rl_optimize into fresh numpy arrays every call (the bench's leg)
  opt_fresh_noovl the same with RL_OVERLAP_DOWNLOAD=0
Also: the kernel, the page-population call and the host-copy rates of this box."""
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402


def host_probe():
    libc = C.CDLL("libc.so.6", use_errno=True)
    libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    n = 64 << 20
    a = np.empty(n, dtype=np.uint8)
    base = a.ctypes.data & ~4095
    t0 = time.perf_counter()
    rc = libc.madvise(C.c_void_p(base), C.c_size_t(n - 8192), 23)      # MADV_POPULATE_WRITE
    t_pop = time.perf_counter() - t0
    err = C.get_errno()
    src = np.ones(n, dtype=np.uint8)
    fresh = np.empty(n, dtype=np.uint8)
    t0 = time.perf_counter()
    C.memmove(fresh.ctypes.data, src.ctypes.data, n)
    t_fresh = time.perf_counter() - t0
    t0 = time.perf_counter()
    C.memmove(fresh.ctypes.data, src.ctypes.data, n)
    t_warm = time.perf_counter() - t0
    thp = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip() \
        if os.path.exists("/sys/kernel/mm/transparent_hugepage/enabled") else None
    return {"kernel": platform.release(), "madvise_populate_rc": rc, "errno": err,
            "populate_64MB_ms": round(t_pop * 1e3, 2), "memcpy_64MB_fresh_ms": round(t_fresh * 1e3, 2),
            "memcpy_64MB_warm_ms": round(t_warm * 1e3, 2), "thp": thp}


def main():
    print(json.dumps(host_probe()), flush=True)
    lib = abi.load_library()
    case = O.load_case("cmap1_n2000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    B, N, MO = 1024, prob.N, int(cfg.max_outer_iters)
    seeds = np.arange(B, dtype=np.uint64)
    plan = raceline.Plan(prob, cfg, seeds=seeds, B=B, modes=abi.RL_MODE_MINCURV)
    pre = abi.Outputs.alloc(B, N, MO, False)
    pre_c = pre.as_c()
    reuse = abi.Outputs.alloc(B, N, MO, False)
    reuse_c = reuse.as_c()
    xonly = abi.Outputs.alloc(B, N, MO, False)
    xo = abi.RlOut()
    xo.x = xonly.as_c().x
    p = prob.as_c()
    arr, n = abi.cfg_array(cfg)
    sd = abi.u64ptr(seeds)

    def mc_ms():
        run, kmc, call = C.c_float(), C.c_float(), C.c_float()
        lib.rl_last_call_times(C.byref(run), C.byref(kmc), None, C.byref(call))
        return kmc.value

    def plan_b2b():
        plan.run()
        return plan.kernel_ms(1)

    def plan_fetch():
        plan.run()
        k = plan.kernel_ms(1)
        assert lib.rl_plan_fetch(plan._h, C.byref(pre_c), None) == 0
        return k

    def opt(o):
        assert lib.rl_optimize(C.byref(p), arr, n, sd, B, C.byref(o), None) == 0
        return mc_ms()

    def opt_fresh():
        out, _ = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
        del out
        return mc_ms()

    def opt_fresh_noovl():
        os.environ["RL_OVERLAP_DOWNLOAD"] = "0"
        try:
            return opt_fresh()
        finally:
            os.environ.pop("RL_OVERLAP_DOWNLOAD")

    cases = {"plan_b2b": plan_b2b, "plan_fetch": plan_fetch, "opt_x_only": lambda: opt(xo),
             "opt_reuse": lambda: opt(reuse_c), "opt_fresh": opt_fresh, "opt_fresh_noovl": opt_fresh_noovl}
    res = {k: [] for k in cases}
    for f in cases.values():
        f()
    for _ in range(6):
        for k, f in cases.items():
            vals = [f() for _ in range(3)]          # three in a row: the later ones are back to back-ish
            res[k].append(vals)
    plan.close()
    print(json.dumps({k: {"first_of_3": round(float(np.median([v[0] for v in vs])), 3),
                          "third_of_3": round(float(np.median([v[2] for v in vs])), 3)} for k, vs in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
