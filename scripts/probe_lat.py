"""Timing probe: time per evaluation of one-instance runs (latency shapes) of the product
against timing-probe variants (probe_nob1: no trial-halo barrier; probe_nozb: every clamp as
maxNum/minNum; their results may be wrong, only the time per evaluation, kernel ms /
evaluations, is read).  Plan path, min-curv.  usage: probe_lat.py [variant ...]"""
import ctypes as C, os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
libs = {"base": abi.load_library()}
for v in (sys.argv[1:] or ["probe_nob1"]):
    libs[v] = abi.load_library(os.path.join(REPO, f"practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_{v}.so"))
for cname in ("track_training_map", "track_competition_map_testday3", "cmap1_n2000"):
    case = O.load_case(cname); prob = O.case_problem(case); cfg = O.case_cfg(case)
    for B in (1, 1024):
        row = {}
        for n, lib in libs.items():
            h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
            seeds = np.arange(B, dtype=np.uint64)
            assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, 1) == 0
            ts = []
            for r in range(6):
                assert lib.rl_plan_run(h, None) == 0
                ms = C.c_float(); lib.rl_plan_kernel_ms(h, 1, C.byref(ms)); ts.append(ms.value)
            o = abi.Outputs.alloc(B, prob.N, 14, False); c = o.as_c()
            assert lib.rl_plan_fetch(h, C.byref(c), None) == 0
            ev = int(o.evals.sum())
            t = float(np.median(ts[1:]))
            row[n] = {"ms": round(t, 3), "evals": ev, "ns_per_eval_instance": round(1e6 * t / ev * B, 1)}
            lib.rl_plan_destroy(h)
        print(cname, "B", B, json.dumps(row), flush=True)
