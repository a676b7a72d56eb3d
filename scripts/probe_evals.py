"""Per-evaluation kernel time of C2-shaped runs for each variant library (probes whose
trajectories differ from the base: time normalised by the evaluation count)."""
import ctypes as C, glob, os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
case = O.load_case("cmap1_n2000"); prob = O.case_problem(case); cfg = O.case_cfg(case)
B = 1024
for path in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so"))):
    lib = abi.load_library(path)
    h = C.c_void_p(); p = prob.as_c(); arr, n = abi.cfg_array(cfg)
    seeds = np.arange(B, dtype=np.uint64)
    assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, n, abi.u64ptr(seeds), B, 1) == 0
    ts = []
    for _ in range(6):
        assert lib.rl_plan_run(h, None) == 0
        ms = C.c_float(); lib.rl_plan_kernel_ms(h, 1, C.byref(ms)); ts.append(ms.value)
    o = abi.Outputs.alloc(B, prob.N, 14, False); c = o.as_c()
    assert lib.rl_plan_fetch(h, C.byref(c), None) == 0
    ev = int(o.evals.sum()); t = float(np.median(ts[1:]))
    print(os.path.basename(path), json.dumps({"ms": round(t, 3), "evals": ev, "ns_per_eval_instance": round(t * 1e6 / ev * B, 2)}), flush=True)
    lib.rl_plan_destroy(h)
