"""Corridor-phase A/B: every variant library in _lib/variants/ runs C2 (cmap1 N=2000) and C5
(oval N=10000), 1024 seeds, min-curv, with max_inner_iters = 0 (per outer only normals,
corridor, lin-geom, one evaluation, update) and with the default cfg; kernel ms medians,
interleaved rounds in one process (experiments only)."""
import ctypes as C, glob, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so")))}
B = 1024
for cname in ("cmap1_n2000", "oval_n10000"):
    case = O.load_case(cname); prob = O.case_problem(case)
    for inner in (0, None):
        cfg = O.case_cfg(case)
        if inner is not None:
            cfg.max_inner_iters = inner
        plans = {}
        for n, lib in libs.items():
            h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
            seeds = np.arange(B, dtype=np.uint64)
            assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, 1) == 0
            plans[n] = (lib, h)
        res = {n: [] for n in libs}
        for r in range(4):
            for n, (lib, h) in plans.items():
                assert lib.rl_plan_run(h, None) == 0
                m = C.c_float(); lib.rl_plan_kernel_ms(h, 1, C.byref(m)); res[n].append(m.value)
        for n, (lib, h) in plans.items():
            print(f"{cname:12s} max_inner={cfg.max_inner_iters:3d} {n:10s} {np.median(res[n][1:]):8.3f} ms", flush=True)
            lib.rl_plan_destroy(h)
