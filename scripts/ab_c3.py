"""A/B kernel times of the C3 workload (competition_map1 N=2000, max_vpass_iters=20, both
modes) at B=256 and B=4096 over the variant libraries in _lib/variants/ (experiments only),
interleaved; checks bit-exactness of the min-time outputs against the first variant."""
import ctypes as C, glob, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so")))}
case = O.load_case("cmap1_n2000_vp20"); prob = O.case_problem(case); cfg = O.case_cfg(case)
for B in (256, 4096):
    plans = {}
    for n, lib in libs.items():
        h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
        seeds = np.arange(B, dtype=np.uint64)
        assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, 3) == 0
        plans[n] = (lib, h)
    res = {n: [] for n in libs}
    for r in range(4):
        for n, (lib, h) in plans.items():
            assert lib.rl_plan_run(h, None) == 0
            m0, m1, m2 = C.c_float(), C.c_float(), C.c_float()
            lib.rl_plan_kernel_ms(h, 0, C.byref(m0))
            lib.rl_plan_kernel_ms(h, 1, C.byref(m1)); lib.rl_plan_kernel_ms(h, 2, C.byref(m2))
            res[n].append((m1.value, m2.value, m0.value))
    outs = {}
    for n, (lib, h) in plans.items():
        o1 = abi.Outputs.alloc(B, prob.N, 14, False); o2 = abi.Outputs.alloc(B, prob.N, 14, True)
        c1, c2 = o1.as_c(), o2.as_c()
        lib.rl_plan_fetch(h, C.byref(c1), C.byref(c2))
        outs[n] = o2
        lib.rl_plan_destroy(h)
    base = next(iter(libs))
    for n in libs:
        a = np.array(res[n][1:])
        same = all(np.array_equal(getattr(outs[n], f), getattr(outs[base], f))
                   for f in ("x", "y", "alpha_last", "v", "ax", "lap"))
        print(f"C3 B={B:5d} {n:8s} min-curv {np.median(a[:, 0]):7.2f} ms  min-time {np.median(a[:, 1]):7.2f} ms  run {np.median(a[:, 2]):7.2f} ms  "
              f"bitexact_vs_{base}: {same}", flush=True)
        if not same:
            print("    differs:", [f for f in ("x", "y", "alpha_last", "v", "ax", "lap", "evals", "accepts")
                                   if not np.array_equal(getattr(outs[n], f), getattr(outs[base], f))],
                  "max |dlap|", float(np.max(np.abs(outs[n].lap - outs[base].lap))),
                  "max |dx|", float(np.max(np.abs(outs[n].x - outs[base].x))), flush=True)
