"""A/B kernel time of the C5 workload (oval N=10000, B instances, min-curv) over the
variant libraries in _lib/variants/ (experiments only), interleaved rounds."""
import ctypes as C, glob, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

pat = sys.argv[1] if len(sys.argv) > 1 else "all"
pat = "*" if pat == "all" else pat
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
modes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_" + pat + ".so")))}
case = O.load_case("oval_n10000"); prob = O.case_problem(case); cfg = O.case_cfg(case)
plans = {}
for n, lib in libs.items():
    h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
    seeds = np.arange(B, dtype=np.uint64)
    assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, modes) == 0, lib.rl_last_error()
    plans[n] = (lib, h)
times = {n: [] for n in libs}
for r in range(4):
    for n, (lib, h) in plans.items():
        assert lib.rl_plan_run(h, None) == 0
        ms = C.c_float(); lib.rl_plan_kernel_ms(h, modes, C.byref(ms))
        times[n].append(ms.value)
for n, t in times.items():
    print(f"C5 B={B} modes={modes} {n:12s} median {np.median(t[1:]):8.2f} ms  min {min(t[1:]):8.2f}", flush=True)
outs = {}
for n, (lib, h) in plans.items():
    o = abi.Outputs.alloc(B, prob.N, 14, modes == 2)
    c = o.as_c()
    lib.rl_plan_fetch(h, C.byref(c), None) if modes == 1 else lib.rl_plan_fetch(h, None, C.byref(c))
    outs[n] = o
base = next(iter(libs))
for n in libs:
    same = all(np.array_equal(getattr(outs[n], f), getattr(outs[base], f)) for f in ("x", "y", "alpha_last", "kappa", "evals", "accepts"))
    print(f"C5 {n:12s} bitexact_vs_{base}: {same}; evals/outer {outs[n].evals.mean():.2f}", flush=True)
