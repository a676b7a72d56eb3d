"""A/B kernel times of C4-shaped plans (each bundled track, B=512 sweep points, both
modes) over the variant libraries in _lib/variants/ (experiments only), interleaved."""
import ctypes as C, glob, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so")))}
tracks = ["track_training_map", "track_competition_map1", "track_competition_map2", "track_competition_map3",
          "track_competition_map_testday1", "track_competition_map_testday2", "track_competition_map_testday3"]
B = 512
res = {n: [] for n in libs}
plans = {}
for t in tracks:
    case = O.load_case(t); prob = O.case_problem(case); cfg = O.case_cfg(case)
    for n, lib in libs.items():
        h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
        seeds = np.arange(B, dtype=np.uint64)
        assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, 3) == 0
        plans[(t, n)] = (lib, h, prob.N)
outs = {}
for r in range(4):
    tot = {n: 0.0 for n in libs}
    for (t, n), (lib, h, N) in plans.items():
        assert lib.rl_plan_run(h, None) == 0
        ms = C.c_float(); lib.rl_plan_kernel_ms(h, 0, C.byref(ms)); tot[n] += ms.value
        if r == 0:
            o1 = abi.Outputs.alloc(B, N, 14, False); o2 = abi.Outputs.alloc(B, N, 14, True)
            c1, c2 = o1.as_c(), o2.as_c()
            lib.rl_plan_fetch(h, C.byref(c1), C.byref(c2))
            outs[(t, n)] = (o1, o2)
    for n in libs: res[n].append(tot[n])
base = next(iter(libs))
for n in libs:
    same = all(np.array_equal(outs[(t, n)][m].x, outs[(t, base)][m].x) and np.array_equal(outs[(t, n)][m].evals, outs[(t, base)][m].evals)
               for t in tracks for m in (0, 1))
    print(f"C4 (7 tracks x {B}, both modes, sequential) {n:10s} sum of run ms: median {np.median(res[n][1:]):8.2f} min {min(res[n][1:]):8.2f}  bitexact_vs_{base}: {same}", flush=True)
