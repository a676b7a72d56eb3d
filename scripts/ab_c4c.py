"""A/B wall time of the C4 sweep as bench.py runs it (7 bundled tracks x 512 (mu, P_max_W,
lambda_smooth) points, both modes, one plan per track on concurrent HIP streams) over the
variant libraries in _lib/variants/ (experiments only), interleaved; checks bit-exactness
of every plan's outputs against the first variant."""
import ctypes as C, glob, os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
from practice_path_planning_for_formula_student_driverless_amd import distributed as D

libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so")))}
B = 512
base_cfg = O.case_cfg(O.load_case("track_training_map"))
cfgs = D.c4_cfgs(base_cfg)
arr, nc = abi.cfg_array(cfgs)
plans = {n: [] for n in libs}
for t in D.C4_TRACKS:
    case = O.load_case("track_" + t); prob = O.case_problem(case)
    for n, lib in libs.items():
        h = C.c_void_p(); p = prob.as_c()
        seeds = np.zeros(B, dtype=np.uint64)
        assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, abi.u64ptr(seeds), B, 3) == 0
        plans[n].append((lib, h, prob.N))
streams = [torch.cuda.Stream() for _ in D.C4_TRACKS]


def launch(n):
    for (lib, h, _), st in zip(plans[n], streams):
        assert lib.rl_plan_run(h, C.c_void_p(st.cuda_stream)) == 0
    for st in streams:
        st.synchronize()


res = {n: [] for n in libs}
for r in range(6):
    for n in libs:
        t0 = time.perf_counter(); launch(n); res[n].append((time.perf_counter() - t0) * 1e3)
outs = {}
for n in libs:
    for i, (lib, h, N) in enumerate(plans[n]):
        o1 = abi.Outputs.alloc(B, N, 14, False); o2 = abi.Outputs.alloc(B, N, 14, True)
        c1, c2 = o1.as_c(), o2.as_c()
        lib.rl_plan_fetch(h, C.byref(c1), C.byref(c2))
        outs[(i, n)] = (o1, o2)
base = next(iter(libs))
for n in libs:
    same = all(np.array_equal(outs[(i, n)][m].x, outs[(i, base)][m].x) and np.array_equal(outs[(i, n)][m].lap, outs[(i, base)][m].lap)
               for i in range(len(D.C4_TRACKS)) for m in (0, 1))
    print(f"C4 concurrent (7 tracks x {B}, both modes) {n:10s} wall ms: median {np.median(res[n][1:]):8.2f} "
          f"min {min(res[n][1:]):8.2f}  bitexact_vs_{base}: {same}", flush=True)
