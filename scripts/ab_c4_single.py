"""A/B wall time of the C4 sweep exactly as bench.run_c4 schedules it (7 bundled tracks x 512
(mu, P_max_W, lambda_smooth) points, one single-mode plan per (track, mode), every plan on its own
HIP stream, all enqueued before any wait) over the variant libraries in _lib/variants/,
interleaved rounds; checks every plan's outputs bit for bit against the first variant.
usage: [AB_MODE=mc|mt] python scripts/ab_c4_single.py [rounds]"""
import ctypes as C, glob, os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
from practice_path_planning_for_formula_student_driverless_amd import distributed as D

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
libs = {os.path.basename(p)[6:-3]: abi.load_library(p)
        for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so")))}
B = 512
MODES = {"mc": (abi.RL_MODE_MINCURV,), "mt": (abi.RL_MODE_MINTIME,)}.get(
    os.environ.get("AB_MODE", ""), (abi.RL_MODE_MINCURV, abi.RL_MODE_MINTIME))
cfgs = D.c4_cfgs(O.case_cfg(O.load_case("track_training_map")))
arr, nc = abi.cfg_array(cfgs)
plans = {n: [] for n in libs}
for t in D.C4_TRACKS:
    prob = O.case_problem(O.load_case("track_" + t))
    for mode in MODES:
        for n, lib in libs.items():
            h = C.c_void_p(); p = prob.as_c()
            assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, None, B, mode) == 0
            if hasattr(lib, "rl_plan_set_shape_batch"):
                assert lib.rl_plan_set_shape_batch(h, len(D.C4_TRACKS) * B) == 0
            plans[n].append((lib, h, prob.N, mode))
streams = [torch.cuda.Stream() for _ in plans[next(iter(libs))]]


def launch(n):
    for (lib, h, _, _), st in zip(plans[n], streams):
        assert lib.rl_plan_run(h, C.c_void_p(st.cuda_stream)) == 0
    for st in streams:
        st.synchronize()


res = {n: [] for n in libs}
for r in range(rounds + 1):
    for n in libs:
        t0 = time.perf_counter(); launch(n); res[n].append((time.perf_counter() - t0) * 1e3)
if os.environ.get("AB_PER_PLAN"):      # each plan alone, its kernel time (min of 3 runs)
    for n in libs:
        per = []
        for (lib, h, N, mode) in plans[n]:
            best = 1e9
            for _ in range(3):
                assert lib.rl_plan_run(h, None) == 0
                ms = C.c_float(); lib.rl_plan_kernel_ms(h, 0, C.byref(ms)); best = min(best, ms.value)
            per.append(f"{N}:{'mt' if mode == abi.RL_MODE_MINTIME else 'mc'}:{best:.2f}")
        print(f"per-plan kernel ms {n:10s} " + " ".join(per), flush=True)
outs = {}
for n in libs:
    for i, (lib, h, N, mode) in enumerate(plans[n]):
        o = abi.Outputs.alloc(B, N, 14, mode == abi.RL_MODE_MINTIME); c = o.as_c()
        lib.rl_plan_fetch(h, C.byref(c) if mode == abi.RL_MODE_MINCURV else None,
                          C.byref(c) if mode == abi.RL_MODE_MINTIME else None)
        outs[(i, n)] = o
base = next(iter(libs))
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}")
for n in libs:
    same = all(np.array_equal(outs[(i, n)].x, outs[(i, base)].x) and np.array_equal(outs[(i, n)].evals, outs[(i, base)].evals)
               for i in range(len(plans[n])))
    print(f"C4 (14 single-mode plans on 14 streams) {n:10s} wall ms: median {np.median(res[n][1:]):8.2f} "
          f"min {min(res[n][1:]):8.2f}  bitexact_vs_{base}: {same}", flush=True)
