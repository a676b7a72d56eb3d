"""A/B of the B=1 (drop-in) kernel latency: variant builds of librl (scripts/build_variants.py)
and the throughput shapes (RL_LAT_SHAPES=0) in ONE process, interleaved rounds; plan path,
kernel ms from the plan's HIP events; each variant checked bit for bit against the base.
usage: python scripts/ab_lat.py [rounds]"""
import ctypes as C, glob, json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

libs = {"base": abi.load_library()}
for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so"))):
    n = os.path.basename(p)[6:-3]
    if not (n in ("stamps", "count") or n.startswith("probe")):
        libs[n] = abi.load_library(p)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
CASES = ["track_training_map", "track_competition_map1", "track_competition_map_testday3", "cmap1_n2000"]
if os.environ.get("AB_LAT_CASES"):
    CASES = os.environ["AB_LAT_CASES"].split(",")
res = {}
for cname in CASES:
    case = O.load_case(cname); prob = O.case_problem(case); cfg = O.case_cfg(case)
    for mode, idx in ((1, 1), (2, 2)):
        runs = {}
        for n, lib in libs.items():
            for thr in ((False, True) if n == "base" else (False,)):
                os.environ["RL_LAT_SHAPES"] = "0" if thr else "1"
                h = C.c_void_p(); p = prob.as_c(); arr, nc = abi.cfg_array(cfg)
                assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, nc, None, 1, mode) == 0
                runs[n + ("_thr" if thr else "")] = (lib, h, thr)
        outs, times = {}, {k: [] for k in runs}
        for r in range(rounds + 1):
            for k, (lib, h, thr) in runs.items():
                os.environ["RL_LAT_SHAPES"] = "0" if thr else "1"
                assert lib.rl_plan_run(h, None) == 0
                ms = C.c_float(); assert lib.rl_plan_kernel_ms(h, idx, C.byref(ms)) == 0
                if r: times[k].append(ms.value)
                if r == 0:
                    o = abi.Outputs.alloc(1, prob.N, 14, mode == 2); c = o.as_c()
                    assert lib.rl_plan_fetch(h, C.byref(c) if mode == 1 else None, C.byref(c) if mode == 2 else None) == 0
                    outs[k] = o
        ref = outs["base_thr"]
        for k in runs:
            same = all(np.array_equal(getattr(outs[k], f), getattr(ref, f)) for f in ("x", "y", "alpha_last", "evals"))
            res.setdefault(k, {})[f"{cname[-12:]}_m{mode}"] = (round(float(np.median(times[k])), 3), same)
            runs[k][0].rl_plan_destroy(runs[k][1])
os.environ.pop("RL_LAT_SHAPES", None)
for k, v in res.items():
    print(k, json.dumps(v), flush=True)
