"""A/B-time variant builds of librl (scripts/build_variants.py) in ONE process,
interleaved rounds (guide §5.4 rule 24).  Prints per-variant kernel ms (median, min)
for C2 (N=2000, B=1024, min-curv) and C3-mt (N=2000 vp20, B=256, min-time), and
checks that each variant reproduces the default build bit for bit."""
import ctypes as C, glob, os, sys, time, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi

libs = {}
for p in sorted(glob.glob(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_*.so"))):
    if not (p.endswith("_stamps.so") or p.endswith("_count.so")):
        libs[os.path.basename(p)[6:-3]] = abi.load_library(p)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5

def make_plan(lib, prob, cfg, B, modes):
    h = C.c_void_p(); p = prob.as_c(); arr, n = abi.cfg_array(cfg)
    seeds = np.arange(B, dtype=np.uint64)
    rc = lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, n, abi.u64ptr(seeds), B, modes)
    assert rc == 0, lib.rl_last_error()
    return h

def run(lib, h, idx):
    assert lib.rl_plan_run(h, None) == 0
    ms = C.c_float(); assert lib.rl_plan_kernel_ms(h, idx, C.byref(ms)) == 0
    return ms.value

def fetch(lib, h, B, N, mo, mt):
    o = abi.Outputs.alloc(B, N, mo, mt); c = o.as_c()
    assert lib.rl_plan_fetch(h, None if mt else C.byref(c), C.byref(c) if mt else None) == 0
    return o

res = {}
CASES = [("C2", "cmap1_n2000", 1024, 1, 1, False), ("C3mt", "cmap1_n2000_vp20", 256, 2, 2, True),
         ("C3big", "cmap1_n2000_vp20", 4096, 2, 2, True), ("C5", "oval_n10000", 1024, 1, 1, False),
         ("C5mt", "oval_n10000", 1024, 2, 2, True), ("C4t3", "track_competition_map_testday3", 512, 3, 0, True)]
sel = os.environ.get("AB_CASES")
CASES += [("O2", "open:cmap1_n2000", 1024, 1, 1, False), ("O2mt", "open:cmap1_n2000", 1024, 2, 2, True),
          # the streaming kernel forced on C2's problem: the accepting regime (E_k 135, 120 accepts)
          ("S2", "cmap1_n2000", 1024, 1, 1, False), ("S2mt", "cmap1_n2000", 1024, 2, 2, True)]
for cname, cfgname, B, modes, idx, mt in [c for c in CASES if not sel or c[0] in sel.split(",")]:
    if cname.startswith("S"):
        os.environ["RL_FORCE_STREAM"] = "1"
    else:
        os.environ.pop("RL_FORCE_STREAM", None)
    if cfgname.startswith("open:"):      # C2's track as an open path (bench.py open_problem)
        import bench
        prob, cfg = bench.open_problem()
    else:
        case = O.load_case(cfgname); prob = O.case_problem(case); cfg = O.case_cfg(case)
    plans = {n: make_plan(l, prob, cfg, B, modes) for n, l in libs.items()}
    outs = {}
    for n, l in libs.items():
        run(l, plans[n], idx); outs[n] = fetch(l, plans[n], B, prob.N, 14, mt)
    ref = outs.get("base", next(iter(outs.values())))
    for n, o in outs.items():
        same = all(np.array_equal(getattr(o, f), getattr(ref, f)) for f in ("x", "y", "alpha_last", "evals"))
        res.setdefault(n, {})[cname + "_bitexact_vs_base"] = bool(same)
    times = {n: [] for n in libs}
    for r in range(rounds):
        for n, l in libs.items():
            times[n].append(run(l, plans[n], idx))
    for n in libs:
        t = np.array(times[n]); res[n][cname + "_ms_med"] = round(float(np.median(t)), 3); res[n][cname + "_ms_min"] = round(float(t.min()), 3)
        libs[n].rl_plan_destroy(plans[n])
for n, r in res.items():
    print(n, json.dumps(r), flush=True)
