"""C5 streaming-kernel phase shares with the v-pass split out (RL_STAMPS build,
_lib/variants/librl_stamps.so): the v-pass split into its
phases (register-resident v-pass: 15 load + v_kappa, 12 forward, 13 backward relaxations, 14
wraps and sweep checks, 11 the stores), slot 2 = gamma^2.  Shares only: a stamped build's time is not the real kernel's.
usage: stamps_c5v.py [B] [mode] [seed0]"""
import ctypes as C, os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
lib = abi.load_library(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_stamps.so"))
names = {0: "setup", 1: "corridor tail (write, seed)", 15: "v-pass: load kappa, v_kappa", 12: "v-pass: forward relaxations",
         13: "v-pass: backward relaxations", 14: "v-pass: wraps, sweep checks", 11: "v-pass: store", 2: "mt: gamma^2 (+ lap)", 3: "lin-geom",
         4: "PGD loop", 5: "update", 6: "normals", 7: "corridor loads", 8: "corridor: inner-ring rays",
         9: "corridor: outer-ring rays", 10: "corridor: fallback search"}
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
MODE = int(sys.argv[2]) if len(sys.argv) > 2 else 2
S0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
case = O.load_case("oval_n10000"); prob = O.case_problem(case); cfg = O.case_cfg(case)
h = C.c_void_p(); p = prob.as_c(); arr, n = abi.cfg_array(cfg)
seeds = np.arange(S0, S0 + B, dtype=np.uint64)
assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, n, abi.u64ptr(seeds), B, MODE) == 0
for _ in range(2):
    assert lib.rl_plan_run(h, None) == 0
ms = C.c_float(); lib.rl_plan_kernel_ms(h, MODE, C.byref(ms))
st = np.zeros((B, 16), dtype=np.uint64)
assert lib.rl_debug_stamps_stream(st.ctypes.data_as(C.c_void_p), B) == 0
tot = st.sum(0).astype(float)
cyc = sum(tot[i] for i in names)
print(f"C5 mode={MODE} B={B} seeds {S0}.. kernel {ms.value:.2f} ms; per-block cycles {cyc/B:.3e}")
for i, nm in names.items():
    if tot[i] > 0: print(f"   {nm:30s} {100*tot[i]/cyc:5.1f}%  {tot[i]/B:.3e} cyc/block")
lib.rl_plan_destroy(h)
