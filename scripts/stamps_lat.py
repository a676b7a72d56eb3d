"""Phase shares of one-instance (drop-in) runs from the RL_STAMPS diagnostic build: the
latency shape (rl_kernels_lat.hip's stamps) against the throughput shape (RL_LAT_SHAPES=0,
rl_kernels.hip's stamps; (4, 512) lives in rl_kernels_mid.hip).  Shares only: a stamped
build's absolute time is not the real kernel's."""
import ctypes as C, os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi
# usage: python scripts/stamps_lat.py [variant]   (stamps, or stamps_eval for the evaluation's phases)
VAR = sys.argv[1] if len(sys.argv) > 1 else "stamps"
lib = abi.load_library(os.path.join(REPO, f"practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_{VAR}.so"))
names = ["setup", "corridor tail", "mt:κ/vpass/γ", "lin-geom", "PGD loop (rest)", "update", "final",
         "normals + corridor loads", "corridor: inner rays", "corridor: outer rays", "corridor: fallback",
         "pgd: projection", "pgd: stencil+partials", "pgd: wave sum", "pgd: barrier+block sum", "pgd: gradient"]
if VAR == "stamps":     # VSPLIT (min-time, K = 1): slot 11 = wave 0's join wait + collect, 12 = the v-pass wave
    names[11], names[12] = "vsplit: join wait + collect (wave 0)", "vsplit: v-pass wave's v-pass [not in the sum]"
    names[13], names[14], names[15] = ("vsplit: wave 0 scan [in 7-10]", "vsplit: wave 1 scan [not in the sum]",
                                       "vsplit: wave 2 scan [not in the sum]")
for cname in [c for c in os.environ.get("ST_CASES", "track_training_map,track_competition_map_testday3,cmap1_n2000").split(",")]:
    case = O.load_case(cname); prob = O.case_problem(case); cfg = O.case_cfg(case)
    for mode in (1, 2):
        for thr in (False, True):
            os.environ["RL_LAT_SHAPES"] = "0" if thr else "1"
            K, T = abi.kernel_shape(prob.N, 1, mode)
            h = C.c_void_p(); p = prob.as_c(); arr, n = abi.cfg_array(cfg)
            assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, n, None, 1, mode) == 0
            lib.rl_plan_run(h, None)
            assert lib.rl_plan_run(h, None) == 0
            ms = C.c_float(); lib.rl_plan_kernel_ms(h, mode, C.byref(ms))
            st = np.zeros((1, 16), dtype=np.uint64)
            f = (lib.rl_debug_stamps_mid if (K, T) == (4, 512) else
                 lib.rl_debug_stamps_lat if not thr else lib.rl_debug_stamps)
            assert f(st.ctypes.data_as(C.c_void_p), 1) == 0
            o = abi.Outputs.alloc(1, prob.N, int(cfg.max_outer_iters), mode == 2)
            c = o.as_c()
            lib.rl_plan_fetch(h, C.byref(c) if mode == 1 else None, C.byref(c) if mode == 2 else None)
            n_ev = int(np.asarray(o.evals).sum())
            tot = st.sum(0).astype(float)
            w0 = tot.sum() - (tot[12:16].sum() if VAR == "stamps" else 0.0)   # wave 0's own cycles
            print(f"{cname} N={prob.N} mode={mode} shape=({K},{T}) kernel {ms.value:.3f} ms (stamped); "
                  f"wave-0 cycles {w0:.3e}, {n_ev} evaluations ({w0 / max(n_ev, 1):.0f} cycles each, all phases): " +
                  ", ".join(f"{nm} {100 * tot[i] / w0:.1f}%" for i, nm in enumerate(names) if tot[i] > 0), flush=True)
            lib.rl_plan_destroy(h)
os.environ.pop("RL_LAT_SHAPES", None)
