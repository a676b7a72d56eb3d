"""Phase shares of the C2-shaped kernel, closed vs open track (RL_STAMPS diagnostic build;
shares and per-block cycles only, a stamped build's absolute time is not the real kernel's)."""
import ctypes as C, os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import bench
from practice_path_planning_for_formula_student_driverless_amd import abi
lib = abi.load_library(os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd/_lib/variants/librl_stamps.so"))
names = ["setup", "corridor tail (combine, LDS, seed)", "mt:κ/vpass/γ", "lin-geom", "PGD loop", "update", "final",
         "normals + corridor loads", "corridor: inner-ring rays", "corridor: outer-ring rays", "corridor: fallback search",
         "-", "-", "-", "-", "-"]
_, closed_prob, cfg = bench.load_problem("cmap1_n2000")
open_prob, _ = bench.open_problem()
B = 1024
for nm, prob in (("closed", closed_prob), ("open", open_prob)):
    for modes in (1, 2):
        h = C.c_void_p(); p = prob.as_c(); arr, n = abi.cfg_array(cfg)
        seeds = np.arange(B, dtype=np.uint64)
        assert lib.rl_plan_create(C.byref(h), 0, C.byref(p), arr, n, abi.u64ptr(seeds), B, modes) == 0
        assert lib.rl_plan_run(h, None) == 0
        ms = C.c_float(); lib.rl_plan_kernel_ms(h, modes, C.byref(ms))
        st = np.zeros((B, 16), dtype=np.uint64)
        assert lib.rl_debug_stamps(st.ctypes.data_as(C.c_void_p), B) == 0
        tot = st.sum(0).astype(float)
        print(f"{nm} mode={modes} B={B} kernel {ms.value:.2f} ms; per-block cycles {tot.sum()/B:.3e}")
        for i, pn in enumerate(names):
            if tot[i] > 0: print(f"   {pn:36s} {100*tot[i]/tot.sum():5.1f}%  {tot[i]/B:.3e} cyc/block")
        lib.rl_plan_destroy(h)
