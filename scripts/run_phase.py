"""Phase isolation by configuration (no code change): C2 (cmap1 N=2000, 1024 seeds) and C5
(oval N=10000) min-curv with max_inner_iters = 0, i.e. per outer iteration only normals,
corridor, lin-geom, one evaluation and the update run.  Kernel ms here vs the full run
gives the PGD loop's share; `python scripts/run_phase.py C2|C5` is also the command
profiled by `PMC_CMD=... scripts/pmc.sh` for a corridor-dominated PMC picture."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O   # fixture loader only
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline
which = sys.argv[1] if len(sys.argv) > 1 else "C2"
name = {"C2": "cmap1_n2000", "C5": "oval_n10000"}[which]
case = O.load_case(name); prob = O.case_problem(case)
B = 1024
for inner in (int(os.environ.get("INNER", "0")), None):
    cfg = O.case_cfg(case)
    if inner is not None:
        cfg.max_inner_iters = inner
    plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B, modes=abi.RL_MODE_MINCURV)
    ms = []
    for _ in range(3):
        plan.run()
        ms.append(plan.kernel_ms(1))
    mc, _ = plan.fetch()
    print(f"{which} max_inner_iters={cfg.max_inner_iters}: kernel {np.median(ms):.3f} ms, evals/outer {mc.evals.mean():.2f}",
          flush=True)
    plan.close()
    if "--only" in sys.argv:
        break
