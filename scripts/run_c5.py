"""C5 workload alone (oval N=10000, 1024 seeds, min-curv, streaming kernel), two launches;
the command profiled by `PMC_CMD="python scripts/run_c5.py" scripts/pmc.sh <outdir>`."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O   # fixture loader only
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline
case = O.load_case("oval_n10000"); prob = O.case_problem(case); cfg = O.case_cfg(case)
B = 1024
plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B, modes=abi.RL_MODE_MINCURV)
for _ in range(2):
    plan.run()
    print(f"C5 kernel {plan.kernel_ms(1):.2f} ms", flush=True)
mc, _ = plan.fetch()
print(f"evals/outer {mc.evals.mean():.2f}")
plan.close()
