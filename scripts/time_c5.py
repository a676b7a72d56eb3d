import os, sys, time, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline
case = O.load_case("oval_n10000"); prob = O.case_problem(case); cfg = O.case_cfg(case)
for B, modes in ((64, 1), (1024, 1), (256, 2)):
    plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B, modes=modes)
    plan.run(); mc, mt = plan.fetch()
    plan.run(); ms = plan.kernel_ms(modes)
    o = mc or mt
    print(f"C5 N=10000 B={B} mode={modes}: kernel {ms:.1f} ms -> {B*14/(ms/1e3):.0f} outer/s; evals/outer {o.evals.mean():.2f}; accepts {o.accepts.mean():.3f}", flush=True)
    plan.close()
