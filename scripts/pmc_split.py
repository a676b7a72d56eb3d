"""Per-evaluation counter cost of the PGD loop: the C2 launch (B=1024, N=2000,
min-curv) run twice under rocprofv3 --pmc, with the default cfg and with
max_inner_iters=0 (one evaluation per outer iteration).  Dispatch 1 = default,
dispatch 2 = no inner iterations; scripts/pmc_split_report.py divides the counter
difference by the difference in evaluations.
usage: rocprofv3 --pmc <counters> --kernel-trace -d DIR -o run --output-format csv -- python scripts/pmc_split.py"""
import json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline

case = O.load_case("cmap1_n2000")
prob, cfg = O.case_problem(case), O.case_cfg(case)
B = 1024
ev = []
for mi in (cfg.max_inner_iters, 0):
    c = abi.RlCfg.from_dict(cfg.to_dict())
    c.max_inner_iters = mi
    plan = raceline.Plan(prob, c, seeds=np.arange(B, dtype=np.uint64), B=B, modes=abi.RL_MODE_MINCURV)
    plan.run()
    mc = plan.fetch()[0]
    ev.append(int(mc.evals.sum()))
    plan.close()
print(json.dumps({"evals": ev, "waves": B * 4}))
