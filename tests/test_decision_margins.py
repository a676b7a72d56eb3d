"""Decision-margin certificate for the accept/stop tests of the PGD loop (CPU, oracle).

The kernels sum J and the Armijo decrease over the same per-sample terms as the reference
(the α iterates are bit-exact, tests/test_gpu_parity.py) but in another order (per lane,
then a butterfly, with fma).  Any two summations of the same n terms differ by at most
2*gamma(n+3)*sum|terms|, so a decision whose margin exceeds that bound comes out the same
for every summation order.  The oracle (oracle/raceline_oracle.c, oracle_margin_*) records
each Armijo test (ref:733 / 1009) and stop test (ref:739 / 1022) of a run with its
margin/bound ratio; this test asserts that no decision of the golden cases lies within the
bound, i.e. the kernels' evals/accepts counters equal the reference's by construction on
these inputs, not only by observation.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O

CASES = ["cmap1_n2000", "oval_n10000", "sweep_hi", "sweep_invv", "sweep_lo", "sweep_mid", "sweep_nototal",
         "track_competition_map1", "track_competition_map2", "track_competition_map3",
         "track_competition_map_testday1", "track_competition_map_testday2", "track_competition_map_testday3",
         "track_training_map", "training_open"]


def margins(prob, cfg, seeds, modes):
    lib = O.oracle()
    lib.oracle_margin_reset()
    O.run_oracle(prob, [cfg], seeds=np.asarray(seeds, dtype=np.uint64), B=len(seeds), modes=modes)
    r, n, b = C.c_double(), C.c_int64(), C.c_int64()
    lib.oracle_margin_get(C.byref(r), C.byref(n), C.byref(b))
    return r.value, n.value, b.value


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode", ["mincurv", "mintime"])
def test_no_decision_within_summation_bound(name, mode):
    case = O.load_case(name)
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    seeds = [0, 1, 7] if prob.N <= 4096 else [1]
    modes = (True, False) if mode == "mincurv" else (False, True)
    ratio, n, below = margins(prob, cfg, seeds, modes)
    assert n > 0
    # measured minimum over these cases: 4.6e5 (testday2 min-curv); 1e3 leaves room
    assert below == 0 and ratio > 1e3, (name, mode, ratio, n, below)


def test_margin_report_counts_every_decision():
    # one instance of C2: evals per outer iteration = Armijo tests + 1, accepts = stop tests run
    case = O.load_case("cmap1_n2000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    lib = O.oracle()
    lib.oracle_margin_reset()
    mc, _ = O.run_oracle(prob, [cfg], seeds=np.array([0], dtype=np.uint64), B=1, modes=(True, False))
    r, n, b = C.c_double(), C.c_int64(), C.c_int64()
    lib.oracle_margin_get(C.byref(r), C.byref(n), C.byref(b))
    armijo = int((mc.evals - 1).sum())
    assert armijo <= n.value <= armijo + int(mc.accepts.sum())
