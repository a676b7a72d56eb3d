#!/usr/bin/env python3
"""A/B of rl_optimize's overlapped download (C2's call: competition_map1, N=2000, B=1024,
min-curv, fresh numpy outputs per call as bench.py's c2_pcie_inclusive leg does): the
overlapped path and RL_OVERLAP_DOWNLOAD=0 (one download after the kernel), interleaved.
Prints one JSON line per variant: call / kernel / ABI medians and the groups signalled."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "cmap1_n2000"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    mt = len(sys.argv) > 4 and sys.argv[4] == "both"
    lib = abi.load_library(os.environ.get("PCIE_LIB", abi.LIB_PATH))
    raceline._lib = lambda: lib          # (a variant build, e.g. the RL_OVL_TRACE one)
    c = O.load_case(case)
    prob, cfg = O.case_problem(c), O.case_cfg(c)
    MO = int(cfg.max_outer_iters)
    seeds = np.arange(B, dtype=np.uint64)
    res = {"1": [], "0": []}
    # PCIE_REUSE=1: every call writes into the same output arrays (optimize_batch(out=...))
    keep = raceline.optimize_batch(prob, cfg, seeds, B, mintime=mt) if os.environ.get("PCIE_REUSE") == "1" else None
    for k in ("1", "0"):
        os.environ["RL_OVERLAP_DOWNLOAD"] = k
        raceline.optimize_batch(prob, cfg, seeds, B, mintime=mt, out=keep)         # warm-up
    for _ in range(reps):
        for k in ("1", "0"):
            os.environ["RL_OVERLAP_DOWNLOAD"] = k
            t0 = time.perf_counter()
            out = raceline.optimize_batch(prob, cfg, seeds, B, mintime=mt, out=keep)
            w = (time.perf_counter() - t0) * 1e3
            del out
            run, kmc, call = C.c_float(), C.c_float(), C.c_float()
            lib.rl_last_call_times(C.byref(run), C.byref(kmc), None, C.byref(call))
            g, s = C.c_int32(), C.c_int32()
            lib.rl_last_call_download(C.byref(g), C.byref(s))
            res[k].append((w, run.value, kmc.value, call.value, g.value, s.value))
    for k, v in res.items():
        a = np.array(v)
        med = lambda i: round(float(np.median(a[:, i])), 3)   # noqa: E731
        print(json.dumps({"overlap": k == "1", "reused_outputs": keep is not None, "case": case, "B": B,
                          "modes": "both" if mt else "mincurv",
                          "call_ms": med(0), "run_ms": med(1), "kernel_ms": med(2), "abi_ms": med(3),
                          "outer_iters_per_s": round(B * MO / (np.median(a[:, 0]) * 1e-3), 1),
                          "groups": int(a[0, 4]), "signalled_min": int(a[:, 5].min()),
                          "call_ms_all": [round(x, 2) for x in a[:, 0]]}), flush=True)


if __name__ == "__main__":
    main()
