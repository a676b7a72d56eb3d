#!/usr/bin/env python3
"""Second drop-in probe (round 6): which host activity before an rl_optimize call makes its
C2 kernel slower?  Every case calls rl_optimize into the SAME preallocated host arrays and
does something else between calls:
  none          nothing
  churn         allocate a fresh 98 MB numpy array, touch every page, free it (mmap, faults, munmap)
  touch_keep    the same, but the array stays alive until the end (faults, no munmap)
  map_unmap     allocate 98 MB and free it untouched (mmap + munmap, no faults)
  sleep         sleep 2 ms (the GPU idle gap alone)
Kernel ms = the optimiser's own HIP events; run it under rocprofv3 --kernel-trace to compare
with the dispatch's own begin/end timestamps."""
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
from practice_path_planning_for_formula_student_driverless_amd import abi  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = abi.load_library()
    case = O.load_case("cmap1_n2000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    B, N, MO = 1024, prob.N, int(cfg.max_outer_iters)
    seeds = np.arange(B, dtype=np.uint64)
    outs = abi.Outputs.alloc(B, N, MO, False)
    oc = outs.as_c()
    p = prob.as_c()
    arr, n = abi.cfg_array(cfg)
    sd = abi.u64ptr(seeds)
    keep = []
    nbytes = B * N * 6 * 8

    def churn():
        a = np.empty(nbytes, dtype=np.uint8)
        a[::4096] = 1
        del a

    def touch_keep():
        a = np.empty(nbytes, dtype=np.uint8)
        a[::4096] = 1
        keep.append(a)

    def map_unmap():
        a = np.empty(nbytes, dtype=np.uint8)
        del a

    cases = {"none": lambda: None, "churn": churn, "touch_keep": touch_keep, "map_unmap": map_unmap,
             "sleep": lambda: time.sleep(0.002)}
    res = {k: [] for k in cases}
    for _ in range(2):
        assert lib.rl_optimize(C.byref(p), arr, n, sd, B, C.byref(oc), None) == 0
    for r in range(rounds):
        for k, f in cases.items():
            f()
            assert lib.rl_optimize(C.byref(p), arr, n, sd, B, C.byref(oc), None) == 0
            run, kmc, call = C.c_float(), C.c_float(), C.c_float()
            lib.rl_last_call_times(C.byref(run), C.byref(kmc), None, C.byref(call))
            res[k].append((kmc.value, call.value))
        if len(keep) > 2:
            keep.clear()
    print(json.dumps({k: {"kernel_ms": round(float(np.median([a for a, _ in v])), 3),
                          "call_ms": round(float(np.median([b for _, b in v])), 3)} for k, v in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
