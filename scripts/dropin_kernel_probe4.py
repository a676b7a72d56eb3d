#!/usr/bin/env python3
"""Fourth drop-in probe (round 6): which part of a fresh-output call pattern slows the next
C2 kernel -- the caller's page faults or its unmaps?  Kernel ms (own HIP events), C2 call
(B=1024, min-curv), interleaved rounds, two calls per case (the second reported):
  reuse          the same output arrays every call
  fresh_keep     fresh arrays every call, all kept alive (faults, no unmap)
  fresh_free     fresh arrays every call, freed after it (faults and unmaps: the bench leg)
  reuse_dontneed the same arrays, their pages dropped (MADV_DONTNEED) before each call
                 (zap + refault, no unmap)"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = abi.load_library()
    libc = C.CDLL("libc.so.6")
    libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    case = O.load_case("cmap1_n2000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    B = 1024
    seeds = np.arange(B, dtype=np.uint64)
    keep = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
    alive = []

    def kmc():
        run, k, call = C.c_float(), C.c_float(), C.c_float()
        lib.rl_last_call_times(C.byref(run), C.byref(k), None, C.byref(call))
        return k.value

    def reuse():
        raceline.optimize_batch(prob, cfg, seeds, B, mintime=False, out=keep)
        return kmc()

    def fresh_keep():
        alive.append(raceline.optimize_batch(prob, cfg, seeds, B, mintime=False))
        return kmc()

    def fresh_free():
        o = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
        del o
        return kmc()

    def reuse_dontneed():
        for f in abi.OUT_F64:
            a = getattr(keep[0], f)
            base = (a.ctypes.data + 4095) & ~4095
            end = (a.ctypes.data + a.nbytes) & ~4095
            if end > base:
                libc.madvise(C.c_void_p(base), C.c_size_t(end - base), 4)      # MADV_DONTNEED
        return reuse()

    cases = {"reuse": reuse, "fresh_keep": fresh_keep, "fresh_free": fresh_free, "reuse_dontneed": reuse_dontneed}
    res = {k: [] for k in cases}
    for f in cases.values():
        f()
    for _ in range(rounds):
        for k, f in cases.items():
            f()
            res[k].append(f())
    print(json.dumps({k: {"median": round(float(np.median(v)), 3), "min": round(float(np.min(v)), 3),
                          "max": round(float(np.max(v)), 3)} for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
