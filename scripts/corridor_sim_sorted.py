#!/usr/bin/env python3
"""Offline simulation (CPU, numpy) for VERDICT r5 item 5: would regrouping C5's corridor
samples into waves by their ray LINE cut the wave-union scan's work enough to build it?

The streaming kernel scans the corridor per wave: 64 lanes x RL_SCK = 2 samples (128
consecutive samples of a work-queue chunk) share one pass over the rings' blocks of 16
entries; a block is visited when some sample's ray line passes within its circle, and a
visited block costs every lane its side tests (16 entries x 2 samples, packed fp32) and the
wave its uniform loads of the block's entries.  So both the executed side tests and the
per-wave uniform loads are proportional to the visited blocks per wave.

Groupings of the same samples into 128-sample waves:
  natural   consecutive samples (the kernel today)
  theta     sorted by the normal's angle mod pi (parallel lines together)
  hough     sorted into (theta, rho) cells of the line space, rho = n x P: lines that are
            close as lines together (the best a wave-uniform regrouping can do cheaply)
  per_lane  lower bound of any per-sample scheme: each sample's own visited blocks (what a
            per-lane work list would test; it pays per-lane loads instead of uniform ones)

Paths: C5's problem (the N = 10000 oval), seeds 1 and 7, the path P entering outer k = 1..13
(the CPU oracle run with max_outer_iters = k: its x, y are the path after k outers; the
corridor of outer k uses its normals).  Ground truth for `natural`: the RL_COUNT counters of
the GPU kernel (profiles/r05/corridor_counts_c5_c2.log: 0.108 / 0.236 = 0.458 of ray blocks).

Decision rule: build only if a grouping predicts >= 25 % fewer executed side
tests AND fewer per-wave uniform loads than `natural` (the regrouping itself -- a sort of
10 000 keys per instance per outer and a permuted write-back -- not even charged here).
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import oracle_lib as O  # noqa: E402
from corridor_sim_alongray import blocks, normals  # noqa: E402

W = 128          # samples per wave (64 lanes x RL_SCK)


def line_hits_block(P, n, c, R):
    """[N] bool: the sample's ray line passes within the block circle (the kernel's rule)."""
    d = c[None, :] - P
    s = d[:, 0] * n[:, 1] - d[:, 1] * n[:, 0]
    return np.abs(s) <= R * 1.000001


def visits(P, n, rings):
    """[N, nblocks] bool: per-sample visited blocks of both rings."""
    cols = []
    for seg in rings:
        for B in blocks(seg):
            cols.append(np.zeros(len(P), bool) if B is None else line_hits_block(P, n, B[0], B[1]))
    return np.stack(cols, 1)


def union_fraction(V, order):
    Vo = V[order]
    tot = 0
    for w0 in range(0, len(Vo), W):
        tot += Vo[w0:w0 + W].any(0).sum()
    nw = (len(Vo) + W - 1) // W
    return tot / (nw * V.shape[1])


def hough_order(P, n, cells_theta):
    th = np.mod(np.arctan2(n[:, 1], n[:, 0]), np.pi)
    rho = P[:, 0] * n[:, 1] - P[:, 1] * n[:, 0]
    tb = np.minimum((th / np.pi * cells_theta).astype(int), cells_theta - 1)
    # within each theta band, order by rho (bands alternate direction: a snake keeps the
    # band edges' lines together)
    key = np.where(tb % 2 == 0, rho, -rho)
    return np.lexsort((key, tb))


def main():
    case = O.load_case("oval_n10000")
    prob, cfg = O.case_problem(case), O.case_cfg(case)
    rings = [prob.inner_seg, prob.outer_seg]
    res = {"natural": [], "theta": [], "hough4": [], "hough9": [], "hough16": [], "per_lane": []}
    for seed in (1, 7):
        for k in range(1, 14, 3):
            c = abi_cfg(cfg, k)
            mc, _ = O.run_oracle(prob, c, seeds=[seed], B=1, modes=(True, False))
            P = np.stack([mc.x[0], mc.y[0]], 1)
            n = normals(P)
            V = visits(P, n, rings)
            N = len(P)
            res["natural"].append(union_fraction(V, np.arange(N)))
            th = np.mod(np.arctan2(n[:, 1], n[:, 0]), np.pi)
            res["theta"].append(union_fraction(V, np.argsort(th)))
            for ct in (4, 9, 16):
                res[f"hough{ct}"].append(union_fraction(V, hough_order(P, n, ct)))
            res["per_lane"].append(V.mean())
            print(json.dumps({"seed": seed, "outer": k, **{key: round(v[-1], 4) for key, v in res.items()}}), flush=True)
    mean = {k: float(np.mean(v)) for k, v in res.items()}
    best = min((k for k in mean if k not in ("natural", "per_lane")), key=lambda k: mean[k])
    saving = 1.0 - mean[best] / mean["natural"]
    print(json.dumps({"mean_visited_fraction": {k: round(v, 4) for k, v in mean.items()},
                      "counters_natural": 0.458, "best_regrouping": best,
                      "side_test_saving_best": round(saving, 4),
                      "per_lane_bound_saving": round(1.0 - mean["per_lane"] / mean["natural"], 4),
                      "decision": "build" if saving >= 0.25 else "do not build (< 25 % fewer side tests)"}),
          flush=True)


def abi_cfg(cfg, k):
    from practice_path_planning_for_formula_student_driverless_amd import abi

    c = abi.RlCfg.from_dict(cfg.to_dict())
    c.max_outer_iters = k
    return c


if __name__ == "__main__":
    main()
