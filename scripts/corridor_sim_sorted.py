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

Paths: C5's problem (the N = 10000 oval), seeds 1 and 7.  The kernel's 14 corridor passes
(outers 0..13) see two paths: the centre line (outer 0), then the path the seeded first
outer iteration left, which no later outer moves (its corridor collapses: every trial is
rejected, E_k = 21) -- the CPU oracle run with max_outer_iters = 1 gives it.  Ground truth
for `natural`: the RL_COUNT counters of the GPU kernel per pass (scripts/counts_c5_outer.py,
profiles/r06/corridor_counts_c5_per_pass.log): first pass 0.177 and later passes 0.500 as
logged, i.e. 0.354 and 0.999 once the counters' denominator is corrected (they counted 4
block slots per 32-entry word, the blocks-of-8 figure, against 2 at blocks of 16; fixed in
rl_corridor.h).  The simulation's `natural` reproduces both (0.354 / 0.998).  So the
round-5 reading "the union scan visits 46 % of C5's ray blocks" was wrong: it visits all of
them on the jittered path.

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
    keys = ["natural", "theta", "hough4", "hough9", "hough16", "per_lane"]

    def fractions(P):
        n = normals(P)
        V = visits(P, n, rings)
        th = np.mod(np.arctan2(n[:, 1], n[:, 0]), np.pi)
        out = {"natural": union_fraction(V, np.arange(len(P))), "theta": union_fraction(V, np.argsort(th))}
        for ct in (4, 9, 16):
            out[f"hough{ct}"] = union_fraction(V, hough_order(P, n, ct))
        out["per_lane"] = float(V.mean())
        return out

    centre = fractions(prob.center.copy())
    print(json.dumps({"path": "centre (pass 0)", **{k: round(v, 4) for k, v in centre.items()}}), flush=True)
    later = []
    for seed in (1, 7):
        mc, _ = O.run_oracle(prob, abi_cfg(cfg, 1), seeds=[seed], B=1, modes=(True, False))
        f = fractions(np.stack([mc.x[0], mc.y[0]], 1))
        later.append(f)
        print(json.dumps({"path": f"seed {seed} after outer 0 (passes 1-13)", **{k: round(v, 4) for k, v in f.items()}}),
              flush=True)
    # the kernel's 14 passes: 1 on the centre line, 13 on the jittered path
    mean = {k: (centre[k] + 13 * float(np.mean([f[k] for f in later]))) / 14 for k in keys}
    best = min((k for k in mean if k not in ("natural", "per_lane")), key=lambda k: mean[k])
    saving = 1.0 - mean[best] / mean["natural"]
    print(json.dumps({"pass_weighted_visited_fraction": {k: round(v, 4) for k, v in mean.items()},
                      "counters_natural_corrected": {"first_pass": 0.3544, "later_passes": 0.9992},
                      "best_regrouping": best, "side_test_saving_best": round(saving, 4),
                      "per_lane_bound_saving": round(1.0 - mean["per_lane"] / mean["natural"], 4),
                      "decision": ("build" if saving >= 0.25 else
                                   "do not build: no wave-uniform regrouping reaches 25 % fewer side tests; the "
                                   "per-lane bound (a work list) needs per-lane loads, built in round 5 and slower")}),
          flush=True)


def abi_cfg(cfg, k):
    from practice_path_planning_for_formula_student_driverless_amd import abi

    c = abi.RlCfg.from_dict(cfg.to_dict())
    c.max_outer_iters = k
    return c


if __name__ == "__main__":
    main()
