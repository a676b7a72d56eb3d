"""Offline simulation (CPU, numpy): work of the corridor's fallback point-to-ring search
(rl_corridor.h ring_mindist) with the current search radius (walked candidates' endpoints,
then the nearest-midpoint pass) against a radius from the ray hit on the same ring
(the distance to the segment that ray hit bounds the ring minimum from above)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)
import oracle_lib as O  # noqa: E402
from corridor_sim_blocks import normals  # noqa: E402

BLK = 16


def seg_arrays(seg):
    x0, y0 = seg[:, 0], seg[:, 1]
    return x0, y0, seg[:, 2] - x0, seg[:, 3] - y0


def hits_idx(P, n, seg):
    x0, y0, vx, vy = seg_arrays(seg)
    ux, uy = n[:, :1], n[:, 1:]
    den = ux * (-vy) + uy * vx
    ax = x0 - P[:, :1]
    ay = y0 - P[:, 1:]
    with np.errstate(divide='ignore', invalid='ignore'):
        t = (ax * (-vy) + ay * vx) / den
        u = (ux * ay - uy * ax) / den
    ok = (np.abs(den) >= 1e-15) & (u >= -1e-12) & (u <= 1 + 1e-12)
    tp = np.where(ok & (t > 0), t, np.inf)
    tn = np.where(ok & (t < 0), -t, np.inf)
    # crossing candidates (the side filter keeps these): endpoints on both sides of the line
    c0 = ux * (y0 - P[:, 1:]) - uy * (x0 - P[:, :1])
    c1 = ux * (y0 + vy - P[:, 1:]) - uy * (x0 + vx - P[:, :1])
    cross = (c0 * c1) <= 0
    return tp.min(1), tn.min(1), tp.argmin(1), tn.argmin(1), cross


def segdist(P, seg):
    x0, y0, vx, vy = seg_arrays(seg)
    apx = P[:, :1] - x0
    apy = P[:, 1:] - y0
    t = np.clip((vx * apx + vy * apy) / np.maximum(1e-30, vx * vx + vy * vy), 0, 1)
    return np.hypot(apx - vx * t, apy - vy * t)


def sim(name, P, rings, CK=2):
    n = normals(P)
    N = len(P)
    H = [hits_idx(P, n, s) for s in rings]
    D = [segdist(P, s) for s in rings]
    res = {"cur": np.zeros(4), "hit": np.zeros(4)}
    nwaves = 0
    for r in range(2):
        seg = rings[r]
        E = len(seg)
        nb = (E + BLK - 1) // BLK
        mids = (seg[:, :2] + seg[:, 2:]) / 2
        hl = np.hypot(*(seg[:, 2:] - seg[:, :2]).T) / 2
        Cb, Rb = [], []
        for b in range(nb):
            s = seg[BLK * b:BLK * b + BLK]
            pts = np.concatenate([s[:, :2], s[:, 2:]])
            lo, hi = pts.min(0), pts.max(0)
            c = (lo + hi) / 2
            Cb.append(c)
            Rb.append(np.max(np.hypot(*(pts - c).T)))
        Cb, Rb = np.array(Cb), np.array(Rb)
        o = 1 - r
        bp, bn, ip, inn, cross = H[r]
        obp, obn = H[o][0], H[o][1]
        mp, mn = np.isinf(bp), np.isinf(bn)
        need = mp | mn
        tau = np.full(N, -np.inf)
        tau = np.where(mp, np.maximum(tau, np.where(np.isfinite(obp), obp, np.inf)), tau)
        tau = np.where(mn, np.maximum(tau, np.where(np.isfinite(obn), obn, np.inf)), tau)
        # current: endpoints of the crossing candidates
        ep = np.minimum(np.hypot(P[:, :1] - seg[:, 0], P[:, 1:] - seg[:, 1]),
                        np.hypot(P[:, :1] - seg[:, 2], P[:, 1:] - seg[:, 3]))
        ub = np.where(cross, ep, np.inf).min(1)
        rad_cur = np.minimum(ub, tau)
        # hit: the segment hit in the other direction on the same ring
        dh = np.full(N, np.inf)
        hp = ~mp
        dh[hp] = D[r][hp, ip[hp]]
        hn = ~mn
        dh[hn] = np.minimum(dh[hn], D[r][hn, inn[hn]])
        rad_hit = np.minimum(rad_cur, dh)
        for w0 in range(0, N, 64 * CK):
            idx = np.arange(w0, min(N, w0 + 64 * CK))
            if r == 0:
                nwaves += 1
            for key, rad, tight in (("cur", rad_cur, True), ("hit", rad_hit, False)):
                lanes = [idx[i:i + CK] for i in range(0, len(idx), CK)]
                Rl, q0, dk = [], [], []
                for ln in lanes:
                    q = P[ln[0]]
                    d = np.abs(P[ln] - q).sum(1)
                    nd = need[ln]
                    Rl.append((rad[ln] + d)[nd].max() if nd.any() else -1.0)
                    q0.append(q)
                    dk.append(d)
                Rl = np.array(Rl)
                q0 = np.array(q0)
                if not (Rl >= 0).any():
                    continue
                dist_c = np.hypot(q0[:, None, 0] - Cb[None, :, 0], q0[:, None, 1] - Cb[None, :, 1])
                vis = ((Rl[:, None] >= 0) & (dist_c <= Rl[:, None] + Rb[None, :])).any(0)
                if tight:
                    res[key][0] += vis.sum()           # pass-1 blocks
                    ent = np.concatenate([np.arange(BLK * b, min(E, BLK * b + BLK)) for b in np.nonzero(vis)[0]])
                    m = np.hypot(q0[:, None, 0] - mids[None, ent, 0], q0[:, None, 1] - mids[None, ent, 1]).min(1)
                    R2 = []
                    for li, ln in enumerate(lanes):
                        nd = need[ln]
                        R2.append((np.minimum(rad[ln], m[li] + dk[li]) + dk[li])[nd].max() if nd.any() else -1.0)
                    Rl = np.array(R2)
                    vis = ((Rl[:, None] >= 0) & (dist_c <= Rl[:, None] + Rb[None, :])).any(0)
                res[key][1] += vis.sum()               # pass-2 blocks
                ent = np.concatenate([np.arange(BLK * b, min(E, BLK * b + BLK)) for b in np.nonzero(vis)[0]]) if vis.any() else np.zeros(0, int)
                dm = np.hypot(q0[:, None, 0] - mids[None, ent, 0], q0[:, None, 1] - mids[None, ent, 1])
                cand = (Rl[:, None] >= 0) & (dm <= Rl[:, None] + hl[None, ent])
                res[key][2] += cand.sum(1).max() if len(ent) else 0   # walk iterations (wave max)
                res[key][3] += cand.sum()                             # lane candidates
    for key in res:
        a = res[key] / nwaves
        print(f"{name:28s} {key}: per wave pass-1 blocks {a[0]:6.2f}  pass-2 blocks {a[1]:6.2f}  "
              f"walk iters {a[2]:6.2f}  lane candidates {a[3]:7.1f}")


if __name__ == '__main__':
    for nm in ("cmap1_n2000", "oval_n10000"):
        case = O.load_case(nm)
        prob = O.case_problem(case)
        P = prob.center.copy()
        rings = [prob.inner_seg, prob.outer_seg]
        sim(nm + " centre", P, rings)
        Pm = np.stack([case["mc_x"], case["mc_y"]], 1)
        sim(nm + " optimised", Pm, rings)
        if nm == "oval_n10000":
            rng = np.random.default_rng(1)
            alpha = 0.25 * rng.uniform(-1, 1, len(P))
            sim(nm + " jittered", P + normals(P) * alpha[:, None], rings, CK=1)
