"""Offline simulation (CPU, numpy): corridor ray-block visitation under line vs half-line culling."""
import sys, numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests')); sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle_lib as O

def blocks_of(seg):
    # entry-stream-like: consecutive segments in chain order, blocks of 8 segments
    nb = (len(seg) + 7) // 8
    C, R = [], []
    for b in range(nb):
        s = seg[8*b:8*b+8]
        pts = np.concatenate([s[:, :2], s[:, 2:]])
        lo, hi = pts.min(0), pts.max(0); c = (lo + hi) / 2
        C.append(c); R.append(np.max(np.hypot(*(pts - c).T)))
    return np.array(C), np.array(R)

def rayhits(P, n, seg):
    # nearest +n and -n hit distances, inf if none (vectorised reference test)
    x0, y0 = seg[:, 0], seg[:, 1]; vx, vy = seg[:, 2] - x0, seg[:, 3] - y0
    ux, uy = n[:, :1], n[:, 1:]
    den = ux * (-vy) + uy * vx
    ax = x0 - P[:, :1]; ay = y0 - P[:, 1:]
    with np.errstate(divide='ignore', invalid='ignore'):
        t = (ax * (-vy) + ay * vx) / den; u = (ux * ay - uy * ax) / den
    ok = (np.abs(den) >= 1e-15) & (u >= -1e-12) & (u <= 1 + 1e-12)
    bp = np.where(ok & (t > 0), t, np.inf).min(1)
    bn = np.where(ok & (t < 0), -t, np.inf).min(1)
    return bp, bn

def mindist(P, seg):
    x0, y0 = seg[:, 0], seg[:, 1]; vx, vy = seg[:, 2] - x0, seg[:, 3] - y0
    apx = P[:, :1] - x0; apy = P[:, 1:] - y0
    t = np.clip((vx * apx + vy * apy) / np.maximum(1e-30, vx*vx+vy*vy), 0, 1)
    return np.hypot(apx - vx * t, apy - vy * t).min(1)

def normals(P):
    t = (np.roll(P, -1, 0) - np.roll(P, 1, 0)) * 0.5
    n = np.stack([-t[:, 1], t[:, 0]], 1)
    return n / np.hypot(*n.T)[:, None]

def sim(name, P, rings, W=128):
    n = normals(P)
    N = len(P)
    res = {}
    blk = [blocks_of(s) for s in rings]
    hits = [rayhits(P, n, s) for s in rings]
    md = [mindist(P, s) for s in rings]
    tot = {"A": 0, "B": 0, "C": 0}
    nblocks = sum(len(b[0]) for b in blk)
    nw = 0
    for w0 in range(0, N, W):
        sl = slice(w0, min(N, w0 + W)); nw += 1
        for r in range(2):
            C, R = blk[r]
            c = (C[None, :, 0] - P[sl, None, 0]) * n[sl, None, 1] - (C[None, :, 1] - P[sl, None, 1]) * n[sl, None, 0]   # side
            a = (C[None, :, 0] - P[sl, None, 0]) * n[sl, None, 0] + (C[None, :, 1] - P[sl, None, 1]) * n[sl, None, 1]   # along
            near = np.abs(c) <= R[None, :] * 1.000001
            tot["A"] += near.any(0).sum()
            bp, bn = hits[r][0][sl, None], hits[r][1][sl, None]
            o = 1 - r
            needp = near & (a + R > 0) & (a - R < bp)
            needn = near & (a - R < 0) & (-a - R < bn)
            tot["B"] += (needp | needn).any(0).sum()
            # relevance: a miss direction matters only if md_r < other ring's hit in that direction
            relp = ~(np.isinf(bp) & (md[r][sl, None] >= hits[o][0][sl, None]))
            reln = ~(np.isinf(bn) & (md[r][sl, None] >= hits[o][1][sl, None]))
            tot["C"] += ((needp & relp) | (needn & reln)).any(0).sum()
    print(f"{name}: N={N} blocks/ring-pair={nblocks} waves={nw}  visited fraction  A(line)={tot['A']/(nw*nblocks):.3f}  "
          f"B(half-line,bounded)={tot['B']/(nw*nblocks):.3f}  C(+relevance)={tot['C']/(nw*nblocks):.3f}")

if __name__ == '__main__':
    for nm in ("cmap1_n2000", "oval_n10000"):
        case = O.load_case(nm); prob = O.case_problem(case)
        P = prob.center.copy()
        sim(nm + " centre", P, [prob.inner_seg, prob.outer_seg])
        Pm = np.stack([case["mc_x"], case["mc_y"]], 1)
        sim(nm + " optimised", Pm, [prob.inner_seg, prob.outer_seg])
        if nm == "oval_n10000":
            rng = np.random.default_rng(1)
            alpha = 0.25 * rng.uniform(-1, 1, len(P))
            Pj = P + normals(P) * alpha[:, None]
            sim(nm + " jittered", Pj, [prob.inner_seg, prob.outer_seg])
