"""Offline simulation (CPU, numpy): corridor ray-block visits of the register/streaming
kernels' scan (blocks of 16 entries, 64 lanes x CK samples per wave, +n and -n rays of a
sample sharing one scan) with and without along-ray block culling.

  line     the kernels' rule: a block is visited when some lane's ray LINE passes within
           the block circle (side test)
  along    a block is also skipped for a sample when, along +n, its circle lies beyond the
           sample's best hit found so far (or behind the sample), and likewise along -n --
           only when every segment of the block makes an angle of more than `guard` with
           the ray (direction cone), where the computed t is well conditioned
Scan orders for `along`: natural entry order, or starting at the word (32 entries) whose
block circle is nearest to the wave's first sample.  `ideal` uses the final best hits
from the start (a lower bound for any order).
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import oracle_lib as O  # noqa: E402

BLK = 16


def entry_stream(seg):
    """Chains of consecutive segments -> entries; entry v carries the segment ending at v."""
    ends, segs = [], []
    for e in range(len(seg)):
        if e == 0 or not (seg[e, 0] == seg[e - 1, 2] and seg[e, 1] == seg[e - 1, 3]):
            ends.append(False); segs.append(None)
        ends.append(True); segs.append(seg[e])
    while len(ends) % 32:
        ends.append(False); segs.append(None)
    return ends, segs


def blocks(seg):
    ends, segs = entry_stream(seg)
    M = len(ends)
    out = []
    for b in range(M // BLK):
        ss = [segs[v] for v in range(b * BLK, (b + 1) * BLK) if ends[v]]
        if not ss:
            out.append(None); continue
        ss = np.array(ss)
        pts = np.concatenate([ss[:, :2], ss[:, 2:]])
        lo, hi = pts.min(0), pts.max(0); c = (lo + hi) / 2
        R = np.max(np.hypot(*(pts - c).T)) * (1 + 1e-9) + 1e-12
        ang = np.mod(np.arctan2(ss[:, 3] - ss[:, 1], ss[:, 2] - ss[:, 0]), np.pi)
        # smallest arc (mod pi) covering every direction: centre and half width
        a = np.sort(ang)
        gaps = np.diff(np.concatenate([a, a[:1] + np.pi]))
        j = int(np.argmax(gaps))
        start = a[(j + 1) % len(a)]
        width = np.pi - gaps[j]
        out.append((c, R, np.mod(start + width / 2, np.pi), width / 2, ss))
    return out


def rayhits(P, n, seg):
    x0, y0 = seg[:, 0], seg[:, 1]; vx, vy = seg[:, 2] - x0, seg[:, 3] - y0
    ux, uy = n[:, :1], n[:, 1:]
    den = ux * (-vy) + uy * vx
    ax = x0 - P[:, :1]; ay = y0 - P[:, 1:]
    with np.errstate(divide='ignore', invalid='ignore'):
        t = (ax * (-vy) + ay * vx) / den; u = (ux * ay - uy * ax) / den
    ok = (np.abs(den) >= 1e-15) & (u >= -1e-12) & (u <= 1 + 1e-12)
    tp = np.where(ok & (t > 0), t, np.inf)
    tn = np.where(ok & (t < 0), -t, np.inf)
    return tp, tn


def normals(P):
    t = (np.roll(P, -1, 0) - np.roll(P, 1, 0)) * 0.5
    n = np.stack([-t[:, 1], t[:, 0]], 1)
    return n / np.hypot(*n.T)[:, None]


def sim(name, P, rings, guard=1e-3, W=128):
    n = normals(P)
    N = len(P)
    th = np.mod(np.arctan2(n[:, 1], n[:, 0]), np.pi)
    tot = {"line": 0, "along_nat": 0, "along_rot": 0, "ideal": 0}
    nblk = 0
    nw = 0
    for r, seg in enumerate(rings):
        bl = blocks(seg)
        nb = len(bl)
        nblk += nb
        # per-block hits of every sample (to update bests when a block is visited)
        hp = np.full((N, nb), np.inf); hn = np.full((N, nb), np.inf)
        for b, B in enumerate(bl):
            if B is None: continue
            tp, tn = rayhits(P, n, B[4])
            hp[:, b] = tp.min(1); hn[:, b] = tn.min(1)
        fbp, fbn = hp.min(1), hn.min(1)
        for w0 in range(0, N, W):
            sl = slice(w0, min(N, w0 + W))
            if r == 0: nw += 1
            Pw, nw_, thw = P[sl], n[sl], th[sl]
            side_ok, a_lo, a_hi, wellc = [], [], [], []
            for b, B in enumerate(bl):
                if B is None:
                    side_ok.append(np.zeros(len(Pw), bool)); a_lo.append(None); a_hi.append(None); wellc.append(None)
                    continue
                c, R, cen, hw, _ = B
                d = c[None, :] - Pw
                s = d[:, 0] * nw_[:, 1] - d[:, 1] * nw_[:, 0]
                a = d[:, 0] * nw_[:, 0] + d[:, 1] * nw_[:, 1]
                side_ok.append(np.abs(s) <= R * 1.000001)
                a_lo.append(a - R); a_hi.append(a + R)
                dist = np.abs(np.mod(thw - cen + np.pi / 2, np.pi) - np.pi / 2)   # angle to the cone centre
                wellc.append(dist > hw + guard)
            line = [so.any() for so in side_ok]
            tot["line"] += sum(line)

            def run(order, ideal=False):
                bp = fbp[sl].copy() if ideal else np.full(len(Pw), np.inf)
                bn = fbn[sl].copy() if ideal else np.full(len(Pw), np.inf)
                cnt = 0
                for b in order:
                    if bl[b] is None or not line[b]: continue
                    needp = side_ok[b] & ((a_hi[b] > 0) & (a_lo[b] < bp) | ~wellc[b])
                    needn = side_ok[b] & ((a_lo[b] < 0) & (-a_hi[b] < bn) | ~wellc[b])
                    if (needp | needn).any():
                        cnt += 1
                        bp = np.minimum(bp, hp[sl, b]); bn = np.minimum(bn, hn[sl, b])
                return cnt
            tot["along_nat"] += run(range(nb))
            # rotated: start at the word whose block circle is nearest to the wave's first sample
            dists = [np.inf if B is None else max(0.0, np.hypot(*(B[0] - Pw[0])) - B[1]) for B in bl]
            b0 = (int(np.argmin(dists)) // 2) * 2
            tot["along_rot"] += run([(b0 + i) % nb for i in range(nb)])
            tot["ideal"] += run(range(nb), ideal=True)
    print(f"{name}: N={N} blocks(2 rings)={nblk} waves={nw} visited fraction " +
          " ".join(f"{k}={v / (nw * nblk):.3f}" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
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
            Pj = P + normals(P) * alpha[:, None]
            sim(nm + " jittered", Pj, rings)
            sim(nm + " jittered guard 1e-2", Pj, rings, guard=1e-2)
