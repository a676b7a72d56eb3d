"""Offline simulation (CPU, numpy): a uniform-grid ray walk with empty-space jumps for the corridor rays."""
import sys, math, numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests')); sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_lib as O
from corridor_sim_blocks import rayhits, mindist, normals

def build(rings, cs):
    allp = np.concatenate([np.concatenate([s[:, :2], s[:, 2:]]) for s in rings])
    lo = allp.min(0) - cs * 0.5; hi = allp.max(0) + cs * 0.5
    nx, ny = int(math.ceil((hi[0]-lo[0])/cs)), int(math.ceil((hi[1]-lo[1])/cs))
    cnt = np.zeros((nx, ny), int)
    for r, s in enumerate(rings):
        for q in s:
            x0, x1 = sorted((q[0], q[2])); y0, y1 = sorted((q[1], q[3]))
            i0, i1 = int((x0-lo[0])//cs), int((x1-lo[0])//cs); j0, j1 = int((y0-lo[1])//cs), int((y1-lo[1])//cs)
            cnt[i0:i1+1, j0:j1+1] += 1
    # chebyshev distance to nearest non-empty cell
    occ = cnt > 0
    dist = np.full((nx, ny), 10**9)
    idx = np.argwhere(occ)
    I, J = np.meshgrid(np.arange(nx), np.arange(ny), indexing='ij')
    for (a, b) in idx:
        dist = np.minimum(dist, np.maximum(abs(I-a), abs(J-b)))
    return lo, cs, nx, ny, cnt, dist

def walk(P, d, tstop, G):
    lo, cs, nx, ny, cnt, dist = G
    x, y = P; steps = 0; tests = 0; t = 0.0
    while True:
        i, j = int((x + d[0]*t - lo[0]) // cs), int((y + d[1]*t - lo[1]) // cs)
        if i < 0 or j < 0 or i >= nx or j >= ny: break
        steps += 1
        k = dist[i, j]
        # box of empty cells [i-k+1, i+k-1] (k>=1), or the cell itself (k=0)
        h = max(k - 1, 0)
        bx0, bx1 = (i - h) * cs + lo[0], (i + h + 1) * cs + lo[0]
        by0, by1 = (j - h) * cs + lo[1], (j + h + 1) * cs + lo[1]
        if k == 0: tests += cnt[i, j]
        tx = ((bx1 if d[0] > 0 else bx0) - x) / d[0] if d[0] != 0 else math.inf
        ty = ((by1 if d[1] > 0 else by0) - y) / d[1] if d[1] != 0 else math.inf
        te = min(tx, ty)
        if te > tstop: break
        t = te + 1e-9
    return steps, tests

def sim(name, P, rings, cs):
    G = build(rings, cs)
    n = normals(P)
    hi_, ho = rayhits(P, n, rings[0]), rayhits(P, n, rings[1])
    N = len(P); st = np.zeros(N); te = np.zeros(N)
    for i in range(N):
        for sgn, bi, bo in ((1, hi_[0][i], ho[0][i]), (-1, hi_[1][i], ho[1][i])):
            s, t = walk(P[i], sgn * n[i], max(bi, bo), G)
            st[i] += s; te[i] += t
    W = 64
    mx = [st[w:w+W].max() for w in range(0, N, W)]
    mt = [te[w:w+W].max() for w in range(0, N, W)]
    print(f"{name} cs={cs}: grid {G[2]}x{G[3]}, occupied {np.mean(G[4]>0):.2f}, mean items/occ cell {G[4][G[4]>0].mean():.1f}; "
          f"steps/sample mean {st.mean():.1f} wave-max mean {np.mean(mx):.1f}; seg tests/sample mean {te.mean():.1f} wave-max {np.mean(mt):.1f}")

for nm in ("cmap1_n2000", "oval_n10000"):
    case = O.load_case(nm); prob = O.case_problem(case)
    rings = [prob.inner_seg, prob.outer_seg]
    P = np.stack([case["mc_x"], case["mc_y"]], 1)
    for cs in (2.0, 4.0):
        sim(nm + " optimised", P, rings, cs)
    if nm == "oval_n10000":
        rng = np.random.default_rng(1)
        Pj = prob.center + normals(prob.center) * (0.25 * rng.uniform(-1, 1, len(P)))[:, None]
        for cs in (2.0, 4.0):
            sim(nm + " jittered", Pj[:3000], rings, cs)
