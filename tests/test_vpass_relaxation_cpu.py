"""CPU model of the kernels' chunked v-pass relaxation: the forward pass
of velocity_profile_forward_backward (ref:829-833, v[i+1] = min(v[i+1], f(v[i], k[i]))) evaluated
as chunks that pass their outgoing value right, round by round, with the early stop (a chunk
re-evaluated with a new incoming value stops at the first value that repeats bit for bit) and a
warm start (round 0 takes an arbitrary guess as incoming value).  Whatever the guess -- exact,
too low, too high, +inf -- the fixed point equals the serial pass bit for bit.  Python floats
are IEEE doubles, so this checks the algorithm, not the kernels (the GPU tests do that)."""
import math

import numpy as np
import pytest


def vstep(v, k, h=0.17):
    """ax_max_at (ref:797-824) with the default cfg, then the forward step (ref:830-832)."""
    a_tot, m, kfd, fr, pmax = 11.4777, 255.0, 0.5 * 1.225 * 0.30 * 1.0, 255.0 * 9.81 * 0.015, 80000.0
    alat = v * v * abs(k)
    a_res = math.sqrt(max(0.0, a_tot * a_tot - alat * alat))
    a_pow = (pmax / (m * v) - (kfd * v * v + fr) / m) if v > 1e-6 else 1e9
    a = max(0.0, min(a_res, 8.0, a_pow))
    return math.sqrt(max(0.0, v * v + 2.0 * a * h))


def serial(cap, kap):
    v = list(cap)
    for i in range(len(v) - 1):
        v[i + 1] = min(v[i + 1], vstep(v[i], kap[i]))
    return v


def relaxed(cap, kap, C, guesses):
    """Chunks of C samples; chunk t gets chunk t-1's outgoing value (guess in round 0)."""
    n = len(cap)
    nch = (n + C - 1) // C
    v = list(cap)
    out = [math.inf] * nch
    in_prev = [None] * nch
    rnd = 0
    while True:
        pub = list(out)                      # the values published in the previous round
        changed = False
        for t in range(nch):
            r0, r1 = t * C, min(n, t * C + C)
            inc = math.inf if t == 0 else (guesses[t] if rnd == 0 else pub[t - 1])
            if inc == in_prev[t]:
                continue
            in_prev[t] = inc
            cur = min(cap[r0], inc)
            go = rnd == 0 or cur != v[r0]
            v[r0] = cur
            for i in range(r0, r1 - 1):
                if not go:
                    break
                nv = min(cap[i + 1], vstep(v[i], kap[i]))
                go = rnd == 0 or nv != v[i + 1]
                v[i + 1] = nv
            if go and r1 < n:
                o = vstep(v[r1 - 1], kap[r1 - 1])
                if o != out[t]:
                    changed = True
                out[t] = o
        if rnd > 0 and not changed:
            return v, rnd
        rnd += 1


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("C", [1, 4, 10])
def test_relaxation_equals_serial_for_any_warm_start(seed, C):
    rng = np.random.default_rng(seed)
    n = 300
    kap = np.abs(rng.normal(0.0, 0.05, n)) * (rng.random(n) < 0.3) + 1e-5
    cap = [min(27.0, math.sqrt(11.0 / max(abs(k), 1e-6))) for k in kap]
    ref = serial(cap, kap)
    nch = (n + C - 1) // C
    exact = [math.inf] + [vstep(ref[t * C - 1], kap[t * C - 1]) for t in range(1, nch)]
    starts = {"inf": [math.inf] * nch, "exact": exact,
              "low": [x * 0.5 for x in exact], "high": [x * 1.7 for x in exact],
              "noise": [x * (1 + 1e-12 * rng.normal()) for x in exact]}
    rounds = {}
    for name, g in starts.items():
        v, r = relaxed(cap, kap, C, g)
        assert v == ref, f"start {name}: relaxation differs from the serial pass"
        rounds[name] = r
    assert rounds["exact"] == 1            # an exact start: one round to confirm, nothing re-walked
    assert rounds["exact"] <= rounds["inf"]
