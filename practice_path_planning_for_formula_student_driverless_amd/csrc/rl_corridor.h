// rl_corridor.h — exact corridor bounds (ref = /root/reference/src/main.cpp):
//   rayIntersectSegment ref:478-490, rayToRingDistance ref:491-500,
//   minDistanceToSegments_global ref:501-512, safe_ray ref:694-699,
//   corridor blocks ref:701-711 / 749-756.
//
// For CK samples per lane (P, n), both rings:
//   1. a uniform pass over blocks of 64 segments computes, per sample, the cheap
//      pretest of the ray test (u numerator vs denominator) and sets a bit in a
//      per-lane 64-bit candidate mask; it also tracks |P - S0|^2, an upper bound
//      of the ring's point-to-segment distance;
//   2. each lane then walks only ITS set bits (ctz loop, per-lane loads of the
//      64-B segment record from L1) and evaluates the reference expressions
//      exactly — the wave no longer runs the exact path for the union of all
//      lanes' candidates;
//   3. where a ray missed, the point-to-segment fallback does the same with the
//      conservative lower bound |P - mid| - half_len <= upper bound as filter.
// The ±n rays share one test: d -> -d gives den' = -den, t' = -t, u' = u bit-exactly.
// Every skipped pair provably cannot change the reference's minimum.
#pragma once
#include <hip/hip_runtime.h>

#include "rl_device.h"
#include "rl_math.h"

namespace rl {

// exact rayIntersectSegment for +n and -n at once, folded into the running minima
__device__ __forceinline__ void ray_exact(const SegRec& s, double qx, double qy, double ux, double uy,
                                          double& bp, double& bn) {
    double den = ux * (-s.vy) + uy * (s.vx);
    if (fabs(den) < 1e-15) return;
    double ax = s.x0 - qx, ay = s.y0 - qy;
    double inv = 1.0 / den;
    double t = (ax * (-s.vy) + ay * (s.vx)) * inv;
    double u = (ux * ay - uy * ax) * inv;
    if (u >= -1e-12 && u <= 1.0 + 1e-12) {
        if (t > 0.0 && t < bp) bp = t;       // ref:496-497
        double tn = -t;
        if (tn > 0.0 && tn < bn) bn = tn;
    }
}

// exact point-to-segment distance term of minDistanceToSegments_global (ref:504-509)
__device__ __forceinline__ double seg_dist_exact(const SegRec& s, double qx, double qy) {
    double apx = qx - s.x0, apy = qy - s.y0;
    double t = sclamp((s.vx * apx + s.vy * apy) / s.denom, 0.0, 1.0);
    double Qx = s.x0 + s.vx * t, Qy = s.y0 + s.vy * t;
    return hypot_ref(qx - Qx, qy - Qy);
}

// one ring: rays (bp, bn) and, where needed, the point-to-segment fallback (md)
template <int CK>
__device__ __forceinline__ void ring_scan(const SegRec* __restrict__ S, int e0, int e1, const double (&qx)[CK],
                                          const double (&qy)[CK], const double (&ux)[CK], const double (&uy)[CK],
                                          const bool (&act)[CK], double (&bp)[CK], double (&bn)[CK],
                                          double (&md)[CK]) {
    double ub2[CK];
#pragma unroll
    for (int k = 0; k < CK; ++k) { bp[k] = bn[k] = md[k] = INFINITY; ub2[k] = INFINITY; }
    for (int b0 = e0; b0 < e1; b0 += 64) {
        const int nb = min(64, e1 - b0);
        unsigned long long m[CK];
#pragma unroll
        for (int k = 0; k < CK; ++k) m[k] = 0ull;
        for (int j = 0; j < nb; ++j) {
            const double x0 = S[b0 + j].x0, y0 = S[b0 + j].y0, vx = S[b0 + j].vx, vy = S[b0 + j].vy;
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                const double ax = x0 - qx[k], ay = y0 - qy[k];
                const double nu = ux[k] * ay - uy[k] * ax;          // u = nu * (1/den)
                const double den = ux[k] * (-vy) + uy[k] * (vx);
                const double ad = fabs(den), anu = fabs(nu);
                // conservative: u can only land in [-1e-12, 1+1e-12] when this holds
                const bool cand = !(ad < 1e-15) && (anu <= 1.0000001 * ad) && (((nu < 0) == (den < 0)) || anu <= 4e-12 * ad);
                m[k] |= (unsigned long long)cand << j;
                ub2[k] = fmin(ub2[k], ax * ax + ay * ay);
            }
        }
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            unsigned long long mm = act[k] ? m[k] : 0ull;
            while (mm) {
                const int j = __builtin_ctzll(mm);
                mm &= mm - 1;
                ray_exact(S[b0 + j], qx[k], qy[k], ux[k], uy[k], bp[k], bn[k]);
            }
        }
    }
    // fallback only where a ray of this ring missed (safe_ray ref:696)
    bool need[CK];
    bool any = false;
#pragma unroll
    for (int k = 0; k < CK; ++k) { need[k] = act[k] && (!isfinite(bp[k]) || !isfinite(bn[k])); any |= need[k]; }
    if (!__any(any)) return;
    double lim[CK];
#pragma unroll
    for (int k = 0; k < CK; ++k) lim[k] = sqrt(ub2[k]) * (1.0 + 1e-9) + 1e-12;
    for (int b0 = e0; b0 < e1; b0 += 64) {
        const int nb = min(64, e1 - b0);
        unsigned long long m[CK];
#pragma unroll
        for (int k = 0; k < CK; ++k) m[k] = 0ull;
        for (int j = 0; j < nb; ++j) {
            const double mx = S[b0 + j].mx, my = S[b0 + j].my, hr = S[b0 + j].hr;
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                const double dx = qx[k] - mx, dy = qy[k] - my, r = lim[k] + hr;
                const bool cand = need[k] && !(dx * dx + dy * dy > r * r);
                m[k] |= (unsigned long long)cand << j;
            }
        }
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            unsigned long long mm = m[k];
            while (mm) {
                const int j = __builtin_ctzll(mm);
                mm &= mm - 1;
                md[k] = smin(md[k], seg_dist_exact(S[b0 + j], qx[k], qy[k]));
            }
        }
    }
}

// corridor bounds for CK samples (ref:702-711); guard = width*0.5 + margin.
// Inactive samples (act false: padding of a ragged chunk) do no exact work; their
// outputs are meaningless and the caller zeroes them.
template <int CK>
__device__ __forceinline__ void corridor_bounds(const SegRec* __restrict__ S, int Ei, int Eo, const double (&qx)[CK],
                                                const double (&qy)[CK], const double (&ux)[CK],
                                                const double (&uy)[CK], const bool (&act)[CK], double guard,
                                                double (&lo)[CK], double (&hi)[CK]) {
    double bpi[CK], bni[CK], mdi[CK], bpo[CK], bno[CK], mdo[CK];
    ring_scan<CK>(S, 0, Ei, qx, qy, ux, uy, act, bpi, bni, mdi);
    ring_scan<CK>(S, Ei, Ei + Eo, qx, qy, ux, uy, act, bpo, bno, mdo);
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        // safe_ray ref:694-699: ray distance, else point-to-segment minimum, else 0; max(0, .)
        double spi = bpi[k], sni = bni[k], spo = bpo[k], sno = bno[k];
        if (!isfinite(spi)) spi = mdi[k];
        if (!isfinite(spi)) spi = 0.0;
        if (!isfinite(sni)) sni = mdi[k];
        if (!isfinite(sni)) sni = 0.0;
        if (!isfinite(spo)) spo = mdo[k];
        if (!isfinite(spo)) spo = 0.0;
        if (!isfinite(sno)) sno = mdo[k];
        if (!isfinite(sno)) sno = 0.0;
        double dpos = smin(smax(0.0, spi), smax(0.0, spo));
        double dneg = smin(smax(0.0, sni), smax(0.0, sno));
        double hk = smax(0.0, dpos - guard);
        double lk = -smax(0.0, dneg - guard);
        if (!isfinite(hk)) hk = 0.0;
        if (!isfinite(lk)) lk = 0.0;
        hi[k] = hk;
        lo[k] = lk;
    }
}

}  // namespace rl
