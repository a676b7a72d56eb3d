// rl_corridor.h — exact corridor bounds (ref = /root/reference/src/main.cpp):
//   rayIntersectSegment ref:478-490, rayToRingDistance ref:491-500,
//   minDistanceToSegments_global ref:501-512, safe_ray ref:694-699,
//   corridor blocks ref:701-711 / 749-756.
//
// Rings arrive as an ENTRY STREAM (built by rl_abi.cpp make_ring): the vertices of
// each chain of segments in order, padded to blocks of 32 entries; entry v carries
// the record of the segment that ENDS at v (flag bit set) or a dummy (chain start,
// padding).  For CK samples (P, n) per lane:
//   1. filter: per entry, the side of the ray line c_v = n x (V_v - P) (two fma with
//      a per-sample constant, two compares); a segment is a candidate unless both its endpoints lie
//      strictly on the same side by more than dl (see below).  The candidate bit
//      shifts into a per-lane 32-bit word (w = 2w + cand, MSB = first entry);
//   2. each lane walks only ITS candidates (clz loop; the CK samples' record loads
//      issued together) and evaluates the reference expressions exactly;
//   3. where a ray missed, the point-to-segment fallback: an upper bound ub from
//      the walked candidates' endpoints, then the conservative lower bound
//      |P - mid| - half_len <= ub as filter and the exact walk again.
// The ±n rays share one test: d -> -d gives den' = -den, t' = -t, u' = u bit-exactly.
//
// Why skipping is exact: with C0, C1 the true sides of the two endpoints, the
// reference's u = nu/den has nu = c0 up to rounding, den = (C0-C1) + eta with
// |eta| <= 7e-16|v|, |nu_f - C| <= 4.5e-16 (|ax|+|ay|) and |c_f - C| <= 6e-16 (Rv+|qx|+|qy|).  If both c0, c1 > dl
// (or both < -dl) with dl = 4e-12 (1 + Vmax) + 4e-15 (Rv + |qx|+|qy|)
// (Vmax = max |vx|+|vy|, Rv = max |x|+|y| over the ring), then u < -1e-12
// (|u| >= dl/|v| >= 4e-12), or u > 1 + 1e-12 ((u-1) >= (dl - 1.1e-15 R - 7e-16|v|)/|v|),
// or the pair is near-parallel with |u| >> 1 — the reference rejects the pair.
#pragma once
#include <hip/hip_runtime.h>

#include "rl_device.h"
#include "rl_math.h"

namespace rl {

// uniform (wave-invariant) reads of the ring streams go through the constant address
// space so they become scalar (SMEM) loads; the kernel never writes these buffers
typedef __attribute__((address_space(4))) const double cdbl;
typedef __attribute__((address_space(4))) const uint32_t cu32;
__device__ __forceinline__ cdbl* as_cdbl(const void* p) { return (cdbl*)p; }
__device__ __forceinline__ cu32* as_cu32(const void* p) { return (cu32*)p; }

// one ring in entry-stream form (device pointers); M is a multiple of 32
struct RingDesc {
    const double2* vtx;       // [M] entry vertex (NaN for padding)
    const SegRec* rec;        // [M] record of the segment ending at the entry
    const uint32_t* flag;     // [M/32] bit (31-j): entry 32b+j ends a segment
    const double* blk;        // ring_blk_doubles(M): [M/B][4] block circles (cx, cy, R, 0), R < 0: no segment
                              // ends in the block; then the side filter's fp32 copies: vertices [M][2] f32
                              // and block circles [M/B][4] f32 (radius rounded up), and the fallback
                              // filters' segment midpoints [M][4] f32 (mx, my, half length rounded up, 0)
    int32_t M, E;             // padded entry count, segment count
    double dl0;               // 4e-12*(1+Vmax) + 4e-15*Rv
    double dl32;              // 1e-6*Rv: the fp32 side filter's extra margin (see ring_rays)
};
#ifndef RL_BLKSZ
#define RL_BLKSZ 16      // entries per culling block (4, 8, 16 or 32; A/B in DESIGN 3d)
#endif
constexpr int RL_BLK = RL_BLKSZ;
static_assert(RL_BLK == 4 || RL_BLK == 8 || RL_BLK == 16 || RL_BLK == 32, "culling blocks of 4, 8, 16 or 32 entries");
// the side bits of a visited block are assembled RL_SUB entries at a time (RL_SUB + 1 bits per word)
constexpr int RL_SUB = RL_BLK < 16 ? RL_BLK : 16;
// a candidate word shifted past one skipped block
__device__ __forceinline__ uint32_t shl_blk(uint32_t w) { return RL_BLK >= 32 ? 0u : (w << (RL_BLK & 31)); }
// layout of RingDesc::blk: [M/B][4] fp64 circles, then fp32 vertices [M][2], fp32 circles
// [M/B][4] and fp32 midpoints [M][4] (counted in doubles)
__host__ __device__ constexpr size_t ring_blk_off_vtx32(size_t M) { return 4 * M / RL_BLK; }
__host__ __device__ constexpr size_t ring_blk_off_blk32(size_t M) { return 4 * M / RL_BLK + M; }
__host__ __device__ constexpr size_t ring_blk_off_mid32(size_t M) { return 4 * M / RL_BLK + M + 2 * M / RL_BLK; }
__host__ __device__ constexpr size_t ring_blk_doubles(size_t M) { return ring_blk_off_mid32(M) + 2 * M; }
typedef __attribute__((address_space(4))) const float cflt;

// (Along-ray block culling, round 4: built bit-exact with a per-block direction-cone guard and
// measured slower on every configuration, then removed)

// Block culling. Entries come in blocks of RL_BLK. The host gives each block a circle (C, R)
// that contains both endpoints of every segment ending in the block (rl_abi.cpp
// make_ring), so every point of those segments lies within R of C.
//  * Ray filter: |n x (V - C)| <= |n| R for every such vertex V. If the centre's side
//    value satisfies |c_C| > R(1+1e-9) + 2 dl, every endpoint's computed side value is
//    beyond dl on the same side (the error of a computed side value is below dl/6), so
//    no segment of the block is a candidate for that sample.
//  * Fallback: the distance to any segment of the block is >= |q - C| - R.
// A block is skipped only when every lane's samples skip it, so the entry loop stays
// wave-uniform. What survives is exactly what the entry tests would keep.

// Diagnostic build only (-DRL_COUNT=1): corridor work counters (lane-level events),
// summed with atomics into a device array no other code reads.
#ifdef RL_COUNT
static __device__ unsigned long long rl_dbg_count[8];   // one per translation unit
#define RL_CNT(slot, n) atomicAdd(&rl_dbg_count[slot], (unsigned long long)(n))
#else
#define RL_CNT(slot, n) do {} while (0)
#endif

// exact rayIntersectSegment for +n and -n at once, folded into the running minima
__device__ __forceinline__ void ray_exact(double x0, double y0, double vx, double vy, double qx, double qy,
                                          double ux, double uy, double& bp, double& bn) {
    double den = ux * (-vy) + uy * (vx);
    if (fabs(den) < 1e-15) return;
    double ax = x0 - qx, ay = y0 - qy;
    double inv = 1.0 / den;
    double t = (ax * (-vy) + ay * (vx)) * inv;
    double u = (ux * ay - uy * ax) * inv;
    if (u >= -1e-12 && u <= 1.0 + 1e-12) {
        if (t > 0.0 && t < bp) bp = t;       // ref:496-497
        double tn = -t;
        if (tn > 0.0 && tn < bn) bn = tn;
    }
}

// exact point-to-segment distance term of minDistanceToSegments_global (ref:504-509)
__device__ __forceinline__ double seg_dist_exact(double x0, double y0, double vx, double vy, double denom,
                                                 double qx, double qy) {
    double apx = qx - x0, apy = qy - y0;
    double t = sclamp((vx * apx + vy * apy) / denom, 0.0, 1.0);
    double Qx = x0 + vx * t, Qy = y0 + vy * t;
    return hypot_ref(qx - Qx, qy - Qy);
}

// next candidate of each sample's word: entry offset j (0 if none), cleared from w
template <int CK>
__device__ __forceinline__ bool next_bits(uint32_t (&w)[CK], bool (&h)[CK], int (&j)[CK]) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        h[k] = w[k] != 0u;
        j[k] = h[k] ? __clz(w[k]) : 0;
        w[k] &= ~(0x80000000u >> j[k]);
        any |= h[k];
    }
    return __any(any);
}

// one ring's rays: nearest hit along +n (bp) and -n (bn), +inf if none, and ub2 >= the
// squared point-to-segment minimum (from the walked candidates' endpoints; +inf if none)
template <int CK>
__device__ __forceinline__ void ring_rays(const RingDesc& R, const double (&qx)[CK], const double (&qy)[CK],
                                          const double (&ux)[CK], const double (&uy)[CK], const bool (&act)[CK],
                                          double (&bp)[CK], double (&bn)[CK], double (&ub2)[CK]) {
    cu32* F = as_cu32(R.flag);
    cflt* V = (cflt*)(R.blk + ring_blk_off_vtx32(R.M));     // fp32 vertices [M][2]
    cflt* BK = (cflt*)(R.blk + ring_blk_off_blk32(R.M));    // fp32 block circles [M/B][4]
    const SegRec* __restrict__ S = R.rec;  // per-lane (divergent) reads
    // The side filter runs in fp32 (packed for two samples per lane).  c = n x (V - P) =
    // ux*vy - uy*vx - g.  With e = 2^-24 and |n| <= 1, the fp32 value built from fp32
    // copies of n, V, g differs from the exact one by <= 5e(|vx|+|vy|+|g|) <= 3e-7(Rv+|q|_1),
    // and the fp64 value (the one the skip proof above bounds by dl) by <= dl/6; so with
    // dl32 = dl + 1e-6(Rv+|q|_1), c32 > dl32 implies c64 > dl: a pair the fp32 filter skips
    // is one the fp64 filter would skip.  Block test: the fp32 centre is within e|C|_1 of
    // the exact one and R is rounded up, so |c32(C)| > R(1+1e-6) + 2 dl32 leaves every
    // endpoint with |c32| > 2 dl32 - 11e(Rv+|q|_1) >= dl32 on the centre's side.
    float dl[CK], g[CK], uxf[CK], uyf[CK];
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        const double q1 = fabs(qx[k]) + fabs(qy[k]);
        g[k] = (float)(ux[k] * qy[k] - uy[k] * qx[k]);
        dl[k] = (float)((R.dl0 + 4e-15 * q1) + (R.dl32 + 1e-6 * q1));
        uxf[k] = (float)ux[k];
        uyf[k] = (float)uy[k];
        bp[k] = bn[k] = ub2[k] = INFINITY;
    }
    auto side = [&](int k, float vx, float vy) -> float { return __builtin_fmaf(uxf[k], vy, -__builtin_fmaf(uyf[k], vx, g[k])); };
    // Side bits without mask logic: c > dl <=> sign(dl - c) and c < -dl <=> sign(c + dl), exact
    // for finite operands (a rounded difference keeps the sign of the exact one, equality gives
    // +0); v_alignbit shifts each sign bit straight into a per-lane word.  A lane whose sample or
    // margin is not finite takes every pair as a candidate (as the compare form did with NaN).
    // NaN sides only come from the padding entries at the end of the stream, whose bits the
    // segment flags mask.
    bool bad[CK];
    uint32_t lp[CK], lq[CK];       // side bits of the entry just before the next block
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        bad[k] = !(isfinite(g[k]) && isfinite(dl[k]) && isfinite(uxf[k]) && isfinite(uyf[k]));
        lp[k] = lq[k] = 0u;
    }
    auto sgn = [](float x) -> uint32_t { return __float_as_uint(x) >> 31; };
    bool prev_ok = false;          // lp/lq hold the sides of the entry just before the next block
    for (int b0 = 0; b0 < R.M; b0 += 32) {
        uint32_t w[CK];
#pragma unroll
        for (int k = 0; k < CK; ++k) w[k] = 0u;
        // which of the word's 32/RL_BLK blocks some lane's ray line may cross (wave-uniform)
        uint32_t visit = 0u;
#pragma unroll
        for (int q = 0; q < 32 / RL_BLK; ++q) {
            cflt* bk = BK + 4 * ((b0 / RL_BLK) + q);
            const float cx = bk[0], cy = bk[1], rb = bk[2];
            bool need = false;
            if (rb >= 0.0f) {
#pragma unroll
                for (int k = 0; k < CK; ++k) {
                    const float c = side(k, cx, cy);
                    need |= act[k] && !(fabsf(c) > rb * (1.0f + 1e-6f) + 2.0f * dl[k]);
                }
            }
            if (__any(need)) visit |= 1u << q;
        }
        // (block slots per 32-entry word: 32 / RL_BLK; round 5 counted 4, the blocks-of-8
        // figure, which halved the visited fractions reported at blocks of 16)
        if (threadIdx.x % 64 == 0) { RL_CNT(0, 32 / RL_BLK); RL_CNT(1, __popc(visit)); }
        if (visit == 0u) { prev_ok = false; continue; }
#pragma unroll
        for (int q = 0; q < 32 / RL_BLK; ++q) {
            if (!((visit >> q) & 1u)) {
#pragma unroll
                for (int k = 0; k < CK; ++k) w[k] = shl_blk(w[k]);
                prev_ok = false;
                continue;
            }
#pragma unroll
          for (int sb = 0; sb < RL_BLK / RL_SUB; ++sb) {
            const int e0 = b0 + q * RL_BLK + sb * RL_SUB;
            uint32_t pb[CK], qb[CK];   // bit S: the entry before the sub-block, bit S-1-j: entry e0+j
#pragma unroll
            for (int k = 0; k < CK; ++k) { pb[k] = lp[k]; qb[k] = lq[k]; }
            if (!prev_ok) {
                if (e0 > 0) {          // sides of the entry before the block
                    const float vx = V[2 * (e0 - 1)], vy = V[2 * (e0 - 1) + 1];
#pragma unroll
                    for (int k = 0; k < CK; ++k) {
                        const float c = side(k, vx, vy);
                        pb[k] = sgn(dl[k] - c);
                        qb[k] = sgn(c + dl[k]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < CK; ++k) pb[k] = qb[k] = 0u;
                }
            }
#pragma unroll
            for (int j = 0; j < RL_SUB; ++j) {
                const float vx = V[2 * (e0 + j)], vy = V[2 * (e0 + j) + 1];
#pragma unroll
                for (int k = 0; k < CK; ++k) {
                    const float c = side(k, vx, vy);
                    pb[k] = __builtin_amdgcn_alignbit(pb[k], __float_as_uint(dl[k] - c), 31);
                    qb[k] = __builtin_amdgcn_alignbit(qb[k], __float_as_uint(c + dl[k]), 31);
                }
            }
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                // a pair is skipped only when both endpoints lie beyond dl on the same side
                constexpr uint32_t BM = (1u << RL_SUB) - 1u;
                uint32_t cand = ~((pb[k] & (pb[k] >> 1)) | (qb[k] & (qb[k] >> 1))) & BM;
                if (bad[k]) cand = BM;
                w[k] = (RL_SUB >= 32 ? 0u : (w[k] << (RL_SUB & 31))) | cand;
                lp[k] = pb[k] & 1u;
                lq[k] = qb[k] & 1u;
            }
            prev_ok = true;
          }
        }
        const uint32_t f = F[b0 >> 5];
#pragma unroll
        for (int k = 0; k < CK; ++k) w[k] = act[k] ? (w[k] & f) : 0u;
        bool h[CK];
        int j[CK];
        while (next_bits<CK>(w, h, j)) {
            double x0[CK], y0[CK], sx[CK], sy[CK];
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                const SegRec* s = S + b0 + j[k];
                x0[k] = s->x0; y0[k] = s->y0; sx[k] = s->vx; sy[k] = s->vy;
            }
            if (threadIdx.x % 64 == 0) RL_CNT(2, 1);          // walk iterations (wave)
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                if (h[k]) {
                    RL_CNT(3, 1);                                 // exact ray tests (lane)
                    ray_exact(x0[k], y0[k], sx[k], sy[k], qx[k], qy[k], ux[k], uy[k], bp[k], bn[k]);
                    // any segment endpoint bounds the point-to-segment minimum from above
                    const double ax = qx[k] - x0[k], ay = qy[k] - y0[k];
                    const double ex = ax - sx[k], ey = ay - sy[k];
                    ub2[k] = fmin(ub2[k], fmin(ax * ax + ay * ay, ex * ex + ey * ey));
                }
            }
        }
    }
}

// (A work-list form of the ray scan -- each lane's samples testing only their own blocks
// from a compacted (sample, block) list in LDS, per-lane vertex loads and LDS atomic minima --
// was built in round 5 and measured 40 % slower on C5: DESIGN.md §3f.)

// minDistanceToSegments_global (ref:501-512) for the samples with need[k], exact for
// every sample whose minimum is <= rad[k] (md[k] = +inf or a value > rad[k] otherwise).
// Lane-level filters per block and per entry: the samples' bounding circle (centre q0,
// radius max_k r_k + |q_k - q0|_1) against the block circle, then against
// |mid - q0| <= r + half_len.  Two passes over the surviving entries:
//   1. the nearest segment midpoint to q0, at distance m: a midpoint lies on its
//      segment, so md_k <= m + |q_k - q0| and the search radius of sample k drops to
//      r_k = min(rad_k, m + |q_k - q0|);
//   2. the candidates within that radius, walked in entry order; a candidate whose
//      lower bound |q_k - mid| - half_len already exceeds the running minimum md_k
//      cannot lower it (std::min keeps the first of equal values), so only the others
//      get the exact reference distance.
template <int CK, bool TIGHT = true, bool PRUNE = true>
__device__ __forceinline__ void ring_mindist(const RingDesc& R, const double (&qx)[CK], const double (&qy)[CK],
                                             const bool (&need)[CK], const double (&rad)[CK], double (&md)[CK]) {
    cu32* F = as_cu32(R.flag);
    cflt* BK = (cflt*)(R.blk + ring_blk_off_blk32(R.M));    // fp32 block circles [M/B][4]
    cflt* MD = (cflt*)(R.blk + ring_blk_off_mid32(R.M));    // fp32 (mx, my, hr, 0) [M][4]
    const SegRec* __restrict__ S = R.rec;
    const double cx = qx[0], cy = qy[0];
    double dk[CK];                         // |q_k - q0|_1, rounded up
    double Rl = -1.0;
    bool lneed = false;
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        md[k] = INFINITY;
        dk[k] = (fabs(qx[k] - cx) + fabs(qy[k] - cy)) * (1.0 + 1e-12);
        if (need[k]) Rl = fmax(Rl, rad[k] + dk[k]);
        lneed |= need[k];
    }
    // The block and midpoint filters run in fp32 on fp32 copies (circle radii and half
    // lengths rounded up).  |q0 - C| computed so differs from the exact distance by at most
    // 2e(|q0|_1 + Rv) + 3e|q0 - C| (e = 2^-24, |C|_1 <= Rv for circle centres and
    // midpoints); dm = dl32 + 1e-6|q0|_1 >= 1e-6(Rv + |q0|_1) covers the first term, the
    // (1 + 1e-6) factors the second: a skip in fp32 is a skip in exact arithmetic, and the
    // nearest-midpoint distance + dm bounds the exact one from above.
    const float cxf = (float)cx, cyf = (float)cy;
    const float dm = (float)(R.dl32 + 1e-6 * (fabs(cx) + fabs(cy)));
    auto d2f = [&](float px, float py) -> float {
        const float dx = cxf - px, dy = cyf - py;
        return __builtin_fmaf(dx, dx, dy * dy);
    };
    float Rlf = (float)(Rl * (1.0 + 1e-6));
    // blocks whose circle meets the search circle (wave-uniform mask of one word)
    auto visit_of = [&](int b0) -> uint32_t {
        uint32_t visit = 0u;
#pragma unroll
        for (int q = 0; q < 32 / RL_BLK; ++q) {
            cflt* bk = BK + 4 * ((b0 / RL_BLK) + q);
            const float rb = bk[2];
            const float r = (Rlf + rb + dm) * (1.0f + 1e-6f);
            const bool nb = lneed && rb >= 0.0f && !(d2f(bk[0], bk[1]) > r * r);
            if (__any(nb)) visit |= 1u << q;
        }
        return visit;
    };
    // pass 1: nearest midpoint (padding and chain starts carry NaN mids: fmin skips them)
    float m2 = INFINITY;
    for (int b0 = 0; TIGHT && b0 < R.M; b0 += 32) {
        const uint32_t visit = visit_of(b0);
        if (visit == 0u) continue;
#pragma unroll
        for (int q = 0; q < 32 / RL_BLK; ++q) {
            if (!((visit >> q) & 1u)) continue;
#pragma unroll
            for (int j = 0; j < RL_BLK; ++j) {
                cflt* mr = MD + 4 * (b0 + q * RL_BLK + j);
                m2 = fminf(m2, d2f(mr[0], mr[1]));
            }
        }
    }
    if (isfinite(m2)) {
        const double m = (double)(sqrtf(m2) * (1.0f + 1e-6f) + dm) * (1.0 + 1e-12) + 1e-12;
        double R2 = -1.0;
#pragma unroll
        for (int k = 0; k < CK; ++k)
            if (need[k]) R2 = fmax(R2, fmin(rad[k], m + dk[k]) + dk[k]);
        Rl = R2;
        Rlf = (float)(Rl * (1.0 + 1e-6));
    }
    // pass 2: candidates and the exact distances
    for (int b0 = 0; b0 < R.M; b0 += 32) {
        const uint32_t visit = visit_of(b0);
        if (threadIdx.x % 64 == 0) { RL_CNT(4, 32 / RL_BLK); RL_CNT(5, __popc(visit)); }
        if (visit == 0u) continue;
        uint32_t w = 0u;
#pragma unroll
        for (int q = 0; q < 32 / RL_BLK; ++q) {
            if (!((visit >> q) & 1u)) { w = shl_blk(w); continue; }
#pragma unroll
            for (int j = 0; j < RL_BLK; ++j) {
                cflt* mr = MD + 4 * (b0 + q * RL_BLK + j);
                const float r = (Rlf + mr[2] + dm) * (1.0f + 1e-6f);
                const bool skip = d2f(mr[0], mr[1]) > r * r;
                w = (w << 1) | (uint32_t)!skip;
            }
        }
        w = lneed ? (w & F[b0 >> 5]) : 0u;
        while (__any(w != 0u)) {
            const bool h = w != 0u;
            const int j = h ? __clz(w) : 0;
            w &= ~(0x80000000u >> j);
            const SegRec* s = S + b0 + j;
            const double x0 = s->x0, y0 = s->y0, sx = s->vx, sy = s->vy, dn = s->denom;
            const double mx = s->mx, my = s->my, hr = s->hr;
            if (threadIdx.x % 64 == 0) RL_CNT(6, 1);              // fallback walk iterations (wave)
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                const double ex = qx[k] - mx, ey = qy[k] - my, lim = md[k] + hr;
                const bool may = h && need[k] && (!PRUNE || !(ex * ex + ey * ey > lim * lim));
                if (may) {
                    RL_CNT(7, 1);                                 // exact distance evaluations (lane)
                    md[k] = smin(md[k], seg_dist_exact(x0, y0, sx, sy, dn, qx[k], qy[k]));
                }
            }
        }
    }
}

// squared distance upper bound from every vertex of the ring (NaN padding ignored)
template <int CK>
__device__ __forceinline__ void ring_vertex_ub(const RingDesc& R, const double (&qx)[CK], const double (&qy)[CK],
                                               double (&ub2)[CK]) {
    cdbl* V = as_cdbl(R.vtx);
    for (int v = 0; v < R.M; ++v) {
        const double vx = V[2 * v], vy = V[2 * v + 1];
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            const double dx = qx[k] - vx, dy = qy[k] - vy;
            ub2[k] = fmin(ub2[k], dx * dx + dy * dy);
        }
    }
}

// corridor bounds for CK samples (ref:694-711); guard = width*0.5 + margin.
// dpos = min(safe(+n, inner), safe(+n, outer)), dneg likewise, where
// safe(t, md) = max(0, t finite ? t : (md finite ? md : 0)) (ref:694-699).
// A ring's fallback minimum md_r only enters through min(., other ring's value):
// when the other ring's ray in that direction hit at s, any md_r >= s yields s
// (std::min returns the same value on ties), so md_r is searched only within
// rad = min(ub, s_max) and reported as +inf when it exceeds it.
// Inactive samples (act false) do no exact work; the caller zeroes their outputs.
// phase hook of the diagnostic stamp builds (RL_STAMPS): called with 8 after the inner
// ring's rays, 9 after the outer ring's, 10 after the fallback searches
struct NoStamp {
    __device__ __forceinline__ void operator()(int) const {}
};
// the fallback searches and the bounds from both rings' ray results (bp/bn/ub2 [ring][k])
template <int CK, bool TIGHT, bool PRUNE, class Stamp>
__device__ __forceinline__ void corridor_finish(const RingDesc& Ri, const RingDesc& Ro, const double (&qx)[CK],
                                                const double (&qy)[CK], const bool (&act)[CK], double guard,
                                                double (&bp)[2][CK], double (&bn)[2][CK], double (&ub2)[2][CK],
                                                double (&lo)[CK], double (&hi)[CK], Stamp stamp) {
    double md[2][CK];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const RingDesc& R = r == 0 ? Ri : Ro;
        const int o = 1 - r;
        bool need[CK], any_need = false, any_ub = false;
        double rad[CK];
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            const bool mp = !isfinite(bp[r][k]), mn = !isfinite(bn[r][k]);
            need[k] = act[k] && (mp || mn);
            // largest value md_r can take and still matter (+inf: the other ring missed too)
            double tau = -INFINITY;
            if (mp) tau = fmax(tau, isfinite(bp[o][k]) ? smax(0.0, bp[o][k]) : INFINITY);
            if (mn) tau = fmax(tau, isfinite(bn[o][k]) ? smax(0.0, bn[o][k]) : INFINITY);
            rad[k] = tau;
            any_need |= need[k];
            any_ub |= need[k] && !isfinite(ub2[r][k]) && !isfinite(tau);
        }
        if (!__any(any_need)) {
#pragma unroll
            for (int k = 0; k < CK; ++k) md[r][k] = INFINITY;
            continue;
        }
        if (__any(any_ub)) ring_vertex_ub<CK>(R, qx, qy, ub2[r]);   // no candidate at all (rare)
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            const double lim = sqrt(ub2[r][k]) * (1.0 + 1e-9) + 1e-12;   // >= the true minimum
            rad[k] = fmin(lim, rad[k] * (1.0 + 1e-9) + 1e-12);
        }
        ring_mindist<CK, TIGHT, PRUNE>(R, qx, qy, need, rad, md[r]);
    }
    stamp(10);
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        double s[2][2];            // [ring][+n, -n]
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int E = r == 0 ? Ri.E : Ro.E;
            // md = +inf from a non-empty ring means "beyond the other ring's value"
            const double mdv = isfinite(md[r][k]) ? smax(0.0, md[r][k]) : (E == 0 ? 0.0 : INFINITY);
            s[r][0] = isfinite(bp[r][k]) ? smax(0.0, bp[r][k]) : mdv;
            s[r][1] = isfinite(bn[r][k]) ? smax(0.0, bn[r][k]) : mdv;
        }
        double dpos = smin(s[0][0], s[1][0]);
        double dneg = smin(s[0][1], s[1][1]);
        double hk = smax(0.0, dpos - guard);
        double lk = -smax(0.0, dneg - guard);
        if (!isfinite(hk)) hk = 0.0;
        if (!isfinite(lk)) lk = 0.0;
        hi[k] = hk;
        lo[k] = lk;
    }
}

template <int CK, bool TIGHT = true, bool PRUNE = true, class Stamp = NoStamp>
__device__ __forceinline__ void corridor_bounds(const RingDesc& Ri, const RingDesc& Ro, const double (&qx)[CK],
                                                const double (&qy)[CK], const double (&ux)[CK],
                                                const double (&uy)[CK], const bool (&act)[CK], double guard,
                                                double (&lo)[CK], double (&hi)[CK], Stamp stamp = Stamp()) {
    double bp[2][CK], bn[2][CK], ub2[2][CK];
    ring_rays<CK>(Ri, qx, qy, ux, uy, act, bp[0], bn[0], ub2[0]);
    stamp(8);
    ring_rays<CK>(Ro, qx, qy, ux, uy, act, bp[1], bn[1], ub2[1]);
    stamp(9);
    corridor_finish<CK, TIGHT, PRUNE>(Ri, Ro, qx, qy, act, guard, bp, bn, ub2, lo, hi, stamp);
}


}  // namespace rl
