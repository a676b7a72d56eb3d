// rl_geom.hip — step 6 on gfx950: the rows of pipeline::compute_geom_and_save
// (ref = /root/reference/src/main.cpp:1295-1335), one thread per output row.
//   s_k = s0 + L*(k/denomN); x, y and derivatives from the Spline1D pieces
//   (eval_with_deriv ref:435-445, binary search + cubic in the reference's
//   operation order); heading = atan2(y', x'); curvature with pow(max(1e-12,
//   x'^2+y'^2), 1.5) (pow15, rl_math.h); n = normalize(-y', x', 1e-12) (ref:132);
//   distancesToRings (ref:513-524) through the exact candidate scan of rl_corridor.h;
//   width; v_kappa = min(v_cap, sqrt(a_lat_max / max(|kappa|, kappa_eps))).
// Compiled with -ffp-contract=off like the optimiser kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_corridor.h"
#include "rl_device.h"
#include "rl_kernels.h"
#include "rl_math.h"

namespace rl {

// Spline1D::eval_with_deriv (ref:435-445); K = knots [5][n] (s,a,b,c,d) of one axis
__device__ __forceinline__ void spline_eval_d(const double* __restrict__ K, int n, double si, double& f, double& fp,
                                              double& fpp) {
    if (n == 0) { f = fp = fpp = 0.0; return; }
    if (n == 1) { f = K[n]; fp = fpp = 0.0; return; }
    const double* s = K;
    int lo = 0, hi = n - 1;
    if (si <= s[0]) lo = 0;
    else if (si >= s[n - 1]) lo = n - 2;
    else {
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (s[mid] <= si) lo = mid;
            else hi = mid;
        }
    }
    const double a = K[n + lo], b = K[2 * n + lo], c = K[3 * n + lo], d = K[4 * n + lo];
    const double t = si - s[lo];
    f = a + b * t + c * t * t + d * t * t * t;
    fp = b + 2.0 * c * t + 3.0 * d * t * t;
    fpp = 2.0 * c + 6.0 * d * t;
}

// distancesToRings for one ring: the nearer ray hit along ±n, else the exact
// point-to-segment minimum (ref:519-522); +inf stays +inf (the caller maps it to 0)
__device__ __forceinline__ double ring_distance(const RingDesc& R, double qx, double qy, double ux, double uy,
                                                bool act) {
    const double QX[1] = {qx}, QY[1] = {qy}, UX[1] = {ux}, UY[1] = {uy};
    const bool A[1] = {act};
    double bp[1], bn[1], ub2[1];
    ring_rays<1>(R, QX, QY, UX, UY, A, bp, bn, ub2);
    const bool hit = isfinite(bp[0]) || isfinite(bn[0]);
    const bool need[1] = {act && !hit};
    double md[1] = {INFINITY};
    if (__any(need[0])) {
        if (__any(need[0] && !isfinite(ub2[0]))) ring_vertex_ub<1>(R, QX, QY, ub2);
        const double rad[1] = {sqrt(ub2[0]) * (1.0 + 1e-9) + 1e-12};
        ring_mindist<1>(R, QX, QY, need, rad, md);
    }
    return hit ? smin(bp[0], bn[0]) : md[0];
}

__global__ __launch_bounds__(256) void rl_geom_kernel(GeomParams g) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = k < g.Kmax;
    double si = g.s0 + g.L * ((double)(active ? k : 0) / (double)g.denomN);
    double x, xp, xpp, y, yp, ypp;
    spline_eval_d(g.kx, g.nk, si, x, xp, xpp);
    spline_eval_d(g.ky, g.nk, si, y, yp, ypp);
    const double heading = atan2_cr(yp, xp);   // correctly rounded (rl_math.h)
    const double speed2 = xp * xp + yp * yp;
    const double denom = pow15(smax(1e-12, speed2));
    const double curv = (xp * ypp - yp * xpp) / denom;
    // geom::normalize({-yp, xp}, 1e-12) (ref:132)
    const double vx = -yp, vy = xp, nn = sqrt(vx * vx + vy * vy);
    double nx = 0.0, ny = 0.0;
    if (!(nn < 1e-12)) { nx = vx / nn; ny = vy / nn; }
    const bool scan = active && (nx != 0 || ny != 0);
    double d_in = ring_distance(g.ring[0], x, y, nx, ny, scan);
    double d_out = ring_distance(g.ring[1], x, y, nx, ny, scan);
    if (!scan) { d_in = 0.0; d_out = 0.0; }
    if (!isfinite(d_in)) d_in = 0.0;
    if (!isfinite(d_out)) d_out = 0.0;
    const double width = d_in + d_out;
    const double denom_k = smax(fabs(curv), g.kappa_eps);
    double v_kappa = sqrt(g.a_lat_max / denom_k);
    if (v_kappa > g.v_cap) v_kappa = g.v_cap;
    if (!active) return;
    const double r[9] = {si - g.s0, x, y, heading, curv, d_in, d_out, width, v_kappa};
    double* out = g.rows + 9 * (size_t)k;
#pragma unroll
    for (int j = 0; j < 9; ++j) out[j] = r[j];
    if (k == 0 && g.emit_dup) {               // closed duplicate: L, then row 0 (ref:1331-1334)
        double* d = g.rows + 9 * (size_t)g.Kmax;
        d[0] = g.L;
#pragma unroll
        for (int j = 1; j < 9; ++j) d[j] = r[j];
    }
}

hipError_t launch_geom(const GeomParams& g, hipStream_t st) {
    if (g.Kmax <= 0) return hipSuccess;
    const int T = 256;
    hipLaunchKernelGGL(rl_geom_kernel, dim3((g.Kmax + T - 1) / T), dim3(T), 0, st, g);
    return hipGetLastError();
}

// rl_corridor: each lane takes 2 adjacent samples (the optimiser's corridor scan
// mapping, rl_kernels.hip), normals_from_points_generic at each (ref:581-593) and the
// exact corridor bounds of rl_corridor.h.
__global__ __launch_bounds__(256) void rl_corridor_kernel(CorrParams c) {
    constexpr int CK = 2;
    const int N = c.N;
    const int i0 = (blockIdx.x * blockDim.x + threadIdx.x) * CK;
    double qx[CK], qy[CK], ux[CK], uy[CK], lo[CK], hi[CK];
    bool act[CK];
    auto P = [&](int j, int a) { return c.center[2 * j + a]; };
#pragma unroll
    for (int k = 0; k < CK; ++k) {
        const int i = min(i0 + k, N - 1);
        act[k] = i0 + k < N;
        double tx, ty;
        if (N == 1) { tx = 1; ty = 0; }
        else if (c.closed) {
            const int ip = (i + 1 == N) ? 0 : i + 1, im = (i == 0) ? N - 1 : i - 1;
            tx = (P(ip, 0) - P(im, 0)) * 0.5; ty = (P(ip, 1) - P(im, 1)) * 0.5;
        } else if (i == 0) { tx = P(1, 0) - P(0, 0); ty = P(1, 1) - P(0, 1); }
        else if (i == N - 1) { tx = P(N - 1, 0) - P(N - 2, 0); ty = P(N - 1, 1) - P(N - 2, 1); }
        else { tx = (P(i + 1, 0) - P(i - 1, 0)) * 0.5; ty = (P(i + 1, 1) - P(i - 1, 1)) * 0.5; }
        if (sqrt(tx * tx + ty * ty) < 1e-15) { tx = 1; ty = 0; }
        const double vx = -ty, vy = tx, n = sqrt(vx * vx + vy * vy);   // geom::normalize ref:132
        ux[k] = 0.0; uy[k] = 0.0;
        if (!(n < 1e-15)) { ux[k] = vx / n; uy[k] = vy / n; }
        qx[k] = P(i, 0);
        qy[k] = P(i, 1);
    }
    corridor_bounds<CK>(c.ring[0], c.ring[1], qx, qy, ux, uy, act, c.guard, lo, hi);
#pragma unroll
    for (int k = 0; k < CK; ++k)
        if (act[k]) { c.lo[i0 + k] = lo[k]; c.hi[i0 + k] = hi[k]; }
}

#ifdef RL_COUNT
int debug_counts_geom(unsigned long long* host, int reset) {
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(rl_dbg_count), z, sizeof(z)) == hipSuccess ? 0 : -3;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_count), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_corridor(const CorrParams& c, hipStream_t st) {
    if (c.N <= 0) return hipSuccess;
    const int T = 256, per = T * 2;
    hipLaunchKernelGGL(rl_corridor_kernel, dim3((c.N + per - 1) / per), dim3(T), 0, st, c);
    return hipGetLastError();
}

}  // namespace rl
