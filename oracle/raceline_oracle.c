/*
 * raceline_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C99, single-threaded, fp64 restatement of the reference hot path
 * (steps 7-8 of /root/reference/src/main.cpp, cited below as "ref:<line>").
 * It is the CHECKER for the HIP kernels: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library
 * (librl.so) never links or calls it.
 *
 * Pinning: tests/test_oracle_golden.py checks every output of this file
 * BIT-FOR-BIT against fixtures produced by the reference itself (compiled from
 * /root/reference/src/main.cpp where it lies, oracle/ref_harness.cpp), on all 7
 * bundled tracks, N=2000, open mode and cfg sweep points.
 *
 * Arithmetic contract: same operations in the same
 * order as the reference; std::min/std::max/std::clamp are restated with the
 * reference library's exact comparison forms; build with -ffp-contract=off.
 *
 * Beyond the reference it adds only instrumentation (evals/accepts per outer
 * iteration, v-pass sweeps that changed something) and the build-defined
 * alpha seeds of SURVEY.md §8d (seed 0 == the reference exactly).
 */
#ifndef ORACLE_FMA
#define ORACLE_FMA 0   /* 1: liboracle_fma.so, the checker of the RL_FMA kernel build */
#endif
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rl_abi.h"

/* libstdc++ semantics: std::max(a,b) = (a<b)?b:a ; std::min(a,b) = (b<a)?b:a */
static inline double smax(double a, double b) { return (a < b) ? b : a; }
static inline double smin(double a, double b) { return (b < a) ? b : a; }
/* std::clamp(v,lo,hi) = (v<lo)?lo:(hi<v)?hi:v */
static inline double sclamp(double v, double lo, double hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }

/* ------------------------------------------------------------------ cfg */
/* cfg::Config defaults, ref:77-113 (a_total_max = mu*9.81 evaluated once, ref:102) */
void oracle_cfg_default(rl_cfg* c) {
    memset(c, 0, sizeof(*c));
    c->veh_width_m = 1.0;
    c->safety_margin_m = 0.05;
    c->lambda_smooth = 1.6e-3;
    c->max_outer_iters = 14;
    c->max_inner_iters = 120;
    c->step_init = 0.65;
    c->step_min = 1e-6;
    c->armijo_c = 1e-5;
    c->kappa_eps = 1e-6;
    c->v_cap_mps = 27.0;
    c->mass_kg = 255.0;
    c->Cd = 0.30;
    c->A_front_m2 = 1.00;
    c->rho_air = 1.225;
    c->c_rr = 0.015;
    c->P_max_W = 80000.0;
    c->mu = 1.17;
    c->a_total_max = c->mu * 9.81;
    c->a_lat_max = 11.0;
    c->a_long_acc_cap = 8.0;
    c->a_long_brake_cap = 11.0;
    c->w_time_gain = 1.0;
    c->time_gamma_power = 2.0;
    c->time_weight_use_inv_v = 0;
    c->inv_v_gain = 0.1;
    c->max_vpass_iters = 6;
    c->use_total_ge_lat = 1;
}

/* ------------------------------------------------------------ α seeds */
/* xi ~ U(-1,1) from splitmix64(seed, counter=i); seed 0 -> 0 */
double oracle_seed_value(uint64_t seed, int32_t i, double sigma) {
    if (seed == 0) return 0.0;
    uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    double u = (double)(z >> 11) * 0x1.0p-53;
    return sigma * (2.0 * u - 1.0);
}

/* --------------------------------------------------------- ray utilities */
/* rayIntersectSegment, ref:478-490 */
static int ray_seg(double Ax, double Ay, double dx, double dy, const double* s, double* t_out) {
    double vx = s[2] - s[0], vy = s[3] - s[1];
    double den = dx * (-vy) + dy * (vx);
    if (fabs(den) < 1e-15) return 0;
    double ax = s[0] - Ax, ay = s[1] - Ay;
    double inv = 1.0 / den;
    double t = (ax * (-vy) + ay * (vx)) * inv;
    double u = (dx * ay - dy * ax) * inv;
    if (t >= 0.0 && u >= -1e-12 && u <= 1.0 + 1e-12) { *t_out = t; return 1; }
    return 0;
}
/* rayToRingDistance, ref:491-500 */
static double ray_ring(double Px, double Py, double dx, double dy, const double* seg, int E) {
    double best = INFINITY;
    for (int e = 0; e < E; ++e) {
        double t;
        if (ray_seg(Px, Py, dx, dy, seg + 4 * e, &t))
            if (t > 0.0 && t < best) best = t;
    }
    return best;
}
/* minDistanceToSegments_global, ref:501-512 */
static double min_dist_segs(double Px, double Py, const double* seg, int E) {
    double best = INFINITY;
    for (int e = 0; e < E; ++e) {
        const double* s = seg + 4 * e;
        double abx = s[2] - s[0], aby = s[3] - s[1], apx = Px - s[0], apy = Py - s[1];
        double denom = smax(1e-30, abx * abx + aby * aby);
        double t = sclamp((abx * apx + aby * apy) / denom, 0.0, 1.0);
        double Qx = s[0] + abx * t, Qy = s[1] + aby * t;
        best = smin(best, hypot(Px - Qx, Py - Qy));
    }
    return best;
}
/* safe_ray lambda, ref:694-699 / 917-922 */
static double safe_ray(double Px, double Py, double dx, double dy, const double* seg, int E) {
    double t = ray_ring(Px, Py, dx, dy, seg, E);
    if (!isfinite(t)) t = min_dist_segs(Px, Py, seg, E);
    if (!isfinite(t)) t = 0.0;
    return smax(0.0, t);
}
/* corridor block, ref:701-711 (initial, guard from veh_width argument) and
 * ref:749-756 (updates, guard from cfg veh_width_m) */
static void corridor(const double* Px, const double* Py, const double* nx, const double* ny, int N,
                     const rl_problem* pr, double veh_width, double safety, double* lo, double* hi) {
    for (int i = 0; i < N; ++i) {
        double vx = nx[i], vy = ny[i], x0 = Px[i], y0 = Py[i], mx = -vx, my = -vy;
        double dpos = smin(safe_ray(x0, y0, vx, vy, pr->inner_seg, pr->Ei), safe_ray(x0, y0, vx, vy, pr->outer_seg, pr->Eo));
        double dneg = smin(safe_ray(x0, y0, mx, my, pr->inner_seg, pr->Ei), safe_ray(x0, y0, mx, my, pr->outer_seg, pr->Eo));
        double guard = veh_width * 0.5 + safety;
        hi[i] = smax(0.0, dpos - guard);
        lo[i] = -smax(0.0, dneg - guard);
        if (!isfinite(hi[i])) hi[i] = 0.0;
        if (!isfinite(lo[i])) lo[i] = 0.0;
    }
}

/* ------------------------------------------------------------ geometry */
/* normals_from_points_generic, ref:581-593 */
static void normals(const double* Px, const double* Py, int N, int closed, double* nx, double* ny) {
    for (int i = 0; i < N; ++i) {
        double tx, ty;
        if (N == 1) { tx = 1; ty = 0; }
        else if (closed) {
            int ip = (i + 1) % N, im = (i - 1 + N) % N;
            tx = (Px[ip] - Px[im]) * 0.5; ty = (Py[ip] - Py[im]) * 0.5;
        } else if (i == 0) { tx = Px[1] - Px[0]; ty = Py[1] - Py[0]; }
        else if (i == N - 1) { tx = Px[N - 1] - Px[N - 2]; ty = Py[N - 1] - Py[N - 2]; }
        else { tx = (Px[i + 1] - Px[i - 1]) * 0.5; ty = (Py[i + 1] - Py[i - 1]) * 0.5; }
        if (sqrt(tx * tx + ty * ty) < 1e-15) { tx = 1; ty = 0; }
        double vx = -ty, vy = tx;
        double n = sqrt(vx * vx + vy * vy);                 /* geom::normalize, ref:132 */
        if (n < 1e-15) { nx[i] = 0; ny[i] = 0; } else { nx[i] = vx / n; ny[i] = vy / n; }
    }
}
/* the `deriv` lambdas of ref:599-613 and ref:625-639 (identical) */
static void deriv(const double* Px, const double* Py, int N, int closed, double h, int i,
                  double* xp, double* yp, double* xpp, double* ypp) {
    if (N == 1) { *xp = 1; *yp = 0; *xpp = *ypp = 0; return; }
    if (closed) {
        int ip = (i + 1) % N, im = (i - 1 + N) % N;
        *xp = (Px[ip] - Px[im]) / (2 * h); *yp = (Py[ip] - Py[im]) / (2 * h);
        *xpp = (Px[ip] - 2 * Px[i] + Px[im]) / (h * h); *ypp = (Py[ip] - 2 * Py[i] + Py[im]) / (h * h);
    } else if (i == 0) {
        *xp = (Px[1] - Px[0]) / h; *yp = (Py[1] - Py[0]) / h;
        if (N >= 3) { *xpp = (Px[2] - 2 * Px[1] + Px[0]) / (h * h); *ypp = (Py[2] - 2 * Py[1] + Py[0]) / (h * h); }
        else *xpp = *ypp = 0;
    } else if (i == N - 1) {
        *xp = (Px[N - 1] - Px[N - 2]) / h; *yp = (Py[N - 1] - Py[N - 2]) / h;
        if (N >= 3) { *xpp = (Px[N - 1] - 2 * Px[N - 2] + Px[N - 3]) / (h * h); *ypp = (Py[N - 1] - 2 * Py[N - 2] + Py[N - 3]) / (h * h); }
        else *xpp = *ypp = 0;
    } else {
        *xp = (Px[i + 1] - Px[i - 1]) / (2 * h); *yp = (Py[i + 1] - Py[i - 1]) / (2 * h);
        *xpp = (Px[i + 1] - 2 * Px[i] + Px[i - 1]) / (h * h); *ypp = (Py[i + 1] - 2 * Py[i] + Py[i - 1]) / (h * h);
    }
}
/* heading_curv_from_points_generic, ref:595-620 */
static void heading_curv(const double* Px, const double* Py, int N, int closed, double h, double* heading, double* kappa) {
    for (int i = 0; i < N; ++i) {
        double xp, yp, xpp, ypp;
        deriv(Px, Py, N, closed, h, i, &xp, &yp, &xpp, &ypp);
        heading[i] = atan2(yp, xp);
        double denom = pow(smax(1e-12, xp * xp + yp * yp), 1.5);
        kappa[i] = (xp * ypp - yp * xpp) / denom;
    }
}
/* precompute_lin_geom_generic, ref:622-651 */
static void lin_geom(const double* Px, const double* Py, const double* nx, const double* ny, int N, int closed,
                     double h, double* A1, double* A2, double* N0, double* W) {
    for (int i = 0; i < N; ++i) {
        double xp, yp, xpp, ypp;
        deriv(Px, Py, N, closed, h, i, &xp, &yp, &xpp, &ypp);
        A1[i] = nx[i] * ypp - ny[i] * xpp;
        A2[i] = xp * ny[i] - yp * nx[i];
        N0[i] = xp * ypp - yp * xpp;
        double denom = pow(smax(1e-12, xp * xp + yp * yp), 1.5);
        W[i] = 1.0 / denom;
    }
}

/* ------------------------------------------------------ difference operators */
typedef struct { int N, closed; double h, invh, inv2h, invh2; } Ops;
static Ops make_ops(int N, double h, int closed) {
    Ops o; o.N = N; o.closed = closed; o.h = h;
    o.invh = 1.0 / h; o.inv2h = 1.0 / (2 * h); o.invh2 = 1.0 / (h * h);   /* ref:547, 562 */
    return o;
}
static inline int wrapi(int i, int N) { i %= N; if (i < 0) i += N; return i; }
/* DiffOps::D1 ref:549-551 / DiffOpsOpen::D1 ref:563-566 */
static void D1(const Ops* o, const double* a, double* out) {
    int N = o->N;
    if (o->closed) {
        for (int i = 0; i < N; ++i) out[i] = (a[wrapi(i + 1, N)] - a[wrapi(i - 1, N)]) * o->inv2h;
        return;
    }
    for (int i = 0; i < N; ++i) out[i] = 0.0;
    if (N == 0) return;
    if (N == 1) { out[0] = 0; return; }
    out[0] = (a[1] - a[0]) * o->invh;
    for (int i = 1; i <= N - 2; ++i) out[i] = (a[i + 1] - a[i - 1]) * o->inv2h;
    out[N - 1] = (a[N - 1] - a[N - 2]) * o->invh;
}
/* DiffOps::D2 ref:552-554 / DiffOpsOpen::D2 ref:573-575 */
static void D2(const Ops* o, const double* a, double* out) {
    int N = o->N;
    if (o->closed) {
        for (int i = 0; i < N; ++i) out[i] = (a[wrapi(i + 1, N)] - 2 * a[i] + a[wrapi(i - 1, N)]) * o->invh2;
        return;
    }
    for (int i = 0; i < N; ++i) out[i] = 0.0;
    if (N <= 2) return;
    for (int i = 1; i <= N - 2; ++i) out[i] = (a[i + 1] - 2 * a[i] + a[i - 1]) * o->invh2;
}
/* DiffOps::D1T ref:555-557 / DiffOpsOpen::D1T ref:567-572 (scatter order kept) */
static void D1T(const Ops* o, const double* v, double* out) {
    int N = o->N;
    if (o->closed) {
        for (int i = 0; i < N; ++i) out[i] = (v[wrapi(i - 1, N)] - v[wrapi(i + 1, N)]) * o->inv2h;
        return;
    }
    for (int i = 0; i < N; ++i) out[i] = 0.0;
    if (N <= 1) return;
    out[0] += (-o->invh) * v[0]; out[1] += (+o->invh) * v[0];
    for (int i = 1; i <= N - 2; ++i) { out[i - 1] += (-o->inv2h) * v[i]; out[i + 1] += (+o->inv2h) * v[i]; }
    out[N - 2] += (-o->invh) * v[N - 1]; out[N - 1] += (+o->invh) * v[N - 1];
}
/* DiffOps::D2T = D2 ref:558 / DiffOpsOpen::D2T ref:576-578 (scatter order kept) */
static void D2T(const Ops* o, const double* v, double* out) {
    int N = o->N;
    if (o->closed) { D2(o, v, out); return; }
    for (int i = 0; i < N; ++i) out[i] = 0.0;
    if (N <= 2) return;
    for (int i = 1; i <= N - 2; ++i) {
        out[i - 1] += (+o->invh2) * v[i]; out[i] += (-2 * o->invh2) * v[i]; out[i + 1] += (+o->invh2) * v[i];
    }
}

/* ----------------------------------------------------------- cost / grad */
typedef struct { double *a1, *a2, *r, *q1, *q2, *g1, *g2, *gsm, *D1a; } Work;

/* eval_cost_grad_frozen ref:654-675 (gamma2==NULL) and
 * eval_cost_grad_timeweighted ref:866-895 (gamma2!=NULL) */
static double cost_grad(const Ops* o, const double* A1, const double* A2, const double* N0, const double* W,
                        const double* gamma2, double lambda, const double* alpha, double* grad, Work* w,
                        double* absJ) {
    int N = o->N;
    D1(o, alpha, w->a1);
    D2(o, alpha, w->a2);
#if ORACLE_FMA
    /* the contracted evaluation of the RL_FMA kernels (checker of that build only) */
    for (int i = 0; i < N; ++i) w->r[i] = W[i] * fma(A2[i], w->a2[i], fma(A1[i], w->a1[i], N0[i]));
#else
    for (int i = 0; i < N; ++i) w->r[i] = W[i] * (N0[i] + A1[i] * w->a1[i] + A2[i] * w->a2[i]);
#endif
    double J = 0;
    if (gamma2) { for (int i = 0; i < N; ++i) J += gamma2[i] * w->r[i] * w->r[i]; }
    else { for (int i = 0; i < N; ++i) J += w->r[i] * w->r[i]; }
    double Jsm = 0;
    for (int i = 0; i < N; ++i) Jsm += w->a1[i] * w->a1[i];
    *absJ = fabs(J) + fabs(lambda) * Jsm;   /* margin report: sum of |terms| (instrumentation) */
    J += lambda * Jsm;
    for (int i = 0; i < N; ++i) {
        double Wz = gamma2 ? W[i] * gamma2[i] * w->r[i] : W[i] * w->r[i];
        w->q1[i] = A1[i] * Wz; w->q2[i] = A2[i] * Wz;
    }
    D1T(o, w->q1, w->g1);
    D2T(o, w->q2, w->g2);
    D1(o, alpha, w->D1a);
    D1T(o, w->D1a, w->gsm);
#if ORACLE_FMA
    for (int i = 0; i < N; ++i) grad[i] = fma(2.0 * lambda, w->gsm[i], 2.0 * (w->g1[i] + w->g2[i]));
#else
    for (int i = 0; i < N; ++i) grad[i] = 2.0 * (w->g1[i] + w->g2[i]) + 2.0 * lambda * w->gsm[i];
#endif
    return J;
}

/* ------------------------------------------------------------- v(s) pass */
typedef struct { double a_acc, a_brk; } AxMax;
/* ax_max_at lambda, ref:797-824 */
static AxMax ax_max_at(const rl_cfg* C, double vi, double ki) {
    double alat = vi * vi * fabs(ki);
    double a_total = C->use_total_ge_lat ? smax(C->a_total_max, C->a_lat_max) : C->a_total_max;
    double a_res = sqrt(smax(0.0, a_total * a_total - alat * alat));
    double Fd = 0.5 * C->rho_air * C->Cd * C->A_front_m2 * vi * vi;
    double Fr = C->mass_kg * 9.81 * C->c_rr;
    double a_power = (C->P_max_W > 0 && vi > 1e-6) ? (C->P_max_W / (C->mass_kg * vi) - (Fd + Fr) / C->mass_kg) : 1e9;
    double a_acc = smin(smin(a_res, C->a_long_acc_cap), a_power);   /* std::min({..}) */
    a_acc = smax(0.0, a_acc);
    double a_brk = smin(a_res, C->a_long_brake_cap) + (Fd + Fr) / C->mass_kg;
    a_brk = smax(0.0, a_brk);
    AxMax r = {a_acc, a_brk};
    return r;
}

/* velocity_profile_forward_backward, ref:782-862.  All max_vpass_iters sweeps
 * are executed as in the reference; *sweeps_changed reports the 1-based index
 * of the first sweep that changed nothing (or max_vpass_iters), which is the
 * number of sweeps an exact early-exiting implementation executes. */
double oracle_vpass(const rl_cfg* C, const double* kappa, int N, double h, int closed,
                    double* v, double* ax, int32_t* sweeps_changed) {
    if (N == 0) { if (sweeps_changed) *sweeps_changed = 0; return 0.0; }
    for (int i = 0; i < N; ++i) v[i] = C->v_cap_mps;
    for (int i = 0; i < N; ++i) {
        double k = fabs(kappa[i]);
        double v_kappa = sqrt(C->a_lat_max / smax(k, C->kappa_eps));
        v[i] = smin(v[i], v_kappa);
    }
    int iters = C->max_vpass_iters, sweep = 0, first_idle = -1;
    while (iters--) {
        int changed = 0;
        ++sweep;
        for (int i = 0; i + 1 < N; ++i) {
            AxMax a = ax_max_at(C, v[i], kappa[i]);
            double vf = sqrt(smax(0.0, v[i] * v[i] + 2.0 * a.a_acc * h));
            double nv = smin(v[i + 1], vf);
            changed |= (nv != v[i + 1]);
            v[i + 1] = nv;
        }
        if (closed) {
            AxMax a = ax_max_at(C, v[N - 1], kappa[N - 1]);
            double vf0 = sqrt(smax(0.0, v[N - 1] * v[N - 1] + 2.0 * a.a_acc * h));
            double nv = smin(v[0], vf0);
            changed |= (nv != v[0]);
            v[0] = nv;
        }
        for (int i = N - 2; i >= 0; --i) {
            AxMax a = ax_max_at(C, v[i + 1], kappa[i + 1]);
            double vb = sqrt(smax(0.0, v[i + 1] * v[i + 1] + 2.0 * a.a_brk * h));
            double nv = smin(v[i], vb);
            changed |= (nv != v[i]);
            v[i] = nv;
        }
        if (closed) {
            AxMax a = ax_max_at(C, v[0], kappa[0]);
            double vbN = sqrt(smax(0.0, v[0] * v[0] + 2.0 * a.a_brk * h));
            double nv = smin(v[N - 1], vbN);
            changed |= (nv != v[N - 1]);
            v[N - 1] = nv;
        }
        if (!changed && first_idle < 0) first_idle = sweep;
    }
    if (sweeps_changed) *sweeps_changed = (first_idle < 0) ? C->max_vpass_iters : first_idle;
    double t = 0.0;
    for (int i = 0; i < N; ++i) {
        int j = (i + 1 < N) ? i + 1 : (closed ? 0 : i);
        double v0 = v[i], v1 = v[j];
        if (ax) ax[i] = (v1 * v1 - v0 * v0) / (2.0 * h);
        t += h / smax(1e-6, v[i]);
    }
    return t;
}

/* ------------------------------------------------------------- drivers */
typedef struct {
    double *Px, *Py, *nx, *ny, *lo, *hi, *alpha, *accum, *last, *anew, *grad, *gnew;
    double *A1, *A2, *N0, *W, *gamma2, *heading, *kappa, *v, *ax;
    Work w;
    double* block;
} State;

static int state_alloc(State* s, int N) {
    int n = N > 0 ? N : 1;
    const int narr = 21 + 9;
    s->block = (double*)malloc(sizeof(double) * (size_t)n * narr);
    if (!s->block) return -1;
    double* p = s->block;
    double** a[] = {&s->Px, &s->Py, &s->nx, &s->ny, &s->lo, &s->hi, &s->alpha, &s->accum, &s->last, &s->anew,
                    &s->grad, &s->gnew, &s->A1, &s->A2, &s->N0, &s->W, &s->gamma2, &s->heading, &s->kappa,
                    &s->v, &s->ax, &s->w.a1, &s->w.a2, &s->w.r, &s->w.q1, &s->w.q2, &s->w.g1, &s->w.g2,
                    &s->w.gsm, &s->w.D1a};
    for (int k = 0; k < narr; ++k) { *a[k] = p; p += n; }
    return 0;
}

/* Decision-margin report (instrumentation, not in the reference).  The kernels compute J
 * and the Armijo decrease from the same per-sample terms in another summation order (per
 * lane, then a butterfly).  Two summations of the same n terms differ by at most
 * 2*gamma(n+3)*sum|terms| (gamma(m) = m*u/(1-m*u), u = 2^-53; +3 covers the rounded
 * products and the lambda*Jsm fold), and the comparison's own additions by a few u of
 * their operands.  A decision whose margin exceeds that bound is taken the same way by any
 * such summation: the report counts the decisions (Armijo tests ref:733 / 1009, stop tests
 * ref:739 / 1022) and the smallest margin/bound ratio seen. */
static double mg_min_ratio = INFINITY;
static int64_t mg_n = 0, mg_below = 0;
void oracle_margin_reset(void) { mg_min_ratio = INFINITY; mg_n = 0; mg_below = 0; }
void oracle_margin_get(double* min_ratio, int64_t* n_decisions, int64_t* n_below) {
    *min_ratio = mg_min_ratio; *n_decisions = mg_n; *n_below = mg_below;
}
static void mg_note(double margin, double bound) {
    ++mg_n;
    /* bound 0: every term is an exact zero, so any summation gives the same zero sums */
    double r = (bound > 0) ? fabs(margin) / bound : INFINITY;
    if (r < mg_min_ratio) mg_min_ratio = r;
    if (r <= 1.0) ++mg_below;
}
static double mg_gamma(int n) { const double u = 0x1p-53; return 2.0 * (n + 3) * u / (1.0 - (n + 3) * u); }

/* compute_min_curvature_raceline ref:683-764 (mintime=0) and
 * compute_min_time_raceline ref:905-1052 (mintime=1), one instance. */
static void run_instance(const rl_problem* pr, const rl_cfg* C, uint64_t seed, int mintime, State* s,
                         rl_out* out, int b) {
    const int N = pr->N;
    const int closed = pr->closed != 0;
    const size_t off = (size_t)b * (size_t)N;
    const int MO = C->max_outer_iters;
    if (out->evals) for (int k = 0; k < MO; ++k) out->evals[(size_t)b * MO + k] = 0;
    if (out->accepts) for (int k = 0; k < MO; ++k) out->accepts[(size_t)b * MO + k] = 0;
    if (mintime && out->vpass_sweeps) for (int k = 0; k <= MO; ++k) out->vpass_sweeps[(size_t)b * (MO + 1) + k] = 0;
    if (N == 0) { if (mintime && out->lap) out->lap[b] = 0.0; return; }  /* ref:689 / 912 */
    const double h = pr->L / (double)N;                                 /* ref:690 / 913 */
    Ops o = make_ops(N, h, closed);
    for (int i = 0; i < N; ++i) { s->Px[i] = pr->center_xy[2 * i]; s->Py[i] = pr->center_xy[2 * i + 1]; }
    normals(s->Px, s->Py, N, closed, s->nx, s->ny);                     /* ref:692 / 915 */
    corridor(s->Px, s->Py, s->nx, s->ny, N, pr, pr->veh_width, C->safety_margin_m, s->lo, s->hi); /* ref:701-711 */
    for (int i = 0; i < N; ++i) {                                        /* ref:720 (+ seed, §8d) */
        s->alpha[i] = (seed == 0) ? 0.0 : smin(s->hi[i], smax(s->lo[i], oracle_seed_value(seed, i, RL_SEED_SIGMA)));
        s->accum[i] = 0.0; s->last[i] = 0.0;
    }
    for (int outer = 0; outer < MO; ++outer) {
        lin_geom(s->Px, s->Py, s->nx, s->ny, N, closed, h, s->A1, s->A2, s->N0, s->W);  /* ref:722 / 941 */
        const double* g2w = NULL;
        if (mintime) {
            heading_curv(s->Px, s->Py, N, closed, h, s->heading, s->kappa);               /* ref:943-944 */
            int32_t sw = 0;
            oracle_vpass(C, s->kappa, N, h, closed, s->v, NULL, &sw);                      /* ref:947 */
            if (out->vpass_sweeps) out->vpass_sweeps[(size_t)b * (MO + 1) + outer] = sw;
            double v_avg = 0.0;                                                            /* ref:951 */
            for (int i = 0; i < N; ++i) v_avg += s->v[i];
            v_avg /= (N > 1 ? N : 1);
            for (int i = 0; i < N; ++i) {                                                  /* ref:954-977 */
                double k = fabs(s->kappa[i]);
                double vkappa = sqrt(C->a_lat_max / smax(k, C->kappa_eps));
                double r = pow(smin(1.0, s->v[i] / smax(1e-6, vkappa)), 2.0);
                r = smin(1.0, smax(0.0, r));
                double corner_w = 1.0 + C->w_time_gain * pow(r, C->time_gamma_power);
                double invv_w = 1.0;
                if (C->time_weight_use_inv_v) {
                    double ratio = v_avg / smax(1e-6, s->v[i]);
                    invv_w = 1.0 + C->inv_v_gain * (ratio - 1.0);
                    if (invv_w < 1.0) invv_w = 1.0;
                    if (invv_w > 3.0) invv_w = 3.0;
                }
                double gamma = corner_w * invv_w;
                s->gamma2[i] = gamma * gamma;
            }
            g2w = s->gamma2;
        }
        double step = C->step_init;                                                        /* ref:723 / 996 */
        double absJ, absJn, absJprev;
        double J = cost_grad(&o, s->A1, s->A2, s->N0, s->W, g2w, C->lambda_smooth, s->alpha, s->grad, &s->w, &absJ);
        int evals = 1, accepts = 0;
        double J_prev = J;
        absJprev = absJ;
        const double gam = mg_gamma(N), u = 0x1p-53;
        for (int it = 0; it < C->max_inner_iters; ++it) {                                  /* ref:727-742 */
            int accepted = 0, bt = 0;
            while (bt < 20) {
                for (int i = 0; i < N; ++i) {
#if ORACLE_FMA
                    double ai = fma(-step, s->grad[i], s->alpha[i]);
#else
                    double ai = s->alpha[i] - step * s->grad[i];
#endif
                    s->anew[i] = smin(s->hi[i], smax(s->lo[i], ai));
                }
                double Jn = cost_grad(&o, s->A1, s->A2, s->N0, s->W, g2w, C->lambda_smooth, s->anew, s->gnew, &s->w,
                                      &absJn);
                ++evals;
                double dec = 0.0, absdec = 0.0;
                for (int i = 0; i < N; ++i) dec += s->grad[i] * (s->anew[i] - s->alpha[i]);
                for (int i = 0; i < N; ++i) absdec += fabs(s->grad[i] * (s->anew[i] - s->alpha[i]));
                {
                    const double cd = C->armijo_c * dec, rhs = J + cd;
                    mg_note(rhs - Jn, gam * (absJn + absJ + fabs(C->armijo_c) * absdec) +
                                          4.0 * u * (fabs(J) + fabs(cd) + fabs(Jn) + fabs(rhs)));
                }
                if (Jn <= J + C->armijo_c * dec) {
                    double* t = s->alpha; s->alpha = s->anew; s->anew = t;
                    t = s->grad; s->grad = s->gnew; s->gnew = t;
                    J = Jn; absJ = absJn; accepted = 1; ++accepts;
                    break;
                }
                step *= 0.5; bt++;
                if (step < C->step_min) break;
            }
            if (!accepted) break;
            mg_note(fabs(J_prev - J) - 1e-10, gam * (absJprev + absJ) + 4.0 * u * (fabs(J_prev) + fabs(J)));
            if (fabs(J_prev - J) < 1e-10) break;
            J_prev = J;
            absJprev = absJ;
        }
        if (out->evals) out->evals[(size_t)b * MO + outer] = evals;
        if (out->accepts) out->accepts[(size_t)b * MO + outer] = accepts;
        for (int i = 0; i < N; ++i) s->last[i] = s->alpha[i];                              /* ref:743 */
        for (int i = 0; i < N; ++i) {                                                      /* ref:745 */
            s->Px[i] += s->nx[i] * s->alpha[i]; s->Py[i] += s->ny[i] * s->alpha[i]; s->accum[i] += s->alpha[i];
        }
        normals(s->Px, s->Py, N, closed, s->nx, s->ny);                                    /* ref:746 */
        corridor(s->Px, s->Py, s->nx, s->ny, N, pr, C->veh_width_m, C->safety_margin_m, s->lo, s->hi); /* ref:749-756 */
        for (int i = 0; i < N; ++i) s->alpha[i] = 0.0;                                     /* ref:757 */
    }
    heading_curv(s->Px, s->Py, N, closed, h, s->heading, s->kappa);                        /* ref:761 / 1046 */
    double lap = 0.0;
    if (mintime) {
        int32_t sw = 0;
        lap = oracle_vpass(C, s->kappa, N, h, closed, s->v, s->ax, &sw);                   /* ref:1047 */
        if (out->vpass_sweeps) out->vpass_sweeps[(size_t)b * (MO + 1) + MO] = sw;
    }
    for (int i = 0; i < N; ++i) {
        if (out->x) out->x[off + i] = s->Px[i];
        if (out->y) out->y[off + i] = s->Py[i];
        if (out->heading) out->heading[off + i] = s->heading[i];
        if (out->kappa) out->kappa[off + i] = s->kappa[i];
        if (out->alpha_total) out->alpha_total[off + i] = s->accum[i];
        if (out->alpha_last) out->alpha_last[off + i] = s->last[i];
        if (mintime) {
            if (out->v) out->v[off + i] = s->v[i];
            if (out->ax) out->ax[off + i] = s->ax[i];
        }
    }
    if (mintime && out->lap) out->lap[b] = lap;
}

/* Same contract as rl_optimize (include/rl_abi.h), CPU, single thread.
 * Instances [b_begin, b_end) only, so callers can time a bounded sample. */
int oracle_optimize_range(const rl_problem* pr, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds,
                          int32_t B, int32_t b_begin, int32_t b_end, rl_out* out_mc, rl_out* out_mt) {
    if (!pr || !cfg || B < 1 || (n_cfg != 1 && n_cfg != B) || pr->N < 0) return RL_EINVAL;
    if (pr->N > 0 && (!pr->center_xy || pr->L <= 0)) return RL_EINVAL;
    if (b_begin < 0 || b_end > B || b_begin > b_end) return RL_EINVAL;
    State s;
    if (state_alloc(&s, pr->N)) return RL_ENOMEM;
    for (int b = b_begin; b < b_end; ++b) {
        const rl_cfg* C = &cfg[n_cfg == 1 ? 0 : b];
        uint64_t seed = seeds ? seeds[b] : 0;
        double* keep[12] = {s.alpha, s.anew, s.grad, s.gnew};
        if (out_mc) run_instance(pr, C, seed, 0, &s, out_mc, b);
        s.alpha = keep[0]; s.anew = keep[1]; s.grad = keep[2]; s.gnew = keep[3];
        if (out_mt) run_instance(pr, C, seed, 1, &s, out_mt, b);
        s.alpha = keep[0]; s.anew = keep[1]; s.grad = keep[2]; s.gnew = keep[3];
    }
    free(s.block);
    return RL_OK;
}

int oracle_optimize(const rl_problem* pr, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds, int32_t B,
                    rl_out* out_mc, rl_out* out_mt) {
    return oracle_optimize_range(pr, cfg, n_cfg, seeds, B, 0, B, out_mc, out_mt);
}

/* The optimisers' first corridor for the path pr->center_xy (ref:692-711): normals,
 * then the corridor block with guard = pr->veh_width*0.5 + safety_margin_m.  Checker
 * of rl_corridor. */
int oracle_corridor(const rl_problem* pr, const rl_cfg* cfg, double* lo, double* hi) {
    const int N = pr->N;
    if (N <= 0) return RL_OK;
    double* b = (double*)malloc(sizeof(double) * 4 * (size_t)N);
    if (!b) return RL_ENOMEM;
    double *Px = b, *Py = b + N, *nx = b + 2 * N, *ny = b + 3 * N;
    for (int i = 0; i < N; ++i) { Px[i] = pr->center_xy[2 * i]; Py[i] = pr->center_xy[2 * i + 1]; }
    normals(Px, Py, N, pr->closed != 0, nx, ny);
    corridor(Px, Py, nx, ny, N, pr, pr->veh_width, cfg->safety_margin_m, lo, hi);
    free(b);
    return RL_OK;
}

/* ---------------------------------------------------------- step 6: geometry */
/* Spline1D::eval_with_deriv, ref:435-445 */
static void spline_eval_d(const rl_spline* sp, double si, double* f, double* fp, double* fpp) {
    const int n = sp->n;
    if (n == 0) { *f = *fp = *fpp = 0; return; }
    if (n == 1) { *f = sp->a[0]; *fp = *fpp = 0; return; }
    int lo = 0, hi = n - 1;
    if (si <= sp->s[0]) lo = 0;
    else if (si >= sp->s[n - 1]) lo = n - 2;
    else { while (hi - lo > 1) { int mid = (lo + hi) >> 1; if (sp->s[mid] <= si) lo = mid; else hi = mid; } }
    double t = si - sp->s[lo];
    *f = sp->a[lo] + sp->b[lo] * t + sp->c[lo] * t * t + sp->d[lo] * t * t * t;
    *fp = sp->b[lo] + 2.0 * sp->c[lo] * t + 3.0 * sp->d[lo] * t * t;
    *fpp = 2.0 * sp->c[lo] + 6.0 * sp->d[lo] * t;
}
/* distancesToRings, ref:513-524: per ring the nearer ray hit along ±n, else the
 * point-to-segment minimum, non-finite -> 0 */
static void dist_to_rings(double Px, double Py, double nx, double ny, const double* in, int Ei,
                          const double* out, int Eo, double* d_in, double* d_out) {
    double di1 = ray_ring(Px, Py, nx, ny, in, Ei), di2 = ray_ring(Px, Py, -nx, -ny, in, Ei);
    *d_in = (isfinite(di1) || isfinite(di2)) ? smin(di1, di2) : min_dist_segs(Px, Py, in, Ei);
    double do1 = ray_ring(Px, Py, nx, ny, out, Eo), do2 = ray_ring(Px, Py, -nx, -ny, out, Eo);
    *d_out = (isfinite(do1) || isfinite(do2)) ? smin(do1, do2) : min_dist_segs(Px, Py, out, Eo);
    if (!isfinite(*d_in)) *d_in = 0.0;
    if (!isfinite(*d_out)) *d_out = 0.0;
}
/* pipeline::compute_geom_and_save rows, ref:1295-1335 (the CSV text is the caller's) */
int oracle_geom(const rl_geom_problem* gp, const rl_cfg* C, double* rows) {
    if (!gp || !C || !rows || gp->Kmax < 0 || gp->denomN == 0) return RL_EINVAL;
    const int Kmax = gp->Kmax;
    double r0[RL_GEOM_COLS] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < Kmax; ++k) {
        double si = gp->s0 + gp->L * ((double)k / (double)gp->denomN);
        double x, xp, xpp, y, yp, ypp;
        spline_eval_d(&gp->spx, si, &x, &xp, &xpp);
        spline_eval_d(&gp->spy, si, &y, &yp, &ypp);
        double heading = atan2(yp, xp);
        double speed2 = xp * xp + yp * yp;
        double denom = pow(smax(1e-12, speed2), 1.5);
        double curv = (xp * ypp - yp * xpp) / denom;
        /* geom::normalize({-yp, xp}, 1e-12), ref:132 */
        double vx = -yp, vy = xp, nn = sqrt(vx * vx + vy * vy), nx = 0.0, ny = 0.0;
        if (!(nn < 1e-12)) { nx = vx / nn; ny = vy / nn; }
        double d_in = 0.0, d_out = 0.0;
        if (nx != 0 || ny != 0) dist_to_rings(x, y, nx, ny, gp->inner_seg, gp->Ei, gp->outer_seg, gp->Eo, &d_in, &d_out);
        double width = d_in + d_out;
        double denom_k = smax(fabs(curv), C->kappa_eps);
        double v_kappa = sqrt(C->a_lat_max / denom_k);
        if (v_kappa > C->v_cap_mps) v_kappa = C->v_cap_mps;
        double* r = rows + RL_GEOM_COLS * k;
        r[0] = si - gp->s0; r[1] = x; r[2] = y; r[3] = heading; r[4] = curv;
        r[5] = d_in; r[6] = d_out; r[7] = width; r[8] = v_kappa;
        if (k == 0) for (int j = 0; j < RL_GEOM_COLS; ++j) r0[j] = r[j];
    }
    if (gp->emit_closed_duplicate) {
        double* r = rows + RL_GEOM_COLS * Kmax;
        for (int j = 0; j < RL_GEOM_COLS; ++j) r[j] = r0[j];
        r[0] = gp->L;
    }
    return Kmax + (gp->emit_closed_duplicate ? 1 : 0);
}

/* CSV rows of a [rows][cols] table with glibc "%.9f" (what std::fixed/precision(9)
 * produces, ref:1303) — the CPU side of the formatter benchmark and checker.
 * Returns the byte count, or -1 if cap is too small. */
long long oracle_format_rows(const double* t, long long rows, int cols, char* out, long long cap) {
    long long n = 0;
    char tmp[64];
    for (long long r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            int k = snprintf(tmp, sizeof tmp, "%.9f", t[r * cols + c]);
            if (n + k + 1 > cap) return -1;
            memcpy(out + n, tmp, (size_t)k);
            n += k;
            out[n++] = (c + 1 < cols) ? ',' : '\n';
        }
    return n;
}

/* edges::ringEdges ref:251-255 / polylineEdges ref:256-260 */
int oracle_ring_segments(const double* ring_xy, int32_t n, int32_t closed, double* seg_out) {
    if (n < 0 || (n > 0 && (!ring_xy || !seg_out))) return RL_EINVAL;
    if (closed) {
        for (int i = 0; i < n; ++i) {
            int j = (i + 1) % n;
            seg_out[4 * i] = ring_xy[2 * i]; seg_out[4 * i + 1] = ring_xy[2 * i + 1];
            seg_out[4 * i + 2] = ring_xy[2 * j]; seg_out[4 * i + 3] = ring_xy[2 * j + 1];
        }
        return n;
    }
    if (n < 2) return 0;
    for (int i = 0; i + 1 < n; ++i) {
        seg_out[4 * i] = ring_xy[2 * i]; seg_out[4 * i + 1] = ring_xy[2 * i + 1];
        seg_out[4 * i + 2] = ring_xy[2 * i + 2]; seg_out[4 * i + 3] = ring_xy[2 * i + 3];
    }
    return n - 1;
}
