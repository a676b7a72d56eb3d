// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Compiles the reference translation unit /root/reference/src/main.cpp AS IT LIES
// (no copy, no patch: REF_MAIN_CPP is passed by oracle/Makefile and `main` is
// renamed with -Dmain=...) and exposes its own functions through a small C
// interface, so that tests/golden/gen_golden.py can:
//   * run the reference steps 1-6 on the bundled cone CSVs and capture the exact
//     (full-precision) inputs of the hot path: center_for_opt, L, s0 and the
//     inner/outer rings (main.cpp:1617-1693);
//   * call raceline_min_curv::compute_min_curvature_raceline (main.cpp:683) and
//     raceline_min_time::compute_min_time_raceline (main.cpp:905) on those inputs
//     with a chosen cfg::Config, and capture every output at full precision.
// Output goes to oracle/_ref/ only (git-ignored).  /root/reference does not
// exist on the GPU box; nothing at GPU run time may depend on this file.
#include REF_MAIN_CPP

#include <cstring>
#include <stdexcept>
#include "../include/rl_abi.h"

namespace {
thread_local std::string g_err;

struct CerrMute {
    std::streambuf* old;
    CerrMute() : old(std::cerr.rdbuf(nullptr)) {}
    ~CerrMute() { std::cerr.rdbuf(old); std::cerr.clear(); }
};

void to_cfg(const rl_cfg* c, cfg::Config& C) {
    C.veh_width_m = c->veh_width_m;
    C.safety_margin_m = c->safety_margin_m;
    C.lambda_smooth = c->lambda_smooth;
    C.max_outer_iters = c->max_outer_iters;
    C.max_inner_iters = c->max_inner_iters;
    C.step_init = c->step_init;
    C.step_min = c->step_min;
    C.armijo_c = c->armijo_c;
    C.kappa_eps = c->kappa_eps;
    C.v_cap_mps = c->v_cap_mps;
    C.mass_kg = c->mass_kg;
    C.Cd = c->Cd;
    C.A_front_m2 = c->A_front_m2;
    C.rho_air = c->rho_air;
    C.c_rr = c->c_rr;
    C.P_max_W = c->P_max_W;
    C.mu = c->mu;
    C.a_total_max = c->a_total_max;
    C.a_lat_max = c->a_lat_max;
    C.a_long_acc_cap = c->a_long_acc_cap;
    C.a_long_brake_cap = c->a_long_brake_cap;
    C.w_time_gain = c->w_time_gain;
    C.time_gamma_power = c->time_gamma_power;
    C.time_weight_use_inv_v = c->time_weight_use_inv_v != 0;
    C.inv_v_gain = c->inv_v_gain;
    C.max_vpass_iters = c->max_vpass_iters;
    C.use_total_ge_lat = c->use_total_ge_lat != 0;
}

void from_cfg(const cfg::Config& C, rl_cfg* c) {
    std::memset(c, 0, sizeof(*c));
    c->veh_width_m = C.veh_width_m;
    c->safety_margin_m = C.safety_margin_m;
    c->lambda_smooth = C.lambda_smooth;
    c->max_outer_iters = C.max_outer_iters;
    c->max_inner_iters = C.max_inner_iters;
    c->step_init = C.step_init;
    c->step_min = C.step_min;
    c->armijo_c = C.armijo_c;
    c->kappa_eps = C.kappa_eps;
    c->v_cap_mps = C.v_cap_mps;
    c->mass_kg = C.mass_kg;
    c->Cd = C.Cd;
    c->A_front_m2 = C.A_front_m2;
    c->rho_air = C.rho_air;
    c->c_rr = C.c_rr;
    c->P_max_W = C.P_max_W;
    c->mu = C.mu;
    c->a_total_max = C.a_total_max;
    c->a_lat_max = C.a_lat_max;
    c->a_long_acc_cap = C.a_long_acc_cap;
    c->a_long_brake_cap = C.a_long_brake_cap;
    c->w_time_gain = C.w_time_gain;
    c->time_gamma_power = C.time_gamma_power;
    c->time_weight_use_inv_v = C.time_weight_use_inv_v ? 1 : 0;
    c->inv_v_gain = C.inv_v_gain;
    c->max_vpass_iters = C.max_vpass_iters;
    c->use_total_ge_lat = C.use_total_ge_lat ? 1 : 0;
}

using geom::Vec2;
using SegVec = vector<pair<Vec2, Vec2>>;

SegVec segs_from(const double* s, int E) {
    SegVec out;
    out.reserve(E);
    for (int e = 0; e < E; ++e) out.push_back({{s[4 * e], s[4 * e + 1]}, {s[4 * e + 2], s[4 * e + 3]}});
    return out;
}
vector<Vec2> pts_from(const double* p, int N) {
    vector<Vec2> out(N);
    for (int i = 0; i < N; ++i) out[i] = {p[2 * i], p[2 * i + 1]};
    return out;
}
}  // namespace

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }

// Reset the reference's global config to its compiled defaults (main.cpp:47-119),
// with logging/debug dumps off.
void ref_cfg_reset() {
    cfg::get() = cfg::Config{};
    cfg::get().verbose = false;
    cfg::get().debug_dump = false;
}
void ref_cfg_get(rl_cfg* out) { from_cfg(cfg::get(), out); }
void ref_cfg_apply(const rl_cfg* c) { to_cfg(c, cfg::get()); }
void ref_set_sampling(int use_dynamic, int samples) {
    cfg::get().use_dynamic_samples = use_dynamic != 0;
    cfg::get().samples = samples;
}
void ref_set_closed(int closed) { cfg::get().is_closed_track = closed != 0; }
void ref_set_debug(int on) { cfg::get().debug_dump = on != 0; }

// heading_curv_from_points_generic + velocity_profile_forward_backward on a path with
// a given h (main.cpp:1466-1478: the debug dump's centreline / min-curvature laps).
int ref_lap_eval(const double* path_xy, int N, double h, int closed, double* heading, double* kappa, double* v,
                 double* ax, double* lap) {
    auto P = pts_from(path_xy, N);
    vector<double> hd, kp;
    raceline_min_curv::heading_curv_from_points_generic(P, h, closed != 0, hd, kp);
    auto VP = raceline_min_time::velocity_profile_forward_backward(kp, h, closed != 0);
    for (int i = 0; i < N; ++i) { heading[i] = hd[i]; kappa[i] = kp[i]; v[i] = VP.v[i]; ax[i] = VP.ax[i]; }
    *lap = VP.lap_time;
    return 0;
}

// Steps 1-6 of main (main.cpp:1617-1693) up to the hot-path inputs.
// Capacities: center_cap points, ring_cap points per ring.  Returns 0 or -1.
int ref_prepare(const char* inner_path, const char* outer_path, const char* out_csv,
                double* center_xy, int center_cap, int* N_out, double* L_out, double* s0_out,
                double* inner_xy, int* Ni_out, double* outer_xy, int* No_out, int ring_cap,
                int* samples_out) {
    CerrMute mute;
    try {
        auto& C = cfg::get();
        const string base = io::dropExt(out_csv);
        auto inner = io::loadCSV_XY(inner_path);
        auto outer = io::loadCSV_XY(outer_path);
        if (inner.size() < 2 || outer.size() < 2) { g_err = "need >=2 points per ring"; return -2; }
        const bool closed_mode = C.is_closed_track;
        auto tri = pipeline::buildDT(inner, outer);
        auto MF = pipeline::extract_mids_with_len_filter(tri, base);
        if (C.use_dynamic_samples) C.samples = pipeline::dynamic_samples_from_mids_count((int)MF.mids.size());
        auto OM = pipeline::order_and_align_mids_open_closed(MF.mids, closed_mode);
        auto RR = pipeline::reconstruct_rings_and_align(OM, MF, tri, base);
        auto CL = pipeline::make_centerline(OM, closed_mode, base);
        vector<Vec2> center_for_opt = CL.center;
        if (closed_mode && center_for_opt.size() >= 2 &&
            geom::almostEq(center_for_opt.front(), center_for_opt.back(), 1e-12))
            center_for_opt.pop_back();
        if ((int)center_for_opt.size() > center_cap || (int)RR.inner_from_mids.size() > ring_cap ||
            (int)RR.outer_from_mids.size() > ring_cap) { g_err = "capacity"; return -3; }
        *N_out = (int)center_for_opt.size();
        for (int i = 0; i < *N_out; ++i) { center_xy[2 * i] = center_for_opt[i].x; center_xy[2 * i + 1] = center_for_opt[i].y; }
        *L_out = CL.L;
        *s0_out = CL.s0;
        *Ni_out = (int)RR.inner_from_mids.size();
        *No_out = (int)RR.outer_from_mids.size();
        for (int i = 0; i < *Ni_out; ++i) { inner_xy[2 * i] = RR.inner_from_mids[i].x; inner_xy[2 * i + 1] = RR.inner_from_mids[i].y; }
        for (int i = 0; i < *No_out; ++i) { outer_xy[2 * i] = RR.outer_from_mids[i].x; outer_xy[2 * i + 1] = RR.outer_from_mids[i].y; }
        *samples_out = C.samples;
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// edges::ringEdges / polylineEdges (main.cpp:251-260) -> [E][4]
int ref_ring_segments(const double* ring_xy, int n, int closed, double* seg_out) {
    auto R = pts_from(ring_xy, n);
    auto E = closed ? edges::ringEdges(R) : edges::polylineEdges(R);
    for (size_t e = 0; e < E.size(); ++e) {
        seg_out[4 * e] = E[e].first.x; seg_out[4 * e + 1] = E[e].first.y;
        seg_out[4 * e + 2] = E[e].second.x; seg_out[4 * e + 3] = E[e].second.y;
    }
    return (int)E.size();
}

// compute_min_curvature_raceline (main.cpp:683).  out_* have N entries each.
int ref_min_curv(const double* center_xy, int N, double L, int closed,
                 const double* inner_seg, int Ei, const double* outer_seg, int Eo, double veh_width,
                 double* x, double* y, double* heading, double* kappa, double* alpha_total, double* alpha_last) {
    CerrMute mute;
    auto res = raceline_min_curv::compute_min_curvature_raceline(
        pts_from(center_xy, N), segs_from(inner_seg, Ei), segs_from(outer_seg, Eo), veh_width, L, closed != 0);
    if ((int)res.raceline.size() != N) { g_err = "size"; return -1; }
    for (int i = 0; i < N; ++i) {
        x[i] = res.raceline[i].x; y[i] = res.raceline[i].y;
        heading[i] = res.heading[i]; kappa[i] = res.curvature[i];
        alpha_total[i] = res.alpha_total[i]; alpha_last[i] = res.alpha_last[i];
    }
    return 0;
}

// compute_min_time_raceline (main.cpp:905).
int ref_min_time(const double* center_xy, int N, double L, int closed,
                 const double* inner_seg, int Ei, const double* outer_seg, int Eo, double veh_width,
                 double* x, double* y, double* heading, double* kappa, double* alpha_total, double* alpha_last,
                 double* v, double* ax, double* lap) {
    CerrMute mute;
    auto res = raceline_min_time::compute_min_time_raceline(
        pts_from(center_xy, N), segs_from(inner_seg, Ei), segs_from(outer_seg, Eo), veh_width, L, closed != 0);
    if ((int)res.raceline.size() != N) { g_err = "size"; return -1; }
    for (int i = 0; i < N; ++i) {
        x[i] = res.raceline[i].x; y[i] = res.raceline[i].y;
        heading[i] = res.heading[i]; kappa[i] = res.curvature[i];
        alpha_total[i] = res.alpha_total[i]; alpha_last[i] = res.alpha_last[i];
        v[i] = res.v[i]; ax[i] = res.ax[i];
    }
    *lap = res.lap_time;
    return 0;
}

// velocity_profile_forward_backward (main.cpp:782) on a given kappa.
int ref_vpass(const double* kappa, int N, double h, int closed, double* v, double* ax, double* lap) {
    vector<double> k(kappa, kappa + N);
    auto VP = raceline_min_time::velocity_profile_forward_backward(k, h, closed != 0);
    for (int i = 0; i < N; ++i) { v[i] = VP.v[i]; ax[i] = VP.ax[i]; }
    *lap = VP.lap_time;
    return 0;
}

// Step 6, compute_geom_and_save (main.cpp:1295-1335), after steps 1-5 exactly as in
// ref_prepare.  Exports the x(s)/y(s) splines (Spline1D s,a,b,c,d; main.cpp:403),
// s0, L, the row count Kmax and the divisor denomN (main.cpp:1308-1309), the rings,
// and full-precision rows [nrows][9] (s_rel,x,y,heading,curvature,d_in,d_out,width,
// v_kappa) computed with the reference's own functions in the reference's order,
// plus the closed-duplicate row when emit_closed_duplicate.  The reference's own
// writer runs as well and leaves <out_csv base>_with_geom.csv next to out_csv.
int ref_geom(const char* inner_path, const char* outer_path, const char* out_csv,
             double* knots, int knot_cap, int* nknots_out, double* s0_out, double* L_out,
             int* Kmax_out, int* denomN_out, int* closed_out,
             double* inner_xy, int* Ni_out, double* outer_xy, int* No_out, int ring_cap,
             double* rows, int row_cap, int* nrows_out) {
    CerrMute mute;
    try {
        auto& C = cfg::get();
        const string base = io::dropExt(out_csv);
        auto inner = io::loadCSV_XY(inner_path);
        auto outer = io::loadCSV_XY(outer_path);
        if (inner.size() < 2 || outer.size() < 2) { g_err = "need >=2 points per ring"; return -2; }
        const bool closed_mode = C.is_closed_track;
        auto tri = pipeline::buildDT(inner, outer);
        auto MF = pipeline::extract_mids_with_len_filter(tri, base);
        if (C.use_dynamic_samples) C.samples = pipeline::dynamic_samples_from_mids_count((int)MF.mids.size());
        auto OM = pipeline::order_and_align_mids_open_closed(MF.mids, closed_mode);
        auto RR = pipeline::reconstruct_rings_and_align(OM, MF, tri, base);
        auto CL = pipeline::make_centerline(OM, closed_mode, base);
        pipeline::compute_geom_and_save(base, CL.center, CL.spx, CL.spy, CL.s0, CL.L, closed_mode,
                                        RR.inner_from_mids, RR.outer_from_mids);
        const int nk = (int)CL.spx.s.size();
        if (nk > knot_cap || (int)CL.spy.s.size() != nk || (int)RR.inner_from_mids.size() > ring_cap ||
            (int)RR.outer_from_mids.size() > ring_cap) { g_err = "capacity"; return -3; }
        const vector<double>* arr[10] = {&CL.spx.s, &CL.spx.a, &CL.spx.b, &CL.spx.c, &CL.spx.d,
                                         &CL.spy.s, &CL.spy.a, &CL.spy.b, &CL.spy.c, &CL.spy.d};
        for (int j = 0; j < 10; ++j)
            for (int i = 0; i < nk; ++i) knots[j * knot_cap + i] = (*arr[j])[i];
        *nknots_out = nk;
        *s0_out = CL.s0;
        *L_out = CL.L;
        const int Ncenter = (int)CL.center.size();
        const int Kmax = closed_mode ? C.samples : Ncenter;
        const int denomN = closed_mode ? C.samples : std::max(1, C.samples);
        *Kmax_out = Kmax;
        *denomN_out = denomN;
        *closed_out = closed_mode ? 1 : 0;
        *Ni_out = (int)RR.inner_from_mids.size();
        *No_out = (int)RR.outer_from_mids.size();
        for (int i = 0; i < *Ni_out; ++i) { inner_xy[2 * i] = RR.inner_from_mids[i].x; inner_xy[2 * i + 1] = RR.inner_from_mids[i].y; }
        for (int i = 0; i < *No_out; ++i) { outer_xy[2 * i] = RR.outer_from_mids[i].x; outer_xy[2 * i + 1] = RR.outer_from_mids[i].y; }
        // the rows, with the reference's functions (main.cpp:1297-1335)
        SegVec innerE = closed_mode ? edges::ringEdges(RR.inner_from_mids) : edges::polylineEdges(RR.inner_from_mids);
        SegVec outerE = closed_mode ? edges::ringEdges(RR.outer_from_mids) : edges::polylineEdges(RR.outer_from_mids);
        const int nrows = Kmax + (C.emit_closed_duplicate ? 1 : 0);
        if (nrows > row_cap) { g_err = "row capacity"; return -3; }
        for (int k = 0; k < Kmax; ++k) {
            double si = CL.s0 + CL.L * (double(k) / double(denomN));
            double x, xp, xpp, y, yp, ypp;
            CL.spx.eval_with_deriv(si, x, xp, xpp);
            CL.spy.eval_with_deriv(si, y, yp, ypp);
            double heading = std::atan2(yp, xp);
            double speed2 = xp * xp + yp * yp;
            double denom = std::pow(std::max(1e-12, speed2), 1.5);
            double curv = (xp * ypp - yp * xpp) / denom;
            Vec2 nvec = geom::normalize(Vec2{-yp, xp}, 1e-12);
            double d_in = 0.0, d_out = 0.0;
            if (nvec.x != 0 || nvec.y != 0) distancesToRings({x, y}, nvec, innerE, outerE, d_in, d_out);
            double width = d_in + d_out;
            double denom_k = std::max(std::fabs(curv), C.kappa_eps);
            double v_kappa = std::sqrt(C.a_lat_max / denom_k);
            if (v_kappa > C.v_cap_mps) v_kappa = C.v_cap_mps;
            double* r = rows + 9 * k;
            r[0] = si - CL.s0; r[1] = x; r[2] = y; r[3] = heading; r[4] = curv;
            r[5] = d_in; r[6] = d_out; r[7] = width; r[8] = v_kappa;
        }
        if (C.emit_closed_duplicate) {
            double* r = rows + 9 * Kmax;
            for (int j = 0; j < 9; ++j) r[j] = (Kmax > 0) ? rows[j] : 0.0;
            r[0] = CL.L;
        }
        *nrows_out = nrows;
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Whole reference CLI (main.cpp:1598) — used to produce the reference's own CSV
// files for the output-format contract fixtures.
int ref_run_cli(const char* inner_path, const char* outer_path, const char* out_csv) {
    CerrMute mute;
    const char* argv[4] = {"fsd_path", inner_path, outer_path, out_csv};
    try {
        return rl_reference_cli_main(4, const_cast<char**>(argv));
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

}  // extern "C"
