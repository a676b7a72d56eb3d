// raceline.cpp — single-file C++17 host for the MI355X raceline optimizer.
//
// Drop-in for steps 7-8 of the reference pipeline (ref = src/main.cpp of
// tjsdn3065/Practice_path_planning_for_formula_student_driverless):
//   * cfg::Config / cfg::get()                    ref:46-121 (same knob names and defaults)
//   * edges::ringEdges / polylineEdges            ref:251-260
//   * io::loadCSV_XY / io::dropExt                ref:267-279, 298
//   * raceline_min_curv::compute_min_curvature_raceline   ref:683   (same signature, same Result)
//   * raceline_min_time::compute_min_time_raceline        ref:905   (same signature, same Result)
//   * pipeline::compute_raceline_and_save / compute_mintime_and_save   ref:1337-1438 (same CSVs)
// The optimisers call the gfx950 kernels through include/rl_abi.h; there is no
// CPU implementation here.
//
// CLI (the reference's step-6 outputs are the inputs):
//   fsd_raceline <centerline.csv> [options]
//     reads <base>.csv (centerline), <base>_inner_from_mids.csv, <base>_outer_from_mids.csv
//     and L from the last row of <base>_with_geom.csv (s = L, ref:1331-1333), pops the
//     closing duplicate (ref:1681-1683) and writes <base>_raceline*.csv and
//     <base>_mintime*.csv exactly like the reference.
//   options: --L <value>  --s0 <value>  --open  --mode mincurv|mintime|both
//            --seeds B   (optimise B α-seeds in one launch; writes <base>_batch_summary.csv)
//            --repeat R  (time R launches of the batch; prints outer-iters/s)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rl_abi.h"

using std::pair;
using std::string;
using std::vector;

// ================================ Config (ref:46-121) =======================
namespace cfg {
struct Config {
    bool is_closed_track = true;
    bool emit_closed_duplicate = true;
    int samples = 300;
    double veh_width_m = 1.0;
    double safety_margin_m = 0.05;
    double lambda_smooth = 1.6e-3;
    int max_outer_iters = 14;
    int max_inner_iters = 120;
    double step_init = 0.65;
    double step_min = 1e-6;
    double armijo_c = 1e-5;
    double kappa_eps = 1e-6;
    double v_cap_mps = 27.0;
    double mass_kg = 255.0;
    double Cd = 0.30;
    double A_front_m2 = 1.00;
    double rho_air = 1.225;
    double c_rr = 0.015;
    double P_max_W = 80000.0;
    double mu = 1.17;
    double a_total_max = mu * 9.81;
    double a_lat_max = 11.0;
    double a_long_acc_cap = 8.0;
    double a_long_brake_cap = 11.0;
    double w_time_gain = 1.0;
    double time_gamma_power = 2.0;
    bool time_weight_use_inv_v = false;
    double inv_v_gain = 0.1;
    int max_vpass_iters = 6;
    bool use_total_ge_lat = true;
    bool verbose = true;
};
inline Config& get() {
    static Config C;
    return C;
}
inline rl_cfg to_abi(const Config& C) {
    rl_cfg c;
    std::memset(&c, 0, sizeof(c));
    c.veh_width_m = C.veh_width_m;
    c.safety_margin_m = C.safety_margin_m;
    c.lambda_smooth = C.lambda_smooth;
    c.max_outer_iters = C.max_outer_iters;
    c.max_inner_iters = C.max_inner_iters;
    c.step_init = C.step_init;
    c.step_min = C.step_min;
    c.armijo_c = C.armijo_c;
    c.kappa_eps = C.kappa_eps;
    c.v_cap_mps = C.v_cap_mps;
    c.mass_kg = C.mass_kg;
    c.Cd = C.Cd;
    c.A_front_m2 = C.A_front_m2;
    c.rho_air = C.rho_air;
    c.c_rr = C.c_rr;
    c.P_max_W = C.P_max_W;
    c.mu = C.mu;
    c.a_total_max = C.a_total_max;
    c.a_lat_max = C.a_lat_max;
    c.a_long_acc_cap = C.a_long_acc_cap;
    c.a_long_brake_cap = C.a_long_brake_cap;
    c.w_time_gain = C.w_time_gain;
    c.time_gamma_power = C.time_gamma_power;
    c.time_weight_use_inv_v = C.time_weight_use_inv_v ? 1 : 0;
    c.inv_v_gain = C.inv_v_gain;
    c.max_vpass_iters = C.max_vpass_iters;
    c.use_total_ge_lat = C.use_total_ge_lat ? 1 : 0;
    return c;
}
}  // namespace cfg

// =============================== Geometry ===================================
namespace geom {
struct Vec2 { double x = 0, y = 0; };
inline bool almostEq(const Vec2& a, const Vec2& b, double e = 1e-12) {
    return std::fabs(a.x - b.x) <= e && std::fabs(a.y - b.y) <= e;
}
}  // namespace geom
using geom::Vec2;
using SegVec = vector<pair<Vec2, Vec2>>;

namespace edges {
inline SegVec ringEdges(const vector<Vec2>& R) {
    SegVec E;
    int n = (int)R.size();
    for (int i = 0; i < n; i++) E.push_back({R[i], R[(i + 1) % n]});
    return E;
}
inline SegVec polylineEdges(const vector<Vec2>& R) {
    SegVec E;
    int n = (int)R.size();
    for (int i = 0; i + 1 < n; i++) E.push_back({R[i], R[i + 1]});
    return E;
}
}  // namespace edges

// =============================== IO (ref:264-299) ==========================
namespace io {
inline vector<Vec2> loadCSV_XY(const string& path) {
    vector<Vec2> pts;
    std::ifstream fin(path);
    if (!fin) { std::cerr << "[ERR] cannot open: " << path << "\n"; return pts; }
    string line;
    while (std::getline(fin, line)) {
        if (line.empty()) continue;
        for (char& ch : line) if (ch == ';' || ch == '\t' || ch == ',') ch = ' ';
        std::istringstream iss(line);
        double x, y;
        if (iss >> x >> y) pts.push_back({x, y});
    }
    return pts;
}
inline string dropExt(const string& s) {
    size_t p = s.find_last_of('.');
    return (p == string::npos) ? s : s.substr(0, p);
}
}  // namespace io

// ============================ ABI glue ======================================
namespace gpu {
inline void check(int rc, const char* what) {
    if (rc != RL_OK) throw std::runtime_error(string(what) + ": " + rl_last_error());
}
struct Packed {
    vector<double> center, inner, outer;
    rl_problem prob;
};
inline Packed pack(const vector<Vec2>& center, const SegVec& innerE, const SegVec& outerE, double veh_width,
                   double L, bool closed) {
    Packed p;
    for (auto& v : center) { p.center.push_back(v.x); p.center.push_back(v.y); }
    for (auto& e : innerE) p.inner.insert(p.inner.end(), {e.first.x, e.first.y, e.second.x, e.second.y});
    for (auto& e : outerE) p.outer.insert(p.outer.end(), {e.first.x, e.first.y, e.second.x, e.second.y});
    std::memset(&p.prob, 0, sizeof(p.prob));
    p.prob.center_xy = p.center.data();
    p.prob.N = (int)center.size();
    p.prob.closed = closed ? 1 : 0;
    p.prob.L = L;
    p.prob.inner_seg = p.inner.data();
    p.prob.Ei = (int)innerE.size();
    p.prob.outer_seg = p.outer.data();
    p.prob.Eo = (int)outerE.size();
    p.prob.veh_width = veh_width;
    return p;
}
}  // namespace gpu

// ======================= Raceline (min-curv), ref:677-764 ===================
namespace raceline_min_curv {
struct Result {
    vector<Vec2> raceline;
    vector<double> heading, curvature;
    vector<double> alpha_total, alpha_last;
};
static Result compute_min_curvature_raceline(const vector<Vec2>& center, const SegVec& innerE, const SegVec& outerE,
                                             double veh_width, double L, bool closed) {
    const int N = (int)center.size();
    if (N == 0) return {};   // ref:689
    auto pk = gpu::pack(center, innerE, outerE, veh_width, L, closed);
    rl_cfg c = cfg::to_abi(cfg::get());
    vector<double> x(N), y(N), hd(N), ka(N), at(N), al(N);
    rl_out o;
    std::memset(&o, 0, sizeof(o));
    o.x = x.data(); o.y = y.data(); o.heading = hd.data(); o.kappa = ka.data();
    o.alpha_total = at.data(); o.alpha_last = al.data();
    gpu::check(rl_optimize(&pk.prob, &c, 1, nullptr, 1, &o, nullptr), "rl_optimize(min-curv)");
    Result r;
    for (int i = 0; i < N; ++i) r.raceline.push_back({x[i], y[i]});
    r.heading = std::move(hd); r.curvature = std::move(ka); r.alpha_total = std::move(at); r.alpha_last = std::move(al);
    return r;
}
}  // namespace raceline_min_curv

// ======================= Raceline (min-time), ref:897-1052 ==================
namespace raceline_min_time {
struct Result {
    vector<Vec2> raceline;
    vector<double> heading, curvature;
    vector<double> alpha_total, alpha_last;
    vector<double> v, ax;
    double lap_time = 0.0;
};
static Result compute_min_time_raceline(const vector<Vec2>& center, const SegVec& innerE, const SegVec& outerE,
                                        double veh_width, double L, bool closed) {
    const int N = (int)center.size();
    if (N == 0) return {};   // ref:912
    auto pk = gpu::pack(center, innerE, outerE, veh_width, L, closed);
    rl_cfg c = cfg::to_abi(cfg::get());
    vector<double> x(N), y(N), hd(N), ka(N), at(N), al(N), v(N), ax(N);
    double lap = 0;
    rl_out o;
    std::memset(&o, 0, sizeof(o));
    o.x = x.data(); o.y = y.data(); o.heading = hd.data(); o.kappa = ka.data();
    o.alpha_total = at.data(); o.alpha_last = al.data(); o.v = v.data(); o.ax = ax.data(); o.lap = &lap;
    gpu::check(rl_optimize(&pk.prob, &c, 1, nullptr, 1, nullptr, &o), "rl_optimize(min-time)");
    Result r;
    for (int i = 0; i < N; ++i) r.raceline.push_back({x[i], y[i]});
    r.heading = std::move(hd); r.curvature = std::move(ka); r.alpha_total = std::move(at); r.alpha_last = std::move(al);
    r.v = std::move(v); r.ax = std::move(ax); r.lap_time = lap;
    return r;
}
}  // namespace raceline_min_time

// =============================== Pipeline ===================================
namespace pipeline {
static void compute_raceline_and_save(const string& base, const vector<Vec2>& center_for_opt, double s0, double L,
                                      bool closed_mode, const vector<Vec2>& inner_from_mids,
                                      const vector<Vec2>& outer_from_mids) {   // ref:1337-1383
    auto& C = cfg::get();
    SegVec innerE = closed_mode ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    SegVec outerE = closed_mode ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    auto res = raceline_min_curv::compute_min_curvature_raceline(center_for_opt, innerE, outerE, C.veh_width_m, L,
                                                                 closed_mode);
    {
        std::ofstream fo(base + "_raceline.csv");
        if (!fo) throw std::runtime_error("save raceline failed");
        fo.setf(std::ios::fixed); fo.precision(9);
        for (auto& p : res.raceline) fo << p.x << "," << p.y << "\n";
        if (C.emit_closed_duplicate && !res.raceline.empty()) fo << res.raceline[0].x << "," << res.raceline[0].y << "\n";
    }
    {
        std::ofstream fo(base + "_raceline_with_geom.csv");
        if (!fo) throw std::runtime_error("save raceline_with_geom failed");
        fo.setf(std::ios::fixed); fo.precision(9);
        fo << "s,x,y,heading_rad,curvature,alpha_last,v_kappa_mps\n";
        int Nrl = (int)res.raceline.size();
        auto vk = [&](double k) {
            double d = std::max(std::fabs(k), C.kappa_eps);
            double v = std::sqrt(C.a_lat_max / d);
            return v > C.v_cap_mps ? C.v_cap_mps : v;
        };
        for (int k = 0; k < Nrl; ++k) {
            double si = s0 + L * (double(k) / double(std::max(1, Nrl)));
            fo << si - s0 << "," << res.raceline[k].x << "," << res.raceline[k].y << "," << res.heading[k] << ","
               << res.curvature[k] << "," << res.alpha_last[k] << "," << vk(res.curvature[k]) << "\n";
        }
        if (C.emit_closed_duplicate && Nrl > 0)
            fo << L << "," << res.raceline[0].x << "," << res.raceline[0].y << "," << res.heading[0] << ","
               << res.curvature[0] << "," << res.alpha_last[0] << "," << vk(res.curvature[0]) << "\n";
    }
}

static void compute_mintime_and_save(const string& base, const vector<Vec2>& center_for_opt, double s0, double L,
                                     bool closed_mode, const vector<Vec2>& inner_from_mids,
                                     const vector<Vec2>& outer_from_mids) {   // ref:1385-1438
    auto& C = cfg::get();
    SegVec innerE = closed_mode ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    SegVec outerE = closed_mode ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    auto res = raceline_min_time::compute_min_time_raceline(center_for_opt, innerE, outerE, C.veh_width_m, L,
                                                            closed_mode);
    {
        std::ofstream fo(base + "_mintime_raceline.csv");
        if (!fo) throw std::runtime_error("save mintime_raceline failed");
        fo.setf(std::ios::fixed); fo.precision(9);
        for (auto& p : res.raceline) fo << p.x << "," << p.y << "\n";
        if (C.emit_closed_duplicate && !res.raceline.empty()) fo << res.raceline[0].x << "," << res.raceline[0].y << "\n";
    }
    {
        std::ofstream fo(base + "_mintime_with_geom.csv");
        if (!fo) throw std::runtime_error("save mintime_with_geom failed");
        fo.setf(std::ios::fixed); fo.precision(9);
        fo << "s,x,y,heading_rad,curvature,alpha_last,v_mps,ax_mps2\n";
        int N = (int)res.raceline.size();
        for (int k = 0; k < N; ++k) {
            double si = s0 + L * (double(k) / double(std::max(1, N)));
            fo << si - s0 << "," << res.raceline[k].x << "," << res.raceline[k].y << "," << res.heading[k] << ","
               << res.curvature[k] << "," << res.alpha_last[k] << "," << res.v[k] << "," << res.ax[k] << "\n";
        }
        if (C.emit_closed_duplicate && N > 0)
            fo << L << "," << res.raceline[0].x << "," << res.raceline[0].y << "," << res.heading[0] << ","
               << res.curvature[0] << "," << res.alpha_last[0] << "," << res.v[0] << "," << res.ax[0] << "\n";
    }
    std::cerr << "[mintime] Estimated laptime: " << std::fixed << std::setprecision(3) << res.lap_time << " s\n";
}

// B α-seeds in one launch (beyond the reference): one summary row per instance.
static void batch_and_save(const string& base, const vector<Vec2>& center, double L, bool closed,
                           const vector<Vec2>& inner_from_mids, const vector<Vec2>& outer_from_mids, int B, int modes,
                           int repeat) {
    auto& C = cfg::get();
    SegVec innerE = closed ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    SegVec outerE = closed ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    auto pk = gpu::pack(center, innerE, outerE, C.veh_width_m, L, closed);
    rl_cfg c = cfg::to_abi(C);
    vector<uint64_t> seeds(B);
    for (int b = 0; b < B; ++b) seeds[b] = (uint64_t)b;
    rl_plan* plan = nullptr;
    gpu::check(rl_plan_create(&plan, 0, &pk.prob, &c, 1, seeds.data(), B, modes), "rl_plan_create");
    gpu::check(rl_plan_run(plan, nullptr), "rl_plan_run");
    const size_t BN = (size_t)B * center.size();
    vector<double> lap(B), al(BN), x(BN), y(BN);
    vector<int32_t> ev((size_t)B * C.max_outer_iters);
    rl_out o;
    std::memset(&o, 0, sizeof(o));
    o.x = x.data(); o.y = y.data(); o.alpha_last = al.data(); o.evals = ev.data();
    const bool mt = modes & RL_MODE_MINTIME;
    if (mt) o.lap = lap.data();
    gpu::check(rl_plan_fetch(plan, mt ? nullptr : &o, mt ? &o : nullptr), "rl_plan_fetch");
    if (repeat > 0) {
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < repeat; ++r) gpu::check(rl_plan_run(plan, nullptr), "rl_plan_run");
        float ms = 0;
        gpu::check(rl_plan_kernel_ms(plan, 0, &ms), "rl_plan_kernel_ms");
        double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        double outers = (double)B * C.max_outer_iters * (mt && (modes & RL_MODE_MINCURV) ? 2 : 1);
        std::cerr << "[batch] B=" << B << " last run " << ms << " ms, " << repeat << " runs " << wall * 1e3
                  << " ms -> " << outers * repeat / wall << " PGD outer-iters/s\n";
    }
    rl_plan_destroy(plan);
    std::ofstream fo(base + "_batch_summary.csv");
    fo.setf(std::ios::fixed); fo.precision(9);
    fo << "seed,lap_time_s,mean_abs_alpha_last,evals_total\n";
    for (int b = 0; b < B; ++b) {
        double s = 0;
        for (size_t i = 0; i < center.size(); ++i) s += std::fabs(al[b * center.size() + i]);
        long et = 0;
        for (int k = 0; k < C.max_outer_iters; ++k) et += ev[(size_t)b * C.max_outer_iters + k];
        fo << b << "," << (mt ? lap[b] : 0.0) << "," << s / std::max<size_t>(1, center.size()) << "," << et << "\n";
    }
}
}  // namespace pipeline

// ================================== MAIN ====================================
static double last_s_of(const string& path) {   // L = s of the closing row (ref:1331-1333)
    std::ifstream f(path);
    string line, last;
    while (std::getline(f, line)) if (!line.empty()) last = line;
    if (last.empty()) return NAN;
    return std::strtod(last.c_str(), nullptr);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::cerr << "Usage: " << argv[0]
                  << " centerline.csv [--L v] [--s0 v] [--open] [--mode mincurv|mintime|both] [--seeds B] [--repeat R]\n";
        return 1;
    }
    auto& C = cfg::get();
    const string outPath = argv[1];
    const string base = io::dropExt(outPath);
    double L = NAN, s0 = 0.0;
    string mode = "both";
    int B = 0, repeat = 0;
    for (int i = 2; i < argc; ++i) {
        string a = argv[i];
        auto next = [&]() -> string { if (i + 1 >= argc) throw std::runtime_error("missing value for " + a); return argv[++i]; };
        if (a == "--L") L = std::stod(next());
        else if (a == "--s0") s0 = std::stod(next());
        else if (a == "--open") C.is_closed_track = false;
        else if (a == "--mode") mode = next();
        else if (a == "--seeds") B = std::stoi(next());
        else if (a == "--repeat") repeat = std::stoi(next());
        else { std::cerr << "unknown option " << a << "\n"; return 1; }
    }
    const bool closed_mode = C.is_closed_track;
    auto center = io::loadCSV_XY(outPath);
    auto inner = io::loadCSV_XY(base + "_inner_from_mids.csv");
    auto outer = io::loadCSV_XY(base + "_outer_from_mids.csv");
    if (std::isnan(L)) L = last_s_of(base + "_with_geom.csv");
    if (center.size() < 2 || inner.size() < 2 || outer.size() < 2 || !(L > 0)) {
        std::cerr << "[ERR] need centerline, inner/outer_from_mids and L (--L or <base>_with_geom.csv)\n";
        return 2;
    }
    vector<Vec2> center_for_opt = center;   // ref:1681-1683
    if (closed_mode && center_for_opt.size() >= 2 && geom::almostEq(center_for_opt.front(), center_for_opt.back(), 1e-12))
        center_for_opt.pop_back();
    try {
        if (B > 0) {
            int modes = (mode == "mincurv" ? RL_MODE_MINCURV : mode == "mintime" ? RL_MODE_MINTIME
                                                                                 : RL_MODE_MINCURV | RL_MODE_MINTIME);
            pipeline::batch_and_save(base, center_for_opt, L, closed_mode, inner, outer, B, modes, repeat);
            return 0;
        }
        auto t0 = std::chrono::steady_clock::now();
        if (mode != "mintime")
            pipeline::compute_raceline_and_save(base, center_for_opt, s0, L, closed_mode, inner, outer);
        auto t1 = std::chrono::steady_clock::now();
        if (mode != "mincurv")
            pipeline::compute_mintime_and_save(base, center_for_opt, s0, L, closed_mode, inner, outer);
        auto t2 = std::chrono::steady_clock::now();
        std::cerr.setf(std::ios::fixed);
        std::cerr << "[TIME][SUMMARY] mincurv_race=" << std::chrono::duration<double, std::milli>(t1 - t0).count()
                  << ", mintime_race=" << std::chrono::duration<double, std::milli>(t2 - t1).count() << "\n";
    } catch (const std::exception& e) {
        std::cerr << "[ERR] " << e.what() << "\n";
        return 3;
    }
    return 0;
}
