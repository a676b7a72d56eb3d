// raceline.cpp — single-file C++17 host for the MI355X raceline optimizer.
//
// A drop-in for the reference CLI (ref = src/main.cpp of
// tjsdn3065/Practice_path_planning_for_formula_student_driverless):
//   fsd_raceline inner.csv outer.csv centerline.csv        (ref:1598-1714, same usage)
// writes every CSV the reference writes, with the same bytes.
//
// Steps 1-5 are host code, as in the reference. They are serial, O(n^2) in the cone
// count and take milliseconds; SURVEY §8f row 4 lists them:
//   * cfg::Config / cfg::get()                          ref:46-121 (same knob names and defaults)
//   * geom:: Vec2, filtered orient2d / incircle         ref:124-171
//   * delaunay::bowyerWatson, edge map                  ref:174-247
//   * edges::ringEdges / polylineEdges                  ref:251-260
//   * io:: loadCSV_XY and the CSV savers                ref:264-299
//   * centerline:: boundary edges, MST ordering, natural cubic spline, uniform resample
//                                                      ref:300-474
//   * pipeline:: buildDT, extract_mids_with_len_filter, order_and_align_mids_open_closed,
//     reconstruct_rings_and_align, dynamic_samples_from_mids_count, make_centerline,
//     save_centerline_csv                              ref:1060-1286
// The GPU runs the rest through include/rl_abi.h. There is no CPU path behind these calls:
//   * step 6   pipeline::compute_geom_and_save          ref:1288-1335  -> rl_geom
//   * step 7   raceline_min_curv::compute_min_curvature_raceline ref:683 -> rl_optimize
//   * step 8   raceline_min_time::compute_min_time_raceline      ref:905 -> rl_optimize
//   * pipeline::compute_raceline_and_save / compute_mintime_and_save  ref:1337-1593
//     (the debug dump's centreline and min-curvature laps go through rl_lap_eval)
//
// Every restated host function keeps the reference's operations in the reference's
// order. Its containers are libstdc++'s (unordered_map iteration order, nth_element,
// mt19937_64 + uniform_real_distribution), so the intermediate CSVs are byte-identical.
// tests/test_host_cli.py checks this against the reference CLI's own files.
//
// Other modes:
//   fsd_raceline <centerline.csv> [options]     the reference's step-6 outputs are the inputs:
//     reads <base>.csv, <base>_inner_from_mids.csv, <base>_outer_from_mids.csv and L from the
//     last row of <base>_with_geom.csv (s = L, ref:1331-1333), then runs steps 7-8.
// options (both modes):
//   --set key=value   override any cfg::Config knob (e.g. --set samples=2000
//                     --set use_dynamic_samples=0 --set is_closed_track=0)
//   --stop-after centerline   run steps 1-5 only and write their CSVs (no GPU is touched)
//   --mode mincurv|mintime|both   --L v  --s0 v  --open
//   --seeds B   optimise B α-seeds in one launch; writes <base>_batch_summary.csv
//   --repeat R  time R launches of the batch; prints outer-iters/s
//   --device D  HIP device
//   --devices 0,1,...  shard the --seeds batch over these devices: contiguous instance
//               blocks, one plan/stream per device, results gathered to the host
//               (rl_optimize_multi; --repeat then times whole calls, PCIe included)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <queue>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "rl_abi.h"

using std::pair;
using std::string;
using std::vector;

// ================================ Config (ref:46-121) =======================
namespace cfg {
struct Config {
    // anchors (ref:49-52)
    double current_pos_x = 4.994457593, current_pos_y = -0.108866966;
    double current_heading_rad = 0.046698693;
    double start_anchor_x = 0.0, start_anchor_y = 0.0;
    double start_heading_rad = 0.0;
    bool is_closed_track = true;
    bool emit_closed_duplicate = true;
    bool force_closed_ccw = false;
    // triangulation (ref:60-61)
    bool add_micro_jitter = true;
    double jitter_eps = 1e-9;
    // sampling / ordering (ref:64-69)
    int samples = 300;
    bool use_dynamic_samples = true;
    double sample_factor_n = 1.1;
    int samples_min = 10;
    int samples_max = 1000;
    int knn_k = 6;
    // boundary-edge length filter (ref:72-74)
    bool enable_boundary_len_filter = true;
    double boundary_edge_len_scale = 1.5;
    double boundary_edge_abs_max = 5.5;
    // optimiser and vehicle (ref:77-113)
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
    // logging / debug (ref:116-118)
    bool verbose = true;
    bool debug_dump = true;
    double debug_offset_warn_m = 0.04;
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
// --set key=value. The reference configures by recompiling, so this has no reference
// counterpart. `mu` recomputes a_total_max = mu*9.81, the way a recompiled reference would
// (ref:102).
inline bool set_knob(Config& C, const string& kv) {
    const size_t eq = kv.find('=');
    if (eq == string::npos) return false;
    const string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    const double d = std::strtod(v.c_str(), nullptr);
    const bool b = !(v == "0" || v == "false");
    std::map<string, double*> dk = {
        {"current_pos_x", &C.current_pos_x}, {"current_pos_y", &C.current_pos_y},
        {"current_heading_rad", &C.current_heading_rad}, {"start_anchor_x", &C.start_anchor_x},
        {"start_anchor_y", &C.start_anchor_y}, {"start_heading_rad", &C.start_heading_rad},
        {"jitter_eps", &C.jitter_eps}, {"sample_factor_n", &C.sample_factor_n},
        {"boundary_edge_len_scale", &C.boundary_edge_len_scale}, {"boundary_edge_abs_max", &C.boundary_edge_abs_max},
        {"veh_width_m", &C.veh_width_m}, {"safety_margin_m", &C.safety_margin_m}, {"lambda_smooth", &C.lambda_smooth},
        {"step_init", &C.step_init}, {"step_min", &C.step_min}, {"armijo_c", &C.armijo_c}, {"kappa_eps", &C.kappa_eps},
        {"v_cap_mps", &C.v_cap_mps}, {"mass_kg", &C.mass_kg}, {"Cd", &C.Cd}, {"A_front_m2", &C.A_front_m2},
        {"rho_air", &C.rho_air}, {"c_rr", &C.c_rr}, {"P_max_W", &C.P_max_W}, {"a_total_max", &C.a_total_max},
        {"a_lat_max", &C.a_lat_max}, {"a_long_acc_cap", &C.a_long_acc_cap}, {"a_long_brake_cap", &C.a_long_brake_cap},
        {"w_time_gain", &C.w_time_gain}, {"time_gamma_power", &C.time_gamma_power}, {"inv_v_gain", &C.inv_v_gain},
        {"debug_offset_warn_m", &C.debug_offset_warn_m}};
    std::map<string, int*> ik = {{"samples", &C.samples}, {"samples_min", &C.samples_min},
                                 {"samples_max", &C.samples_max}, {"knn_k", &C.knn_k},
                                 {"max_outer_iters", &C.max_outer_iters}, {"max_inner_iters", &C.max_inner_iters},
                                 {"max_vpass_iters", &C.max_vpass_iters}};
    std::map<string, bool*> bk = {
        {"is_closed_track", &C.is_closed_track}, {"emit_closed_duplicate", &C.emit_closed_duplicate},
        {"force_closed_ccw", &C.force_closed_ccw}, {"add_micro_jitter", &C.add_micro_jitter},
        {"use_dynamic_samples", &C.use_dynamic_samples}, {"enable_boundary_len_filter", &C.enable_boundary_len_filter},
        {"time_weight_use_inv_v", &C.time_weight_use_inv_v}, {"use_total_ge_lat", &C.use_total_ge_lat},
        {"verbose", &C.verbose}, {"debug_dump", &C.debug_dump}};
    if (k == "mu") { C.mu = d; C.a_total_max = d * 9.81; return true; }
    if (dk.count(k)) { *dk[k] = d; return true; }
    if (ik.count(k)) { *ik[k] = (int)std::strtol(v.c_str(), nullptr, 10); return true; }
    if (bk.count(k)) { *bk[k] = b; return true; }
    return false;
}
}  // namespace cfg

// =============================== Geometry (ref:124-171) =====================
namespace geom {
struct Vec2 { double x = 0, y = 0; };
inline Vec2 operator+(const Vec2& p, const Vec2& q) { return {p.x + q.x, p.y + q.y}; }
inline Vec2 operator-(const Vec2& p, const Vec2& q) { return {p.x - q.x, p.y - q.y}; }
inline Vec2 operator*(const Vec2& p, double s) { return {p.x * s, p.y * s}; }
inline double dot(const Vec2& p, const Vec2& q) { return p.x * q.x + p.y * q.y; }
inline double norm(const Vec2& p) { return std::sqrt(dot(p, p)); }
inline Vec2 normalize(const Vec2& v, double eps = 1e-12) {
    const double len = norm(v);
    if (len < eps) return Vec2{0, 0};
    return Vec2{v.x / len, v.y / len};
}
inline bool almostEq(const Vec2& a, const Vec2& b, double e = 1e-12) {
    return std::fabs(a.x - b.x) <= e && std::fabs(a.y - b.y) <= e;
}
inline Vec2 heading_dir(double rad) { return {std::cos(rad), std::sin(rad)}; }   // ref:525

// Sign of the orientation determinant. The double value is used when it clears the
// static error bound 4·eps·|ab|₁|ac|₁; otherwise x87 long double is used (ref:141-153).
inline double orient2d_filt(const Vec2& a, const Vec2& b, const Vec2& c) {
    const double ux = b.x - a.x, uy = b.y - a.y, wx = c.x - a.x, wy = c.y - a.y;
    const double det = ux * wy - uy * wx;
    const double bound = ((std::fabs(ux) + std::fabs(uy)) * (std::fabs(wx) + std::fabs(wy))) *
                         std::numeric_limits<double>::epsilon() * 4.0;
    if (std::fabs(det) > bound) return det;
    const long double lux = (long double)b.x - (long double)a.x, luy = (long double)b.y - (long double)a.y;
    const long double lwx = (long double)c.x - (long double)a.x, lwy = (long double)c.y - (long double)a.y;
    return (double)(lux * lwy - luy * lwx);
}
// In-circle determinant of d against the circle (a,b,c), lifted about d. The static
// bound is 16·eps; the fallback uses long double (ref:154-168).
inline double incircle_filt(const Vec2& a, const Vec2& b, const Vec2& c, const Vec2& d) {
    const double ax = a.x - d.x, ay = a.y - d.y, bx = b.x - d.x, by = b.y - d.y, cx = c.x - d.x, cy = c.y - d.y;
    const double la = ax * ax + ay * ay, lb = bx * bx + by * by, lc = cx * cx + cy * cy;
    const double det = ax * (by * lc - lb * cy) - ay * (bx * lc - lb * cx) + la * (bx * cy - by * cx);
    const double mags =
        (std::fabs(ax) + std::fabs(ay)) * (std::fabs(bx) + std::fabs(by)) * (std::fabs(cx) + std::fabs(cy));
    if (std::fabs(det) > mags * std::numeric_limits<double>::epsilon() * 16.0) return det;
    typedef long double LD;
    const LD Ax = (LD)a.x - (LD)d.x, Ay = (LD)a.y - (LD)d.y, Bx = (LD)b.x - (LD)d.x, By = (LD)b.y - (LD)d.y,
             Cx = (LD)c.x - (LD)d.x, Cy = (LD)c.y - (LD)d.y;
    const LD La = Ax * Ax + Ay * Ay, Lb = Bx * Bx + By * By, Lc = Cx * Cx + Cy * Cy;
    return (double)(Ax * (By * Lc - Lb * Cy) - Ay * (Bx * Lc - Lb * Cx) + La * (Bx * Cy - By * Cx));
}
inline bool ccw(const Vec2& a, const Vec2& b, const Vec2& c) { return orient2d_filt(a, b, c) > 0; }
}  // namespace geom
using geom::Vec2;
using SegVec = vector<pair<Vec2, Vec2>>;

// ============================ Delaunay (ref:174-247) ========================
namespace delaunay {
struct Tri { int a, b, c; };   // counter-clockwise once touched

// Incremental Bowyer-Watson over the cones. The caller's points get a deterministic
// micro-jitter (mt19937_64 seeded 1234567, U(-eps, eps) to x then y). A super-triangle
// is scaled 1000x the bounding box. Returns the triangles whose three vertices are all
// real points (ref:179-232).
static vector<Tri> bowyerWatson(const vector<Vec2>& pts) {
    const auto& C = cfg::get();
    vector<Vec2> P(pts);
    if (C.add_micro_jitter) {
        std::mt19937_64 gen(1234567);
        std::uniform_real_distribution<double> jit(-C.jitter_eps, C.jitter_eps);
        for (Vec2& p : P) {
            p.x += jit(gen);
            p.y += jit(gen);
        }
    }
    Vec2 bmin{+1e300, +1e300}, bmax{-1e300, -1e300};
    for (const Vec2& p : P) {
        bmin.x = std::min(bmin.x, p.x);
        bmin.y = std::min(bmin.y, p.y);
        bmax.x = std::max(bmax.x, p.x);
        bmax.y = std::max(bmax.y, p.y);
    }
    const Vec2 mid{(bmin.x + bmax.x) * 0.5, (bmin.y + bmax.y) * 0.5};
    const double span = std::max(bmax.x - bmin.x, bmax.y - bmin.y) * 1000.0 + 1.0;
    const int nreal = (int)P.size();
    P.push_back({mid.x - 2 * span, mid.y - span});
    P.push_back({mid.x + 2 * span, mid.y - span});
    P.push_back({mid.x, mid.y + 2 * span});

    vector<Tri> tris{Tri{nreal, nreal + 1, nreal + 2}};
    struct HalfEdge { int u, v; };
    for (int ip = 0; ip < nreal; ++ip) {
        const Vec2& q = P[ip];
        // cavity: triangles whose circumcircle strictly contains q (orientation fixed in place)
        vector<int> cavity;
        cavity.reserve(tris.size() / 3);
        for (int t = 0; t < (int)tris.size(); ++t) {
            Tri& tr = tris[t];
            if (!geom::ccw(P[tr.a], P[tr.b], P[tr.c])) std::swap(tr.b, tr.c);
            if (geom::incircle_filt(P[tr.a], P[tr.b], P[tr.c], q) > 0) cavity.push_back(t);
        }
        // cavity boundary: a half-edge cancels against its twin, order of first appearance kept
        vector<HalfEdge> rim;
        auto toggle = [&rim](int u, int v) {
            for (auto it = rim.begin(); it != rim.end(); ++it)
                if (it->u == v && it->v == u) { rim.erase(it); return; }
            rim.push_back({u, v});
        };
        vector<char> gone(tris.size(), 0);
        for (int t : cavity) {
            gone[t] = 1;
            const Tri tr = tris[t];
            toggle(tr.a, tr.b);
            toggle(tr.b, tr.c);
            toggle(tr.c, tr.a);
        }
        vector<Tri> next;
        next.reserve(tris.size());
        for (int t = 0; t < (int)tris.size(); ++t)
            if (!gone[t]) next.push_back(tris[t]);
        tris.swap(next);
        for (const HalfEdge& e : rim) {
            Tri nt{e.u, e.v, ip};
            if (!geom::ccw(P[nt.a], P[nt.b], P[nt.c])) std::swap(nt.b, nt.c);
            tris.push_back(nt);
        }
    }
    vector<Tri> real;
    real.reserve(tris.size());
    for (const Tri& t : tris)
        if (t.a < nreal && t.b < nreal && t.c < nreal) real.push_back(t);
    return real;
}

// Undirected edge -> the triangles using it. Hash, reserve and insertion order follow
// ref:234-246, so that libstdc++ iterates the map in the same order.
struct EdgeKey {
    int u, v;
    EdgeKey() {}
    EdgeKey(int a, int b) { u = std::min(a, b); v = std::max(a, b); }
    bool operator==(const EdgeKey& o) const { return u == o.u && v == o.v; }
};
struct EdgeKeyHash {
    size_t operator()(const EdgeKey& k) const { return ((uint64_t)k.u << 32) ^ (uint64_t)k.v; }
};
struct EdgeRef { int tri; int a, b; };
using EdgeMap = std::unordered_map<EdgeKey, vector<EdgeRef>, EdgeKeyHash>;

inline void buildEdgeMap(const vector<Tri>& T, EdgeMap& M) {
    M.clear();
    M.reserve(T.size() * 2);
    for (int t = 0; t < (int)T.size(); ++t) {
        const int v3[3] = {T[t].a, T[t].b, T[t].c};
        for (int i = 0; i < 3; ++i) M[EdgeKey(v3[i], v3[(i + 1) % 3])].push_back({t, v3[i], v3[(i + 1) % 3]});
    }
}
}  // namespace delaunay

// =========================== Edge helpers (ref:251-260) =====================
namespace edges {
inline SegVec ringEdges(const vector<Vec2>& R) {
    SegVec E;
    const int n = (int)R.size();
    E.reserve(n);
    for (int i = 0; i < n; i++) E.push_back({R[i], R[(i + 1) % n]});
    return E;
}
inline SegVec polylineEdges(const vector<Vec2>& R) {
    SegVec E;
    const int n = (int)R.size();
    for (int i = 0; i + 1 < n; i++) E.push_back({R[i], R[i + 1]});
    return E;
}
}  // namespace edges

// =============================== IO (ref:264-299) ==========================
namespace io {
// one point per line; ',', ';' and tab separate fields; unparsable lines are skipped
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
// every CSV of the reference is std::fixed + precision(9) (= glibc "%.9f")
struct Csv {
    std::ofstream f;
    explicit Csv(const string& path) : f(path) {
        f.setf(std::ios::fixed);
        f.precision(9);
    }
    explicit operator bool() const { return (bool)f; }
};
inline bool saveCSV_pointsXY(const string& path, const vector<Vec2>& pts) {
    Csv o(path);
    if (!o) { std::cerr << "[ERR] write failed: " << path << "\n"; return false; }
    for (const Vec2& p : pts) o.f << p.x << "," << p.y << "\n";
    return true;
}
inline bool saveCSV_pointsLabeled(const string& path, const vector<Vec2>& pts, const vector<int>& label) {
    Csv o(path);
    if (!o) { std::cerr << "[ERR] write failed: " << path << "\n"; return false; }
    o.f << "id,x,y,label\n";
    for (size_t i = 0; i < pts.size(); ++i) o.f << i << "," << pts[i].x << "," << pts[i].y << "," << label[i] << "\n";
    return true;
}
inline bool saveCSV_edgesIdx(const string& path, const vector<pair<int, int>>& E) {
    std::ofstream f(path);
    if (!f) { std::cerr << "[ERR] write failed: " << path << "\n"; return false; }
    for (const auto& e : E) f << e.first << "," << e.second << "\n";
    return true;
}
inline bool saveCSV_trisIdx(const string& path, const vector<delaunay::Tri>& T) {
    std::ofstream f(path);
    if (!f) { std::cerr << "[ERR] write failed: " << path << "\n"; return false; }
    for (const auto& t : T) f << t.a << "," << t.b << "," << t.c << "\n";
    return true;
}
inline string dropExt(const string& s) {
    const size_t p = s.find_last_of('.');
    return (p == string::npos) ? s : s.substr(0, p);
}
}  // namespace io

// ============================ Centerline (ref:300-474) ======================
namespace centerline {
using delaunay::Tri;

struct BoundaryEdgeInfo {
    int u, v;
    double len;
    bool is_hull;
    Vec2 mid;
};

// Triangle edges joining an inner cone to an outer cone, in edge-map order (ref:307-327)
inline vector<BoundaryEdgeInfo> labelBoundaryEdges_with_len(const vector<Vec2>& all, const delaunay::EdgeMap& M,
                                                            const vector<int>& labels) {
    vector<BoundaryEdgeInfo> out;
    out.reserve(M.size());
    const int n = (int)all.size();
    for (const auto& kv : M) {
        const int u = kv.first.u, v = kv.first.v;
        if (u < 0 || v < 0 || u >= n || v >= n) continue;
        if (labels[u] < 0 || labels[v] < 0 || labels[u] == labels[v]) continue;
        out.push_back({u, v, geom::norm(all[v] - all[u]), kv.second.size() == 1, (all[u] + all[v]) * 0.5});
    }
    return out;
}

// Orders the midpoints along the track (ref:329-383):
//  1. a k-nearest-neighbour graph with Euclidean weights (nth_element on squared distance);
//  2. its Prim MST from vertex 0;
//  3. the tree's diameter path by two BFS sweeps, with hypot lengths;
//  4. off-path vertices appended in index order.
// Also returns the index permutation. The reference recomputes it by nearest matching
// (orderIndicesByMST, ref:385-401); that matching is run here on the same ordering.
inline vector<Vec2> orderByMST(const vector<Vec2>& pts) {
    const int n = (int)pts.size();
    if (n <= 2) return pts;
    const int K = std::min(cfg::get().knn_k, n - 1);
    vector<vector<pair<int, double>>> adj(n);
    for (int i = 0; i < n; i++) {
        vector<pair<double, int>> near;
        near.reserve(n - 1);
        for (int j = 0; j < n; j++) {
            if (j == i) continue;
            const double dx = pts[i].x - pts[j].x, dy = pts[i].y - pts[j].y;
            near.push_back({dx * dx + dy * dy, j});
        }
        if ((int)near.size() > K) {
            std::nth_element(near.begin(), near.begin() + K, near.end(),
                             [](const pair<double, int>& p, const pair<double, int>& q) { return p.first < q.first; });
            near.resize(K);
        }
        for (const auto& c : near) {
            const double w = std::sqrt(std::max(0.0, c.first));
            adj[i].push_back({c.second, w});
            adj[c.second].push_back({i, w});
        }
    }
    // Prim, O(n^2) selection (first minimum wins)
    vector<double> key(n, 1e300);
    vector<int> parent(n, -1);
    vector<char> done(n, 0);
    key[0] = 0;
    for (int it = 0; it < n; ++it) {
        int u = -1;
        double best = 1e301;
        for (int i = 0; i < n; i++)
            if (!done[i] && key[i] < best) { best = key[i]; u = i; }
        if (u < 0) break;
        done[u] = 1;
        for (const auto& e : adj[u])
            if (!done[e.first] && e.second < key[e.first]) { key[e.first] = e.second; parent[e.first] = u; }
    }
    vector<vector<int>> tree(n);
    for (int v = 0; v < n; v++)
        if (parent[v] >= 0) { tree[v].push_back(parent[v]); tree[parent[v]].push_back(v); }
    // BFS over the tree: distances (1e300 = unreached) and the farthest vertex (first max)
    auto sweep = [&](int src, vector<int>& from) {
        vector<double> dist(n, 1e300);
        from.assign(n, -1);
        std::queue<int> q;
        q.push(src);
        dist[src] = 0;
        while (!q.empty()) {
            const int u = q.front();
            q.pop();
            for (int v : tree[u]) {
                if (!(dist[v] > 1e299)) continue;
                dist[v] = dist[u] + std::hypot(pts[u].x - pts[v].x, pts[u].y - pts[v].y);
                from[v] = u;
                q.push(v);
            }
        }
        int far = src;
        for (int i = 0; i < n; i++)
            if (dist[i] > dist[far]) far = i;
        return far;
    };
    vector<int> from;
    const int end1 = sweep(0, from);
    const int end2 = sweep(end1, from);
    vector<char> used(n, 0);
    vector<Vec2> out;
    out.reserve(n);
    for (int v = end2; v != -1; v = from[v]) { out.push_back(pts[v]); used[v] = 1; }
    for (int i = 0; i < n; i++)
        if (!used[i]) out.push_back(pts[i]);
    return out;
}

// indices of `ordered` in `pts` by greedy nearest matching (ref:385-401)
inline vector<int> matchIndices(const vector<Vec2>& pts, const vector<Vec2>& ordered) {
    vector<int> idx;
    idx.reserve(pts.size());
    vector<char> taken(pts.size(), 0);
    for (const Vec2& p : ordered) {
        int pick = -1;
        double best = 1e300;
        for (int i = 0; i < (int)pts.size(); ++i) {
            if (taken[i]) continue;
            const double dx = pts[i].x - p.x, dy = pts[i].y - p.y, d2 = dx * dx + dy * dy;
            if (d2 < best) { best = d2; pick = i; }
        }
        if (pick < 0) pick = 0;
        taken[pick] = 1;
        idx.push_back(pick);
    }
    return idx;
}

// Natural cubic spline y(s) = a + b t + c t^2 + d t^3 on [s_i, s_{i+1}) (ref:403-446).
// The tridiagonal elimination weights row i with dl[i-1]/dm[i-1], as the reference does.
struct Spline1D {
    vector<double> s, a, b, c, d;
    void fit(const vector<double>& knots, const vector<double>& y) {
        const int n = (int)knots.size();
        s = knots;
        a = y;
        b.assign(n, 0.0);
        c.assign(n, 0.0);
        d.assign(n, 0.0);
        if (n < 3) {
            if (n == 2) b[0] = (a[1] - a[0]) / std::max(1e-30, s[1] - s[0]);
            return;
        }
        vector<double> h(n - 1);
        for (int i = 0; i + 1 < n; ++i) h[i] = std::max(1e-30, s[i + 1] - s[i]);
        const int m = n - 2;
        vector<double> lo(m), dg(m), up(m), r(m);
        for (int i = 1; i <= m; ++i) {
            lo[i - 1] = h[i - 1];
            dg[i - 1] = 2.0 * (h[i - 1] + h[i]);
            up[i - 1] = h[i];
            r[i - 1] = 3.0 * ((a[i + 1] - a[i]) / h[i] - (a[i] - a[i - 1]) / h[i - 1]);
        }
        for (int i = 1; i < m; ++i) {
            const double w = lo[i - 1] / dg[i - 1];
            dg[i] -= w * up[i - 1];
            r[i] -= w * r[i - 1];
        }
        r[m - 1] /= dg[m - 1];
        for (int i = m - 2; i >= 0; --i) r[i] = (r[i] - up[i] * r[i + 1]) / dg[i];
        for (int i = 1; i <= m; ++i) c[i] = r[i - 1];
        c[0] = 0.0;
        c[n - 1] = 0.0;
        for (int i = 0; i + 1 < n; ++i) {
            b[i] = (a[i + 1] - a[i]) / h[i] - (2.0 * c[i] + c[i + 1]) * h[i] / 3.0;
            d[i] = (c[i + 1] - c[i]) / (3.0 * h[i]);
        }
    }
    int piece(double si) const {   // clamped binary search (ref:422-425)
        const int n = (int)s.size();
        if (si <= s.front()) return 0;
        if (si >= s.back()) return n - 2;
        int lo = 0, hi = n - 1;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s[mid] <= si) lo = mid;
            else hi = mid;
        }
        return lo;
    }
    double eval(double si) const {
        const int n = (int)s.size();
        if (n == 0) return 0.0;
        if (n == 1) return a[0];
        const int k = piece(si);
        const double t = si - s[k];
        return a[k] + b[k] * t + c[k] * t * t + d[k] * t * t * t;
    }
};

// Pads the ordered midpoints with paddingK wrapped points per side and parametrises by
// chord length. Fits x(s) and y(s), then samples `samples` points uniformly over the
// unpadded span. Returns the input unchanged when it has fewer than 3 points
// (ref:448-474).
inline vector<Vec2> splineUniformResample(const vector<Vec2>& ordered, int samples, int paddingK, bool close_loop,
                                          Spline1D& spx_out, Spline1D& spy_out, double& s0_out, double& L_out) {
    const int n = (int)ordered.size();
    if (n < 3) return ordered;
    vector<Vec2> P;
    P.reserve(n + 2 * paddingK);
    for (int i = 0; i < paddingK; ++i) P.push_back(ordered[n - paddingK + i]);
    P.insert(P.end(), ordered.begin(), ordered.end());
    for (int i = 0; i < paddingK; ++i) P.push_back(ordered[i]);
    const int M = (int)P.size();
    vector<double> s(M, 0.0), xs(M), ys(M);
    for (int i = 1; i < M; ++i) {
        const double dx = P[i].x - P[i - 1].x, dy = P[i].y - P[i - 1].y;
        s[i] = s[i - 1] + std::sqrt(dx * dx + dy * dy);
    }
    for (int i = 0; i < M; ++i) { xs[i] = P[i].x; ys[i] = P[i].y; }
    Spline1D spx, spy;
    spx.fit(s, xs);
    spy.fit(s, ys);
    const double s0 = s[paddingK], L = std::max(1e-30, s[M - paddingK - 1] - s0);
    vector<Vec2> out;
    out.reserve(samples + (close_loop ? 1 : 0));
    for (int k = 0; k < samples; k++) {
        const double si = s0 + L * (double(k) / double(samples));
        out.push_back({spx.eval(si), spy.eval(si)});
    }
    if (close_loop) out.push_back(out.front());
    spx_out = std::move(spx);
    spy_out = std::move(spy);
    s0_out = s0;
    L_out = L;
    return out;
}
}  // namespace centerline

// ============================ ABI glue ======================================
namespace gpu {
inline int device = 0;
inline vector<int32_t> devices;   // --devices: a batch sharded over these (rl_optimize_multi)
inline void check(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(string(what) + ": " + rl_last_error());
}
inline vector<double> flat_segments(const SegVec& E) {
    vector<double> s;
    s.reserve(4 * E.size());
    for (const auto& e : E) s.insert(s.end(), {e.first.x, e.first.y, e.second.x, e.second.y});
    return s;
}
struct Packed {
    vector<double> center, inner, outer;
    rl_problem prob;
};
inline Packed pack(const vector<Vec2>& center, const SegVec& innerE, const SegVec& outerE, double veh_width,
                   double L, bool closed) {
    Packed p;
    for (const Vec2& v : center) { p.center.push_back(v.x); p.center.push_back(v.y); }
    p.inner = flat_segments(innerE);
    p.outer = flat_segments(outerE);
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
// normals_from_points_generic (ref:581-593): host-side, for the debug dump's signed offsets
static void normals_from_points_generic(const vector<Vec2>& P, bool closed, vector<Vec2>& n) {
    const int N = (int)P.size();
    n.assign(N, Vec2{0, 0});
    for (int i = 0; i < N; ++i) {
        Vec2 t;
        if (N == 1) t = {1, 0};
        else if (closed) {
            const int ip = (i + 1) % N, im = (i - 1 + N) % N;
            t = {(P[ip].x - P[im].x) * 0.5, (P[ip].y - P[im].y) * 0.5};
        } else if (i == 0) t = P[1] - P[0];
        else if (i == N - 1) t = P[N - 1] - P[N - 2];
        else t = {(P[i + 1].x - P[i - 1].x) * 0.5, (P[i + 1].y - P[i - 1].y) * 0.5};
        if (geom::norm(t) < 1e-15) t = {1, 0};
        n[i] = geom::normalize(Vec2{-t.y, t.x}, 1e-15);
    }
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
// Lap times of given paths: heading/curvature with h = L_b/N and the v(s) passes
// (ref:1466-1478), one GPU launch for all paths (rl_lap_eval). All paths have N points.
static vector<double> lap_times(const vector<const vector<Vec2>*>& paths, const vector<double>& Ls, bool closed) {
    const int B = (int)paths.size();
    if (B == 0) return {};
    const int N = (int)paths[0]->size();
    vector<double> xy;
    xy.reserve((size_t)2 * B * N);
    for (const auto* p : paths)
        for (const Vec2& q : *p) { xy.push_back(q.x); xy.push_back(q.y); }
    vector<double> hd((size_t)B * N), ka((size_t)B * N), v((size_t)B * N), ax((size_t)B * N), lap(B);
    vector<int32_t> sweeps(B);
    rl_out o;
    std::memset(&o, 0, sizeof(o));
    o.heading = hd.data(); o.kappa = ka.data(); o.v = v.data(); o.ax = ax.data(); o.lap = lap.data();
    o.vpass_sweeps = sweeps.data();
    rl_cfg c = cfg::to_abi(cfg::get());
    gpu::check(rl_lap_eval(xy.data(), Ls.data(), N, B, closed ? 1 : 0, &c, 1, gpu::device, &o, nullptr), "rl_lap_eval");
    return lap;
}
}  // namespace raceline_min_time

// =============================== Pipeline ===================================
namespace pipeline {
struct Triangulation {
    vector<Vec2> all;
    vector<int> label;   // 0 inner, 1 outer
    vector<delaunay::Tri> tris;
};
// ref:1066-1073
static Triangulation buildDT(const vector<Vec2>& inner, const vector<Vec2>& outer) {
    Triangulation R;
    R.all = inner;
    R.all.insert(R.all.end(), outer.begin(), outer.end());
    R.label.assign(R.all.size(), 1);
    std::fill(R.label.begin(), R.label.begin() + inner.size(), 0);
    R.tris = delaunay::bowyerWatson(R.all);
    return R;
}

struct MidsFiltered {
    vector<centerline::BoundaryEdgeInfo> binfo;
    vector<Vec2> mids;
    vector<int> keep_edge_idx;
};
// Inner-outer edges, their midpoints, and a cutoff at min(abs_max, scale·median length).
// The median is the linear-interpolated quantile of the sorted lengths. Writes the three
// edge CSVs (ref:1081-1140).
static MidsFiltered extract_mids_with_len_filter(const Triangulation& T, const string& base) {
    const auto& C = cfg::get();
    MidsFiltered R;
    delaunay::EdgeMap M;
    delaunay::buildEdgeMap(T.tris, M);
    R.binfo = centerline::labelBoundaryEdges_with_len(T.all, M, T.label);
    if (R.binfo.empty()) throw std::runtime_error("no label-different boundary edges");
    {
        vector<pair<int, int>> all_e, mixed;
        all_e.reserve(M.size());
        for (const auto& kv : M) all_e.push_back({kv.first.u, kv.first.v});
        io::saveCSV_edgesIdx(base + "_edges_all_idx.csv", all_e);
        for (const auto& e : R.binfo) mixed.push_back({e.u, e.v});
        io::saveCSV_edgesIdx(base + "_edges_labeldiff_idx.csv", mixed);
        if (C.verbose) std::cerr << "[edges] label-different edges = " << mixed.size() << "\n";
    }
    vector<double> lens;
    lens.reserve(R.binfo.size());
    for (const auto& e : R.binfo) lens.push_back(e.len);
    std::sort(lens.begin(), lens.end());
    const double qpos = 0.5 * (lens.size() - 1);
    const size_t qi = (size_t)std::floor(qpos), qj = std::min(qi + 1, lens.size() - 1);
    const double qt = qpos - qi;
    const double Lmed = (1.0 - qt) * lens[qi] + qt * lens[qj];
    const double cutoff = std::min(C.boundary_edge_abs_max, C.boundary_edge_len_scale * std::max(1e-12, Lmed));
    for (int i = 0; i < (int)R.binfo.size(); ++i) {
        if (C.enable_boundary_len_filter && !(R.binfo[i].len <= cutoff)) continue;
        R.mids.push_back(R.binfo[i].mid);
        R.keep_edge_idx.push_back(i);
    }
    if (R.mids.size() < 2) {
        io::saveCSV_pointsXY(base + "_mids_raw.csv", R.mids);
        throw std::runtime_error("not enough midpoints after length filter");
    }
    vector<pair<int, int>> kept;
    for (int i : R.keep_edge_idx) kept.push_back({R.binfo[i].u, R.binfo[i].v});
    io::saveCSV_edgesIdx(base + "_edges_labeldiff_kept_idx.csv", kept);
    if (C.verbose) std::cerr << "[edges] kept (len-filtered) = " << kept.size() << " / " << R.binfo.size() << "\n";
    return R;
}

struct OrderedMids {
    vector<Vec2> ordered;
    vector<int> mids_order_idx;
};
// MST order, then direction and start (ref:1149-1202):
//  * open: along the car's heading, starting nearest the start anchor;
//  * closed: along start_heading_rad (unless force_closed_ccw), rotated so that the
//    midpoint nearest the anchor comes first.
static OrderedMids order_and_align_mids_open_closed(const vector<Vec2>& mids, bool closed_mode) {
    const auto& C = cfg::get();
    OrderedMids R;
    R.ordered = centerline::orderByMST(mids);
    R.mids_order_idx = centerline::matchIndices(mids, R.ordered);
    auto nearest = [](const vector<Vec2>& S, const Vec2& t) {
        size_t k = 0;
        double best = 1e300;
        for (size_t i = 0; i < S.size(); ++i) {
            const double dx = S[i].x - t.x, dy = S[i].y - t.y, d2 = dx * dx + dy * dy;
            if (d2 < best) { best = d2; k = i; }
        }
        return k;
    };
    auto step_dir = [&](size_t i) -> Vec2 {   // local_dir_open / local_dir_closed
        const vector<Vec2>& S = R.ordered;
        if (S.size() < 2) return {1, 0};
        if (closed_mode) return geom::normalize(S[(i + 1) % S.size()] - S[i], 1e-12);
        if (i + 1 < S.size()) return geom::normalize(S[i + 1] - S[i], 1e-12);
        return geom::normalize(S[i] - S[i - 1], 1e-12);
    };
    auto flip = [&]() {
        std::reverse(R.ordered.begin(), R.ordered.end());
        std::reverse(R.mids_order_idx.begin(), R.mids_order_idx.end());
    };
    auto rotate_to = [&](size_t k) {
        std::rotate(R.ordered.begin(), R.ordered.begin() + k, R.ordered.end());
        std::rotate(R.mids_order_idx.begin(), R.mids_order_idx.begin() + k, R.mids_order_idx.end());
    };
    const Vec2 anchor{C.start_anchor_x, C.start_anchor_y};
    if (!closed_mode) {
        const Vec2 car{C.current_pos_x, C.current_pos_y};
        const Vec2 want = geom::normalize(geom::heading_dir(C.current_heading_rad), 1e-12);
        if (geom::dot(step_dir(nearest(R.ordered, car)), want) < 0.0) flip();
        rotate_to(nearest(R.ordered, anchor));
    } else {
        const Vec2 want = geom::normalize(geom::heading_dir(C.start_heading_rad), 1e-12);
        if (!C.force_closed_ccw && geom::dot(step_dir(nearest(R.ordered, anchor)), want) < 0.0) flip();
        rotate_to(nearest(R.ordered, anchor));
    }
    return R;
}

struct ReconstructedRings {
    vector<Vec2> inner_from_mids, outer_from_mids;
};
// The cones of the kept edges, visited in midpoint order, first use only. Each ring is
// reversed when its first step points against the midpoints' first step (ref:1209-1254).
static ReconstructedRings reconstruct_rings_and_align(const OrderedMids& OM, const MidsFiltered& MF,
                                                      const Triangulation& T, const string& base) {
    ReconstructedRings R;
    vector<char> seen_in(T.all.size(), 0), seen_out(T.all.size(), 0);
    for (int local : OM.mids_order_idx) {
        const auto& e = MF.binfo[MF.keep_edge_idx[local]];
        int iv = -1, ov = -1;
        if (T.label[e.u] == 0 && T.label[e.v] == 1) { iv = e.u; ov = e.v; }
        else if (T.label[e.u] == 1 && T.label[e.v] == 0) { iv = e.v; ov = e.u; }
        if (iv >= 0 && !seen_in[iv]) { R.inner_from_mids.push_back(T.all[iv]); seen_in[iv] = 1; }
        if (ov >= 0 && !seen_out[ov]) { R.outer_from_mids.push_back(T.all[ov]); seen_out[ov] = 1; }
    }
    auto first_dir = [](const vector<Vec2>& S) -> Vec2 {
        if (S.size() < 2) return Vec2{1, 0};
        return geom::normalize(S[1] - S[0], 1e-12);
    };
    const Vec2 ref_dir = first_dir(OM.ordered);
    for (vector<Vec2>* ring : {&R.inner_from_mids, &R.outer_from_mids})
        if (ring->size() >= 2 && geom::dot(ref_dir, first_dir(*ring)) < 0.0) std::reverse(ring->begin(), ring->end());
    io::saveCSV_pointsXY(base + "_inner_from_mids.csv", R.inner_from_mids);
    io::saveCSV_pointsXY(base + "_outer_from_mids.csv", R.outer_from_mids);
    if (cfg::get().verbose) {
        const int want_in = (int)std::count(T.label.begin(), T.label.end(), 0);
        const int want_out = (int)std::count(T.label.begin(), T.label.end(), 1);
        std::cerr << "[cones-from-mids] inner used " << R.inner_from_mids.size() << "/" << want_in << ", outer used "
                  << R.outer_from_mids.size() << "/" << want_out << "\n";
    }
    return R;
}

struct CenterlineOut {
    vector<Vec2> center;
    centerline::Spline1D spx, spy;
    double s0 = 0.0, L = 0.0;
};
// llround(factor·mids), clamped to [samples_min, samples_max] and to at least 4 (ref:1262-1269)
static int dynamic_samples_from_mids_count(int mids_n) {
    const auto& C = cfg::get();
    int n = (int)std::llround(C.sample_factor_n * std::max(0, mids_n));
    n = std::max(n, C.samples_min);
    if (C.samples_max > 0) n = std::min(n, C.samples_max);
    return std::max(n, 4);
}
// ref:1271-1280 (closed: 3 padding points per side; the duplicate follows emit_closed_duplicate)
static CenterlineOut make_centerline(const OrderedMids& OM, bool closed_mode, const string& base) {
    const auto& C = cfg::get();
    CenterlineOut R;
    R.center = centerline::splineUniformResample(OM.ordered, C.samples, closed_mode ? 3 : 0, C.emit_closed_duplicate,
                                                 R.spx, R.spy, R.s0, R.L);
    io::saveCSV_pointsXY(base + "_mids_raw.csv", OM.ordered);
    return R;
}
static void save_centerline_csv(const string& outPath, const vector<Vec2>& center) {   // ref:1282-1286
    io::Csv o(outPath);
    if (!o) throw std::runtime_error("save centerline failed: " + outPath);
    for (const Vec2& p : center) o.f << p.x << "," << p.y << "\n";
}

// Step 6 on the GPU (rl_geom): <base>_with_geom.csv (ref:1288-1335)
static void compute_geom_and_save(const string& base, const vector<Vec2>& center, const centerline::Spline1D& spx,
                                  const centerline::Spline1D& spy, double s0, double L, bool closed_mode,
                                  const vector<Vec2>& inner_from_mids, const vector<Vec2>& outer_from_mids) {
    const auto& C = cfg::get();
    const SegVec innerE = closed_mode ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    const SegVec outerE = closed_mode ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    const vector<double> si = gpu::flat_segments(innerE), so = gpu::flat_segments(outerE);
    rl_geom_problem gp;
    std::memset(&gp, 0, sizeof(gp));
    auto spline = [](const centerline::Spline1D& sp) {
        rl_spline r;
        std::memset(&r, 0, sizeof(r));
        r.s = sp.s.data(); r.a = sp.a.data(); r.b = sp.b.data(); r.c = sp.c.data(); r.d = sp.d.data();
        r.n = (int32_t)sp.s.size();
        return r;
    };
    gp.spx = spline(spx);
    gp.spy = spline(spy);
    gp.s0 = s0;
    gp.L = L;
    gp.Kmax = closed_mode ? C.samples : (int)center.size();
    gp.denomN = closed_mode ? C.samples : std::max(1, C.samples);
    gp.emit_closed_duplicate = C.emit_closed_duplicate ? 1 : 0;
    gp.closed = closed_mode ? 1 : 0;
    gp.inner_seg = si.data();
    gp.outer_seg = so.data();
    gp.Ei = (int)innerE.size();
    gp.Eo = (int)outerE.size();
    vector<double> rows((size_t)RL_GEOM_COLS * (gp.Kmax + 1));
    rl_cfg c = cfg::to_abi(C);
    const int nrows = rl_geom(&gp, &c, gpu::device, rows.data(), nullptr);
    gpu::check(nrows, "rl_geom");
    io::Csv o(base + "_with_geom.csv");
    if (!o) throw std::runtime_error("save centerline_with_geom failed");
    o.f << "s,x,y,heading_rad,curvature,dist_to_inner,dist_to_outer,width,v_kappa_mps\n";
    for (int r = 0; r < nrows; ++r) {
        const double* q = &rows[(size_t)RL_GEOM_COLS * r];
        for (int j = 0; j < RL_GEOM_COLS; ++j) o.f << q[j] << (j + 1 < RL_GEOM_COLS ? "," : "\n");
    }
}

static void compute_raceline_and_save(const string& base, const vector<Vec2>& center_for_opt, double s0, double L,
                                      bool closed_mode, const vector<Vec2>& inner_from_mids,
                                      const vector<Vec2>& outer_from_mids) {   // ref:1337-1383
    auto& C = cfg::get();
    SegVec innerE = closed_mode ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    SegVec outerE = closed_mode ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    auto res = raceline_min_curv::compute_min_curvature_raceline(center_for_opt, innerE, outerE, C.veh_width_m, L,
                                                                 closed_mode);
    {
        io::Csv o(base + "_raceline.csv");
        if (!o) throw std::runtime_error("save raceline failed");
        for (auto& p : res.raceline) o.f << p.x << "," << p.y << "\n";
        if (C.emit_closed_duplicate && !res.raceline.empty()) o.f << res.raceline[0].x << "," << res.raceline[0].y << "\n";
    }
    {
        io::Csv o(base + "_raceline_with_geom.csv");
        if (!o) throw std::runtime_error("save raceline_with_geom failed");
        o.f << "s,x,y,heading_rad,curvature,alpha_last,v_kappa_mps\n";
        const int Nrl = (int)res.raceline.size();
        auto vk = [&](double k) {
            const double v = std::sqrt(C.a_lat_max / std::max(std::fabs(k), C.kappa_eps));
            return v > C.v_cap_mps ? C.v_cap_mps : v;
        };
        for (int k = 0; k < Nrl; ++k) {
            const double si = s0 + L * (double(k) / double(std::max(1, Nrl)));
            o.f << si - s0 << "," << res.raceline[k].x << "," << res.raceline[k].y << "," << res.heading[k] << ","
                << res.curvature[k] << "," << res.alpha_last[k] << "," << vk(res.curvature[k]) << "\n";
        }
        if (C.emit_closed_duplicate && Nrl > 0)
            o.f << L << "," << res.raceline[0].x << "," << res.raceline[0].y << "," << res.heading[0] << ","
                << res.curvature[0] << "," << res.alpha_last[0] << "," << vk(res.curvature[0]) << "\n";
    }
}

// The cfg::debug_dump block (ref:1440-1593): centreline and min-curvature laps (GPU),
// then <base>_debug_compare_paths.csv and its summary. The rows are O(N) host arithmetic
// in the reference's order.
static void debug_dump(const string& base, const vector<Vec2>& center_for_opt, double s0, double L, bool closed_mode,
                       const raceline_min_time::Result& res) {
    const auto& C = cfg::get();
    const double nan = std::numeric_limits<double>::quiet_NaN();
    auto path_length = [](const vector<Vec2>& P, bool closed) {
        const int n = (int)P.size();
        double tot = 0.0;
        if (n <= 1) return tot;
        for (int i = 0; i + 1 < n; ++i) tot += std::hypot(P[i + 1].x - P[i].x, P[i + 1].y - P[i].y);
        if (closed) tot += std::hypot(P[0].x - P[n - 1].x, P[0].y - P[n - 1].y);
        return tot;
    };
    vector<Vec2> mc = io::loadCSV_XY(base + "_raceline.csv");
    if (!mc.empty() && closed_mode && mc.size() >= 2 && geom::almostEq(mc.front(), mc.back(), 1e-12)) mc.pop_back();
    vector<Vec2> nc;
    raceline_min_curv::normals_from_points_generic(center_for_opt, closed_mode, nc);

    double lap_c = 0.0, lap_mc = -1.0;
    if (!center_for_opt.empty()) {
        vector<const vector<Vec2>*> paths{&center_for_opt};
        vector<double> Ls{L};
        const bool together = !mc.empty() && mc.size() == center_for_opt.size();
        if (together) { paths.push_back(&mc); Ls.push_back(path_length(mc, closed_mode)); }
        const vector<double> laps = raceline_min_time::lap_times(paths, Ls, closed_mode);
        lap_c = laps[0];
        if (together) lap_mc = laps[1];
        else if (!mc.empty()) lap_mc = raceline_min_time::lap_times({&mc}, {path_length(mc, closed_mode)}, closed_mode)[0];
    }
    if (!mc.empty())
        std::cerr << "[debug] centerline lap ≈ " << std::setprecision(3) << lap_c << " s,  min-curv lap ≈ " << lap_mc
                  << " s,  min-time lap ≈ " << res.lap_time << " s\n";
    else
        std::cerr << "[debug] centerline lap ≈ " << std::setprecision(3) << lap_c
                  << " s,  (min-curv not found),  min-time lap ≈ " << res.lap_time << " s\n";

    const int N = (int)std::min(res.raceline.size(), center_for_opt.size());
    io::Csv o(base + "_debug_compare_paths.csv");
    if (!o) {
        std::cerr << "[debug] cfg::debug_dump=false\n";
        return;
    }
    o.f << "s,cx,cy,mt_x,mt_y,mc_x,mc_y,d_mt_signed_m,d_mc_signed_m,d_mt_abs_m,d_mc_abs_m,kappa_mt,v_mt,ax_mt,"
           "alat_mt,alat_ratio,gamma,a_acc_cap,a_brk_cap,a_power_cap\n";
    double sum_mt = 0, sq_mt = 0, max_mt = 0, sum_mc = 0, sq_mc = 0, max_mc = 0;
    int at_mt = 0, at_mc = 0, near = 0;
    const double Fr = C.mass_kg * 9.81 * C.c_rr;
    for (int k = 0; k < N; ++k) {
        const double si = s0 + L * (double(k) / double(std::max(1, N)));
        const Vec2& cp = center_for_opt[k];
        const Vec2& mt = res.raceline[k];
        const Vec2 mcp = (int)mc.size() > k ? mc[k] : Vec2{nan, nan};
        const double dmt = (mt.x - cp.x) * nc[k].x + (mt.y - cp.y) * nc[k].y;
        const double dmc = std::isfinite(mcp.x) ? (mcp.x - cp.x) * nc[k].x + (mcp.y - cp.y) * nc[k].y : nan;
        const double admt = std::fabs(dmt), admc = std::isfinite(dmc) ? std::fabs(dmc) : nan;
        const double kap = k < (int)res.curvature.size() ? res.curvature[k] : 0.0;
        const double v = k < (int)res.v.size() ? res.v[k] : 0.0;
        const double ax = k < (int)res.ax.size() ? res.ax[k] : 0.0;
        const double alat = v * v * std::fabs(kap);
        const double alat_ratio = (C.a_total_max > 1e-9) ? std::min(1.0, alat / C.a_total_max) : 0.0;
        const double vkappa = std::sqrt(C.a_lat_max / std::max(std::fabs(kap), C.kappa_eps));
        const double pr = (vkappa - v) / std::max(1e-6, vkappa);
        const double gamma = 1.0 + C.w_time_gain * (pr < 0 ? 0 : (pr > 1 ? 1 : pr));
        // longitudinal caps at (v, κ), as ax_max_at (ref:1529-1539)
        const double al2 = v * v * std::fabs(kap);
        const double a_res = std::sqrt(std::max(0.0, C.a_total_max * C.a_total_max - al2 * al2));
        const double Fd = 0.5 * C.rho_air * C.Cd * C.A_front_m2 * v * v;
        const double a_power = (C.P_max_W > 0 && v > 1e-6) ? (C.P_max_W / (C.mass_kg * v) - (Fd + Fr) / C.mass_kg) : 1e9;
        const double a_acc = std::max(0.0, std::min({a_res, C.a_long_acc_cap, a_power}));
        const double a_brk = std::max(0.0, std::min(a_res, C.a_long_brake_cap) + (Fd + Fr) / C.mass_kg);
        const double row[20] = {si - s0, cp.x, cp.y, mt.x, mt.y, mcp.x, mcp.y, dmt, dmc, admt,
                                admc, kap, v, ax, alat, alat_ratio, gamma, a_acc, a_brk, std::max(0.0, a_power)};
        for (int j = 0; j < 20; ++j) o.f << row[j] << (j < 19 ? "," : "\n");
        sum_mt += admt;
        sq_mt += admt * admt;
        if (admt > max_mt) { max_mt = admt; at_mt = k; }
        if (std::isfinite(admc)) {
            sum_mc += admc;
            sq_mc += admc * admc;
            if (admc > max_mc) { max_mc = admc; at_mc = k; }
        }
        if (admt < C.debug_offset_warn_m) near++;
    }
    o.f.close();
    const double mean_mt = sum_mt / std::max(1, N);
    std::cerr << std::setprecision(3) << "[debug] min-time vs center: mean|offset|=" << mean_mt
              << " m, rms=" << std::sqrt(sq_mt / std::max(1, N)) << " m, max=" << max_mt << " m @i=" << at_mt
              << ", within " << C.debug_offset_warn_m << " m : " << near << "/" << N << "\n";
    if (max_mc > 0.0 && std::isfinite(max_mc))
        std::cerr << "[debug] min-curv vs center: mean|offset|=" << sum_mc / std::max(1, N)
                  << " m, rms=" << std::sqrt(sq_mc / std::max(1, N)) << " m, max=" << max_mc << " m @i=" << at_mc
                  << "\n";
    if (mean_mt < 0.01 && max_mt < 0.03)
        std::cerr << "[hint] the min-time path stays very close to the centreline (narrow track or tight "
                     "curvature/dynamics limits)\n";
    if (lap_mc > 0.0) std::cerr << "[debug] lap gain vs min-curv: " << (lap_mc - res.lap_time) / lap_mc * 100.0 << " %\n";
}

static void compute_mintime_and_save(const string& base, const vector<Vec2>& center_for_opt, double s0, double L,
                                     bool closed_mode, const vector<Vec2>& inner_from_mids,
                                     const vector<Vec2>& outer_from_mids) {   // ref:1385-1593
    auto& C = cfg::get();
    SegVec innerE = closed_mode ? edges::ringEdges(inner_from_mids) : edges::polylineEdges(inner_from_mids);
    SegVec outerE = closed_mode ? edges::ringEdges(outer_from_mids) : edges::polylineEdges(outer_from_mids);
    auto res = raceline_min_time::compute_min_time_raceline(center_for_opt, innerE, outerE, C.veh_width_m, L,
                                                            closed_mode);
    {
        io::Csv o(base + "_mintime_raceline.csv");
        if (!o) throw std::runtime_error("save mintime_raceline failed");
        for (auto& p : res.raceline) o.f << p.x << "," << p.y << "\n";
        if (C.emit_closed_duplicate && !res.raceline.empty()) o.f << res.raceline[0].x << "," << res.raceline[0].y << "\n";
    }
    {
        io::Csv o(base + "_mintime_with_geom.csv");
        if (!o) throw std::runtime_error("save mintime_with_geom failed");
        o.f << "s,x,y,heading_rad,curvature,alpha_last,v_mps,ax_mps2\n";
        const int N = (int)res.raceline.size();
        for (int k = 0; k < N; ++k) {
            const double si = s0 + L * (double(k) / double(std::max(1, N)));
            o.f << si - s0 << "," << res.raceline[k].x << "," << res.raceline[k].y << "," << res.heading[k] << ","
                << res.curvature[k] << "," << res.alpha_last[k] << "," << res.v[k] << "," << res.ax[k] << "\n";
        }
        if (C.emit_closed_duplicate && N > 0)
            o.f << L << "," << res.raceline[0].x << "," << res.raceline[0].y << "," << res.heading[0] << ","
                << res.curvature[0] << "," << res.alpha_last[0] << "," << res.v[0] << "," << res.ax[0] << "\n";
    }
    std::cerr << "[mintime] Estimated laptime: " << std::fixed << std::setprecision(3) << res.lap_time << " s\n";
    if (C.debug_dump) debug_dump(base, center_for_opt, s0, L, closed_mode, res);
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
    const size_t BN = (size_t)B * center.size();
    vector<double> lap(B), al(BN), x(BN), y(BN);
    vector<int32_t> ev((size_t)B * C.max_outer_iters);
    rl_out o;
    std::memset(&o, 0, sizeof(o));
    o.x = x.data(); o.y = y.data(); o.alpha_last = al.data(); o.evals = ev.data();
    const bool mt = modes & RL_MODE_MINTIME;
    if (mt) o.lap = lap.data();
    rl_plan* plan = nullptr;
    if (!gpu::devices.empty()) {
        // sharded over the listed devices (one mode per call: the summary reads one)
        auto call = [&]() {
            gpu::check(rl_optimize_multi(&pk.prob, &c, 1, seeds.data(), B, gpu::devices.data(),
                                         (int32_t)gpu::devices.size(), mt ? nullptr : &o, mt ? &o : nullptr),
                       "rl_optimize_multi");
        };
        call();
        if (repeat > 0) {
            auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < repeat; ++r) call();
            double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::cerr << "[batch] B=" << B << " over " << gpu::devices.size() << " devices, " << repeat
                      << " calls " << wall * 1e3 << " ms (PCIe included) -> "
                      << (double)B * C.max_outer_iters * repeat / wall << " PGD outer-iters/s\n";
        }
        repeat = 0;
    } else {
        gpu::check(rl_plan_create(&plan, gpu::device, &pk.prob, &c, 1, seeds.data(), B, modes), "rl_plan_create");
        gpu::check(rl_plan_run(plan, nullptr), "rl_plan_run");
        gpu::check(rl_plan_fetch(plan, mt ? nullptr : &o, mt ? &o : nullptr), "rl_plan_fetch");
    }
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
    if (plan) rl_plan_destroy(plan);
    io::Csv fo(base + "_batch_summary.csv");
    fo.f << "seed,lap_time_s,mean_abs_alpha_last,evals_total\n";
    for (int b = 0; b < B; ++b) {
        double s = 0;
        for (size_t i = 0; i < center.size(); ++i) s += std::fabs(al[b * center.size() + i]);
        long et = 0;
        for (int k = 0; k < C.max_outer_iters; ++k) et += ev[(size_t)b * C.max_outer_iters + k];
        fo.f << b << "," << (mt ? lap[b] : 0.0) << "," << s / std::max<size_t>(1, center.size()) << "," << et << "\n";
    }
}
}  // namespace pipeline

// ================================== MAIN ====================================
namespace {
using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

double last_s_of(const string& path) {   // L = s of the closing row (ref:1331-1333)
    std::ifstream f(path);
    string line, last;
    while (std::getline(f, line)) if (!line.empty()) last = line;
    if (last.empty()) return NAN;
    return std::strtod(last.c_str(), nullptr);
}

vector<Vec2> opt_input(const vector<Vec2>& center, bool closed) {   // ref:1681-1683
    vector<Vec2> c = center;
    if (closed && c.size() >= 2 && geom::almostEq(c.front(), c.back(), 1e-12)) c.pop_back();
    return c;
}

// The reference CLI: cones -> every CSV (ref:1598-1714). Steps 1-5 on the host, the rest
// on the GPU. stop_after_centerline ends after step 5 (no GPU call).
int run_pipeline(const string& innerPath, const string& outerPath, const string& outPath, const string& mode,
                 bool stop_after_centerline) {
    auto& C = cfg::get();
    const string base = io::dropExt(outPath);
    double t_load, t_dt, t_mids, t_mst, t_spline, t_saveC, t_geom = 0, t_mc = 0, t_mt = 0;
    auto t = Clock::now();
    const vector<Vec2> inner = io::loadCSV_XY(innerPath), outer = io::loadCSV_XY(outerPath);
    t_load = ms_since(t);
    if (inner.size() < 2 || outer.size() < 2) { std::cerr << "[ERR] need >=2 points per ring\n"; return 2; }
    const bool closed_mode = C.is_closed_track;

    t = Clock::now();
    const pipeline::Triangulation tri = pipeline::buildDT(inner, outer);
    if (C.verbose) std::cerr << "[DT] points=" << tri.all.size() << " faces=" << tri.tris.size() << "\n";
    io::saveCSV_pointsLabeled(base + "_all_points.csv", tri.all, tri.label);
    io::saveCSV_trisIdx(base + "_tri_raw_idx.csv", tri.tris);
    t_dt = ms_since(t);

    t = Clock::now();
    const pipeline::MidsFiltered MF = pipeline::extract_mids_with_len_filter(tri, base);
    if (C.use_dynamic_samples) {
        C.samples = pipeline::dynamic_samples_from_mids_count((int)MF.mids.size());
        if (C.verbose)
            std::cerr << "[samples] dynamic=" << C.samples << " (n=" << C.sample_factor_n << ", mids=" << MF.mids.size()
                      << ")\n";
    }
    t_mids = ms_since(t);

    t = Clock::now();
    const pipeline::OrderedMids OM = pipeline::order_and_align_mids_open_closed(MF.mids, closed_mode);
    io::saveCSV_pointsXY(base + "_mids_ordered.csv", OM.ordered);
    const pipeline::ReconstructedRings RR = pipeline::reconstruct_rings_and_align(OM, MF, tri, base);
    t_mst = ms_since(t);

    t = Clock::now();
    const pipeline::CenterlineOut CL = pipeline::make_centerline(OM, closed_mode, base);
    t_spline = ms_since(t);
    t = Clock::now();
    pipeline::save_centerline_csv(outPath, CL.center);
    t_saveC = ms_since(t);

    if (!stop_after_centerline) {
        t = Clock::now();
        pipeline::compute_geom_and_save(base, CL.center, CL.spx, CL.spy, CL.s0, CL.L, closed_mode, RR.inner_from_mids,
                                        RR.outer_from_mids);
        t_geom = ms_since(t);
        const vector<Vec2> center_for_opt = opt_input(CL.center, closed_mode);
        t = Clock::now();
        if (mode != "mintime")
            pipeline::compute_raceline_and_save(base, center_for_opt, CL.s0, CL.L, closed_mode, RR.inner_from_mids,
                                                RR.outer_from_mids);
        t_mc = ms_since(t);
        t = Clock::now();
        if (mode != "mincurv")
            pipeline::compute_mintime_and_save(base, center_for_opt, CL.s0, CL.L, closed_mode, RR.inner_from_mids,
                                               RR.outer_from_mids);
        t_mt = ms_since(t);
    }
    std::cerr.setf(std::ios::fixed);
    std::cerr << std::setprecision(3) << "[TIME][SUMMARY] load=" << t_load << ", dt=" << t_dt << ", mids=" << t_mids
              << ", mst=" << t_mst << ", spline=" << t_spline << ", saveC=" << t_saveC << ", geom=" << t_geom
              << ", mincurv_race=" << t_mc << ", mintime_race=" << t_mt << "\n";
    return 0;
}

// Steps 7-8 from the reference's step-6 files.
int run_from_centerline(const string& outPath, double L, double s0, const string& mode, int B, int repeat) {
    auto& C = cfg::get();
    const string base = io::dropExt(outPath);
    const bool closed_mode = C.is_closed_track;
    const auto center = io::loadCSV_XY(outPath);
    const auto inner = io::loadCSV_XY(base + "_inner_from_mids.csv");
    const auto outer = io::loadCSV_XY(base + "_outer_from_mids.csv");
    if (std::isnan(L)) L = last_s_of(base + "_with_geom.csv");
    if (center.size() < 2 || inner.size() < 2 || outer.size() < 2 || !(L > 0)) {
        std::cerr << "[ERR] need centerline, inner/outer_from_mids and L (--L or <base>_with_geom.csv)\n";
        return 2;
    }
    const vector<Vec2> center_for_opt = opt_input(center, closed_mode);
    if (B > 0) {
        const int modes = mode == "mincurv" ? RL_MODE_MINCURV
                                            : mode == "mintime" ? RL_MODE_MINTIME : RL_MODE_MINCURV | RL_MODE_MINTIME;
        pipeline::batch_and_save(base, center_for_opt, L, closed_mode, inner, outer, B, modes, repeat);
        return 0;
    }
    auto t0 = Clock::now();
    if (mode != "mintime") pipeline::compute_raceline_and_save(base, center_for_opt, s0, L, closed_mode, inner, outer);
    const double t_mc = ms_since(t0);
    t0 = Clock::now();
    if (mode != "mincurv") pipeline::compute_mintime_and_save(base, center_for_opt, s0, L, closed_mode, inner, outer);
    std::cerr.setf(std::ios::fixed);
    std::cerr << "[TIME][SUMMARY] mincurv_race=" << t_mc << ", mintime_race=" << ms_since(t0) << "\n";
    return 0;
}
}  // namespace

int main(int argc, char** argv) {
    std::ios::sync_with_stdio(false);
    auto& C = cfg::get();
    vector<string> pos;
    double L = NAN, s0 = 0.0;
    string mode = "both", stop_after;
    int B = 0, repeat = 0;
    try {
        for (int i = 1; i < argc; ++i) {
            const string a = argv[i];
            auto next = [&]() -> string {
                if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
                return argv[++i];
            };
            if (a.rfind("--", 0) != 0) pos.push_back(a);
            else if (a == "--L") L = std::stod(next());
            else if (a == "--s0") s0 = std::stod(next());
            else if (a == "--open") C.is_closed_track = false;
            else if (a == "--mode") mode = next();
            else if (a == "--seeds") B = std::stoi(next());
            else if (a == "--repeat") repeat = std::stoi(next());
            else if (a == "--device") gpu::device = std::stoi(next());
            else if (a == "--devices") {
                std::stringstream ss(next());
                string tok;
                while (std::getline(ss, tok, ',')) gpu::devices.push_back(std::stoi(tok));
            }
            else if (a == "--stop-after") stop_after = next();
            else if (a == "--set") {
                const string kv = next();
                if (!cfg::set_knob(C, kv)) throw std::runtime_error("unknown cfg knob: " + kv);
            } else throw std::runtime_error("unknown option " + a);
        }
        if (pos.size() != 1 && pos.size() != 3) {
            std::cerr << "Usage: " << argv[0] << " inner.csv outer.csv centerline.csv [--set key=value ...]"
                      << " [--mode mincurv|mintime|both] [--stop-after centerline]\n"
                      << "       " << argv[0]
                      << " centerline.csv [--L v] [--s0 v] [--open] [--mode m] [--seeds B] [--repeat R]\n";
            return 1;
        }
        if (pos.size() == 3) return run_pipeline(pos[0], pos[1], pos[2], mode, stop_after == "centerline");
        return run_from_centerline(pos[0], L, s0, mode, B, repeat);
    } catch (const std::exception& e) {
        std::cerr << "[ERR] " << e.what() << "\n";
        return 3;
    }
}
