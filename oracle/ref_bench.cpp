// ref_bench.cpp — TEST INFRASTRUCTURE ONLY: the CPU baseline timer (bench.py's
// cpu_baseline leg), never shipped, never on the product path.
//
// Compiles the reference translation unit /root/reference/src/main.cpp AS IT LIES
// (REF_MAIN_CPP from oracle/Makefile, `main` renamed with -Dmain=...) with the
// reference's own build flags, `g++ -std=c++17 -O3` (/root/reference/README.md:28),
// and times its optimisers on one problem:
//   ref_bench_o3 <problem.bin> <mincurv|mintime> <budget_s> <min_calls>
// calls raceline_min_curv::compute_min_curvature_raceline (main.cpp:683) or
// raceline_min_time::compute_min_time_raceline (main.cpp:905) repeatedly, on the
// calling thread, until budget_s seconds have passed and at least min_calls calls
// ran, and prints one JSON line with the per-call wall times.  The reference's
// unconditional stderr diagnostics of the min-time driver (main.cpp:980-991,
// 1017-1022) are muted (the stream's buffer is detached, so nothing is formatted).
//
// problem.bin (little endian, written by bench.py):
//   int32 N, closed, Ei, Eo; double L, veh_width; rl_cfg; double center[N][2],
//   inner[Ei][4], outer[Eo][4].
#define main rl_reference_cli_main      // the reference's CLI entry, not called here
#include REF_MAIN_CPP
#undef main

#include <chrono>
#include <cstdio>
#include <cstring>
#include "../include/rl_abi.h"

namespace {
using geom::Vec2;
using SegVec = vector<pair<Vec2, Vec2>>;

bool read_all(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

void apply(const rl_cfg& c) {
    cfg::Config& C = cfg::get();
    C = cfg::Config{};
    C.verbose = false;
    C.debug_dump = false;
    C.veh_width_m = c.veh_width_m;
    C.safety_margin_m = c.safety_margin_m;
    C.lambda_smooth = c.lambda_smooth;
    C.max_outer_iters = c.max_outer_iters;
    C.max_inner_iters = c.max_inner_iters;
    C.step_init = c.step_init;
    C.step_min = c.step_min;
    C.armijo_c = c.armijo_c;
    C.kappa_eps = c.kappa_eps;
    C.v_cap_mps = c.v_cap_mps;
    C.mass_kg = c.mass_kg;
    C.Cd = c.Cd;
    C.A_front_m2 = c.A_front_m2;
    C.rho_air = c.rho_air;
    C.c_rr = c.c_rr;
    C.P_max_W = c.P_max_W;
    C.mu = c.mu;
    C.a_total_max = c.a_total_max;
    C.a_lat_max = c.a_lat_max;
    C.a_long_acc_cap = c.a_long_acc_cap;
    C.a_long_brake_cap = c.a_long_brake_cap;
    C.w_time_gain = c.w_time_gain;
    C.time_gamma_power = c.time_gamma_power;
    C.time_weight_use_inv_v = c.time_weight_use_inv_v != 0;
    C.inv_v_gain = c.inv_v_gain;
    C.max_vpass_iters = c.max_vpass_iters;
    C.use_total_ge_lat = c.use_total_ge_lat != 0;
}
}  // namespace

int main(int argc, char** argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s problem.bin mincurv|mintime budget_s min_calls\n", argv[0]);
        return 1;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", argv[1]); return 1; }
    int32_t hdr[4];
    double lw[2];
    rl_cfg c;
    bool ok = read_all(f, hdr, sizeof hdr) && read_all(f, lw, sizeof lw) && read_all(f, &c, sizeof c);
    const int N = hdr[0], closed = hdr[1], Ei = hdr[2], Eo = hdr[3];
    ok = ok && N >= 0 && Ei >= 0 && Eo >= 0;
    vector<double> ctr(ok ? 2 * (size_t)N : 0), in(ok ? 4 * (size_t)Ei : 0), out(ok ? 4 * (size_t)Eo : 0);
    ok = ok && read_all(f, ctr.data(), ctr.size() * 8) && read_all(f, in.data(), in.size() * 8) &&
         read_all(f, out.data(), out.size() * 8);
    fclose(f);
    if (!ok) { fprintf(stderr, "bad problem file\n"); return 1; }
    const bool mintime = std::strcmp(argv[2], "mintime") == 0;
    const double budget = std::atof(argv[3]);
    const int min_calls = std::atoi(argv[4]);

    vector<Vec2> center((size_t)N);
    for (int i = 0; i < N; ++i) center[i] = {ctr[2 * i], ctr[2 * i + 1]};
    auto segs = [](const vector<double>& s) {
        SegVec e(s.size() / 4);
        for (size_t k = 0; k < e.size(); ++k) e[k] = {{s[4 * k], s[4 * k + 1]}, {s[4 * k + 2], s[4 * k + 3]}};
        return e;
    };
    const SegVec innerE = segs(in), outerE = segs(out);
    apply(c);
    std::streambuf* old = std::cerr.rdbuf(nullptr);

    vector<double> ms;
    double lap = 0.0, xsum = 0.0;
    const auto t_start = std::chrono::steady_clock::now();
    for (;;) {
        const auto t0 = std::chrono::steady_clock::now();
        if (mintime) {
            auto r = raceline_min_time::compute_min_time_raceline(center, innerE, outerE, lw[1], lw[0], closed != 0);
            lap = r.lap_time;
            xsum = r.raceline.empty() ? 0.0 : r.raceline[0].x;
        } else {
            auto r = raceline_min_curv::compute_min_curvature_raceline(center, innerE, outerE, lw[1], lw[0], closed != 0);
            xsum = r.raceline.empty() ? 0.0 : r.raceline[0].x;
        }
        const auto t1 = std::chrono::steady_clock::now();
        ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        const double el = std::chrono::duration<double>(t1 - t_start).count();
        if ((int)ms.size() >= min_calls && el >= budget) break;
    }
    std::cerr.rdbuf(old);
    const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    printf("{\"calls\": %zu, \"seconds\": %.6f, \"lap\": %.17g, \"x0\": %.17g, \"ms\": [", ms.size(), total, lap, xsum);
    for (size_t k = 0; k < ms.size(); ++k) printf("%s%.4f", k ? ", " : "", ms[k]);
    printf("]}\n");
    return 0;
}
