// rl_device.h — device-side math shared by the raceline kernels (gfx950, fp64).
//
// Every helper restates one reference expression (ref = /root/reference/src/main.cpp)
// with the same operations in the same order; the translation unit is compiled
// with -ffp-contract=off so no a*b+c is fused.  f64 +,-,*,/ and sqrt are
// correctly rounded on gfx950 (div_scale/div_fmas/div_fixup and the
// Newton-refined rsq sequence), so they reproduce the CPU bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rl {

// libstdc++ std::max / std::min / std::clamp comparison forms (NaN behaviour included)
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }
// a - 2*b as the reference evaluates it (two roundings: 2*b, then the difference), in one
// instruction: 2*b is exact (barring overflow past 8.9e307), so the fused form rounds the
// same exact value once, zero signs included
__device__ __forceinline__ double sub2x(double a, double b) { return __builtin_fma(-2.0, b, a); }
// a wave-uniform double held in an SGPR pair (readfirstlane): fp64 values computed on the
// VALU land in VGPRs, where a kernel-lifetime constant would occupy two registers per lane
__device__ __forceinline__ double uni(double x) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                            __builtin_amdgcn_readfirstlane(__double2loint(x)));
}
__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double sclamp(double v, double lo, double hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }

// SURVEY.md §8d α-seed: splitmix64(seed, counter=i) -> U(-1,1), seed 0 -> 0
__host__ __device__ __forceinline__ double seed_value(uint64_t seed, int32_t i, double sigma) {
    if (seed == 0) return 0.0;
    uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    double u = (double)(z >> 11) * 0x1.0p-53;
    return sigma * (2.0 * u - 1.0);
}

// Segment record prepared on the host from a reference segment pair (S0,S1):
//   vx,vy = S1-S0             (rayIntersectSegment ref:482; minDistance ab ref:505)
//   denom = max(1e-30, |ab|^2) (ref:506)
//   mx,my,hr = midpoint and half-length(+slack) for conservative culling
struct SegRec {
    double x0, y0, vx, vy, denom, mx, my, hr;
};
static_assert(sizeof(SegRec) == 64, "SegRec must be 64 B");

// Derived v-pass constants, evaluated exactly as the reference expressions
// of ax_max_at (ref:797-824) evaluate their constant prefixes.
// 72 bytes: it sits in every kernel's LDS block, whose size is allocated in 512-byte granules
// (one field more put the (4, 64) / (8, 64) blocks one granule over: C4 concurrent wall
// +30% at equal kernel times, profiles/r05/ab_c4_lds.log)
struct VConst {
    double a_total2;    // a_total^2, a_total = use_total_ge_lat ? max(a_total_max, a_lat_max) : a_total_max
    double kFd;         // (0.5*rho_air)*Cd*A_front_m2
    double Fr;          // mass_kg*9.81*c_rr
    double mass, Pmax, acc_cap, brk_cap;
    double h;
    int32_t pw_free;    // the power limit can never bind (see power_never_binds); read per step
    int32_t _pad;
};

#ifndef RL_VC_UNI
#define RL_VC_UNI 1      // v-pass constants in SGPRs (A/B knob)
#endif
// the v-pass constants as wave-uniform values (SGPR pairs) rather than per-lane VGPR copies
// of the LDS table: the register-resident relaxations hold 3 x Cr doubles per lane already
__device__ __forceinline__ VConst vconst_uniform(const VConst& s) {
    VConst c;
    c.a_total2 = uni(s.a_total2); c.kFd = uni(s.kFd); c.Fr = uni(s.Fr);
    c.mass = uni(s.mass); c.Pmax = uni(s.Pmax); c.acc_cap = uni(s.acc_cap); c.brk_cap = uni(s.brk_cap);
    c.h = uni(s.h);
    c.pw_free = __builtin_amdgcn_readfirstlane(s.pw_free);
    c._pad = 0;
    return c;
}

// True when the power limit of ax_max_at (ref:812-817) can never be the smallest of
// std::min({a_res, a_long_acc_cap, a_power}) (ref:818) for any speed the v-pass produces,
// so the forward step may skip its two divisions: every v of the profile is <= v_cap
// (ref:787-794 caps the start values, every later value is a std::min with them), and for
// 1e-6 < v <= v_cap the exact a_power(v) = P/(m v) - (kFd v^2 + Fr)/m is decreasing in v,
// so a_power(v) >= a_power(v_cap).  The computed a_power differs from the exact one by a
// few ulps of P/(m v) + (Fd + Fr)/m, far below the margin 1e-9 (1 + cap) required here, so
// it stays strictly above acc_cap >= min(a_res, acc_cap), and std::min never picks it (a
// NaN a_power is never picked either; v <= 1e-6 gives 1e9 > acc_cap).  The minimum is then
// min(a_res, acc_cap) bit for bit.
__device__ __forceinline__ bool power_never_binds(double Pmax, double mass, double kFd, double Fr, double v_cap,
                                                  double acc_cap) {
#if defined(RL_PWF) && RL_PWF == 0
    return false;                    // A/B knob: always evaluate the power limit
#endif
    if (!(Pmax > 0.0) || !(mass > 0.0) || !(v_cap > 1e-6) || !(kFd >= 0.0) || !(Fr >= 0.0)) return false;
    if (!(Pmax < 1e300) || !(mass < 1e300) || !(v_cap < 1e150) || !(kFd < 1e300) || !(Fr < 1e300)) return false;
    if (!(acc_cap < 1e8) || !(acc_cap > -1e300)) return false;
    const double lb = Pmax / (mass * v_cap) - (kFd * v_cap * v_cap + Fr) / mass;
    return lb > acc_cap + 1e-9 * (1.0 + fabs(acc_cap)) + 1e-9 * (Pmax / (mass * v_cap));
}

// IEEE maxNum / minNum on the fp64 VALU (one instruction each).  They equal the
// reference's std::max(lo, x) / std::min(hi, x) select forms for every x unless a
// bound is a zero: v_max_f64(-0, +0) = +0 where std::max(-0, +0) = -0, and
// v_min_f64(+0, -0) = -0 where std::min(+0, -0) = +0.  The projection uses them only
// in waves whose bounds hold no such zero (PGD loop, `zb`).  Inline asm: the operands
// need no canonicalisation (a NaN trial value would be a quiet NaN, and maxNum then
// returns the bound, as the select form does).
__device__ __forceinline__ double vmax_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// The v-pass steps below sit on the velocity profile's serial dependency chain (each
// step needs the previous one's value), so their latency, not their throughput, sets the
// v-pass time.  RL_VSTEP_FAST (A/B knob) shortens that chain without changing a bit:
//  * std::max(0.0, x) as v_max_f64(+0, x): equal for every x that is not a signalling NaN
//    (x > 0: x; x = +0, -0, < 0, -inf or a quiet NaN: +0 both ways); one instruction
//    instead of a compare and two selects;
//  * the std::min's ahead of each max(0, .) as v_min_f64: the two forms differ only in
//    the sign of a zero result (which the max(0, .) right after turns into +0 either way,
//    also through the brake path's `+ (Fd+Fr)/m`: -0 + y and +0 + y differ only in a zero
//    sign) or when the FIRST operand is a NaN (a_res = sqrt(max(0, .)) never is; a quiet
//    NaN cap or power limit gives the other operand in both forms);
//  * the power limit's divisions evaluated unconditionally (see vstep_fwd).
// A signalling-NaN cap would make v_min_f64 return a quiet NaN where the select form
// returns the other operand, so the caps are loaded canonicalised (vs_cap: a signalling
// NaN quieted, every other value unchanged, zero signs included).
#ifndef RL_VSTEP_FAST
#define RL_VSTEP_FAST 1
#endif
#if RL_VSTEP_FAST
__device__ __forceinline__ double vs_cap(double x) { return __builtin_canonicalize(x); }
__device__ __forceinline__ double vs_max0(double x) { return vmax_f64(0.0, x); }
__device__ __forceinline__ double vs_min(double a, double b) { return vmin_f64(a, b); }
#else
__device__ __forceinline__ double vs_cap(double x) { return x; }
__device__ __forceinline__ double vs_max0(double x) { return smax(0.0, x); }
__device__ __forceinline__ double vs_min(double a, double b) { return smin(a, b); }
#endif

// forward step of velocity_profile_forward_backward (ref:829-833):
//   a_acc = ax_max_at(v,k).first ; return sqrt(max(0, v*v + 2*a_acc*h))
__device__ __forceinline__ double vstep_fwd(const VConst& c, double vi, double ki) {
    double alat = vi * vi * fabs(ki);
    double a_res = sqrt(vs_max0(c.a_total2 - alat * alat));
    double a_acc = vs_min(a_res, c.acc_cap);
#if defined(RL_PW_BRANCH) && RL_PW_BRANCH == 0
    if (true) {
#else
    if (!__builtin_amdgcn_readfirstlane(c.pw_free)) {
#endif   // uniform per instance (power_never_binds)
        double Fd = c.kFd * vi * vi;
#if RL_VSTEP_FAST
        // evaluated unconditionally and selected: as the arm of a branch its two divisions ran
        // after the a_res chain instead of beside it (a discarded value has no effect)
        const double ap = c.Pmax / (c.mass * vi) - (Fd + c.Fr) / c.mass;
        double a_power = (c.Pmax > 0 && vi > 1e-6) ? ap : 1e9;
#else
        double a_power = (c.Pmax > 0 && vi > 1e-6) ? (c.Pmax / (c.mass * vi) - (Fd + c.Fr) / c.mass) : 1e9;
#endif
        a_acc = vs_min(a_acc, a_power);     // std::min({a_res, cap, a_power}) ref:818
    }
    a_acc = vs_max0(a_acc);
    return sqrt(vs_max0(__builtin_fma(2.0, a_acc * c.h, vi * vi)));   // 2*(a*h) is exact: the sum's one rounding
}
// backward step (ref:841-845): a_brk = ax_max_at(v,k).second
__device__ __forceinline__ double vstep_bwd(const VConst& c, double vi, double ki) {
    double alat = vi * vi * fabs(ki);
    double a_res = sqrt(vs_max0(c.a_total2 - alat * alat));
    double Fd = c.kFd * vi * vi;
    double a_brk = vs_min(a_res, c.brk_cap) + (Fd + c.Fr) / c.mass;
    a_brk = vs_max0(a_brk);
    return sqrt(vs_max0(__builtin_fma(2.0, a_brk * c.h, vi * vi)));
}

}  // namespace rl
