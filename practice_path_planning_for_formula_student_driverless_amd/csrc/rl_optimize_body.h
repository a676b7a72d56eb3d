// rl_optimize_body.h — the register-resident optimiser kernel template
// (rl_optimize_kernel<K, T, CLOSED, MT, RAGGED>), shared by the translation units that
// instantiate its shapes (rl_kernels.hip: throughput shapes, rl_kernels_lat.hip: latency
// shapes for small batches).
//
// MI355X (gfx950) batched raceline optimizer: steps 7-8 of the
// reference pipeline (ref = /root/reference/src/main.cpp) as one persistent
// kernel per (problem, mode).
//
// Mapping:
//   * one workgroup = one track instance (α-seed / cfg sweep point); the whole
//     optimiser (max_outer_iters linearisations x PGD/Armijo inner loop x
//     corridor updates, and for min-time the v(s) passes) runs in one launch;
//   * thread t owns K contiguous samples [t*K, t*K+K).  The mutable inner-loop
//     state (α, grad, α_trial, lo, hi, q1, q2, D1α[, γ²]) lives in VGPRs; the
//     read-only linearisation (A1,A2 | N0,W) is staged once per outer
//     iteration in LDS as [pair][k][t] double2 (lane-consecutive 16-B reads,
//     bank-conflict free, each thread reads only its own entries);
//   * the tridiagonal stencils need one neighbour on each side: chunk edges
//     move lane-to-lane with DPP wave_shr/wave_shl and across waves through a
//     per-wave LDS edge table; an evaluation costs two workgroup barriers;
//   * J, Jsm and the Armijo decrease are reduced per wave then across waves in
//     a fixed order, so the accept/backtrack decision is uniform;
//   * outer-level state (P, n, α_total, α_last) lives in the instance's slice of
//     the result arrays in HBM and is touched once per outer iteration;
//   * the serial v(s) recurrence runs as an exact chunked relaxation: every
//     thread recomputes its chunk from the pass-start values with the value its
//     neighbour published, until no published value changes; the fixed point
//     is the serial result bit for bit.
// All arithmetic is IEEE fp64 (-ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_abi.h"
#include "rl_corridor.h"
#include "rl_device.h"
#include "rl_kernels.h"
#include "rl_math.h"

#define RL_AI __attribute__((always_inline))

namespace rl {

#ifndef RL_CK
#define RL_CK 2
#endif
constexpr int CK = (RL_CK < 8 ? RL_CK : 8);   // corridor sub-chunk (samples per ring pass)
#ifndef RL_MD_TIGHT
#define RL_MD_TIGHT 0    // fallback search: nearest-midpoint radius pass (rl_corridor.h ring_mindist; A/B: +0.8% C2 here, -21% C5 in the streaming kernel)
#endif
// v-pass: in-wave relaxation rounds between two cross-wave exchanges (barriers), per shape.
// A/B (scripts/ab_variants.py, caps 1 (= one barrier per round), 2, 4, 8, 16): the (4, 512)
// latency shape gains 5 % from 8-16 rounds; the (8, 256) throughput shape at two instances
// per CU loses 1-3 % with any cap above 1 (a chain that reaches a wave edge waits for the
// slowest wave's rounds), so it keeps one barrier per round; single-wave instances need
// no barrier at all.
#ifndef RL_VP_ROUNDS
#define RL_VP_ROUNDS 16
#endif
template <int K, int T>
struct VpRounds {
    // latency shapes (K <= 2 or 1024 lanes: one instance per CU, rl_kernels_lat.hip) take
    // the in-wave rounds like the (4, 512) latency shape
    static constexpr int value = (T == 64) ? 0x7fffffff
                                 : ((K == 4 && T == 512) || K <= 2 || T >= 1024) ? RL_VP_ROUNDS : 1;
};
#ifndef RL_MD_PRUNE
#define RL_MD_PRUNE 1    // fallback search: running-minimum pruning in the exact walk
#endif

// Diagnostic build only (-DRL_STAMPS=1): per-phase s_memtime totals of each
// workgroup's wave 0, written to a device array no other code reads.
#ifdef RL_STAMPS
static __device__ unsigned long long rl_dbg_stamps[16384][16];   // per translation unit
#define RL_STAMP(slot)                                              \
    do {                                                            \
        __builtin_amdgcn_sched_barrier(0);                          \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
        st_acc[slot] += t_ - st_last;                               \
        st_last = t_;                                               \
        __builtin_amdgcn_sched_barrier(0);                          \
    } while (0)
#else
#define RL_STAMP(slot) do {} while (0)
#endif
// finer stamps inside the latency shapes' evaluation (-DRL_STAMPS_EVAL=1 with RL_STAMPS):
// 11 projection, 12 stencil + partial sums + LDS writes, 13 wave sum, 14 barrier + block
// sum + Armijo test, 15 gradient.  Each stamp serialises the code around it, so the shares
// are indicative only.
#if defined(RL_STAMPS) && defined(RL_STAMPS_EVAL)
#define RL_ESTAMP(slot) RL_STAMP(slot)
#else
#define RL_ESTAMP(slot) do {} while (0)
#endif

// std::pow for a non-default time_gamma_power (ref:960), out of line: inlined, its
// temporaries competed with the kernel's live state for registers (min-time (8,256):
// 328 -> 192 B/lane scratch); the default power 2 never calls it
static __device__ __attribute__((noinline)) double pow_noinline(double x, double y) { return pow(x, y); }
// heading (ref:616), correctly rounded (rl_math.h atan2_cr), out of line for the same reason
static __device__ __attribute__((noinline)) double atan2_noinline(double y, double x) { return atan2_cr(y, x); }

// ------------------------------------------------------------ wave primitives
// x from another lane for patterns where every lane has a source (quad_perm, row_ror):
// no `old` operand, so no register has to be zeroed first
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
// wave-uniform sum of x over the 64 lanes: DPP butterflies inside each 16-lane row
// (quad_perm, row_ror:4, row_ror:8), then the four row sums via readlane, combined
// in a fixed order.  No LDS round trip.
// row_bcast steps: rows outside ROWS keep an unspecified value.  Only lane 63 of the
// reduction is read, and those rows never feed it, so no register is zeroed first.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_rows(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, ROWS, 0xf, false);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, ROWS, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum(double x) {
    x += dpp<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dpp<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dpp<0x124>(x);   // row_ror:4
    x += dpp<0x128>(x);   // row_ror:8  -> every lane holds its row sum r0..r3
    x += dpp_rows<0x142, 0xa>(x);   // row_bcast:15 into rows 1,3: r0+r1, r2+r3 (rows 0,2: unused)
    x += dpp_rows<0x143, 0xc>(x);   // row_bcast:31 into rows 2,3: lane 63 = (r2+r3)+(r0+r1)
    return readlane(x, 63);
}
// two wave sums at once, step by step (each chain fills the other's DPP hazard
// window); same association as wave_sum, so bit-identical results
__device__ __forceinline__ void wave_sum2(double& x, double& y) {
    x += dpp<0xB1>(x);  y += dpp<0xB1>(y);
    x += dpp<0x4E>(x);  y += dpp<0x4E>(y);
    x += dpp<0x124>(x); y += dpp<0x124>(y);
    x += dpp<0x128>(x); y += dpp<0x128>(y);
    x += dpp_rows<0x142, 0xa>(x); y += dpp_rows<0x142, 0xa>(y);
    x += dpp_rows<0x143, 0xc>(x); y += dpp_rows<0x143, 0xc>(y);
    x = readlane(x, 63);
    y = readlane(y, 63);
}
// (vmax_f64 / vmin_f64: rl_device.h)
// x + (the same register of the lane 16 (permlane16) / 32 (permlane32) rows away): the
// swap exchanges the odd rows of one copy with the even rows of the other, so the two
// copies afterwards hold (r0,r0,r2,r2) and (r1,r1,r3,r3) (resp. the half-waves), and their
// sum is r0+r1 in rows 0-1 and r2+r3 in rows 2-3 (resp. lo+hi everywhere)
__device__ __forceinline__ double swap16_add(double x) {
    const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
    return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ double swap32_add(double x) {
    const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
    return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
// Two wave sums in one butterfly: the first step leaves x-pair sums in the even lanes
// and y-pair sums in the odd lanes; every later step (quad_perm [2,3,0,1], row_ror 4/8,
// the row and half-wave swaps) keeps lane parity, so one chain serves both sums.
// Returns Σx in every even lane and Σy in every odd lane.
__device__ __forceinline__ double wave_sum_xy(double x, double y, bool odd) {
    const double send = odd ? x : y, keep = odd ? y : x;
    double z = keep + dpp<0xB1>(send);    // quad_perm [1,0,3,2]: the partner lane l^1
    z += dpp<0x4E>(z);                     // quad_perm [2,3,0,1]
    z += dpp<0x124>(z);                    // row_ror:4
    z += dpp<0x128>(z);                    // row_ror:8: row sums
    z = swap16_add(z);
    return swap32_add(z);
}
// lane l <- lane l-1 (wave_shr:1); lane 0 keeps `edge` (bound_ctrl off: no write)
__device__ __forceinline__ double dpp_from_left_or(double x, double edge) {
    int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(x), 0x138, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// lane l <- lane l+1 (wave_shl:1); lane 63 keeps `edge`
__device__ __forceinline__ double dpp_from_right_or(double x, double edge) {
    int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(x), 0x130, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(x), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// keep v opaque to loop-invariant code motion (stops hoisting of per-sample addresses)
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// materialise x here (the value cannot be sunk past this point into a later branch)
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }

// a[idx] for a runtime idx as a bit-mask blend: a select chain would be turned
// into an indexed load, which forces the whole array out of VGPRs into scratch
template <int K>
__device__ __forceinline__ double pick(const double (&a)[K], int idx) {
    unsigned long long r = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned long long m = 0ull - (unsigned long long)(k == idx);
        r |= (unsigned long long)__double_as_longlong(a[k]) & m;
    }
    return __longlong_as_double((long long)r);
}
template <int K>
__device__ __forceinline__ void put(double (&a)[K], int idx, double v) {
    const unsigned long long vb = (unsigned long long)__double_as_longlong(v);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned long long m = 0ull - (unsigned long long)(k == idx);
        const unsigned long long ab = (unsigned long long)__double_as_longlong(a[k]);
        a[k] = __longlong_as_double((long long)((ab & ~m) | (vb & m)));
    }
}

// v-pass warm starts (min-time, see vpass): 0 off, 1 multi-wave shapes only, 2 every
// min-time shape.  In the one-wave (K, 64) throughput shapes (C1/C4) the in-wave rounds are
// cheap DPP steps and the starts leave the kernel time as it is, while their 2 KB table
// costs LDS granules that concurrent plans share (C4 min-time 8.7 -> 11.9 ms wall at equal
// kernel times, scripts/ab_c4_single.py, profiles/r05/ab_c4_lds.log)
#ifndef RL_WARM
#define RL_WARM 1
#endif
template <int T, bool MT>
struct WarmStart {
    static constexpr bool value = MT && (RL_WARM == 2 || (RL_WARM == 1 && T > 64));
};

// min-time: warm start of the v-pass relaxations, per thread the incoming value its chunk
// ended with in [0] the first forward sweep of the previous v pass, [1] the latest forward
// sweep, [2] / [3] the same for the backward sweeps (+inf: none yet; see vpass).  An empty
// base (no bytes) in the shapes without warm starts.
template <int T, bool WARM>
struct WarmTab {
    double vg[4][T];
};
template <int T>
struct WarmTab<T, false> {};

// Edge tables of the neighbour exchange, one row per exchange slot.  Every lane stores
// (branch-free): the lane that publishes into its row's tail, every other lane into its own
// entry of the row's head (a sink nobody reads).  One address register per table serves
// all four slots (the slot is an immediate offset).  One wave exchanges by readlane and
// needs none: an empty base, 6 KB less LDS per (K, 64) block.
template <int NW>
struct PubTab {
    static constexpr int RF = 64 + NW;
    double pubF[4][RF];          // [s][64 + w]: first value of lane 0 of wave w
    double pubL[4][RF];          // [s][64 + w]: last value of lane 63 of wave w
    double pubW[4][65];          // [s][64]: last valid value of the last active thread (closed wrap)
};
template <>
struct PubTab<1> {};

// The small tables come first: their (mostly wave-uniform) addresses then fit the 16-bit
// offset field of ds_read/ds_write, so one base register serves them all.  The block size
// is allocated in 512-byte LDS granules and sets how many blocks of concurrent plans share
// a CU: one granule more on the (4, 64) / (8, 64) min-time blocks cost the C4 concurrent
// sweep 30% at equal kernel times (profiles/r05/ab_c4_lds.log).
template <int K, int T, bool WARM>
struct alignas(16) Smem : PubTab<T / 64>, WarmTab<T, WARM> {
    static constexpr int NW = T / 64;
    double red[3][NW];           // per-wave partial sums of an evaluation
    double red2[2][NW];          // other block reductions
    double bc[4];                // broadcast scalars
    int ctr;                     // corridor work queue: next chunk of 64*CK samples
    VConst vc;                   // v-pass constants (read per v pass: no registers held across the kernel)
    union {
        double2 coef[2][K][T];   // [0]: (A1,A2)  [1]: (N0,W)   (precompute_lin_geom_generic)
        double vin[2][T];        // v-pass relaxation: published outgoing values
    } u;
};

// --------------------------------------------------------------- the kernel
// Variant for 1024 < N <= 2048 (the C2/C3 tracks): RL_MID_K samples per lane,
// RL_MID_T lanes per instance, RL_MID_W waves per SIMD requested from the
// register allocator.  Build-time knobs so variants can be A/B-timed.
#ifndef RL_MID_K
#define RL_MID_K 8
#endif
#ifndef RL_MID_T
#define RL_MID_T 256
#endif
#ifndef RL_MID_W
#define RL_MID_W 2
#endif
// min-time at 1024 < N <= 2048: the extra γ² state favours 4 samples per lane
#ifndef RL_MIDMT_K
#define RL_MIDMT_K 4
#endif
#ifndef RL_MIDMT_T
#define RL_MIDMT_T 512
#endif
#ifndef RL_MIDMT_W
#define RL_MIDMT_W 2
#endif

// single-wave (4, 64) variant (N <= 256: the bundled tracks, C1/C4) per mode.  A/B on
// C4-shaped plans (scripts/ab_c4.py, kernel-time sum): 4 waves/SIMD (128 VGPRs) spilled
// 148 B/lane (min-curv) and 596 B/lane (min-time); 2 waves/SIMD: 61.9 -> 51.1 ms
#ifndef RL_SMALL_W
#define RL_SMALL_W 2
#endif
#ifndef RL_SMALLMT_W
#define RL_SMALLMT_W 2
#endif
// (8, 64) (256 < N <= 512) and (8, 128) (512 < N <= 1024) per mode; (8, 64) min-time
// spills 540 B/lane at 2 waves/SIMD, 1 wave/SIMD lets it use the AGPRs (C4: -2.5%)
#ifndef RL_S8_W
#define RL_S8_W 2
#endif
#ifndef RL_S8MT_W
#define RL_S8MT_W 1
#endif
#ifndef RL_M8_W
#define RL_M8_W 2
#endif
#ifndef RL_M8MT_W
#define RL_M8MT_W 2
#endif

// latency shapes (rl_kernels_lat.hip: K <= 2, or 1024 lanes): one instance per CU, so one
// wave per SIMD may use the whole register file (1024 lanes need 4 per SIMD regardless)
#ifndef RL_LAT_W
#define RL_LAT_W 1
#endif
// waves per SIMD to keep resident (caps the register budget the compiler may use)
template <int K, int T, bool MT>
struct MinWaves {
    static constexpr int value = (K <= 2 || T >= 1024)                   ? RL_LAT_W
                                 : (K == RL_MID_K && T == RL_MID_T)       ? RL_MID_W
                                 : (K == RL_MIDMT_K && T == RL_MIDMT_T) ? RL_MIDMT_W
                                 : (T >= 512)                           ? 1
                                 : (T == 64 && K == 4)                  ? (MT ? RL_SMALLMT_W : RL_SMALL_W)
                                 : (T == 64 && K == 8)                  ? (MT ? RL_S8MT_W : RL_S8_W)
                                 : (T == 128 && K == 8)                 ? (MT ? RL_M8MT_W : RL_M8_W)
                                                                        : 2;
};

// RAGGED: N % K != 0, i.e. one thread holds a partial chunk (decided per launch; the
// exact-multiple version carries no partial-chunk bookkeeping).  One workgroup runs instance b
// of the launch p; the kernels below call it with their own (p, b).
template <int K, int T, bool CLOSED, bool MT, bool RAGGED>
__device__ __forceinline__ void rl_optimize_body(const KParams& p, const int b) {
    constexpr int NW = T / 64;
    constexpr bool WARM = WarmStart<T, MT>::value;
    __shared__ Smem<K, T, WARM> sm;
#ifdef RL_STAMPS
    unsigned long long st_acc[16] = {};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int N = p.N;
    const int base = tid * K;
    const int Ta = (N + K - 1) / K;
    const bool active = tid < Ta;
    // samples of this thread (without a partial chunk: K or 0, one lane mask for every k)
    const int cnt = RAGGED ? min(K, max(0, N - base)) : (tid < Ta ? K : 0);
    const int cntL = N - (Ta - 1) * K;                  // samples of the last active thread
    // wave-uniform: does this wave hold the (only) partial chunk?  Every other
    // lane is either full (cnt == K) or inactive, and inactive lanes carry exact
    // zeros (coefficients, corridor, state, neighbour values), so their sums
    // need no masking.
    const int wid_u = __builtin_amdgcn_readfirstlane(wid);
    const bool part_wave = RAGGED && (cntL != K) && (((Ta - 1) >> 6) == wid_u);
    // wave-uniform: this wave holds the last active thread or lies beyond it
    const bool tail_wave = wid_u >= ((Ta - 1) >> 6);
    // Open tracks without a partial chunk (OPEN_FAST): the boundary forms of DiffOpsOpen
    // (ref:560-579) touch samples 0, 1, N-2 and N-1 only, i.e. chunk positions k = 0, 1
    // of lane 0 (fl) and K-2, K-1 of the last active lane (ll).  Every lane evaluates the
    // interior forms; in a wave holding one of those lanes (edge_wave, uniform) the four
    // positions take their boundary coefficients and operands by lane-masked selects
    // (eval_j / eval_grad below), so the boundary costs a few selects, not general forms
    // with per-sample conditions (whose lane masks, held across the PGD loop, spilled).
    // (K >= 4: lane 0 holds samples 0, 1 and the last active lane N-2, N-1; the latency
    // shapes with K <= 2 take the general per-sample forms)
    constexpr bool OPEN_FAST = !CLOSED && !RAGGED && K >= 4;
    const bool edge_wave = OPEN_FAST && (wid_u == 0 || wid_u == ((Ta - 1) >> 6));
    const bool fl = tid == 0, ll = tid == Ta - 1;
    const rl_cfg& C = p.cfg[p.ncfg == 1 ? 0 : b];
    const uint64_t seed = p.seeds ? p.seeds[b] : 0ull;

    const double Lb = p.Ls ? p.Ls[b] : p.L;
    // (uni: the kernel-lifetime constants live in SGPR pairs, not in VGPRs.  Besides the
    // registers this saves, it keeps them out of the register allocator's VGPR/AGPR
    // live-range copies: with this compiler such a copy can be placed inside a divergent
    // region (the ragged init loop below), so the lanes outside EXEC kept a stale copy --
    // seen as ax = 0/(garbage 2h) = -0 on the last, partial chunk of an open track; an SGPR
    // copy is lane-independent)
    const double h = uni(Lb / (double)N);                // ref:690 / 913
    const double* __restrict__ CEN = p.center + (size_t)b * (size_t)p.center_stride;
    const double invh = uni(1.0 / h), inv2h = uni(1.0 / (2 * h)), invh2 = uni(1.0 / (h * h));   // ref:547, 562
    const double m2invh2 = uni(-2 * invh2);              // ref:577 (-2*invh2)
    const double two_h = uni(2 * h), hh = uni(h * h);    // ref:602-603 divisors
    const double lam = C.lambda_smooth;
    const double lam2 = uni(2.0 * lam);                  // ref:673 2.0*lambda_smooth*gsm
    const double lam_act = active ? lam : 0.0;           // inactive lanes' Σa1² drops out of J
    const bool is_last = tid == Ta - 1;
    const bool wrap_lane = tail_wave && is_last;         // the closed wrap's right neighbour is sample 0
    // PGD constants in registers (the cfg lives in global memory the kernel also writes)
    const double step_init = C.step_init, step_min = C.step_min, armijo_c = C.armijo_c;
    const int max_inner = C.max_inner_iters;

    const size_t off = (size_t)b * (size_t)N;
    double* __restrict__ X = p.x + off;                  // P.x (state, then output)
    double* __restrict__ Y = p.y + off;
    double* __restrict__ NX = p.nx + off;                // normals (scratch)
    double* __restrict__ NY = p.ny + off;
    double* __restrict__ ATOT = p.alpha_total + off;
    double* __restrict__ ALAST = p.alpha_last + off;

    // ---- neighbour exchange (DPP in-wave, LDS across waves and for the wrap) ----
    // before a barrier: the wave's edge values (and the wrap value) go to LDS
    double* aF = nullptr;
    double* aL = nullptr;
    double* aW = nullptr;
    if constexpr (NW > 1) {
        aF = &sm.pubF[0][(lane == 0) ? 64 + wid : lane];
        aL = &sm.pubL[0][(lane == 63) ? 64 + wid : lane];
        aW = &sm.pubW[0][(tid == Ta - 1) ? 64 : lane];
    }
    auto xpub = [&](int slot, const double (&a)[K]) RL_AI {
        if constexpr (NW > 1) {              // one wave: xget reads the edges with readlane
            constexpr int RF = PubTab<NW>::RF;
            const double first = a[0], last = a[K - 1];
            aF[slot * RF] = first;
            aL[slot * RF] = last;
            if (!RAGGED || cntL == K) {
                aW[slot * 65] = last;
            } else if (part_wave) {
                const double lv = pick(a, cntL - 1);
                if (tid == Ta - 1) sm.pubW[slot][64] = lv;
            }
        }
    };
    // after the barrier: lv = value at sample base-1, rv = value at base+cnt (wrapped).
    // In-wave neighbours by DPP; lanes 0 / 63 keep the other wave's edge value.
    auto xget = [&](int slot, const double (&a)[K], double& lv, double& rv) RL_AI {
        double el, ef;
        if constexpr (NW == 1) {
            // the same values as the LDS tables hold: the last valid value of the last
            // active thread (closed wrap) and lane 0's first value
            const double lastv = (!RAGGED || cntL == K) ? a[K - 1] : pick(a, cnt - 1);
            el = readlane(lastv, Ta - 1);
            ef = readlane(a[0], 0);
        } else {
            el = (wid > 0) ? sm.pubL[slot][64 + ((wid > 0) ? wid - 1 : 0)] : sm.pubW[slot][64];   // wave-uniform reads
            ef = sm.pubF[slot][64 + ((wid + 1 < NW) ? wid + 1 : 0)];
        }
        lv = dpp_from_left_or(a[K - 1], el);
        rv = dpp_from_right_or(a[0], ef);
        // the closed wrap for the last active thread; inactive lanes keep whatever
        // their neighbours hold (finite) -- their coefficients and bounds are zero,
        // so only their Σa1² term could leak, and lam_act removes it
        // (one lane-masked select: a wave-uniform branch on tail_wave would be if-converted
        // into a second select pair)
        if (CLOSED) {
            double e0 = ef;
            if constexpr (NW > 1) e0 = sm.pubF[slot][64];
            rv = wrap_lane ? e0 : rv;
        }
    };
    // the last active thread's padding slots take the right neighbour, so every
    // stencil reads a[k+1] (k<K-1) or rv (k=K-1) uniformly
    auto fill_pad = [&](double (&a)[K], double rv) RL_AI {
        if (part_wave && cnt != K && active) {
#pragma unroll
            for (int k = 0; k < K; ++k) a[k] = (k < cnt) ? a[k] : rv;
        }
    };

    // ---- ghost samples (latency shapes: K <= 2 samples per lane, several waves) ----
    // Each thread keeps the PGD state of its chunk's two neighbour samples (base-1 and
    // base+cnt): α, gradient and corridor bounds.  A trial's neighbour values are then its
    // own projections of them (select forms, the reference's std::min/std::max, which the
    // owner's maxNum/minNum forms equal bit for bit), so the trial needs no exchange and no
    // barrier; after an accepted step each thread recomputes the neighbours' gradients
    // from the q1, q2, D1α the evaluation left in LDS (every sample's, double-buffered by
    // the parity of the evaluation's one barrier), with the same expressions the owners
    // use.  One barrier per evaluation instead of two: in a one-instance launch the
    // barrier and its LDS round trip, not the arithmetic, set the latency.
#ifndef RL_GHOST
#define RL_GHOST 1
#endif
#ifndef RL_GHOST_KMAX
#define RL_GHOST_KMAX 2      // ghost samples for K <= this (A/B knob)
#endif
    constexpr bool GHOST = RL_GHOST && NW > 1 && K <= RL_GHOST_KMAX;
    // min-time latency shapes: the v-pass on one wave beside the corridor (VSPLIT, see vpass1w)
#ifndef RL_VSPLIT
#define RL_VSPLIT 1
#endif
    constexpr bool VSPLIT = RL_VSPLIT && MT && K == 1 && NW >= 2 && T <= 512;
    // Speculative gradient (latency shapes): every trial's gradient is evaluated before its
    // Armijo test (the bundled tracks accept 120 of 122-137 trials per outer iteration), so
    // the gradient's LDS reads and arithmetic run beside the J/decrease sums instead of
    // after them.  A rejected trial's gradient is discarded; nothing else changes.
#ifndef RL_SPEC_GRAD
#define RL_SPEC_GRAD 1
#endif
    constexpr bool SPEC = RL_SPEC_GRAD && GHOST;
    constexpr int KT = K * T;
    __shared__ double gq[GHOST ? 2 * 3 * KT : 1];      // [parity][q1 | q2 | D1α][sample]
    __shared__ double gred[GHOST ? 2 * 2 * NW : 1];    // [parity][J | decrease][wave]
    auto wrapj = [&](int j) RL_AI -> int {
        if (CLOSED) { j %= N; return j < 0 ? j + N : j; }
        return j < 0 ? 0 : (j >= N ? N - 1 : j);      // open: the boundary forms read none of these
    };
    const int jl2 = wrapj(base - 2), jl1 = wrapj(base - 1), jr1 = wrapj(base + cnt), jr2 = wrapj(base + cnt + 1);
    double cL = 0.0, gL = 0.0, loL = 0.0, hiL = 0.0, tL = 0.0;   // sample base-1
    double cR = 0.0, gR = 0.0, loR = 0.0, hiR = 0.0, tR = 0.0;   // sample base+cnt
    int gpar = 0, gpar_last = 0;

    // ---- P-neighbourhood helpers --------------------------------------------
    // P with a halo of 2 on each side: px[j] = P[base-2+j] (wrapped / clamped)
    auto loadP = [&](double (&px)[K + 4], double (&py)[K + 4]) RL_AI {
        const int bs = opaque(base);
        if (bs >= 2 && bs + K + 2 <= N) {
            const double* xb = X + (bs - 2);
            const double* yb = Y + (bs - 2);
#pragma unroll
            for (int j = 0; j < K + 4; ++j) { px[j] = xb[j]; py[j] = yb[j]; }
        } else {
#pragma unroll
            for (int j = 0; j < K + 4; ++j) {
                int g = bs - 2 + j;
                if (CLOSED) { g %= N; if (g < 0) g += N; }
                else g = g < 0 ? 0 : (g >= N ? N - 1 : g);
                px[j] = X[g];
                py[j] = Y[g];
            }
        }
    };
    // own sample k (clamped for padding)
    auto own = [&](int k) RL_AI -> int { return min(opaque(base) + k, N - 1); };
    // the `deriv` lambdas of ref:599-613 / 625-639 for own sample k (P index k+2)
    auto deriv = [&](const double (&px)[K + 4], const double (&py)[K + 4], int k, double& xp, double& yp,
                     double& xpp, double& ypp) RL_AI {
        const int i = base + k;
        if (N == 1) { xp = 1; yp = 0; xpp = ypp = 0; return; }
        if (CLOSED) {
            xp = (px[k + 3] - px[k + 1]) / two_h; yp = (py[k + 3] - py[k + 1]) / two_h;
            xpp = (sub2x(px[k + 3], px[k + 2]) + px[k + 1]) / hh; ypp = (sub2x(py[k + 3], py[k + 2]) + py[k + 1]) / hh;
        } else if (i == 0) {
            xp = (px[k + 3] - px[k + 2]) / h; yp = (py[k + 3] - py[k + 2]) / h;
            if (N >= 3) { xpp = (sub2x(px[k + 4], px[k + 3]) + px[k + 2]) / hh; ypp = (sub2x(py[k + 4], py[k + 3]) + py[k + 2]) / hh; }
            else xpp = ypp = 0;
        } else if (i == N - 1) {
            xp = (px[k + 2] - px[k + 1]) / h; yp = (py[k + 2] - py[k + 1]) / h;
            if (N >= 3) { xpp = (sub2x(px[k + 2], px[k + 1]) + px[k]) / hh; ypp = (sub2x(py[k + 2], py[k + 1]) + py[k]) / hh; }
            else xpp = ypp = 0;
        } else {
            xp = (px[k + 3] - px[k + 1]) / two_h; yp = (py[k + 3] - py[k + 1]) / two_h;
            xpp = (sub2x(px[k + 3], px[k + 2]) + px[k + 1]) / hh; ypp = (sub2x(py[k + 3], py[k + 2]) + py[k + 1]) / hh;
        }
    };
    // normals_from_points_generic ref:581-593, own valid samples -> NX/NY
    auto normals = [&]() RL_AI {
        if (!active) return;
        double px[K + 4], py[K + 4];
        loadP(px, py);
        const int bs = opaque(base);     // per-phase addresses (nothing hoisted across the PGD loop)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = bs + k;
            double tx, ty;
            if (N == 1) { tx = 1; ty = 0; }
            else if (CLOSED) { tx = (px[k + 3] - px[k + 1]) * 0.5; ty = (py[k + 3] - py[k + 1]) * 0.5; }
            else if (i == 0) { tx = px[k + 3] - px[k + 2]; ty = py[k + 3] - py[k + 2]; }
            else if (i == N - 1) { tx = px[k + 2] - px[k + 1]; ty = py[k + 2] - py[k + 1]; }
            else { tx = (px[k + 3] - px[k + 1]) * 0.5; ty = (py[k + 3] - py[k + 1]) * 0.5; }
            if (sqrt(tx * tx + ty * ty) < 1e-15) { tx = 1; ty = 0; }
            double vx = -ty, vy = tx;
            double n = sqrt(vx * vx + vy * vy);              // geom::normalize ref:132
            double ox = 0, oy = 0;
            if (!(n < 1e-15)) { ox = vx / n; oy = vy / n; }
            if (k < cnt) { NX[i] = ox; NY[i] = oy; }
        }
    };
    // normals (as `normals`) and the curvature of heading_curv_from_points_generic
    // (ref:595-620) from one load of the path: the min-time latency shapes (VSPLIT) need the
    // curvature before the v-pass wave starts, and computing it beside the normals takes it
    // off the path to the split
    auto normals_kappa = [&](double (&kaout)[K]) RL_AI {
        double px[K + 4], py[K + 4];
        loadP(px, py);
        const int bs = opaque(base);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = bs + k;
            double tx, ty;
            if (N == 1) { tx = 1; ty = 0; }
            else if (CLOSED) { tx = (px[k + 3] - px[k + 1]) * 0.5; ty = (py[k + 3] - py[k + 1]) * 0.5; }
            else if (i == 0) { tx = px[k + 3] - px[k + 2]; ty = py[k + 3] - py[k + 2]; }
            else if (i == N - 1) { tx = px[k + 2] - px[k + 1]; ty = py[k + 2] - py[k + 1]; }
            else { tx = (px[k + 3] - px[k + 1]) * 0.5; ty = (py[k + 3] - py[k + 1]) * 0.5; }
            if (sqrt(tx * tx + ty * ty) < 1e-15) { tx = 1; ty = 0; }
            double vx = -ty, vy = tx;
            double n = sqrt(vx * vx + vy * vy);              // geom::normalize ref:132
            double ox = 0, oy = 0;
            if (!(n < 1e-15)) { ox = vx / n; oy = vy / n; }
            if (active && k < cnt) { NX[i] = ox; NY[i] = oy; }
            double xp, yp, xpp, ypp;
            deriv(px, py, k, xp, yp, xpp, ypp);
            const double kav = (xp * ypp - yp * xpp) / pow15(smax(1e-12, xp * xp + yp * yp));
            kaout[k] = (active && k < cnt) ? kav : 0.0;
        }
    };
    // corridor blocks ref:701-711 / 749-756 (guard = width*0.5 + margin). The scan runs
    // in its own mapping: pass c gives lane t the CKK adjacent samples from (c*T+t)*CKK,
    // so a wave holds 64*CKK consecutive samples whose rays are spatially coherent and
    // the block culling of rl_corridor.h skips most of both rings. The bounds reach their
    // owner threads through LDS, in the coefficient area, which is free until lin-geom
    // fills it: slot k*T+t holds (lo, hi) of sample t*K+k.
    constexpr int CKK = CK < K ? CK : K;
    // the scan (no barrier): the chunks of the work queue, bounds into the coefficient area
    // pre: outer iteration 0 with the batch's precomputed bounds (KParams::lo0/hi0): the same
    // chunks, the bounds loaded instead of cast
    auto corridor_scan = [&](double guard, bool pre) RL_AI {
        double2* bnd = &sm.u.coef[0][0][0];
        // Several waves: chunks of 64*CKK samples from a work queue in LDS, so a wave whose
        // rays are cheap takes the next chunk instead of waiting at the barrier below for
        // the slowest wave (the bounds of a sample depend only on that sample).
        for (int c = (NW == 1) ? 0 : -1;; c = (NW == 1) ? c + 1 : -1) {
            if constexpr (NW > 1) {
                int q = 0;
                if (lane == 0) q = atomicAdd(&sm.ctr, 1);
                c = __builtin_amdgcn_readlane(q, 0);
            }
            if (c * 64 * CKK >= N) break;
            const int i0 = (c * 64 + lane) * CKK;
            double qx[CKK], qy[CKK], ux[CKK], uy[CKK], lc[CKK], hc[CKK];
            bool act[CKK];
#pragma unroll
            for (int k = 0; k < CKK; ++k) {
                const int i = min(i0 + k, N - 1);
                qx[k] = X[i]; qy[k] = Y[i]; ux[k] = NX[i]; uy[k] = NY[i];
                act[k] = i0 + k < N;
            }
            if (pre) {
#pragma unroll
                for (int k = 0; k < CKK; ++k) {
                    const int i = min(i0 + k, N - 1);
                    lc[k] = p.lo0[i];
                    hc[k] = p.hi0[i];
                }
            } else {
#ifdef RL_STAMPS
            RL_STAMP(7);
            corridor_bounds<CKK, RL_MD_TIGHT != 0, RL_MD_PRUNE != 0>(p.ring[0], p.ring[1], qx, qy, ux, uy, act, guard,
                                                                      lc, hc, [&](int s) { RL_STAMP(s); });
#else
            corridor_bounds<CKK, RL_MD_TIGHT != 0, RL_MD_PRUNE != 0>(p.ring[0], p.ring[1], qx, qy, ux, uy, act, guard,
                                                                      lc, hc);
#endif
            }
#pragma unroll
            for (int k = 0; k < CKK; ++k) {
                const int i = i0 + k;
                if (act[k]) bnd[(i % K) * T + i / K] = make_double2(lc[k], hc[k]);
            }
        }
    };
    // every thread's own bounds (and its ghost samples') from the coefficient area
    auto corridor_collect = [&](double (&lo)[K], double (&hi)[K]) RL_AI {
        const double2* bnd = &sm.u.coef[0][0][0];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double2 v = bnd[k * T + tid];
            lo[k] = (k < cnt) ? v.x : 0.0;
            hi[k] = (k < cnt) ? v.y : 0.0;
        }
        if constexpr (GHOST) {                                // the neighbour samples' bounds
            const double2 vl = bnd[(jl1 % K) * T + jl1 / K], vr = bnd[(jr1 % K) * T + jr1 / K];
            loL = vl.x; hiL = vl.y; loR = vr.x; hiR = vr.y;
        }
        __syncthreads();      // the area is written again (v-pass relaxation, coefficients)
    };
    auto corridor = [&](double guard, bool pre, double (&lo)[K], double (&hi)[K]) RL_AI {
        corridor_scan(guard, pre);
        corridor_collect(lo, hi);
    };

    // ---- v(s) profile: velocity_profile_forward_backward ref:782-862 ---------
    if (tid == 0) {
        VConst vc;
        const double a_total = C.use_total_ge_lat ? smax(C.a_total_max, C.a_lat_max) : C.a_total_max;   // ref:802-804
        vc.a_total2 = a_total * a_total;
        vc.kFd = 0.5 * C.rho_air * C.Cd * C.A_front_m2;     // ref:810 constant prefix
        vc.Fr = C.mass_kg * 9.81 * C.c_rr;                   // ref:811
        vc.mass = C.mass_kg; vc.Pmax = C.P_max_W;
        vc.acc_cap = vs_cap(C.a_long_acc_cap); vc.brk_cap = vs_cap(C.a_long_brake_cap);
        vc.h = h;
        vc.pw_free = power_never_binds(C.P_max_W, C.mass_kg, vc.kFd, vc.Fr, C.v_cap_mps, vc.acc_cap);
        sm.vc = vc;          // first read after the outer loop's first barrier
    }
    if constexpr (WARM) {    // v-pass warm starts: none yet (each thread reads only its own)
#pragma unroll
        for (int j = 0; j < 4; ++j) sm.vg[j][tid] = INFINITY;
    }

    auto same_bits = [](double a, double b) RL_AI -> bool { return __double_as_longlong(a) == __double_as_longlong(b); };
    // returns sweeps executed; padding samples hold ka=0, v=+inf (never bind)
    auto vpass = [&](const double (&ka)[K], double (&v)[K]) RL_AI -> int {
        const VConst vc = RL_VC_UNI ? vconst_uniform(sm.vc) : sm.vc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double kk = fabs(ka[k]);
            double v_kappa = sqrt(C.a_lat_max / smax(kk, C.kappa_eps));
            v[k] = (k < cnt) ? smin(C.v_cap_mps, v_kappa) : INFINITY;   // ref:787-794
        }
        const int iters = C.max_vpass_iters;
        int sweeps = 0;
        const bool has_right = active && (base + cnt < N);   // chunk feeds a right neighbour
        const bool has_left = active && (base > 0);
        for (int s = 0; s < iters; ++s) {
            ++sweeps;
            double vstart[K];
#pragma unroll
            for (int k = 0; k < K; ++k) vstart[k] = v[k];
            // ---- forward pass (ref:829-833)
            // Exact chunked relaxation.  Every chunk first evaluates with no incoming constraint;
            // then, within each wave, a lane takes its left neighbour's outgoing value by DPP
            // (lane 0 the previous wave's, through LDS) and re-evaluates while that value
            // changes: the in-wave rounds need no barrier, and one barrier per round across
            // waves passes the wave edges on until no published edge changes.  A chunk
            // re-evaluated with a new incoming value stops as soon as a value equals, bit for
            // bit, the one it already holds (each step depends only on the previous value), so
            // its outgoing value would repeat.  Each chunk's result is a deterministic function
            // of its incoming value, so the fixed point is the serial result bit for bit.
            // Warm start: the first round takes as incoming value the one this chunk ended with
            // in the same sweep of the previous v pass (sweep 0) or in the previous sweep (lane
            // 0 also keeps it as the previous wave's value until that wave publishes).  Any
            // start reaches the same fixed point -- chunk t is exact from round t on, and the
            // rounds end only when every incoming value equals its neighbour's outgoing one --
            // and a start that is already exact leaves nothing to re-evaluate.
            {
                double g = INFINITY;
                if constexpr (WARM) g = sm.vg[s == 0 ? 0 : 1][tid];
                double in_prev = -1.0;       // sentinel (valid values are >= 0 or +inf)
                double out = INFINITY;       // the value this chunk passes right
                double wave_in = g;          // lane 0: the previous wave's last outgoing value
                double pub = -1.0;           // lane 63: the value last published for the next wave
                bool first = true;
                for (int ro = 0;; ++ro) {
                    bool conv = false;         // wave-uniform: the in-wave relaxation settled
                    for (int ir = 0; ir < VpRounds<K, T>::value; ++ir) {
                        double in = dpp_from_left_or(out, wave_in);
                        if (first) in = g;
                        if (!has_left) in = INFINITY;
                        bool ch = false;
                        if (active && in != in_prev) {
                            in_prev = in;
                            double cur = vstart[0];
                            if (has_left) cur = smin(vstart[0], in);     // v[i+1] = min(v[i+1], vf)
                            bool go = first || !same_bits(cur, v[0]);
                            v[0] = cur;
#pragma unroll
                            for (int k = 0; k + 1 < K; ++k) {
                                if (!__any(go)) break;
                                if (go) {
                                    const double vf = vstep_fwd(vc, v[k], ka[k]);
                                    const double nv = (k + 1 < cnt) ? smin(vstart[k + 1], vf) : INFINITY;
                                    go = first || !same_bits(nv, v[k + 1]);
                                    v[k + 1] = nv;
                                }
                            }
                            if (has_right && go) {
                                const double o = vstep_fwd(vc, v[K - 1], ka[K - 1]);
                                ch = o != out;
                                out = o;
                            }
                        }
                        if (first) { first = false; continue; }
                        if (!__any(ch)) { conv = true; break; }
                    }
                    if constexpr (NW == 1) break;
                    bool pch = false;
                    if (lane == 63 && has_right) {
                        pch = out != pub;
                        pub = out;
                        sm.u.vin[ro & 1][wid] = out;
                    }
                    if (!__syncthreads_or(pch || !conv) && ro > 0) break;
                    if (wid > 0) wave_in = sm.u.vin[ro & 1][wid - 1];
                }
                if constexpr (WARM) {
                    sm.vg[1][tid] = in_prev;
                    if (s == 0) sm.vg[0][tid] = in_prev;
                }
            }
            // closed wrap (ref:834-839): v[0] = min(v[0], f(v[N-1], k[N-1]))
            if (CLOSED) {
                if (active && base + cnt == N) {
                    double vl = (cnt == K) ? v[K - 1] : pick(v, cnt - 1);
                    double kl = (cnt == K) ? ka[K - 1] : pick(ka, cnt - 1);
                    sm.bc[0] = vstep_fwd(vc, vl, kl);
                }
                __syncthreads();
                if (tid == 0) v[0] = smin(v[0], sm.bc[0]);
                __syncthreads();
            }
            // ---- backward pass (ref:841-845): the same relaxation from the right
            {
                double vpre[K];
#pragma unroll
                for (int k = 0; k < K; ++k) vpre[k] = v[k];
                double g = INFINITY;                 // warm start (as forward)
                if constexpr (WARM) g = sm.vg[s == 0 ? 2 : 3][tid];
                double in_prev = -1.0;
                double out = INFINITY;
                double wave_in = g;          // lane 63: the next wave's first outgoing value
                double pub = -1.0;           // lane 0: the value last published for the previous wave
                bool first = true;
                for (int ro = 0;; ++ro) {
                    bool conv = false;         // wave-uniform: the in-wave relaxation settled
                    for (int ir = 0; ir < VpRounds<K, T>::value; ++ir) {
                        double in = dpp_from_right_or(out, wave_in);
                        if (first) in = g;
                        if (!has_right) in = INFINITY;
                        bool ch = false;
                        if (active && in != in_prev) {
                            in_prev = in;
                            // has_right => full chunk (only the last thread can be partial)
                            const double cur = has_right ? smin(vpre[K - 1], in) : vpre[K - 1];
                            bool go = first || !same_bits(cur, v[K - 1]);
                            v[K - 1] = cur;
#pragma unroll
                            for (int k = K - 2; k >= 0; --k) {
                                if (!__any(go)) break;
                                if (go) {
                                    const double vb = vstep_bwd(vc, v[k + 1], ka[k + 1]);
                                    const double nv = (k < cnt) ? smin(vpre[k], vb) : INFINITY;
                                    go = first || !same_bits(nv, v[k]);
                                    v[k] = nv;
                                }
                            }
                            if (has_left && go) {
                                const double o = vstep_bwd(vc, v[0], ka[0]);
                                ch = o != out;
                                out = o;
                            }
                        }
                        if (first) { first = false; continue; }
                        if (!__any(ch)) { conv = true; break; }
                    }
                    if constexpr (NW == 1) break;
                    bool pch = false;
                    if (lane == 0 && has_left) {
                        pch = out != pub;
                        pub = out;
                        sm.u.vin[ro & 1][wid] = out;
                    }
                    if (!__syncthreads_or(pch || !conv) && ro > 0) break;
                    if (wid + 1 < NW) wave_in = sm.u.vin[ro & 1][wid + 1];
                }
                if constexpr (WARM) {
                    sm.vg[3][tid] = in_prev;
                    if (s == 0) sm.vg[2][tid] = in_prev;
                }
            }
            // closed wrap (ref:846-850): v[N-1] = min(v[N-1], b(v[0], k[0]))
            if (CLOSED) {
                if (tid == 0) sm.bc[1] = vstep_bwd(vc, v[0], ka[0]);
                __syncthreads();
                if (active && base + cnt == N) {
                    if (cnt == K) v[K - 1] = smin(v[K - 1], sm.bc[1]);
                    else put(v, cnt - 1, smin(pick(v, cnt - 1), sm.bc[1]));
                }
                __syncthreads();
            }
            bool any_change = false;
#pragma unroll
            for (int k = 0; k < K; ++k) any_change |= (k < cnt) && (v[k] != vstart[k]);
            if (!__syncthreads_or(any_change)) break;   // later sweeps are exact repeats
        }
        return sweeps;
    };

    // ---- min-time latency shapes (K = 1, several waves): the v-pass on one wave -------
    // VSPLIT: the v-pass (ref:782-862) runs on the last wave while the other waves scan the
    // corridor (the two are independent: both need only the updated path), so a one-instance
    // launch pays the longer of the two instead of their sum.  The v-pass wave holds KP = T/64
    // consecutive samples per lane and relaxes them within the wave (DPP only, no barrier),
    // with the warm start and early stops of `vpass`; curvature in and speeds out go through
    // LDS (vsv).  Same fixed point, so the same values bit for bit.
    constexpr int KP = VSPLIT ? T / 64 : 1;
    __shared__ double vsv[VSPLIT ? T : 1];
    double vwg[4] = {INFINITY, INFINITY, INFINITY, INFINITY};   // warm starts (the v-pass wave's lanes)
    auto vpass1w = [&]() RL_AI -> int {
        const VConst vc = RL_VC_UNI ? vconst_uniform(sm.vc) : sm.vc;
        const int b0 = lane * KP;
        const int c1 = min(KP, max(0, N - b0));
        double ka1[KP], v[KP];
#pragma unroll
        for (int j = 0; j < KP; ++j) {
            ka1[j] = (j < c1) ? vsv[b0 + j] : 0.0;
            const double kk = fabs(ka1[j]);
            const double v_kappa = sqrt(C.a_lat_max / smax(kk, C.kappa_eps));
            v[j] = (j < c1) ? smin(C.v_cap_mps, v_kappa) : INFINITY;   // ref:787-794
        }
        const bool act1 = c1 > 0, hasL = act1 && b0 > 0, hasR = act1 && b0 + c1 < N;
        const int lastl = (N - 1) / KP;                 // the lane holding sample N-1
        const int iters = C.max_vpass_iters;
        int sweeps = 0;
        for (int s = 0; s < iters; ++s) {
            ++sweeps;
            double vstart[KP];
#pragma unroll
            for (int j = 0; j < KP; ++j) vstart[j] = v[j];
            {   // forward (ref:829-833)
                const double g = vwg[s == 0 ? 0 : 1];
                double in_prev = -1.0, out = INFINITY;
                bool first = true;
                for (;;) {
                    double in = dpp_from_left_or(out, INFINITY);
                    if (first) in = g;
                    if (!hasL) in = INFINITY;
                    bool ch = false;
                    if (act1 && in != in_prev) {
                        in_prev = in;
                        double cur = vstart[0];
                        if (hasL) cur = smin(vstart[0], in);
                        bool go = first || !same_bits(cur, v[0]);
                        v[0] = cur;
#pragma unroll
                        for (int j = 0; j + 1 < KP; ++j) {
                            if (!__any(go)) break;
                            if (go) {
                                const double vf = vstep_fwd(vc, v[j], ka1[j]);
                                const double nv = (j + 1 < c1) ? smin(vstart[j + 1], vf) : INFINITY;
                                go = first || !same_bits(nv, v[j + 1]);
                                v[j + 1] = nv;
                            }
                        }
                        if (hasR && go) {                     // hasR => full chunk
                            const double o = vstep_fwd(vc, v[KP - 1], ka1[KP - 1]);
                            ch = o != out;
                            out = o;
                        }
                    }
                    if (first) { first = false; continue; }
                    if (!__any(ch)) break;
                }
                vwg[1] = in_prev;
                if (s == 0) vwg[0] = in_prev;
            }
            if (CLOSED) {                                     // ref:834-839
                const double f = readlane(vstep_fwd(vc, pick(v, c1 - 1), pick(ka1, c1 - 1)), lastl);
                if (lane == 0) v[0] = smin(v[0], f);
            }
            {   // backward (ref:841-845)
                double vpre[KP];
#pragma unroll
                for (int j = 0; j < KP; ++j) vpre[j] = v[j];
                const double g = vwg[s == 0 ? 2 : 3];
                double in_prev = -1.0, out = INFINITY;
                bool first = true;
                for (;;) {
                    double in = dpp_from_right_or(out, INFINITY);
                    if (first) in = g;
                    if (!hasR) in = INFINITY;
                    bool ch = false;
                    if (act1 && in != in_prev) {
                        in_prev = in;
                        const double cur = hasR ? smin(vpre[KP - 1], in) : vpre[KP - 1];
                        bool go = first || !same_bits(cur, v[KP - 1]);
                        v[KP - 1] = cur;
#pragma unroll
                        for (int j = KP - 2; j >= 0; --j) {
                            if (!__any(go)) break;
                            if (go) {
                                const double vb = vstep_bwd(vc, v[j + 1], ka1[j + 1]);
                                const double nv = (j < c1) ? smin(vpre[j], vb) : INFINITY;
                                go = first || !same_bits(nv, v[j]);
                                v[j] = nv;
                            }
                        }
                        if (hasL && go) {
                            const double o = vstep_bwd(vc, v[0], ka1[0]);
                            ch = o != out;
                            out = o;
                        }
                    }
                    if (first) { first = false; continue; }
                    if (!__any(ch)) break;
                }
                vwg[3] = in_prev;
                if (s == 0) vwg[2] = in_prev;
            }
            if (CLOSED) {                                     // ref:846-850
                const double f = readlane(vstep_bwd(vc, v[0], ka1[0]), 0);
                if (lane == lastl) put(v, c1 - 1, smin(pick(v, c1 - 1), f));
            }
            bool any_change = false;
#pragma unroll
            for (int j = 0; j < KP; ++j) any_change |= (j < c1) && (v[j] != vstart[j]);
            if (!__any(any_change)) break;                    // later sweeps are exact repeats
        }
#pragma unroll
        for (int j = 0; j < KP; ++j)
            if (j < c1) vsv[b0 + j] = v[j];
        return sweeps;
    };

    // ---- difference operators (DiffOps / DiffOpsOpen ref:545-579) -------------
    auto d1_at = [&](int k, double am, double a0, double ap) RL_AI -> double {   // D1 ref:549-551 / 563-566
        if (CLOSED) return (ap - am) * inv2h;
        const int i = base + k;
        if (N == 1) return 0.0;
        if (i == 0) return (ap - a0) * invh;
        if (i == N - 1) return (a0 - am) * invh;
        return (ap - am) * inv2h;
    };
    auto d2_at = [&](int k, double am, double a0, double ap) RL_AI -> double {   // D2 ref:552-554 / 573-575
        if (CLOSED) return (sub2x(ap, a0) + am) * invh2;
        const int i = base + k;
        if (N <= 2 || i == 0 || i == N - 1) return 0.0;
        return (sub2x(ap, a0) + am) * invh2;
    };
    auto d1t_at = [&](int k, double vm, double v0, double vp) RL_AI -> double {  // D1T ref:555-557 / 567-572
        if (CLOSED) return (vm - vp) * inv2h;
        const int j = base + k;
        if (N <= 1) return 0.0;
        double acc = 0.0;     // the scatter order of ref:569-571 restated as a gather
        if (j >= 1) acc += ((j == 1) ? invh : inv2h) * vm;
        if (j == 0) acc += (-invh) * v0;
        else if (j == N - 1) acc += (+invh) * v0;
        if (j <= N - 2) acc += ((j + 1 == N - 1) ? -invh : -inv2h) * vp;
        return acc;
    };

    // gradient at own sample k from the stencil inputs around it (ref:668-673 / 886-893):
    // 2.0*(g1+g2) + lam2*gsm. Scaling by 2 is exact, so 2*(g1+g2) = 2*g1 + 2*g2 and
    // 2*g1 = D1T(q1) with the coefficients doubled (likewise D2T(q2)), bit for bit as
    // long as no product is subnormal: the factor 2 costs no multiplication.
    const double inv2h_x2 = uni(2.0 * inv2h), invh_x2 = uni(2.0 * invh), invh2_x2 = uni(2.0 * invh2),
                 m2invh2_x2 = uni(2.0 * m2invh2);
    auto d1t_x2 = [&](int k, double vm, double v0, double vp) RL_AI -> double {   // 2*D1T (ref:555-557 / 567-572)
        if (CLOSED) return (vm - vp) * inv2h_x2;
        const int j = base + k;
        if (N <= 1) return 0.0;
        double acc = 0.0;
        if (j >= 1) acc += ((j == 1) ? invh_x2 : inv2h_x2) * vm;
        if (j == 0) acc += (-invh_x2) * v0;
        else if (j == N - 1) acc += (+invh_x2) * v0;
        if (j <= N - 2) acc += ((j + 1 == N - 1) ? -invh_x2 : -inv2h_x2) * vp;
        return acc;
    };
    auto d2t_x2 = [&](int k, double vm, double v0, double vp) RL_AI -> double {   // 2*D2T (ref:558 / 576-578)
        if (CLOSED) return (sub2x(vp, v0) + vm) * invh2_x2;
        const int j = base + k;
        if (N <= 2) return 0.0;
        double acc = 0.0;
        if (j - 1 >= 1 && j - 1 <= N - 2) acc += (+invh2_x2) * vm;
        if (j >= 1 && j <= N - 2) acc += m2invh2_x2 * v0;
        if (j + 1 >= 1 && j + 1 <= N - 2) acc += (+invh2_x2) * vp;
        return acc;
    };
    auto grad_at = [&](int k, double q1m, double q10, double q1p, double q2m, double q20, double q2p, double am,
                       double a0, double ap) RL_AI -> double {
        double g1 = d1t_x2(k, q1m, q10, q1p);
        double g2 = d2t_x2(k, q2m, q20, q2p);
        double gsm = d1t_at(k, am, a0, ap);
        return (g1 + g2) + lam2 * gsm;
    };
    // the same gathers for an open interior sample (2 <= j <= N-3), term for term as the
    // general forms evaluate them there: acc = 0.0, then the products in the same order
    // (0.0 + x keeps the reference's zero signs)
    auto grad_int = [&](double q1m, double q1p, double q2m, double q20, double q2p, double am, double ap) RL_AI
        -> double {
        const double g1 = (0.0 + inv2h_x2 * q1m) + (-inv2h_x2) * q1p;
        const double g2 = ((0.0 + invh2_x2 * q2m) + m2invh2_x2 * q20) + invh2_x2 * q2p;
        const double gsm = (0.0 + inv2h * am) + (-inv2h) * ap;
        return (g1 + g2) + lam2 * gsm;
    };

    // ---- state ------------------------------------------------------------
    double G2[K];                                   // γ² (min-time)
    // corridor, α and α_trial, the gradient at α; al and an swap roles on every accepted
    // step (PGD loop), so nothing is copied.  One gradient array: an accepted trial's
    // gradient overwrites the old one, which nothing reads after the trial's evaluation
    double lo[K], hi[K], al[K], gr[K], an[K];
    double q1[K], q2[K], a1v[K];                    // gradient stencil inputs of the last evaluation
    // Min-curv keeps A1, A2, N0 of its own samples in registers from lin-geom on (the single
    // gradient array left the room: 247 VGPRs, no scratch) and reads only W from LDS per
    // evaluation.  A/B (build knob RL_A12_REG = 0 / 1 / 2: none / A1,A2 / A1,A2,N0 in
    // registers): C2 8.81 / 8.71 / 8.69 ms, bit-exact.  Min-time has no room (γ²), nor has
    // the open K = 8 min-curv kernel (its boundary stencils: scratch 100 -> 172 B/lane, the
    // open C2-shaped run 21.4 -> 25.0 ms).
#ifndef RL_A12_REG
#define RL_A12_REG 2
#endif
#ifndef RL_A12_MT
// min-time, shapes of 256+ lanes: 0 none, 1 N0, 2 A1+A2, 3 all three in registers.  2: C3
// (B = 4096, (8, 256)) min-time 39.19 -> 38.77 ms at 32 B/lane of scratch outside the loop,
// B = 256 ((4, 512)) 7.50 -> 7.34 ms, bit-exact (profiles/r05/ab_c3_a12mt.log)
#define RL_A12_MT 2
#endif
    // The latency shapes (K <= 2 samples per lane, registers to spare) hold all four
    // coefficients in registers: no LDS read on the evaluation's dependency chain
#ifndef RL_LAT_COEF_REG
#define RL_LAT_COEF_REG 1
#endif
    constexpr bool ALLR = RL_LAT_COEF_REG && K <= 2;
    constexpr bool A12R = ALLR || (RL_A12_REG && !MT && (CLOSED || K < 8)) || (MT && CLOSED && T >= 256 && (RL_A12_MT & 2));   // (A1, A2) in registers instead of LDS
    constexpr bool N0R = ALLR || (A12R && !MT && RL_A12_REG >= 2) || (MT && CLOSED && T >= 256 && (RL_A12_MT & 1));            // and N0
    constexpr bool WR = ALLR;                                                                                   // and W
    double A1r[K], A2r[K], N0r[K], Wr[K];

    // One evaluation (eval_cost_grad_frozen ref:654-675 / _timeweighted ref:866-895)
    // of the trial vector a: J (uniform across the workgroup) and the Armijo
    // decrease Σ grad*(a-α) (ref:733 / 1009); q1,q2,D1α and their in-wave
    // neighbours are left for eval_grad.
    // Σ g·(a − cur) over this lane's samples (the Armijo decrease, ref:733 / 1009)
    auto part_dec = [&](const double (&a)[K], const double (&cur)[K], const double (&g)[K]) RL_AI -> double {
        double pdec = 0.0;
        if (part_wave) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k < cnt) pdec = __builtin_fma(g[k], a[k] - cur[k], pdec);
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) pdec = __builtin_fma(g[k], a[k] - cur[k], pdec);
        }
        return pdec;
    };
    // the lane's part of one evaluation of a, given its neighbours' values lv, rv: the
    // residuals, this lane's J terms (returned) and the stencil inputs q1, q2, D1α, published
    // for the gradient (GHOST: LDS buffer gpar; else the halo exchange slots)
    auto eval_part = [&](double (&a)[K], double lv, double rv) RL_AI -> double {
        fill_pad(a, rv);
        double pJ = 0.0, pJsm = 0.0;
        double jr[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double2 c01 = A12R ? make_double2(A1r[k], A2r[k]) : sm.u.coef[0][k][tid];   // (A1, A2)
            const double2 c23 = WR ? make_double2(N0r[k], Wr[k])
                                : N0R ? make_double2(N0r[k], sm.u.coef[1][k][tid].y) : sm.u.coef[1][k][tid];   // (N0, W)
            double am = (k > 0) ? a[k - 1] : lv;
            double ap = (k + 1 < K) ? a[k + 1] : rv;
            double x1, x2;
            if (OPEN_FAST && edge_wave && (k == 0 || k == K - 1)) {
                // D1 one-sided and D2 = 0 at sample 0 (fl, k = 0) and N-1 (ll, k = K-1)
                // (ref:563-566, 573-575); the interior forms on every other lane
                const bool e = (k == 0) ? fl : ll;
                const double om = (k == 0 && fl) ? a[k] : am;
                const double op = (k == K - 1 && ll) ? a[k] : ap;
                x1 = (op - om) * (e ? invh : inv2h);
                const double x2i = (sub2x(ap, a[k]) + am) * invh2;
                x2 = e ? 0.0 : x2i;
            } else if (OPEN_FAST) {             // interior forms (ref:563-575)
                x1 = (ap - am) * inv2h;
                x2 = (sub2x(ap, a[k]) + am) * invh2;
            } else {
                x1 = d1_at(k, am, a[k], ap);
                x2 = d2_at(k, am, a[k], ap);
            }
            double r = c23.y * (c23.x + c01.x * x1 + c01.y * x2);
            jr[k] = r;
            double Wz = MT ? (c23.y * G2[k] * r) : (c23.y * r);
            q1[k] = c01.x * Wz;
            q2[k] = c01.y * Wz;
            a1v[k] = x1;
        }
        auto acc = [&](int k) RL_AI {    // Σ γ²r² (ref:881) / Σ z² (ref:661), Σ a1² (ref:662 / 882)
            pJ = __builtin_fma(MT ? G2[k] * jr[k] : jr[k], jr[k], pJ);
            pJsm = __builtin_fma(a1v[k], a1v[k], pJsm);
        };
        if (part_wave) {            // wave-uniform: only the wave with the partial chunk masks
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k < cnt) acc(k);
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) acc(k);
        }
        pJ = __builtin_fma(lam_act, pJsm, pJ);         // J += λ·Jsm (ref:663 / 883), per lane
        if constexpr (GHOST) {
            // every lane writes its K slots (base + k < K*T): a padding sample's slot is never
            // read, and unmasked stores keep the evaluation one basic block
            double* const Q = &gq[gpar * 3 * KT];
#pragma unroll
            for (int k = 0; k < K; ++k) { Q[base + k] = q1[k]; Q[KT + base + k] = q2[k]; Q[2 * KT + base + k] = a1v[k]; }
        } else {
            xpub(1, q1);
            xpub(2, q2);
            xpub(3, a1v);
        }
        return pJ;
    };
    auto eval_j = [&](double (&a)[K], const double (&cur)[K], const double (&g)[K], bool trial,
                      double& dec) RL_AI -> double {
        // J and the Armijo decrease only steer accept/stop decisions; the α iterates
        // never read them, so their accumulations use fma (their summation order
        // already differs from the reference's serial loop, ref:661-666)
        const double pdec = trial ? part_dec(a, cur, g) : 0.0;
        double lv, rv;
        RL_ESTAMP(11);
        if constexpr (GHOST) {               // the neighbours' values of a: no exchange
            lv = trial ? tL : cL;
            rv = trial ? tR : cR;
        } else {
            xpub(0, a);
#ifndef RL_PROBE_NOB1       // timing probe only (wrong results): the trial halo's barrier removed
            if constexpr (NW > 1) __syncthreads();
#endif
            xget(0, a, lv, rv);
        }
        const double pJ = eval_part(a, lv, rv);
        RL_ESTAMP(12);
        const double z = wave_sum_xy(pJ, pdec, lane & 1);   // lane 0: Σ J terms, lane 1: Σ decrease
        RL_ESTAMP(13);
        if constexpr (NW == 1) {             // the wave sums are the block sums
            dec = readlane(z, 1);
            return readlane(z, 0);
        }
        if constexpr (GHOST) {               // double-buffered: the only barrier of the evaluation
            double* const R = &gred[gpar * 2 * NW];
            if (lane < 2) R[lane * NW + wid] = z;
            __syncthreads();
            double J = R[0], D = R[NW];
#pragma unroll
            for (int w = 1; w < NW; ++w) { J += R[w]; D += R[NW + w]; }
            dec = D;
            gpar_last = gpar;
            gpar ^= 1;
            RL_ESTAMP(14);
            return J;
        }
        if (lane < 2) sm.red[lane][wid] = z;
        __syncthreads();
        double J = sm.red[0][0], D = sm.red[1][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) { J += sm.red[0][w]; D += sm.red[1][w]; }
        dec = D;
        return J;
    };
    // gradient of the last evaluation (ref:668-673 / 886-893)
    auto eval_grad = [&](double (&g)[K]) RL_AI {
        double l1, r1, l2, r2, l3, r3;
        if constexpr (GHOST) {
            const double* const Q = &gq[gpar_last * 3 * KT];
            l1 = Q[jl1]; r1 = Q[jr1]; l2 = Q[KT + jl1]; r2 = Q[KT + jr1]; l3 = Q[2 * KT + jl1]; r3 = Q[2 * KT + jr1];
            // the neighbour samples' gradients (the owners' expressions, index base-1 / base+cnt)
            const double q1a = (!RAGGED || cnt == K) ? q1[K - 1] : pick(q1, cnt > 0 ? cnt - 1 : 0);
            const double q2a = (!RAGGED || cnt == K) ? q2[K - 1] : pick(q2, cnt > 0 ? cnt - 1 : 0);
            const double a1a = (!RAGGED || cnt == K) ? a1v[K - 1] : pick(a1v, cnt > 0 ? cnt - 1 : 0);
            gL = grad_at(-1, Q[jl2], l1, q1[0], Q[KT + jl2], l2, q2[0], Q[2 * KT + jl2], l3, a1v[0]);
            gR = grad_at(cnt, q1a, r1, Q[jr2], q2a, r2, Q[KT + jr2], a1a, r3, Q[2 * KT + jr2]);
        } else {
            xget(1, q1, l1, r1);
            xget(2, q2, l2, r2);
            xget(3, a1v, l3, r3);
        }
        fill_pad(q1, r1);
        fill_pad(q2, r2);
        fill_pad(a1v, r3);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double q1m = (k > 0) ? q1[k - 1] : l1, q1p = (k + 1 < K) ? q1[k + 1] : r1;
            const double q2m = (k > 0) ? q2[k - 1] : l2, q2p = (k + 1 < K) ? q2[k + 1] : r2;
            const double am = (k > 0) ? a1v[k - 1] : l3, ap = (k + 1 < K) ? a1v[k + 1] : r3;
            if (OPEN_FAST && edge_wave && (k < 2 || k >= K - 2)) {
                // the gathers of DiffOpsOpen at samples 0, 1 (fl) and N-2, N-1 (ll) in the
                // interior shape (ref:567-578): a boundary form differs from it only in
                // one term's coefficient and operand, and a term it lacks is added as c*0
                // (the accumulator after 0.0 + x is never -0, so adding a zero leaves it)
                const bool e = (k < 2) ? fl : ll;
                double c1A = inv2h_x2, o1A = q1m, c1C = -inv2h_x2, o1C = q1p;
                double o2A = q2m, o2B = q2[k], o2C = q2p;
                double csA = inv2h, osA = am, csC = -inv2h, osC = ap;
                if (k == 0) {                        // j = 0: -h^-1 v0, no D2T vm, v0 terms
                    c1A = e ? -invh_x2 : c1A; o1A = e ? q1[k] : o1A;
                    o2A = e ? 0.0 : o2A; o2B = e ? 0.0 : o2B;
                    csA = e ? -invh : csA; osA = e ? a1v[k] : osA;
                } else if (k == 1) {                 // j = 1: h^-1 vm, no D2T vm term
                    c1A = e ? invh_x2 : c1A;
                    o2A = e ? 0.0 : o2A;
                    csA = e ? invh : csA;
                } else if (k == K - 2) {             // j = N-2: -h^-1 vp, no D2T vp term
                    c1C = e ? -invh_x2 : c1C;
                    o2C = e ? 0.0 : o2C;
                    csC = e ? -invh : csC;
                } else {                             // j = N-1: +h^-1 v0, no D2T v0, vp terms
                    c1C = e ? invh_x2 : c1C; o1C = e ? q1[k] : o1C;
                    o2B = e ? 0.0 : o2B; o2C = e ? 0.0 : o2C;
                    csC = e ? invh : csC; osC = e ? a1v[k] : osC;
                }
                const double g1 = (0.0 + c1A * o1A) + c1C * o1C;
                const double g2 = ((0.0 + invh2_x2 * o2A) + m2invh2_x2 * o2B) + invh2_x2 * o2C;
                const double gsm = (0.0 + csA * osA) + csC * osC;
                g[k] = (g1 + g2) + lam2 * gsm;
            } else if (OPEN_FAST) {
                g[k] = grad_int(q1m, q1p, q2m, q2[k], q2p, am, ap);
            } else {
                g[k] = grad_at(k, q1m, q1[k], q1p, q2m, q2[k], q2p, am, a1v[k], ap);
            }
        }
    };

    // ======================================================================
    // driver: compute_min_curvature_raceline ref:683-764 /
    //         compute_min_time_raceline ref:905-1052
    // ======================================================================
    if (active) {                                                // P := center
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (k < cnt) {
                X[base + k] = CEN[2 * (base + k)];
                Y[base + k] = CEN[2 * (base + k) + 1];
                ATOT[base + k] = 0.0;
                ALAST[base + k] = 0.0;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) { al[k] = 0.0; gr[k] = 0.0; G2[k] = 0.0; }

    const int MO = C.max_outer_iters;
    RL_STAMP(0);
    for (int outer = 0;; ++outer) {
        if (outer > 0 && active) {
            const int bu = opaque(base);
            // update (ref:743-746 / 1027-1030): alpha_last, P += n*alpha, alpha_accum
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (k < cnt) {
                    const int i = bu + k;
                    ALAST[i] = al[k];
                    X[i] += NX[i] * al[k];
                    Y[i] += NY[i] * al[k];
                    ATOT[i] += al[k];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) { al[k] = 0.0; gr[k] = 0.0; }   // ref:757 / 1041
        cL = cR = gL = gR = 0.0;
        __syncthreads();
        RL_STAMP(5);
        // ref:720 + seed: the first outer iteration starts from the seeded alpha
        auto seed_alpha = [&]() RL_AI {
            if (outer == 0 && seed != 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    // (opaque: keeps the seed values from being hoisted out of the outer
                    // loop, where they would hold 2K VGPRs for the whole kernel)
                    double s0 = seed_value(seed, opaque(base) + k, RL_SEED_SIGMA);
                    al[k] = (k < cnt) ? smin(hi[k], smax(lo[k], s0)) : 0.0;
                }
                if constexpr (GHOST) {
                    cL = smin(hiL, smax(loL, seed_value(seed, jl1, RL_SEED_SIGMA)));
                    cR = smin(hiR, smax(loR, seed_value(seed, jr1, RL_SEED_SIGMA)));
                }
            }
        };
        const double guard = (outer == 0 ? p.veh_width : C.veh_width_m) * 0.5 + C.safety_margin_m;
        const bool pre = outer == 0 && p.lo0 != nullptr;        // (uniform)
        double ka[K];
        bool ka_done = false;                                    // (uniform)
        if (outer < MO) {
            // normals + corridor (ref:692-711 initially with the veh_width argument,
            // ref:746-756 after each update with cfg veh_width_m)
            if (tid == 0) sm.ctr = 0;                            // read after the barrier below
            if constexpr (VSPLIT) {
                normals_kappa(ka);
                vsv[tid] = ka[0];
                ka_done = true;
            } else {
                normals();
            }
            __syncthreads();
            if constexpr (!VSPLIT) {                             // (VSPLIT: beside the v-pass below)
                corridor(guard, pre, lo, hi);
                seed_alpha();
            }
        }
        RL_STAMP(1);
        if ((MT || outer == MO) && !ka_done) {
            // heading_curv_from_points_generic ref:595-620
            double hd[K];
            double px[K + 4], py[K + 4];
            loadP(px, py);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                double xp, yp, xpp, ypp;
                deriv(px, py, k, xp, yp, xpp, ypp);
                double hdv = (outer == MO) ? atan2_noinline(yp, xp) : 0.0;   // heading is an output only
                double denom = pow15(smax(1e-12, xp * xp + yp * yp));
                double kav = (xp * ypp - yp * xpp) / denom;
                hd[k] = (k < cnt) ? hdv : 0.0;
                ka[k] = (k < cnt) ? kav : 0.0;
                __builtin_amdgcn_sched_barrier(0);
            }
            if (outer == MO && active) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (k < cnt) { p.heading[off + opaque(base) + k] = hd[k]; p.kappa[off + opaque(base) + k] = ka[k]; }
            }
        }
        if (MT) {
            double v[K];
            if constexpr (VSPLIT) {
                // the v-pass on the last wave, the corridor on the others, then both results
                // reach their owners through LDS
                if (!ka_done) {                                  // (the final outer iteration)
                    vsv[tid] = ka[0];
                    __syncthreads();
                }
                RL_STAMP(2);                                     // (stamps: curvature)
                if (wid_u == NW - 1) {
                    const int sw = vpass1w();                    // ref:947 / 1047
                    if (lane == 0 && p.sweeps) p.sweeps[(size_t)b * (MO + 1) + outer] = sw;
#if defined(RL_STAMPS) && !defined(RL_STAMPS_EVAL)
                    RL_STAMP(12);                                // (the v-pass wave's own slot)
#endif
                    // then the corridor chunks still in the queue: the 64-sample chunks of a
                    // bundled track (N = 187-261: 3-5 chunks) fall unevenly on the other waves
                    // (phase stamps: the join waited for the wave with two; two samples per lane
                    // instead, 128-sample chunks, was slower: training_map 1.49 -> 1.56 ms)
                    if (outer < MO) corridor_scan(guard, pre);
                } else if (outer < MO) {
#if defined(RL_STAMPS) && !defined(RL_STAMPS_EVAL)
                    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
                    corridor_scan(guard, pre);
                    if (wid_u < 3) st_acc[13 + wid_u] += __builtin_amdgcn_s_memtime() - ts0;   // per-wave scan time
#else
                    corridor_scan(guard, pre);
#endif
                }
                if (outer < MO) {
                    corridor_collect(lo, hi);                    // (its first barrier joins the two)
                    seed_alpha();
                } else {
                    __syncthreads();
                }
#if defined(RL_STAMPS) && !defined(RL_STAMPS_EVAL)
                RL_STAMP(11);                                    // (wave 0: the join's wait + collect)
#endif
                v[0] = active ? vsv[tid] : INFINITY;
            } else {
                const int sw = vpass(ka, v);                     // ref:947 / 1047
                if (tid == 0 && p.sweeps) p.sweeps[(size_t)b * (MO + 1) + outer] = sw;
            }
            if (outer == MO) {
                // ax and lap time (ref:854-860)
                double lv, rv;
                xpub(0, v);
                __syncthreads();
                xget(0, v, lv, rv);
                double lt = 0.0;
                if (active) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (k < cnt) {
                            const int i = base + k;
                            double v1;
                            if (i + 1 < N) v1 = (k + 1 < cnt) ? v[(k + 1 < K) ? k + 1 : k] : rv;
                            else v1 = CLOSED ? rv : v[k];
                            double v0 = v[k];
                            p.ax[off + i] = (v1 * v1 - v0 * v0) / two_h;   // ref:857 (2.0*h)
                            p.v[off + i] = v0;
                            lt += h / smax(1e-6, v[k]);
                        }
                    }
                }
                lt = wave_sum(lt);
                if (lane == 0) sm.red2[1][wid] = lt;
                __syncthreads();
                if (tid == 0 && p.lap) {
                    double tot = sm.red2[1][0];
                    for (int w = 1; w < NW; ++w) tot += sm.red2[1][w];
                    p.lap[b] = tot;
                }
            } else {
                // time weights γ² (ref:950-977)
                double v_avg = 0.0;
                if (C.time_weight_use_inv_v) {                   // ref:951 (read only when enabled)
                    double vs = 0.0;
#pragma unroll
                    for (int k = 0; k < K; ++k) if (k < cnt) vs += v[k];
                    vs = wave_sum(vs);
                    if (lane == 0) sm.red2[0][wid] = vs;
                    __syncthreads();
                    double tot = sm.red2[0][0];
                    for (int w = 1; w < NW; ++w) tot += sm.red2[0][w];
                    v_avg = tot / (double)(N > 1 ? N : 1);
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    double kk = fabs(ka[k]);
                    double vkappa = sqrt(C.a_lat_max / smax(kk, C.kappa_eps));
                    double rr = smin(1.0, v[k] / smax(1e-6, vkappa));
                    double r = rr * rr;                                     // std::pow(.., 2.0)
                    r = smin(1.0, smax(0.0, r));
                    double rp;
                    if (C.time_gamma_power == 2.0) rp = r * r;           // GCC folds pow(r, 2.0) to r*r
                    else rp = pow_noinline(r, C.time_gamma_power);
                    double corner_w = 1.0 + C.w_time_gain * rp;
                    double invv_w = 1.0;
                    if (C.time_weight_use_inv_v) {
                        double ratio = v_avg / smax(1e-6, v[k]);
                        invv_w = 1.0 + C.inv_v_gain * (ratio - 1.0);
                        if (invv_w < 1.0) invv_w = 1.0;
                        if (invv_w > 3.0) invv_w = 3.0;
                    }
                    double gamma = corner_w * invv_w;
                    G2[k] = (k < cnt) ? gamma * gamma : 0.0;
                }
                __syncthreads();   // vin (aliased with coef) fully consumed before coef is written
            }
        }
        RL_STAMP(2);
        if (outer == MO) break;

        // precompute_lin_geom_generic ref:622-651 -> LDS (own entries only)
        {
            double px[K + 4], py[K + 4];
            loadP(px, py);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                double xp, yp, xpp, ypp;
                deriv(px, py, k, xp, yp, xpp, ypp);
                const int i = own(k);
                double nxk = NX[i], nyk = NY[i];
                double a1 = nxk * ypp - nyk * xpp;
                double a2 = xp * nyk - yp * nxk;
                double n0 = xp * ypp - yp * xpp;
                double denom = pow15(smax(1e-12, xp * xp + yp * yp));
                double w = 1.0 / denom;
                const bool v = k < cnt;
                if (A12R) { A1r[k] = v ? a1 : 0.0; A2r[k] = v ? a2 : 0.0; }
                if (N0R) N0r[k] = v ? n0 : 0.0;
                else sm.u.coef[0][k][tid] = make_double2(v ? a1 : 0.0, v ? a2 : 0.0);
                if (WR) Wr[k] = v ? w : 0.0;
                else sm.u.coef[1][k][tid] = make_double2(v ? n0 : 0.0, v ? w : 0.0);
            }
        }
        RL_STAMP(3);
        // PGD + Armijo (ref:723-742 / 996-1026)
        // zb: this wave's bounds hold a zero of the sign that makes maxNum/minNum differ
        // from the reference's select forms (lo = -0, or hi = +0 on a valid sample;
        // padding and inactive lanes hold lo = hi = +0, where both forms agree).
        // Wave-uniform, fixed for the outer iteration.
        bool zb_lane = false;
#pragma unroll
        for (int k = 0; k < K; ++k)
            zb_lane |= (__double_as_longlong(lo[k]) == (long long)0x8000000000000000ull) ||
                       (hi[k] == 0.0 && k < cnt);
#ifdef RL_PROBE_NOZB      // timing probe only (zero signs may differ): every clamp as maxNum/minNum
        const bool zb = false;
        (void)zb_lane;
#else
        const bool zb = __builtin_amdgcn_ballot_w64(zb_lane) != 0;
#endif
        double step = step_init;
        // trial vector std::min(hi, std::max(lo, cur - step*grad)) (ref:731)
        auto project = [&](const double (&cur)[K], const double (&g)[K], double (&nxt)[K]) RL_AI {
            double ai[K];
#pragma unroll
            for (int k = 0; k < K; ++k) ai[k] = cur[k] - step * g[k];
            if (!zb) {
#pragma unroll
                for (int k = 0; k < K; ++k) nxt[k] = vmin_f64(hi[k], vmax_f64(lo[k], ai[k]));
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) nxt[k] = smin(hi[k], smax(lo[k], ai[k]));   // the select forms
            }
            if constexpr (GHOST) {               // the neighbour samples' trial values
#ifdef RL_PROBE_NOZB
                tL = vmin_f64(hiL, vmax_f64(loL, cL - step * gL));
                tR = vmin_f64(hiR, vmax_f64(loR, cR - step * gR));
#else
                tL = smin(hiL, smax(loL, cL - step * gL));
                tR = smin(hiR, smax(loR, cR - step * gR));
#endif
            }
        };
        double dec;
        double J = eval_j(al, al, gr, false, dec);
        eval_grad(gr);
        int evals = 1, accepts = 0, it = 0;
        double J_prev = J;
        // One inner iteration (ref:726-742) from (cur, g): trials in nxt; an accepted trial's
        // gradient replaces g (the projection and the Armijo decrease have read g by then;
        // a rejected trial leaves it).  Returns 2: accepted, go on (nxt is current); 1: stop
        // with nxt current; 0: stop with cur current.  The loop below alternates the roles
        // of al and an, so an accepted step copies nothing.
        auto inner = [&](const double (&cur)[K], double (&g)[K], double (&nxt)[K]) RL_AI -> int {
            if (it >= max_inner) return 0;
            ++it;
            int bt = 0;
            if constexpr (SPEC) {
                for (;;) {
                    project(cur, g, nxt);
                    double Jn = eval_j(nxt, cur, g, true, dec);
                    ++evals;
                    // the trial's gradient before the Armijo test, so its LDS reads and
                    // arithmetic overlap the J sums (pinned here: not sunk into the branch)
                    double gt[K];
                    const double gL0 = gL, gR0 = gR;
                    eval_grad(gt);
#pragma unroll
                    for (int k = 0; k < K; ++k) pin(gt[k]);
                    pin(gL);
                    pin(gR);
                    RL_ESTAMP(15);
                    if (Jn <= J + armijo_c * dec) {
#pragma unroll
                        for (int k = 0; k < K; ++k) g[k] = gt[k];
                        cL = tL; cR = tR;
                        J = Jn;
                        ++accepts;
                        break;
                    }
                    gL = gL0; gR = gR0;                  // a rejected trial keeps the gradient
                    step *= 0.5;
                    bt++;
                    if (step < step_min || bt >= 20) return 0;
                }
                if (fabs(J_prev - J) < 1e-10) return 1;
                J_prev = J;
                return 2;
            }
            for (;;) {
                project(cur, g, nxt);
                double Jn = eval_j(nxt, cur, g, true, dec);
                ++evals;
                if (Jn <= J + armijo_c * dec) {
                    eval_grad(g);
                    if constexpr (GHOST) { cL = tL; cR = tR; }
                    J = Jn;
                    ++accepts;
                    break;
                }
                step *= 0.5;
                bt++;
                if (step < step_min || bt >= 20) return 0;
            }
            if (fabs(J_prev - J) < 1e-10) return 1;
            J_prev = J;
            return 2;
        };
        bool in_an = false;
        for (;;) {
            int r = inner(al, gr, an);
            if (r != 2) { in_an = (r == 1); break; }
            r = inner(an, gr, al);
            if (r != 2) { in_an = (r == 0); break; }
        }
        if (in_an) {
#pragma unroll
            for (int k = 0; k < K; ++k) al[k] = an[k];
        }
        if (tid == 0) {
            if (p.evals) p.evals[(size_t)b * MO + outer] = evals;
            if (p.accepts) p.accepts[(size_t)b * MO + outer] = accepts;
        }
        RL_STAMP(4);
    }
    if (p.done) signal_done(p.done, b, p.epoch);
#ifdef RL_STAMPS
    RL_STAMP(6);
    if (tid == 0 && b < 16384) {
        for (int i = 0; i < 16; ++i)
            if (!(VSPLIT && (i == 12 || i == 14 || i == 15))) rl_dbg_stamps[b][i] = st_acc[i];
    }
    if (VSPLIT && lane == 0 && b < 16384) {                  // the v-pass wave; waves 1, 2's scans
        if (wid == NW - 1) rl_dbg_stamps[b][12] = st_acc[12];
        else if (wid == 1 || wid == 2) rl_dbg_stamps[b][13 + wid] = st_acc[13 + wid];
    }
#endif
}

// one launch of one plan: workgroup b runs instance b
template <int K, int T, bool CLOSED, bool MT, bool RAGGED>
__global__ __launch_bounds__(T, (MinWaves<K, T, MT>::value)) void rl_optimize_kernel(KParams p) {
    rl_optimize_body<K, T, CLOSED, MT, RAGGED>(p, blockIdx.x);
}

// one launch of up to RL_GROUP_MAX plans of one shape (rl_plan_run_group): the plans'
// workgroups follow each other (plan j owns blocks start[j] .. start[j+1]-1), so a grid of
// small plans fills the GPU as one launch instead of one launch per plan.  The launch
// parameters are kernel arguments (constant memory): plan j is found and read with scalar
// instructions, and instance b of it runs exactly as in that plan's own launch.
template <int K, int T, bool CLOSED, bool MT, bool RAGGED>
__global__ __launch_bounds__(T, (MinWaves<K, T, MT>::value)) void rl_optimize_group_kernel(KGroup g) {
    const int blk = blockIdx.x;
    int j = 0;
#pragma unroll
    for (int i = 1; i < RL_GROUP_MAX; ++i)
        if (i < g.n && blk >= g.start[i]) j = i;
    rl_optimize_body<K, T, CLOSED, MT, RAGGED>(g.p[j], blk - g.start[j]);
}

}  // namespace rl
