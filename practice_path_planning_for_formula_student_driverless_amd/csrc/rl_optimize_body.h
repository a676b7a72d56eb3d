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
#ifndef RL_PRIO
// wave priority by progress (rl_kernels.h progress_prio): build.py sets 1 for the throughput
// shapes' translation units (two or more instances per CU); 0 keeps the issue order
#define RL_PRIO 0
#endif
template <int K, int T, bool CLOSED, bool MT, bool RAGGED>
__device__ __forceinline__ void rl_optimize_body(const KParams& p, const int b) {
#define RL_BID_ b
#include "rl_optimize_body.inc"
#undef RL_BID_
}

// one launch of one plan: workgroup b runs instance b.  RL_BODY_CALL (per translation unit,
// build.py): 1 calls rl_optimize_body, 0 expands the body in the kernel itself.  The two forms
// are the same statements, but LLVM optimises them differently: the call form spills fewer
// SGPRs in the throughput shapes (C2 8.54 -> 8.45 ms), the kernel form schedules the
// latency shapes' min-time better (testday1/3 1.71 / 1.80 ms against 1.78 / 1.88,
// profiles/r06/ab_body_refactor.log); results are the same bit for bit.  (The kernel form is
// the round-5 kernel's code exactly, the unsigned workgroup id in the two addresses included.)
#ifndef RL_BODY_CALL
#define RL_BODY_CALL 1
#endif
template <int K, int T, bool CLOSED, bool MT, bool RAGGED>
__global__ __launch_bounds__(T, (MinWaves<K, T, MT>::value)) void rl_optimize_kernel(KParams p) {
#if RL_BODY_CALL
    rl_optimize_body<K, T, CLOSED, MT, RAGGED>(p, blockIdx.x);
#else
    const int b = blockIdx.x;
#define RL_BID_ blockIdx.x
#include "rl_optimize_body.inc"
#undef RL_BID_
#endif
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
