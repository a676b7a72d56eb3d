// rl_stream.hip — large-N (N > 4096) variant of the raceline optimiser for gfx950.
//
// Same algorithm and arithmetic as rl_kernels.hip (ref = /root/reference/src/main.cpp:
// compute_min_curvature_raceline ref:683-764, compute_min_time_raceline ref:905-1052),
// but the per-instance state no longer fits on chip (N=10000: ~1 MB per instance), so
// it streams through HBM / L2:
//   * one 1024-thread workgroup per instance; every state array (α, grad, α_trial,
//     lo, hi, A1, A2, N0, W, q1, q2, D1α, γ², v, κ) is an instance-major [B][N]
//     slice in HBM;
//   * stencil / PGD / corridor / geometry phases use the interleaved mapping
//     i = tile*1024 + tid: consecutive lanes touch consecutive doubles (coalesced),
//     neighbour reads i±1 hit the lines the wave just loaded;
//   * __syncthreads() orders the global writes of one phase before the next phase's
//     neighbour reads (all waves of the instance share one CU);
//   * the v(s) relaxation gives each thread a contiguous range [t*C, t*C+C) and
//     publishes the chunk's outgoing value through LDS, exactly like the
//     register-resident kernel;
//   * reductions: per-thread partial sums in a fixed sample order, DPP wave sums,
//     then the 16 wave partials in order.
// This is the HBM-bound configuration; its roofline is HBM bytes.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "rl_abi.h"
#include "rl_corridor.h"
#include "rl_device.h"
#include "rl_kernels.h"
#include "rl_math.h"

#ifndef RL_SPRIO
#define RL_SPRIO 0         // (A/B build knob: wave priority by progress, rl_kernels.h progress_prio)
#endif

namespace rl {

namespace {
// threads per instance (C5 A/B: 1024 -> 32.5 ms, 512 -> 38.3 ms, 256 -> 36.7 ms;
// profiles/r01/ab_c5_stream_wg.log)
#ifndef RL_STS
#define RL_STS 1024
#endif
constexpr int TS = RL_STS;        // threads per instance
constexpr int NWS = TS / 64;

// The lane's first index of a strided pass, opaque to the optimiser: its addresses (array
// base + 8·tid for each of the ~20 state arrays) are then formed inside the pass instead of
// being hoisted to the kernel's start as 64-bit per-lane pointers live across every outer
// iteration -- at the 128-VGPR budget of 1024 threads those were spilled and reloaded
#ifndef RL_S_OPQ
#define RL_S_OPQ 1
#endif
__device__ __forceinline__ int opq(int x) {
#if RL_S_OPQ
    asm volatile("" : "+v"(x));
#endif
    return x;
}

// The instance's state arrays (StreamBufs: [B][15][N] in one allocation) through one buffer
// resource: a load / store takes the resource (4 SGPRs, one per instance), the array's byte
// offset (an SGPR) and the lane's byte offset i*8 (one VGPR shared by every array indexed by i).
// As plain pointers each array's 64-bit base held an SGPR pair for the whole kernel (30 of its
// 106 SGPRs for these 15 arrays) and the kernel spilled SGPRs to VGPR lanes, VGPRs to scratch.
// Offsets stay below 2^31: 15 * N * 8 B with N <= RL_STREAM_MAX_N.  A/B knob: 0 = pointers.
#ifndef RL_S_BUF
#define RL_S_BUF 1
#endif
#ifndef RL_S_BUF_OPQ
#define RL_S_BUF_OPQ 1
#endif
typedef unsigned int u32x2_s __attribute__((ext_vector_type(2)));
struct BufArr {
    __amdgpu_buffer_rsrc_t r;
    int so;                     // byte offset of the array within the instance's resource
    struct Ref {
        __amdgpu_buffer_rsrc_t r;
        int so, vo;
        __device__ __forceinline__ operator double() const {
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
        }
        __device__ __forceinline__ Ref& operator=(double v) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_s, v), r, vo, so, 0);
            return *this;
        }
        __device__ __forceinline__ Ref& operator=(const Ref& o) { return *this = (double)o; }   // a store, not a copy
        __device__ __forceinline__ Ref& operator+=(double v) { return *this = (double)*this + v; }
    };
    __device__ __forceinline__ Ref operator[](int i) const {
#if RL_S_BUF_OPQ
        int n8 = so;            // (so holds N*8 and k: field k's offset formed at each access)
        asm volatile("" : "+s"(n8));
        return Ref{r, k * n8, i * 8};
#else
        return Ref{r, so, i * 8};
#endif
    }
    int k;
};

template <int CTRL>
__device__ __forceinline__ double dpp_s(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_s(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ double wave_sum_s(double x) {
    x += dpp_s<0xB1>(x);
    x += dpp_s<0x4E>(x);
    x += dpp_s<0x124>(x);
    x += dpp_s<0x128>(x);
    return (readlane_s(x, 0) + readlane_s(x, 16)) + (readlane_s(x, 32) + readlane_s(x, 48));
}

// backtracking trials evaluated per pass over the state once the first trial of an
// inner iteration is rejected (both optimisers)
// corridor samples per lane in the streaming kernel (C5 A/B: 1 -> 36.0 ms, 2 -> 32.4 ms,
// 4 -> 41.6 ms; scripts/ab_c5.py)
#ifndef RL_SFUSE
#define RL_SFUSE 1       // lin-geom (and min-time curvature) in the normals pass (A/B knob)
#endif
#ifndef RL_SVP_REG
#define RL_SVP_REG 1     // register-resident v-pass for RL_SVP_MIN <= ceil(N/1024) <= RL_SVP_MAX (A/B knob)
#endif
#ifndef RL_SVP_MIN
#define RL_SVP_MIN 5
#endif
#ifndef RL_SVP_MAX
#define RL_SVP_MAX 12
#endif
#ifndef RL_SCK
#define RL_SCK 2
#endif
#ifndef RL_BT_FIRST
#define RL_BT_FIRST 1    // the first trial of an inner iteration joins a batch (its vectors stored)
#endif
#ifndef RL_BT_BATCH
#define RL_BT_BATCH 4
#endif
#ifndef RL_BT_FIRST_MT
#define RL_BT_FIRST_MT 0 // min-time: the first trial joins a batch as well (A/B knob)
#endif
// adaptive first trial: it joins a batch exactly when the instance's previous first trial was
// rejected (the all-rejected regime of C5, E_k = 21), and is evaluated alone otherwise (the
// accepting regime, where a batch's three extra steps are wasted work).  Uniform per
// instance; exact either way (a batched step is bit-identical to a lone trial).
#ifndef RL_BT_ADAPT
#define RL_BT_ADAPT 1
#endif
constexpr int RED_SLOTS = 3 * RL_BT_BATCH > 4 ? 3 * RL_BT_BATCH : 4;

struct SSmem {
    double red[RED_SLOTS][NWS];
    struct {
        double vin[2][TS];             // v-pass relaxation
    } u;
    // warm start of the v-pass relaxations: per thread, the incoming value its chunk ended
    // with in [0] the first forward sweep of the previous v pass, [1] the latest forward
    // sweep, [2] / [3] the same for the backward sweeps (+inf: none yet)
    double vg[4][TS];
    double bc[4];
    double* pp[7];    // the instance's output arrays X .. KA (RL_S_PLDS), read where used
    VConst vc;        // v-pass constants (read at the start of each v pass: no registers held)
    int ctr;          // corridor work queue: next chunk of 64*RL_SCK samples
};

// std::pow for a non-default time_gamma_power (ref:960), out of line: inlined, OCML's pow
// held registers across the whole kernel (min-time scratch 416 -> 272 B/lane)
__device__ __attribute__((noinline)) double pow_stream(double x, double y) { return pow(x, y); }
// heading (ref:616), correctly rounded (rl_math.h); out of line so its double-double
// temporaries do not compete with the kernel's live state for registers
__device__ __attribute__((noinline)) double atan2_stream(double y, double x) { return atan2_cr(y, x); }

// block sum of NV values; ends with every thread holding the totals
template <int NV>
__device__ __forceinline__ void block_sum_s(SSmem& sm, double (&v)[NV], int lane, int wid) {
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = wave_sum_s(v[j]);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < NV; ++j) sm.red[j][wid] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        double s = sm.red[j][0];
        for (int w = 1; w < NWS; ++w) s += sm.red[j][w];
        v[j] = s;
    }
    __syncthreads();
}
}  // namespace

#ifdef RL_STAMPS
// Diagnostic build only: per-phase s_memtime totals of each workgroup's wave 0
__device__ unsigned long long rl_dbg_stamps_s[16384][16];
#define RL_SSTAMP(slot)                                             \
    do {                                                            \
        __builtin_amdgcn_sched_barrier(0);                          \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
        st_acc[slot] += t_ - st_last;                               \
        st_last = t_;                                               \
        __builtin_amdgcn_sched_barrier(0);                          \
    } while (0)
#else
#define RL_SSTAMP(slot) do {} while (0)
#endif

// the output arrays' bases: 0 pointers held for the whole kernel, 1 all seven in an LDS table
// read where used, 2 X, Y, NX, NY held (every pass reads them) and alpha_total, alpha_last,
// kappa from the table (once-per-outer passes).  C5 A/B (profiles/r05/ab_c5_scratch.log):
// min-time scratch 112 / 64 / 32 B/lane, 32.3 / 32.7 / 32.2 ms (round-5 head 160 B/lane, 32.3)
#ifndef RL_S_PLDS
#define RL_S_PLDS 2
#endif
// a uniform pointer read from LDS, as an SGPR pair
template <class T>
__device__ __forceinline__ T* unip(T* q) {
    const uint64_t u = (uint64_t)q;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return (T*)(((uint64_t)hi << 32) | lo);
}
#if RL_S_PLDS == 2
#define PPT(k) ((k) < 4 ? PL4[(k) & 3] : unip(sm.pp[(k)]))
#elif RL_S_PLDS
#define PPT(k) (unip(sm.pp[(k)]))
#else
#define PPT(k) (((double* const[]){X, Y, NX, NY, ATOT, ALAST, KA})[(k)])
#endif

template <bool CLOSED, bool MT>
// RL_STS_MINW: minimum waves per SIMD the register budget must allow (0: the compiler's
// choice for TS), e.g. TS = 512 with 4 keeps two instances co-resident per CU (A/B knob)
#ifndef RL_STS_MINW
#define RL_STS_MINW 0
#endif
#if RL_STS_MINW
__global__ __launch_bounds__(TS, RL_STS_MINW) void rl_stream_kernel(KParams p, StreamBufs sb) {
#else
__global__ __launch_bounds__(TS) void rl_stream_kernel(KParams p, StreamBufs sb) {
#endif
    __shared__ SSmem sm;
    // the register-resident v-pass's curvatures (RL_SVP_MAX samples per thread; vpass_reg)
    __shared__ double ska[MT && RL_SVP_REG ? RL_SVP_MAX * TS + RL_SVP_MAX : 1];
#ifdef RL_STAMPS
    unsigned long long st_acc[16] = {};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b = blockIdx.x;
    const int N = p.N;
    const rl_cfg& C = p.cfg[p.ncfg == 1 ? 0 : b];
    const uint64_t seed = p.seeds ? p.seeds[b] : 0ull;

    const double Lb = p.Ls ? p.Ls[blockIdx.x] : p.L;
    // (uni: the kernel-lifetime constants live in SGPR pairs, not in VGPRs)
    const double h = uni(Lb / (double)N);                // ref:690 / 913
    const double* __restrict__ CEN = p.center + (size_t)blockIdx.x * (size_t)p.center_stride;
    const double invh = uni(1.0 / h), inv2h = uni(1.0 / (2 * h)), invh2 = uni(1.0 / (h * h));   // ref:547, 562
    const double m2invh2 = uni(-2 * invh2);
    const double two_h = uni(2 * h), hh = uni(h * h);
    const double lam = C.lambda_smooth, lam2 = uni(2.0 * lam);

    const size_t off = (size_t)b * (size_t)N;
#if RL_S_PLDS
    // the output arrays' bases in LDS, read where they are used: held for the whole kernel they
    // sat in VGPR pairs (no SGPRs left) and were spilled (RL_S_PLDS above)
    if (tid == 0) {
        sm.pp[0] = p.x + off; sm.pp[1] = p.y + off; sm.pp[2] = p.nx + off; sm.pp[3] = p.ny + off;
        sm.pp[4] = p.alpha_total + off; sm.pp[5] = p.alpha_last + off; sm.pp[6] = p.kappa + off;
    }
    __syncthreads();
#if RL_S_PLDS == 2
    double* const PL4[4] = {p.x + off, p.y + off, p.nx + off, p.ny + off};   // (the corridor's, held)
#endif
#else
    double* __restrict__ X = p.x + off;
    double* __restrict__ Y = p.y + off;
    double* __restrict__ NX = p.nx + off;
    double* __restrict__ NY = p.ny + off;
    double* __restrict__ ATOT = p.alpha_total + off;
    double* __restrict__ ALAST = p.alpha_last + off;
    double* __restrict__ KA = p.kappa + off;          // κ scratch, final output at the end
#endif
    // the streaming state ([B][15][N], StreamBufs); al / an swap roles on every accepted step
#if RL_S_BUF
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        sb.base + (size_t)b * RL_STREAM_ARRAYS * (size_t)N, (short)0, RL_STREAM_ARRAYS * N * 8, 0x00020000);
#if RL_S_BUF_OPQ
    auto sfield = [&](int k) { return BufArr{srs, N * 8, k}; };
#else
    auto sfield = [&](int k) { return BufArr{srs, k * N * 8, k}; };
#endif
#else
    double* const sinst = sb.base + (size_t)b * RL_STREAM_ARRAYS * (size_t)N;
    auto sfield = [&](int k) -> double* __restrict__ { return sinst + (size_t)k * N; };
#endif
    const auto AL = sfield(0), AN = sfield(1), GR = sfield(2), LO = sfield(3), HI = sfield(4);
    const auto CA1 = sfield(5), CA2 = sfield(6), CN0 = sfield(7), CW = sfield(8);
    const auto Q1 = sfield(9), Q2 = sfield(10), D1 = sfield(11), G2 = sfield(12), V = sfield(13), VS = sfield(14);

    // neighbour index i-1 / i+1: wrapped when closed, clamped when open (no integer division)
    auto prev_i = [&](int i) -> int { return i > 0 ? i - 1 : (CLOSED ? N - 1 : 0); };
    auto next_i = [&](int i) -> int { return i + 1 < N ? i + 1 : (CLOSED ? 0 : N - 1); };
    // deriv lambdas of ref:599-613 / 625-639 at sample i
    auto deriv = [&](int i, double& xp, double& yp, double& xpp, double& ypp) {
        if (N == 1) { xp = 1; yp = 0; xpp = ypp = 0; return; }
        if (CLOSED) {
            const int ip = next_i(i), im = prev_i(i);
            xp = (PPT(0)[ip] - PPT(0)[im]) / two_h; yp = (PPT(1)[ip] - PPT(1)[im]) / two_h;
            xpp = (sub2x(PPT(0)[ip], PPT(0)[i]) + PPT(0)[im]) / hh; ypp = (sub2x(PPT(1)[ip], PPT(1)[i]) + PPT(1)[im]) / hh;
        } else if (i == 0) {
            xp = (PPT(0)[1] - PPT(0)[0]) / h; yp = (PPT(1)[1] - PPT(1)[0]) / h;
            if (N >= 3) { xpp = (sub2x(PPT(0)[2], PPT(0)[1]) + PPT(0)[0]) / hh; ypp = (sub2x(PPT(1)[2], PPT(1)[1]) + PPT(1)[0]) / hh; }
            else xpp = ypp = 0;
        } else if (i == N - 1) {
            xp = (PPT(0)[N - 1] - PPT(0)[N - 2]) / h; yp = (PPT(1)[N - 1] - PPT(1)[N - 2]) / h;
            if (N >= 3) { xpp = (sub2x(PPT(0)[N - 1], PPT(0)[N - 2]) + PPT(0)[N - 3]) / hh; ypp = (sub2x(PPT(1)[N - 1], PPT(1)[N - 2]) + PPT(1)[N - 3]) / hh; }
            else xpp = ypp = 0;
        } else {
            xp = (PPT(0)[i + 1] - PPT(0)[i - 1]) / two_h; yp = (PPT(1)[i + 1] - PPT(1)[i - 1]) / two_h;
            xpp = (sub2x(PPT(0)[i + 1], PPT(0)[i]) + PPT(0)[i - 1]) / hh; ypp = (sub2x(PPT(1)[i + 1], PPT(1)[i]) + PPT(1)[i - 1]) / hh;
        }
    };
    // normals_from_points_generic ref:581-593
    auto normal_at = [&](int i) {
        double tx, ty;
        if (N == 1) { tx = 1; ty = 0; }
        else if (CLOSED) { const int ip = next_i(i), im = prev_i(i); tx = (PPT(0)[ip] - PPT(0)[im]) * 0.5; ty = (PPT(1)[ip] - PPT(1)[im]) * 0.5; }
        else if (i == 0) { tx = PPT(0)[1] - PPT(0)[0]; ty = PPT(1)[1] - PPT(1)[0]; }
        else if (i == N - 1) { tx = PPT(0)[N - 1] - PPT(0)[N - 2]; ty = PPT(1)[N - 1] - PPT(1)[N - 2]; }
        else { tx = (PPT(0)[i + 1] - PPT(0)[i - 1]) * 0.5; ty = (PPT(1)[i + 1] - PPT(1)[i - 1]) * 0.5; }
        if (sqrt(tx * tx + ty * ty) < 1e-15) { tx = 1; ty = 0; }
        double vx = -ty, vy = tx;
        double n = sqrt(vx * vx + vy * vy);
        double ox = 0, oy = 0;
        if (!(n < 1e-15)) { ox = vx / n; oy = vy / n; }
        PPT(2)[i] = ox;
        PPT(3)[i] = oy;
#if RL_SFUSE
        // precompute_lin_geom_generic (ref:622-651) at i in the same pass over P: it needs
        // only this sample's normal, so the later lin-geom pass (and, for min-time, the
        // curvature pass, ref:595-620) need not read P and n again
        double xp, yp, xpp, ypp;
        deriv(i, xp, yp, xpp, ypp);
        CA1[i] = ox * ypp - oy * xpp;
        CA2[i] = xp * oy - yp * ox;
        const double n0 = xp * ypp - yp * xpp;
        CN0[i] = n0;
        const double d = pow15(smax(1e-12, xp * xp + yp * yp));
        CW[i] = 1.0 / d;
        if (MT) PPT(6)[i] = n0 / d;
#endif
    };
    // corridor (ref:694-711 / 749-756) at sample i via the per-lane candidate scan
    auto corridor_at = [&](int i, double guard) {
        const double qx[1] = {PPT(0)[i]}, qy[1] = {PPT(1)[i]}, ux[1] = {PPT(2)[i]}, uy[1] = {PPT(3)[i]};
        const bool act[1] = {true};
        double lk[1], hk[1];
        corridor_bounds<1>(p.ring[0], p.ring[1], qx, qy, ux, uy, act, guard, lk, hk);
        HI[i] = hk[0];
        LO[i] = lk[0];
    };
    // difference operators at sample i (DiffOps / DiffOpsOpen ref:545-579)
    auto d1_at = [&](int i, double am, double a0, double ap) -> double {
        if (CLOSED) return (ap - am) * inv2h;
        if (N == 1) return 0.0;
        if (i == 0) return (ap - a0) * invh;
        if (i == N - 1) return (a0 - am) * invh;
        return (ap - am) * inv2h;
    };
    auto d2_at = [&](int i, double am, double a0, double ap) -> double {
        if (CLOSED) return (sub2x(ap, a0) + am) * invh2;
        if (N <= 2 || i == 0 || i == N - 1) return 0.0;
        return (sub2x(ap, a0) + am) * invh2;
    };
    auto d1t_at = [&](int j, double vm, double v0, double vp) -> double {
        if (CLOSED) return (vm - vp) * inv2h;
        if (N <= 1) return 0.0;
        double acc = 0.0;
        if (j >= 1) acc += ((j == 1) ? invh : inv2h) * vm;
        if (j == 0) acc += (-invh) * v0;
        else if (j == N - 1) acc += (+invh) * v0;
        if (j <= N - 2) acc += ((j + 1 == N - 1) ? -invh : -inv2h) * vp;
        return acc;
    };
    auto d2t_at = [&](int j, double vm, double v0, double vp) -> double {
        if (CLOSED) return (sub2x(vp, v0) + vm) * invh2;
        if (N <= 2) return 0.0;
        double acc = 0.0;
        if (j - 1 >= 1 && j - 1 <= N - 2) acc += (+invh2) * vm;
        if (j >= 1 && j <= N - 2) acc += m2invh2 * v0;
        if (j + 1 >= 1 && j + 1 <= N - 2) acc += (+invh2) * vp;
        return acc;
    };

    // time weight gamma^2 of one sample (ref:950-977) from its curvature and speed
    auto gamma2_of = [&](double kap, double vv, double v_avg) -> double {
        double vkappa = sqrt(C.a_lat_max / smax(fabs(kap), C.kappa_eps));
        double rr = smin(1.0, vv / smax(1e-6, vkappa));
        double r = smin(1.0, smax(0.0, rr * rr));
        double rp = (C.time_gamma_power == 2.0) ? r * r : pow_stream(r, C.time_gamma_power);
        double corner_w = 1.0 + C.w_time_gain * rp;
        double invv_w = 1.0;
        if (C.time_weight_use_inv_v) {
            double ratio = v_avg / smax(1e-6, vv);
            invv_w = 1.0 + C.inv_v_gain * (ratio - 1.0);
            if (invv_w < 1.0) invv_w = 1.0;
            if (invv_w > 3.0) invv_w = 3.0;
        }
        double gamma = corner_w * invv_w;
        return gamma * gamma;
    };
    // ---- v(s) profile (ref:782-862), contiguous ranges [t*Cr, t*Cr+Cr) --------
    if (tid == 0) {
        VConst vc;
        const double a_total = C.use_total_ge_lat ? smax(C.a_total_max, C.a_lat_max) : C.a_total_max;
        vc.a_total2 = a_total * a_total;
        vc.kFd = 0.5 * C.rho_air * C.Cd * C.A_front_m2;
        vc.Fr = C.mass_kg * 9.81 * C.c_rr;
        vc.mass = C.mass_kg; vc.Pmax = C.P_max_W;
        vc.acc_cap = vs_cap(C.a_long_acc_cap); vc.brk_cap = vs_cap(C.a_long_brake_cap);
        vc.h = h;
        vc.pw_free = power_never_binds(C.P_max_W, C.mass_kg, vc.kFd, vc.Fr, C.v_cap_mps, vc.acc_cap);
        sm.vc = vc;                      // first read after the outer loop's first barrier
    }
    for (int j = 0; j < 4; ++j) sm.vg[j][tid] = INFINITY;   // own entries only, read by this thread
    const int Cr = (N + TS - 1) / TS;
    const int r0_ = min(N, tid * Cr), r1_ = min(N, r0_ + Cr);
    const bool ract = r0_ < r1_;
    const bool has_left = ract && r0_ > 0, has_right = ract && r1_ < N;
    // (A/B, round 3: the register kernel's in-wave DPP relaxation made this kernel's C5
    // min-time run 5-15 % slower at every round cap tried -- one barrier per round stays)
    auto vpass = [&]() -> int {
        const int r0 = opq(r0_), r1 = opq(r1_);   // (opaque: addresses formed per pass, see opq)
        const VConst vc = RL_VC_UNI ? vconst_uniform(sm.vc) : sm.vc;
        for (int i = r0; i < r1; ++i) {
            double kk = fabs(PPT(6)[i]);
            V[i] = smin(C.v_cap_mps, sqrt(C.a_lat_max / smax(kk, C.kappa_eps)));   // ref:787-794
        }
        int sweeps = 0;
        for (int s = 0; s < C.max_vpass_iters; ++s) {
            ++sweeps;
            for (int i = r0; i < r1; ++i) VS[i] = V[i];           // sweep start
            __syncthreads();
            // forward (ref:829-833), warm-started (see vpass_reg)
            double in_prev = -1.0;
            const double gf = sm.vg[s == 0 ? 0 : 1][tid];
            for (int it = 0;; ++it) {
                double in = INFINITY;
                if (has_left) in = (it > 0) ? sm.u.vin[(it - 1) & 1][tid - 1] : gf;
                bool changed = false;
                if (ract && in != in_prev) {
                    changed = (it > 0);
                    in_prev = in;
                    double cur = has_left ? smin(VS[r0], in) : VS[r0];
                    V[r0] = cur;
                    for (int i = r0; i + 1 < r1; ++i) {
                        cur = smin(VS[i + 1], vstep_fwd(vc, cur, PPT(6)[i]));
                        V[i + 1] = cur;
                    }
                    if (has_right) sm.u.vin[it & 1][tid] = vstep_fwd(vc, cur, PPT(6)[r1 - 1]);
                } else if (has_right) {
                    sm.u.vin[it & 1][tid] = sm.u.vin[(it - 1) & 1][tid];
                }
                if (!__syncthreads_or(changed) && it > 0) break;
            }
            if (has_left) {
                sm.vg[1][tid] = in_prev;
                if (s == 0) sm.vg[0][tid] = in_prev;
            }
            if (CLOSED) {                                          // ref:834-839
                if (ract && r1 == N) sm.bc[0] = vstep_fwd(vc, V[N - 1], PPT(6)[N - 1]);
                __syncthreads();
                if (tid == 0) V[0] = smin(V[0], sm.bc[0]);
                __syncthreads();
            }
            // backward (ref:841-845)
            for (int i = r0; i < r1; ++i) Q1[i] = V[i];            // pass start (Q1 is free here)
            __syncthreads();
            in_prev = -1.0;
            const double gb = sm.vg[s == 0 ? 2 : 3][tid];
            for (int it = 0;; ++it) {
                double in = INFINITY;
                if (has_right) in = (it > 0) ? sm.u.vin[(it - 1) & 1][tid + 1] : gb;
                bool changed = false;
                if (ract && in != in_prev) {
                    changed = (it > 0);
                    in_prev = in;
                    double cur = has_right ? smin(Q1[r1 - 1], in) : Q1[r1 - 1];
                    V[r1 - 1] = cur;
                    for (int i = r1 - 2; i >= r0; --i) {
                        cur = smin(Q1[i], vstep_bwd(vc, cur, PPT(6)[i + 1]));
                        V[i] = cur;
                    }
                    if (has_left) sm.u.vin[it & 1][tid] = vstep_bwd(vc, cur, PPT(6)[r0]);
                } else if (has_left) {
                    sm.u.vin[it & 1][tid] = sm.u.vin[(it - 1) & 1][tid];
                }
                if (!__syncthreads_or(changed) && it > 0) break;
            }
            if (has_right) {
                sm.vg[3][tid] = in_prev;
                if (s == 0) sm.vg[2][tid] = in_prev;
            }
            if (CLOSED) {                                          // ref:846-850
                if (tid == 0) sm.bc[1] = vstep_bwd(vc, V[0], PPT(6)[0]);
                __syncthreads();
                if (ract && r1 == N) V[N - 1] = smin(V[N - 1], sm.bc[1]);
                __syncthreads();
            }
            bool any = false;
            for (int i = r0; i < r1; ++i) any |= (V[i] != VS[i]);
            if (!__syncthreads_or(any)) break;
        }
        return sweeps;
    };

    // Register-resident v-pass for Cr = CR samples per thread (RL_SVP_MIN <= Cr <= RL_SVP_MAX,
    // e.g. C5's N = 10000: Cr = 10).  The chunk's κ, its values and the pass-start values stay
    // in registers for the whole v pass (the memory path above reloads them from HBM in every
    // relaxation round), and a re-evaluated chunk stops at the first value that repeats bit for
    // bit (each step depends only on the previous value: the rest would repeat, its outgoing
    // value included).  Rounds end when no published value changes.  Padding slots of the
    // partial last chunk hold ka = 0, v = +inf and never bind.  Same fixed point, bit for bit.
    auto same_bits = [](double a, double b) -> bool { return __double_as_longlong(a) == __double_as_longlong(b); };
    // g2: also finish the outer iteration's time weights from the registers (gamma^2 needs no
    // block-wide value unless time_weight_use_inv_v, which the caller excludes): G2 is written
    // directly and V, which only the weights would read, is not
    auto vpass_reg = [&](auto crc, bool g2) -> int {
        constexpr int CR = decltype(crc)::value;
        const VConst vc = RL_VC_UNI ? vconst_uniform(sm.vc) : sm.vc;
        // (opaque: the chunk's addresses are formed here, not hoisted out of the outer loop
        // as per-lane pointers for every instantiated CR, which were spilled)
        const int rb = opq(r0_);
        const int cnt = opq(r1_ - r0_);             // CR, except the last active thread; 0 beyond N
        // the chunk's curvatures stay in LDS (read-only for the whole v pass; each thread
        // reads only its own entries, so no barrier): in registers they spilled to scratch
        // (the 128-VGPR budget of 1024 threads), reloaded inside every step
        double* const ka = &ska[rb];
        double v[CR];
#pragma unroll
        for (int k = 0; k < CR; ++k) {
            const double kv = (k < cnt) ? PPT(6)[rb + k] : 0.0;
            ka[k] = kv;                           // (the padding slots past N hold 0)
            const double kk = fabs(kv);
            const double vk = smin(C.v_cap_mps, sqrt(C.a_lat_max / smax(kk, C.kappa_eps)));   // ref:787-794
            v[k] = (k < cnt) ? vk : INFINITY;
        }
        int sweeps = 0;
        RL_SSTAMP(15);
        for (int s = 0; s < C.max_vpass_iters; ++s) {
            ++sweeps;
            bool any = false;
            {   // forward (ref:829-833)
                double vst[CR];
#pragma unroll
                for (int k = 0; k < CR; ++k) vst[k] = v[k];
                // warm start: round 0 takes the incoming value this chunk ended with in the
                // same sweep of the previous v pass (sweep 0) or in the previous sweep; any
                // start converges to the same fixed point (chunk t is exact from round t on,
                // and the rounds end only when every input equals its neighbour's output),
                // and a start that is already exact leaves nothing to re-evaluate
                double in_prev = -1.0, out = INFINITY;
                const double gf = sm.vg[s == 0 ? 0 : 1][tid];
                for (int it = 0;; ++it) {
                    double in = INFINITY;
                    if (has_left) in = (it > 0) ? sm.u.vin[(it - 1) & 1][tid - 1] : gf;
                    bool ch = false;
                    if (ract && in != in_prev) {
                        in_prev = in;
                        const double cur = has_left ? smin(vst[0], in) : vst[0];
                        bool go = it == 0 || !same_bits(cur, v[0]);
                        v[0] = cur;
#pragma unroll
                        for (int k = 0; k + 1 < CR; ++k) {
                            if (!__any(go)) break;
                            if (go) {
                                const double vf = vstep_fwd(vc, v[k], ka[k]);
                                const double nv = (k + 1 < cnt) ? smin(vst[k + 1], vf) : INFINITY;
                                go = it == 0 || !same_bits(nv, v[k + 1]);
                                v[k + 1] = nv;
                            }
                        }
                        if (has_right && go) {             // has_right => full chunk
                            const double o = vstep_fwd(vc, v[CR - 1], ka[CR - 1]);
                            ch = o != out;
                            out = o;
                        }
                    }
                    if (has_right) sm.u.vin[it & 1][tid] = out;
                    if (!__syncthreads_or(ch) && it > 0) break;
                }
                RL_SSTAMP(12);
                if (has_left) {
                    sm.vg[1][tid] = in_prev;
                    if (s == 0) sm.vg[0][tid] = in_prev;
                }
                if (CLOSED) {                                  // ref:834-839
                    if (ract && r1_ == N) {
                        double vl = v[0], kl = ka[0];
#pragma unroll
                        for (int k = 1; k < CR; ++k)
                            if (k == cnt - 1) { vl = v[k]; kl = ka[k]; }
                        sm.bc[0] = vstep_fwd(vc, vl, kl);
                    }
                    __syncthreads();
                    if (tid == 0) v[0] = smin(v[0], sm.bc[0]);
                }
#pragma unroll
                for (int k = 0; k < CR; ++k) any |= (k < cnt) && (v[k] != vst[k]);
            }
            {   // backward (ref:841-845)
                double vpre[CR];
#pragma unroll
                for (int k = 0; k < CR; ++k) vpre[k] = v[k];
                __syncthreads();                               // vin reuse: the forward reads are done
                RL_SSTAMP(14);
                double in_prev = -1.0, out = INFINITY;
                const double gb = sm.vg[s == 0 ? 2 : 3][tid];
                for (int it = 0;; ++it) {
                    double in = INFINITY;
                    if (has_right) in = (it > 0) ? sm.u.vin[(it - 1) & 1][tid + 1] : gb;
                    bool ch = false;
                    if (ract && in != in_prev) {
                        in_prev = in;
                        const double cur = has_right ? smin(vpre[CR - 1], in) : vpre[CR - 1];
                        bool go = it == 0 || !same_bits(cur, v[CR - 1]);
                        v[CR - 1] = cur;
#pragma unroll
                        for (int k = CR - 2; k >= 0; --k) {
                            if (!__any(go)) break;
                            if (go) {
                                const double vb = vstep_bwd(vc, v[k + 1], ka[k + 1]);
                                const double nv = (k < cnt) ? smin(vpre[k], vb) : INFINITY;
                                go = it == 0 || !same_bits(nv, v[k]);
                                v[k] = nv;
                            }
                        }
                        if (has_left && go) {
                            const double o = vstep_bwd(vc, v[0], ka[0]);
                            ch = o != out;
                            out = o;
                        }
                    }
                    if (has_left) sm.u.vin[it & 1][tid] = out;
                    if (!__syncthreads_or(ch) && it > 0) break;
                }
                RL_SSTAMP(13);
                if (has_right) {
                    sm.vg[3][tid] = in_prev;
                    if (s == 0) sm.vg[2][tid] = in_prev;
                }
                if (CLOSED) {                                  // ref:846-850
                    if (tid == 0) sm.bc[1] = vstep_bwd(vc, v[0], ka[0]);
                    __syncthreads();
                    if (ract && r1_ == N) {
#pragma unroll
                        for (int k = 0; k < CR; ++k)
                            if (k == cnt - 1) v[k] = smin(v[k], sm.bc[1]);
                    }
                }
#pragma unroll
                for (int k = 0; k < CR; ++k) any |= (k < cnt) && (v[k] != vpre[k]);
            }
            if (!__syncthreads_or(any)) break;                 // later sweeps are exact repeats
            RL_SSTAMP(14);
        }
        RL_SSTAMP(14);
        if (g2) {
#pragma unroll
            for (int k = 0; k < CR; ++k)
                if (k < cnt) G2[rb + k] = gamma2_of(ka[k], v[k], 0.0);
        } else {
#pragma unroll
            for (int k = 0; k < CR; ++k)
                if (k < cnt) V[rb + k] = v[k];
        }
        return sweeps;
    };
    // g2_done: the register path wrote G2 itself (requested by g2)
    auto vpass_any = [&](bool g2, bool& g2_done) -> int {
        g2_done = false;
        if (RL_SVP_REG) {
            switch (Cr) {
#define RL_SVP_CASE(n) case n: if (n >= RL_SVP_MIN && n <= RL_SVP_MAX) { g2_done = g2; return vpass_reg(std::integral_constant<int, n>(), g2); } break;
                RL_SVP_CASE(5) RL_SVP_CASE(6) RL_SVP_CASE(7) RL_SVP_CASE(8)
                RL_SVP_CASE(9) RL_SVP_CASE(10) RL_SVP_CASE(11) RL_SVP_CASE(12)
#undef RL_SVP_CASE
                default: break;
            }
        }
        return vpass();
    };

    // ---- init ---------------------------------------------------------------
    for (int i = opq(tid); i < N; i += TS) {
        PPT(0)[i] = CEN[2 * i];
        PPT(1)[i] = CEN[2 * i + 1];
        PPT(4)[i] = 0.0; PPT(5)[i] = 0.0; AL[i] = 0.0;   // (the gradient needs no zeroing: each outer
    }                                                     // iteration's first evaluation writes it first)
    const int MO = C.max_outer_iters;
    bool first_batch = RL_BT_ADAPT ? false : (RL_BT_FIRST && (!MT || RL_BT_FIRST_MT));
    auto al_p = AL;
    auto an_p = AN;
    RL_SSTAMP(0);
    for (int outer = 0;; ++outer) {
#if RL_SPRIO
        progress_prio(outer, MO, RL_SPRIO);                        // (tail balance, rl_kernels.h)
#endif
        __syncthreads();
        if (outer > 0) {                                           // ref:743-746
            for (int i = opq(tid); i < N; i += TS) {
                const double a = al_p[i];
                PPT(5)[i] = a;
                PPT(0)[i] += PPT(2)[i] * a;
                PPT(1)[i] += PPT(3)[i] * a;
                PPT(4)[i] += a;
                al_p[i] = 0.0;                                     // ref:757
            }
            __syncthreads();
        }
        RL_SSTAMP(5);
        if (outer < MO) {
            if (tid == 0) sm.ctr = 0;                              // read after the barrier below
            for (int i = opq(tid); i < N; i += TS) normal_at(i);
            __syncthreads();
            RL_SSTAMP(6);
            const double guard = (outer == 0 ? p.veh_width : C.veh_width_m) * 0.5 + C.safety_margin_m;
#if RL_SCK > 1
            // RL_SCK adjacent samples per lane (a wave scans 64*RL_SCK consecutive rays).
            // The chunks come from a work queue in LDS: a ray's cost depends on the ring
            // geometry around it, and a static interleave left the other waves waiting at the
            // next barrier for the slowest one (C5 phase stamps: 23 % of the kernel).  Each
            // sample's bounds depend only on that sample, so the assignment does not change them.
            for (;;) {
                int c = 0;
                if (lane == 0) c = atomicAdd(&sm.ctr, 1);
                c = __builtin_amdgcn_readlane(c, 0);
                if (c * 64 * RL_SCK >= N) break;
                const int i0 = (c * 64 + lane) * RL_SCK;
                double qx[RL_SCK], qy[RL_SCK], ux[RL_SCK], uy[RL_SCK], lk[RL_SCK], hk[RL_SCK];
                bool act[RL_SCK];
#pragma unroll
                for (int k = 0; k < RL_SCK; ++k) {
                    const int i = min(i0 + k, N - 1);
                    qx[k] = PPT(0)[i]; qy[k] = PPT(1)[i]; ux[k] = PPT(2)[i]; uy[k] = PPT(3)[i];
                    act[k] = i0 + k < N;
                }
                if (outer == 0 && p.lo0) {                         // the batch's precomputed first corridor
#pragma unroll
                    for (int k = 0; k < RL_SCK; ++k) {
                        const int i = min(i0 + k, N - 1);
                        lk[k] = p.lo0[i];
                        hk[k] = p.hi0[i];
                    }
                } else {
#ifdef RL_STAMPS
                RL_SSTAMP(7);
                corridor_bounds<RL_SCK>(p.ring[0], p.ring[1], qx, qy, ux, uy, act, guard, lk, hk,
                                        [&](int s) { RL_SSTAMP(s); });
#else
                corridor_bounds<RL_SCK>(p.ring[0], p.ring[1], qx, qy, ux, uy, act, guard, lk, hk);
#endif
                }
#pragma unroll
                for (int k = 0; k < RL_SCK; ++k) {
                    const int i = i0 + k;
                    if (act[k]) {
                        HI[i] = hk[k];
                        LO[i] = lk[k];
                        if (outer == 0 && seed != 0)
                            al_p[i] = smin(hk[k], smax(lk[k], seed_value(seed, i, RL_SEED_SIGMA)));
                    }
                }
            }
#else
            for (int i = opq(tid); i < N; i += TS) {
                corridor_at(i, guard);
                if (outer == 0 && seed != 0)
                    al_p[i] = smin(HI[i], smax(LO[i], seed_value(seed, i, RL_SEED_SIGMA)));
            }
#endif
        }
#ifdef RL_STAMPS
        __syncthreads();
#endif
        RL_SSTAMP(1);
        if ((MT && !RL_SFUSE) || outer == MO) {
            for (int i = opq(tid); i < N; i += TS) {                    // ref:595-620
                double xp, yp, xpp, ypp;
                deriv(i, xp, yp, xpp, ypp);
                PPT(6)[i] = (xp * ypp - yp * xpp) / pow15(smax(1e-12, xp * xp + yp * yp));
                if (outer == MO) p.heading[off + i] = MT ? atan2_stream(yp, xp) : atan2_cr(yp, xp);   // ref:616
            }
            __syncthreads();
        }
        if (MT) {
            bool g2_done;
            const int sw = vpass_any(outer < MO && !C.time_weight_use_inv_v, g2_done);   // ref:947 / 1047
            RL_SSTAMP(11);
            if (tid == 0 && p.sweeps) p.sweeps[(size_t)b * (MO + 1) + outer] = sw;
            __syncthreads();
            if (outer == MO) {
                double lt[1] = {0.0};
                for (int i = opq(tid); i < N; i += TS) {                // ref:854-860
                    const int j = (i + 1 < N) ? i + 1 : (CLOSED ? 0 : i);
                    const double v0 = V[i], v1 = V[j];
                    p.ax[off + i] = (v1 * v1 - v0 * v0) / two_h;   // ref:857 (2.0*h)
                    p.v[off + i] = v0;
                    lt[0] += h / smax(1e-6, v0);
                }
                block_sum_s<1>(sm, lt, lane, wid);
                if (tid == 0 && p.lap) p.lap[b] = lt[0];
            } else if (!g2_done) {
                double v_avg = 0.0;
                if (C.time_weight_use_inv_v) {
                    double vs[1] = {0.0};
                    for (int i = opq(tid); i < N; i += TS) vs[0] += V[i];
                    block_sum_s<1>(sm, vs, lane, wid);
                    v_avg = vs[0] / (double)(N > 1 ? N : 1);
                }
                for (int i = opq(tid); i < N; i += TS) G2[i] = gamma2_of(PPT(6)[i], V[i], v_avg);   // ref:950-977
            }
        }
        RL_SSTAMP(2);
        if (outer == MO) break;

        if (!RL_SFUSE) {
            for (int i = opq(tid); i < N; i += TS) {                    // ref:622-651
                double xp, yp, xpp, ypp;
                deriv(i, xp, yp, xpp, ypp);
                const double nx = PPT(2)[i], ny = PPT(3)[i];
                CA1[i] = nx * ypp - ny * xpp;
                CA2[i] = xp * ny - yp * nx;
                CN0[i] = xp * ypp - yp * xpp;
                CW[i] = 1.0 / pow15(smax(1e-12, xp * xp + yp * yp));
            }
        }
        __syncthreads();
        RL_SSTAMP(3);

        // the residual terms of sample i from the stencil values around it (ref:654-675 /
        // 866-895): J term, Σa1² term, and q1, q2, D1α for the gradient
        struct Term { double jz, x1, q1, q2; };
        auto term_at = [&](int i, double am, double a0, double ap) -> Term {
            const double x1 = d1_at(i, am, a0, ap), x2 = d2_at(i, am, a0, ap);
            const double w = CW[i], A1 = CA1[i], A2 = CA2[i];
            const double r = w * (CN0[i] + A1 * x1 + A2 * x2);
            double jz, Wz;
            if (MT) { const double g2 = G2[i]; jz = g2 * r * r; Wz = w * g2 * r; }
            else { jz = r * r; Wz = w * r; }
            return {jz, x1, A1 * Wz, A2 * Wz};
        };
        // one evaluation of the vector `a` (already written and synchronised):
        // J; q1,q2,D1α to global for the gradient
        auto eval_j = [&](const auto a) -> double {
            double s3[2] = {0.0, 0.0};
            for (int i = opq(tid); i < N; i += TS) {
                const Term t = term_at(i, a[prev_i(i)], a[i], a[next_i(i)]);
                Q1[i] = t.q1;
                Q2[i] = t.q2;
                D1[i] = t.x1;
                s3[0] += t.jz;
                s3[1] += t.x1 * t.x1;
            }
            block_sum_s<2>(sm, s3, lane, wid);                     // two barriers: q/D1 visible after
            return s3[0] + lam * s3[1];
        };
        // the trial vector of step st at sample j: std::min(hi, std::max(lo, α - st*g)) (ref:731)
        auto trial_at = [&](int j, double st) -> double { return smin(HI[j], smax(LO[j], al_p[j] - st * GR[j])); };
        // one evaluation of the trial vector of step st: J and the Armijo decrease
        // Σ g(α_trial - α) (ref:733 / 1009). Each sample recomputes its neighbours' trial
        // values from (α, g, lo, hi), so a rejected trial writes nothing; `keep` also
        // stores α_trial, q1, q2 and D1α, which an accepted step needs.
        auto eval_trial = [&](double st, bool keep, double& dec) -> double {
            double s3[3] = {0.0, 0.0, 0.0};
            for (int i = opq(tid); i < N; i += TS) {
                const int im = prev_i(i), ip = next_i(i);
                const double a0 = trial_at(i, st);
                const double am = (im == i) ? a0 : trial_at(im, st);
                const double ap = (ip == i) ? a0 : trial_at(ip, st);
                const Term t = term_at(i, am, a0, ap);
                if (keep) { an_p[i] = a0; Q1[i] = t.q1; Q2[i] = t.q2; D1[i] = t.x1; }
                s3[0] += t.jz;
                s3[1] += t.x1 * t.x1;
                s3[2] += GR[i] * (a0 - al_p[i]);
            }
            block_sum_s<3>(sm, s3, lane, wid);                     // two barriers: writes visible after
            dec = s3[2];
            return s3[0] + lam * s3[1];
        };
        // an accepted trial that was evaluated without `keep`: write what it would have
        auto materialize = [&](double st) {
            for (int i = opq(tid); i < N; i += TS) {
                const int im = prev_i(i), ip = next_i(i);
                const double a0 = trial_at(i, st);
                const double am = (im == i) ? a0 : trial_at(im, st);
                const double ap = (ip == i) ? a0 : trial_at(ip, st);
                const Term t = term_at(i, am, a0, ap);
                an_p[i] = a0; Q1[i] = t.q1; Q2[i] = t.q2; D1[i] = t.x1;
            }
            __syncthreads();
        };
        auto eval_grad = [&]() {
            for (int i = opq(tid); i < N; i += TS) {
                const int im = prev_i(i), ip = next_i(i);
                const double g1 = d1t_at(i, Q1[im], Q1[i], Q1[ip]);
                const double g2 = d2t_at(i, Q2[im], Q2[i], Q2[ip]);
                const double gsm = d1t_at(i, D1[im], D1[i], D1[ip]);
                GR[i] = 2.0 * (g1 + g2) + lam2 * gsm;
            }
            __syncthreads();                                       // the next trial reads g at i±1
        };

        // The next up-to-MB steps of a backtracking run (C5: every trial of an outer
        // iteration is rejected) from one pass over (α, g, lo, hi, coefficients): per
        // step the arithmetic and the per-thread sample order of eval_trial, and
        // block_sum_s reduces each sum on its own, so J and the decrease of every step
        // are bit-identical to one-at-a-time trials.  Writes nothing unless keep0 is set.
        constexpr int MB = RL_BT_BATCH;
        // keep0: step 0 is the first trial of an inner iteration -- also store its α_trial,
        // q1, q2 and D1α (eval_trial's `keep`) into an_p, Q1, Q2, D1, so an accepted first
        // step needs no second pass: the accept path skips materialize() for j == 0 and
        // relies on these writes
        auto eval_trials = [&](const double (&st)[MB], int m, double (&Jn)[MB], double (&dn)[MB], bool keep0) {
            double s3[3 * MB];
#pragma unroll
            for (int j = 0; j < 3 * MB; ++j) s3[j] = 0.0;
            for (int i = opq(tid); i < N; i += TS) {
                const int im = prev_i(i), ip = next_i(i);
                const double a0v = al_p[i], g0 = GR[i], lo0 = LO[i], hi0 = HI[i];
                const double amv = al_p[im], gm = GR[im], lom = LO[im], him = HI[im];
                const double apv = al_p[ip], gp = GR[ip], lop = LO[ip], hip = HI[ip];
                const double w = CW[i], A1 = CA1[i], A2 = CA2[i], n0 = CN0[i];
                const double g2 = MT ? G2[i] : 1.0;
#pragma unroll
                for (int j = 0; j < MB; ++j) {
                    if (j < m) {                                      // uniform
                        const double a0 = smin(hi0, smax(lo0, a0v - st[j] * g0));
                        const double am = (im == i) ? a0 : smin(him, smax(lom, amv - st[j] * gm));
                        const double ap = (ip == i) ? a0 : smin(hip, smax(lop, apv - st[j] * gp));
                        const double x1 = d1_at(i, am, a0, ap), x2 = d2_at(i, am, a0, ap);
                        const double r = w * (n0 + A1 * x1 + A2 * x2);
                        if (j == 0 && keep0) {                         // term_at's q1, q2 (ref:667)
                            const double Wz = MT ? w * g2 * r : w * r;
                            an_p[i] = a0; Q1[i] = A1 * Wz; Q2[i] = A2 * Wz; D1[i] = x1;
                        }
                        s3[3 * j] += MT ? g2 * r * r : r * r;        // term_at's jz (ref:881 / 661)
                        s3[3 * j + 1] += x1 * x1;
                        s3[3 * j + 2] += g0 * (a0 - a0v);
                    }
                }
            }
            block_sum_s<3 * MB>(sm, s3, lane, wid);
#pragma unroll
            for (int j = 0; j < MB; ++j) { Jn[j] = s3[3 * j] + lam * s3[3 * j + 1]; dn[j] = s3[3 * j + 2]; }
        };

        double step = C.step_init;
        double dec;
        double J = eval_j(al_p);
        eval_grad();
        int evals = 1, accepts = 0;
        double J_prev = J;
        for (int it = 0; it < C.max_inner_iters; ++it) {
            bool accepted = false;
            int bt = 0;
            while (bt < 20) {
                // (fixed rules measured before RL_BT_ADAPT: the first trial in a batch for min-curv
                // only, C5 27.8 -> 26.4 ms; min-time 67.2 -> 69.8 ms)
                if (MB > 1 && (first_batch || bt > 0)) {
                    const bool kept = bt == 0;             // step 0's vectors are stored by the pass
                    // the steps ref:737-740 would try next: halve, stop at 20 backtracks
                    // or below step_min
                    double st[MB], Jn[MB], dn[MB];
                    int m = 1;
                    st[0] = step;
#pragma unroll
                    for (int j = 1; j < MB; ++j) {
                        const double sj = st[j - 1] * 0.5;
                        st[j] = sj;
                        if (m == j && bt + j < 20 && !(sj < C.step_min)) m = j + 1;
                    }
                    eval_trials(st, m, Jn, dn, kept);
                    bool stop = false;
                    for (int j = 0; j < m; ++j) {
                        ++evals;
                        if (RL_BT_ADAPT && kept && j == 0) first_batch = !(Jn[0] <= J + C.armijo_c * dn[0]);
                        if (Jn[j] <= J + C.armijo_c * dn[j]) {
                            if (!(kept && j == 0)) materialize(st[j]);
                            const auto t = al_p; al_p = an_p; an_p = t;
                            eval_grad();
                            J = Jn[j];
                            accepted = true;
                            ++accepts;
                            stop = true;
                            break;
                        }
                        step *= 0.5;
                        bt++;
                        if (step < C.step_min) { stop = true; break; }
                    }
                    if (stop) break;
                    continue;
                }
                // the first trial of an inner iteration is the usual accept: keep its
                // vectors; later (backtracked) trials are mostly rejected
                const bool keep = (bt == 0);
                const double Jn = eval_trial(step, keep, dec);
                ++evals;
                if (RL_BT_ADAPT && keep) first_batch = !(Jn <= J + C.armijo_c * dec);
                if (Jn <= J + C.armijo_c * dec) {
                    if (!keep) materialize(step);
                    const auto t = al_p; al_p = an_p; an_p = t;       // α := α_trial (uniform swap)
                    eval_grad();
                    J = Jn;
                    accepted = true;
                    ++accepts;
                    break;
                }
                step *= 0.5;
                bt++;
                if (step < C.step_min) break;
            }
            if (!accepted) break;
            if (fabs(J_prev - J) < 1e-10) break;
            J_prev = J;
        }
        if (tid == 0) {
            if (p.evals) p.evals[(size_t)b * MO + outer] = evals;
            if (p.accepts) p.accepts[(size_t)b * MO + outer] = accepts;
        }
        RL_SSTAMP(4);
    }
    if (p.done) signal_done(p.done, b, p.epoch);
#ifdef RL_STAMPS
    if (tid == 0 && b < 16384) {
        for (int i = 0; i < 16; ++i) rl_dbg_stamps_s[b][i] = st_acc[i];
    }
#endif
}

#ifdef RL_COUNT
int debug_counts(unsigned long long* host, int reset) {
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(rl_dbg_count), z, sizeof(z)) == hipSuccess ? 0 : -3;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_count), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -3;
}
#endif
#ifdef RL_STAMPS
int debug_stamps_stream(unsigned long long* host, int nblocks) {
    if (nblocks > 16384) nblocks = 16384;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_stamps_s), sizeof(unsigned long long) * 16 * nblocks) == hipSuccess ? 0 : -3;
}
#endif

template <bool CL, bool MT>
static hipError_t launch_s(const KParams& p, const StreamBufs& sb, hipStream_t st) {
    hipLaunchKernelGGL((rl_stream_kernel<CL, MT>), dim3(p.B), dim3(TS), 0, st, p, sb);
    return hipGetLastError();
}

#undef PPT

int stream_threads() { return TS; }

hipError_t launch_stream(const KParams& p, const StreamBufs& sb, bool mintime, hipStream_t st) {
    if (p.N <= 0 || p.N > RL_STREAM_MAX_N) return hipErrorInvalidValue;
    if (p.closed) return mintime ? launch_s<true, true>(p, sb, st) : launch_s<true, false>(p, sb, st);
    return mintime ? launch_s<false, true>(p, sb, st) : launch_s<false, false>(p, sb, st);
}

}  // namespace rl
