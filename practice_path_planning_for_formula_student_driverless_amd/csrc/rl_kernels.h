// rl_kernels.h — launch interface between the C-ABI (rl_abi.cpp) and the
// gfx950 kernels (rl_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_abi.h"
#include "rl_corridor.h"
#include "rl_device.h"

namespace rl {

// Device pointers of one (problem, mode) launch.  Result/state arrays are
// instance-major [B][N]; x/y double as the path state P during the run.
struct KParams {
    const double* center;      // [N][2], or [B][N][2] with center_stride = 2N (lap evaluation)
    const double* Ls;          // per-instance L [B] or nullptr (then L)
    RingDesc ring[2];          // inner, outer ring as entry streams (rl_corridor.h)
    const rl_cfg* cfg;         // [ncfg]
    const uint64_t* seeds;     // [B] or nullptr
    double *x, *y, *heading, *kappa, *alpha_total, *alpha_last;
    double *v, *ax, *lap;      // min-time only (may be nullptr for min-curv)
    double *nx, *ny;           // scratch normals [B][N]
    int32_t *evals, *accepts, *sweeps;
    int32_t N, Ei, Eo, ncfg, B, closed;
    int32_t shape_B;           // batch size the kernel shape is chosen for (pick_shape; >= 1)
    int64_t center_stride;     // doubles between instances' centres (0: shared)
    double L, veh_width;
    // Instance completion flags (rl_optimize's overlapped download, rl_abi.cpp run_cached):
    // nullptr, or [B] words in coherent pinned host memory; instance b stores `epoch` into
    // done[b] once every result word of b has reached memory (signal_done below)
    uint32_t* done;
    uint32_t epoch;
    // Outer iteration 0's corridor bounds [N] (lo, hi), computed once for the whole batch by
    // rl_corridor_kernel on the shared centre line (rl_abi.cpp rl_plan_run), or nullptr: the
    // first corridor is the same for every instance of a batch (P = centre, guard = the
    // problem's veh_width * 0.5 + the cfg's margin), so the instances load it instead of each
    // casting it again
    const double* lo0;
    const double* hi0;
};

// Up to RL_GROUP_MAX plans of one kernel shape in one launch (rl_plan_run_group): the plans'
// parameters and their first workgroup index, passed as kernel arguments (8 x 344 B + 36 B)
constexpr int RL_GROUP_MAX = 8;
struct KGroup {
    int32_t n;                          // plans in the launch (1..RL_GROUP_MAX)
    int32_t start[RL_GROUP_MAX];        // first workgroup of plan j; plan j has p[j].B of them
    KParams p[RL_GROUP_MAX];
};
static_assert(sizeof(KGroup) <= 4096, "kernel arguments of a group launch");

// The instance's completion flag: every wave waits until its own result stores have reached
// L2 (vmcnt(0): on gfx9 a store's count drops when L2 acknowledges it), the workgroup joins,
// then one lane writes the L2 back to memory (a system-scope release fence: buffer_wbl2 and
// its wait; all waves of a workgroup share one CU, hence one XCD's L2) and stores the epoch
// into the host-visible flag with a vector store.  One write-back per instance instead of one
// per wave: C2's drop-in kernel 9.08 -> 8.98 ms (profiles/r06/ab_done_one_wb.log).  Called
// once, at the very end of the kernel, uniformly by every thread of the workgroup.
__device__ __forceinline__ void signal_done(uint32_t* done, int b, uint32_t epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(done + b, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Wave priority by progress, set at the top of every outer iteration (`mode` 1: four levels,
// 3 in the first quarter of the instance's outer iterations down to 0 in the last; 2: two
// levels, 3 in the first half, 0 after).  Two instances share a CU (two per CU in C2's shape);
// the arbiter issues the oldest wave first at equal priority, so the first-dispatched
// instance of each pair races ahead and the last instance of every CU runs alone at the
// grid's end.  Favouring the instance that is behind makes the pair end together.
__device__ __forceinline__ void progress_prio(int outer, int MO, int mode) {
    // mode 3 (the product's, build.py): the levels' resolution spent near the end, where the
    // pair's gap decides the tail: 3 for the first half, 2 to three quarters, 1 to the last
    // outer iteration, 0 in it (C2 -0.7..-1 % against mode 1; mode 2 and an even later
    // split were slower: profiles/r06/ab_prio.log, ab_prio3.log)
    const int lvl = mode == 2   ? (2 * outer < MO ? 3 : 0)
                    : mode == 3 ? (2 * outer < MO ? 3 : 4 * outer < 3 * MO ? 2 : outer < MO - 1 ? 1 : 0)
                                : ((MO - outer) * 4) / (MO + 1);
    if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
    else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
    else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// Per-instance HBM state of the large-N streaming kernel (rl_stream.hip): RL_STREAM_ARRAYS
// arrays of N doubles per instance, instance-major [B][RL_STREAM_ARRAYS][N] in one allocation
// (al, an, gr, lo, hi, a1, a2, n0, w, q1, q2, d1, g2, v, vs), so one buffer resource and a
// field offset address any of an instance's arrays.
struct StreamBufs {
    double* base;
};
constexpr int RL_STREAM_ARRAYS = 15;
constexpr int RL_REG_MAX_N = 4096;          // register-resident kernel covers N <= 4096
constexpr int RL_STREAM_MAX_N = 1 << 20;

// samples per lane for N (4, 5 or 8) of the throughput shapes, or -1 if N exceeds the
// register-resident kernel
int pick_k(int N);
// (K samples per lane, T lanes per instance) of a register-resident launch
struct Shape {
    int K, T;
};
// Latency shapes (rl_kernels_lat.hip) by N: one instance spread over a whole CU, for
// batches that leave most of the GPU idle (build knobs for A/B timing).  Above N = 2048
// the throughput shape (8, 512) already spreads an instance over 8 waves (a 1024-lane
// shape would be capped at 128 VGPRs and spill).
#ifndef RL_LAT1_K
#define RL_LAT1_K 1      // N <= 256: (1, 256)
#endif
#ifndef RL_LAT2_K
#define RL_LAT2_K 1      // N <= 512: (1, 512), 8 waves (A/B: testday3 N=261 2.20 -> 1.75 ms vs (2, 256))
#endif
#ifndef RL_LAT3_K
#define RL_LAT3_K 2      // N <= 1024: (2, 512)
#endif
// RL_LAT_FIT: for N <= 512 one sample per lane on just enough waves, T = max(128, N rounded
// up to 64): fewer waves make the evaluation's barrier and cross-wave sum cheaper (A/B:
// testday3 N=261 (1, 512) -> (1, 320) 1.76 -> 1.68 ms min-curv, 2.25 -> 2.16 ms min-time;
// 0 keeps the RL_LAT1_K / RL_LAT2_K table)
#ifndef RL_LAT_FIT
#define RL_LAT_FIT 1
#endif
inline Shape lat_shape(int N) {
    if (RL_LAT_FIT && N <= 512) return {1, N <= 128 ? 128 : (N + 63) / 64 * 64};
    if (N <= 256) return {RL_LAT1_K, 256 / RL_LAT1_K};
    if (N <= 512) return {RL_LAT2_K, 512 / RL_LAT2_K};
    if (N <= 1024) return {RL_LAT3_K, 1024 / RL_LAT3_K};
    if (N <= 2048) return {4, 512};
    return {-1, -1};
}
// the shape launch_optimize uses for N samples and a batch of B instances on a device with
// `cus` CUs: the latency shape while B x its waves <= 4 x cus (one wave per SIMD) and
// RL_LAT_SHAPES is not "0", else the throughput shape; {-1, -1} beyond RL_REG_MAX_N
Shape pick_shape(int N, int B, bool mintime, int cus);
// enqueue one persistent launch (one workgroup per instance) on `st`
hipError_t launch_optimize(const KParams& p, bool mintime, hipStream_t st);
// the shapes a group launch covers (the one-wave throughput shapes, rl_kernels_group.hip)
bool group_shape(const Shape& s);
// one launch of g.n plans whose pick_shape is s (group_shape(s)), all closed or all open,
// all ragged (N % K != 0) or none, one mode: rl_kernels_group.hip
hipError_t launch_optimize_group(const KGroup& g, const Shape& s, bool closed, bool ragged, bool mintime,
                                 hipStream_t st);
// the launches of the latency shapes lat_shape(p.N) and of every (4, 512) shape (also the
// min-time shape for 1024 < N <= 2048 below two instances per CU), rl_kernels_lat.hip
hipError_t launch_optimize_lat(const KParams& p, bool mintime, hipStream_t st);
// the (4, 512) launches (1024 < N <= 2048), rl_kernels_mid.hip
hipError_t launch_optimize_mid(const KParams& p, bool mintime, hipStream_t st);
// large-N variant: one workgroup of stream_threads() threads per instance, state in HBM
hipError_t launch_stream(const KParams& p, const StreamBufs& sb, bool mintime, hipStream_t st);
// threads per instance of the streaming kernel (its build knob RL_STS, 1024 by default)
int stream_threads();
// step 6 geometry (rl_geom.hip): spline knots [5][nk] per axis (s,a,b,c,d), rows [Kmax+dup][9]
struct GeomParams {
    const double* kx;
    const double* ky;
    int32_t nk;
    int32_t Kmax, denomN, emit_dup;
    double s0, L;
    RingDesc ring[2];
    double kappa_eps, a_lat_max, v_cap;
    double* rows;
};
hipError_t launch_geom(const GeomParams& g, hipStream_t st);
// rl_corridor (rl_geom.hip): normals of `center` then the corridor bounds of every sample
struct CorrParams {
    const double* center;      // [N][2]
    int32_t N, closed;
    RingDesc ring[2];
    double guard;
    double *lo, *hi;
};
hipError_t launch_corridor(const CorrParams& c, hipStream_t st);
// "%.9f" CSV rows of a [rows][cols] device table (rl_format.hip): 0, -1 (|x| >= 9.2e9),
// -2 (cap short; *total = needed), -3 (HIP failure)
int format_rows(const double* table, int64_t rows, int cols, char* out, uint64_t cap, uint64_t* offs,
                uint64_t* total, hipStream_t st);
#ifdef RL_STAMPS
int debug_stamps(unsigned long long* host, int nblocks);
int debug_stamps_stream(unsigned long long* host, int nblocks);
int debug_stamps_lat(unsigned long long* host, int nblocks);
int debug_stamps_mid(unsigned long long* host, int nblocks);
#endif
#ifdef RL_COUNT
int debug_counts(unsigned long long* host, int reset);
int debug_counts_geom(unsigned long long* host, int reset);
int debug_counts_reg(unsigned long long* host, int reset);
#endif

}  // namespace rl
