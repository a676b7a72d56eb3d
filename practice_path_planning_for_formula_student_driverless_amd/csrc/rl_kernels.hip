// rl_kernels.hip — MI355X (gfx950) batched raceline optimizer, steps 7-8 of the
// reference pipeline (ref = /root/reference/src/main.cpp): the throughput shapes of the
// register-resident kernel (rl_optimize_body.h) and the launch dispatch by (N, B).
// The latency shapes for small batches are instantiated in rl_kernels_lat.hip.
#include <cstdlib>

#include "rl_optimize_body.h"

namespace rl {

#ifdef RL_STAMPS
int debug_stamps(unsigned long long* host, int nblocks) {
    if (nblocks > 16384) nblocks = 16384;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_stamps), sizeof(unsigned long long) * 16 * nblocks) == hipSuccess ? 0 : -3;
}
#endif

// ------------------------------------------------------------------ launcher
template <int K, int T, bool CL, bool MT>
static hipError_t launch_t(const KParams& p, hipStream_t st) {
    if (p.N % K)
        hipLaunchKernelGGL((rl_optimize_kernel<K, T, CL, MT, true>), dim3(p.B), dim3(T), 0, st, p);
    else
        hipLaunchKernelGGL((rl_optimize_kernel<K, T, CL, MT, false>), dim3(p.B), dim3(T), 0, st, p);
    return hipGetLastError();
}
template <int K, int T>
static hipError_t launch_kt(const KParams& p, bool mt, hipStream_t st) {
    if (p.closed) return mt ? launch_t<K, T, true, true>(p, st) : launch_t<K, T, true, false>(p, st);
    return mt ? launch_t<K, T, false, true>(p, st) : launch_t<K, T, false, false>(p, st);
}
template <int K, int T, bool MT>
static hipError_t launch_ktm(const KParams& p, hipStream_t st) {
    return p.closed ? launch_t<K, T, true, MT>(p, st) : launch_t<K, T, false, MT>(p, st);
}

// variant table by N: (K samples per lane, T lanes per instance)
//   throughput shapes (every batch that fills the GPU):
//   N <= 256          (4, 64)      one wave per instance
//   N <= 320          (5, 64)      one wave per instance (RL_S5)
//   N <= 512          (8, 64)      one wave per instance
//   N <= 1024         (8, 128)
//   N <= 2048         (RL_MID_K, RL_MID_T)   default (8, 256); min-time (RL_MIDMT_K, RL_MIDMT_T) = (4, 512)
//                     below two instances per CU, else (RL_MID_K, RL_MID_T)
//   N <= 4096         (8, 512)
//   latency shapes (rl_kernels_lat.hip, RL_LAT* in rl_kernels.h): while the batch needs at
//   most one wave per SIMD in them (B x T/64 <= 4 x CUs), fewer samples per lane spread
//   one instance over a whole CU -- the drop-in use, one track per call (ref:1347, 1397)
static_assert(RL_MID_K * RL_MID_T == 2048, "mid variant must cover N <= 2048");
static_assert(RL_MIDMT_K == 4 && RL_MIDMT_T == 512, "the mid min-time shape is (4, 512), instantiated in rl_kernels_lat.hip");
// (5, 64) for 256 < N <= 320 (testday1/3 of the bundled tracks): one wave, 5 samples per lane
// instead of 8, 0 B scratch and two waves per SIMD in both modes.  C4 (scripts/ab_c4_single.py,
// profiles/r05/ab_c4_s5.log): those plans alone min-time 4.16 / 4.59 -> 3.32 / 3.74 ms,
// min-curv 3.64 / 3.97 -> 3.07 / 3.36 ms; the concurrent sweep 17.55 -> 16.42 ms, bit-exact
#ifndef RL_S5
#define RL_S5 1
#endif
int pick_k(int N) {
    if (N <= 4 * 64) return 4;
    if (RL_S5 && N <= 5 * 64) return 5;
    if (N <= 8 * 64) return 8;
    if (N <= 8 * 128) return 8;
    if (N <= 2048) return RL_MID_K;
    if (N <= 8 * 512) return 8;
    return -1;
}

#ifndef RL_MIDMT_BIG
#define RL_MIDMT_BIG 1
#endif
static int cu_count() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 256;
    return n > 0 ? n : 256;
}

bool lat_shapes_enabled() {
    const char* e = std::getenv("RL_LAT_SHAPES");
    return !(e && e[0] == '0');
}

Shape pick_shape(int N, int B, bool mintime, int cus) {
    if (N <= 0 || N > RL_REG_MAX_N) return {-1, -1};
    const Shape lat = lat_shape(N);
    if (lat.K > 0 && lat_shapes_enabled() && (int64_t)B * (lat.T / 64) <= (int64_t)4 * cus) return lat;
    if (N <= 4 * 64) return {4, 64};
    if (RL_S5 && N <= 5 * 64) return {5, 64};
    if (N <= 8 * 64) return {8, 64};
    if (N <= 8 * 128) return {8, 128};
    if (N <= 2048) {
        if (!mintime) return {RL_MID_K, RL_MID_T};
#if RL_MIDMT_BIG
        // min-time: (4, 512) holds one instance per CU (8 waves at 2 waves/SIMD), the
        // lower latency while the batch leaves CUs idle; from two instances per CU up,
        // the (RL_MID_K, RL_MID_T) shape keeps two per CU resident for throughput
        if (B >= 2 * cus) return {RL_MID_K, RL_MID_T};
#endif
        return {RL_MIDMT_K, RL_MIDMT_T};
    }
    return {8, 512};
}

#ifdef RL_COUNT
// diagnostic builds: this translation unit's corridor counters (the throughput shapes)
int debug_counts_reg(unsigned long long* host, int reset) {
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(rl_dbg_count), z, sizeof(z)) == hipSuccess ? 0 : -3;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_count), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_optimize(const KParams& p, bool mintime, hipStream_t st) {
    if (p.N <= 0 || pick_k(p.N) < 0) return hipErrorInvalidValue;
#ifdef RL_ANALYZE_ONE   // static analysis builds (scripts/regs_one.sh): the C2/C3 shape only (2: open)
    constexpr bool CL = RL_ANALYZE_ONE != 2;
    return mintime ? launch_t<8, 256, CL, true>(p, st) : launch_t<8, 256, CL, false>(p, st);
#else
    const Shape s = pick_shape(p.N, p.shape_B > 0 ? p.shape_B : p.B, mintime, cu_count());
    const Shape lat = lat_shape(p.N);
    if ((s.K == lat.K && s.T == lat.T) || (s.K == 4 && s.T == 512)) return launch_optimize_lat(p, mintime, st);
    if (s.K == 4 && s.T == 64) return launch_kt<4, 64>(p, mintime, st);
#if RL_S5
    if (s.K == 5 && s.T == 64) return launch_kt<5, 64>(p, mintime, st);
#endif
    if (s.K == 8 && s.T == 64) return launch_kt<8, 64>(p, mintime, st);      // one wave (single-wave paths)
    if (s.K == 8 && s.T == 128) return launch_kt<8, 128>(p, mintime, st);
    if (p.N <= 2048) {
        return mintime ? launch_ktm<RL_MID_K, RL_MID_T, true>(p, st) : launch_ktm<RL_MID_K, RL_MID_T, false>(p, st);
    }
    return launch_kt<8, 512>(p, mintime, st);
#endif
}

}  // namespace rl
