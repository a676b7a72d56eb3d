// rl_kernels_lat.hip — the latency shapes of the register-resident optimiser kernel
// (rl_optimize_body.h): one instance spread over a whole CU with 1-4 samples per lane.
//
// The reference's own use is one track per call (pipeline::compute_raceline_and_save
// ref:1347, compute_mintime_and_save ref:1397): a batch of one leaves 255 of 256 CUs idle,
// and the throughput shapes' per-lane serial work (4-8 samples per lane, one or four
// waves) sets the latency.  Spreading the instance over 4-16 waves cuts each lane's
// chain of dependent fp64 operations per evaluation at the price of the cross-wave
// reductions and exchanges (LDS + barriers).  pick_shape (rl_kernels.hip) selects these
// shapes while the batch needs at most one wave per SIMD in them.  Results equal the
// throughput shapes' bit for bit except the lap sum's tree order (the same kernel
// template; every per-sample expression and every J / decrease sum is the same).
// The (4, 512) shape has a translation unit of its own (rl_kernels_mid.hip) so that each
// can be compiled with the instruction scheduler that suits it (build.py TU_FLAGS).
#include "rl_optimize_body.h"

namespace rl {

template <int K, int T, bool CL, bool MT>
static hipError_t launch_lat_t(const KParams& p, hipStream_t st) {
    if constexpr (K > 1) {
        if (p.N % K) {
            hipLaunchKernelGGL((rl_optimize_kernel<K, T, CL, MT, true>), dim3(p.B), dim3(T), 0, st, p);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((rl_optimize_kernel<K, T, CL, MT, false>), dim3(p.B), dim3(T), 0, st, p);
    return hipGetLastError();
}
template <int K, int T>
static hipError_t launch_lat_kt(const KParams& p, bool mt, hipStream_t st) {
    static_assert(T % 64 == 0 && T <= 512, "latency shape");
    if (p.closed) return mt ? launch_lat_t<K, T, true, true>(p, st) : launch_lat_t<K, T, true, false>(p, st);
    return mt ? launch_lat_t<K, T, false, true>(p, st) : launch_lat_t<K, T, false, false>(p, st);
}

#ifdef RL_STAMPS
// diagnostic builds: this translation unit's copy of the per-phase cycle totals
int debug_stamps_lat(unsigned long long* host, int nblocks) {
    if (nblocks > 16384) nblocks = 16384;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_stamps), sizeof(unsigned long long) * 16 * nblocks) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_optimize_lat(const KParams& p, bool mintime, hipStream_t st) {
    if (p.N <= 0 || p.N > 2048) return hipErrorInvalidValue;
#if RL_LAT_FIT
    if (p.N <= 512) {
        switch (lat_shape(p.N).T) {
            case 128: return launch_lat_kt<1, 128>(p, mintime, st);
            case 192: return launch_lat_kt<1, 192>(p, mintime, st);
            case 256: return launch_lat_kt<1, 256>(p, mintime, st);
            case 320: return launch_lat_kt<1, 320>(p, mintime, st);
            case 384: return launch_lat_kt<1, 384>(p, mintime, st);
            case 448: return launch_lat_kt<1, 448>(p, mintime, st);
            default: return launch_lat_kt<1, 512>(p, mintime, st);
        }
    }
#endif
    if (p.N <= 256) return launch_lat_kt<RL_LAT1_K, 256 / RL_LAT1_K>(p, mintime, st);
    if (p.N <= 512) return launch_lat_kt<RL_LAT2_K, 512 / RL_LAT2_K>(p, mintime, st);
    if (p.N <= 1024) return launch_lat_kt<RL_LAT3_K, 1024 / RL_LAT3_K>(p, mintime, st);
    return launch_optimize_mid(p, mintime, st);       // (4, 512): rl_kernels_mid.hip
}

}  // namespace rl
