// rl_kernels_mid.hip — the (4, 512) shape of the register-resident optimiser kernel
// (rl_optimize_body.h): the latency shape for 1024 < N <= 2048 and the min-time shape for
// that N range below two instances per CU (rl_kernels.hip pick_shape).  A translation unit
// of its own so that it can be compiled with its own instruction scheduler (build.py
// TU_FLAGS; A/B in DESIGN.md §3e).
#include "rl_optimize_body.h"

namespace rl {

template <bool CL, bool MT>
static hipError_t launch_mid_t(const KParams& p, hipStream_t st) {
    if (p.N % 4) {
        hipLaunchKernelGGL((rl_optimize_kernel<4, 512, CL, MT, true>), dim3(p.B), dim3(512), 0, st, p);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((rl_optimize_kernel<4, 512, CL, MT, false>), dim3(p.B), dim3(512), 0, st, p);
    return hipGetLastError();
}

#ifdef RL_STAMPS
// diagnostic builds: this translation unit's copy of the per-phase cycle totals
int debug_stamps_mid(unsigned long long* host, int nblocks) {
    if (nblocks > 16384) nblocks = 16384;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rl_dbg_stamps), sizeof(unsigned long long) * 16 * nblocks) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_optimize_mid(const KParams& p, bool mintime, hipStream_t st) {
    if (p.N <= 1024 || p.N > 2048) return hipErrorInvalidValue;
    if (p.closed) return mintime ? launch_mid_t<true, true>(p, st) : launch_mid_t<true, false>(p, st);
    return mintime ? launch_mid_t<false, true>(p, st) : launch_mid_t<false, false>(p, st);
}

}  // namespace rl
