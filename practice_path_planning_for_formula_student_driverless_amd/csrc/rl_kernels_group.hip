// rl_kernels_group.hip — group launches of the register-resident optimiser (rl_optimize_body.h):
// several plans of one one-wave throughput shape in a single grid (rl_plan_run_group).
//
// Why: a sweep (C4: 7 tracks x 512 sweep points x 2 modes) is 14 plans of 512 one-wave
// instances.  Launched one per plan, at most as many kernels run at once as the process has
// HIP hardware queues (4 on the GPU box), and each kernel's last, longest instances hold
// their queue while most CUs idle.  Grouped, the same instances form a few large grids that
// the dispatcher keeps refilling as instances finish.  The instance code is the plan launch's
// own (rl_optimize_body), so the results are the same bit for bit.
// Same scheduler flags as rl_kernels.hip (build.py TU_FLAGS).
#include "rl_optimize_body.h"

namespace rl {

template <int K, bool CL, bool MT, bool RG>
static hipError_t launch_g(const KGroup& g, hipStream_t st) {
    int blocks = 0;
    for (int j = 0; j < g.n; ++j) blocks += g.p[j].B;
    hipLaunchKernelGGL((rl_optimize_group_kernel<K, 64, CL, MT, RG>), dim3(blocks), dim3(64), 0, st, g);
    return hipGetLastError();
}

template <int K>
static hipError_t launch_gk(const KGroup& g, bool closed, bool ragged, bool mt, hipStream_t st) {
    if (closed) {
        if (ragged) return mt ? launch_g<K, true, true, true>(g, st) : launch_g<K, true, false, true>(g, st);
        return mt ? launch_g<K, true, true, false>(g, st) : launch_g<K, true, false, false>(g, st);
    }
    if (ragged) return mt ? launch_g<K, false, true, true>(g, st) : launch_g<K, false, false, true>(g, st);
    return mt ? launch_g<K, false, true, false>(g, st) : launch_g<K, false, false, false>(g, st);
}

bool group_shape(const Shape& s) {
    return s.T == 64 && (s.K == 4 || s.K == 5 || s.K == 8);
}

hipError_t launch_optimize_group(const KGroup& g, const Shape& s, bool closed, bool ragged, bool mintime,
                                 hipStream_t st) {
    if (g.n < 1 || g.n > RL_GROUP_MAX || !group_shape(s)) return hipErrorInvalidValue;
    for (int j = 0; j < g.n; ++j) {
        const KParams& p = g.p[j];
        // every plan of the launch in the shape, boundary and chunk form it was compiled for
        // (the ragged form covers every N; the exact-multiple form only N % K == 0)
        if (p.N <= 0 || p.N > s.K * s.T || p.B < 1 || (p.closed != 0) != closed || (!ragged && p.N % s.K != 0))
            return hipErrorInvalidValue;
    }
    if (s.K == 4) return launch_gk<4>(g, closed, ragged, mintime, st);
    if (s.K == 5) return launch_gk<5>(g, closed, ragged, mintime, st);
    return launch_gk<8>(g, closed, ragged, mintime, st);
}

}  // namespace rl
