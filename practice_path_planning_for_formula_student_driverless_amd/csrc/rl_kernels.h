// rl_kernels.h — launch interface between the C-ABI (rl_abi.cpp) and the
// gfx950 kernels (rl_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_abi.h"
#include "rl_device.h"

namespace rl {

// Device pointers of one (problem, mode) launch.  Result/state arrays are
// instance-major [B][N]; x/y double as the path state P during the run.
struct KParams {
    const double* center;      // [N][2]
    const SegRec* seg;         // inner ring segments [Ei], then outer [Eo]
    const rl_cfg* cfg;         // [ncfg]
    const uint64_t* seeds;     // [B] or nullptr
    double *x, *y, *heading, *kappa, *alpha_total, *alpha_last;
    double *v, *ax, *lap;      // min-time only (may be nullptr for min-curv)
    double *nx, *ny;           // scratch normals [B][N]
    int32_t *evals, *accepts, *sweeps;
    int32_t N, Ei, Eo, ncfg, B, closed;
    double L, veh_width;
};

// samples per lane for N (4 or 8), or -1 if N exceeds the register-resident kernel
int pick_k(int N);
// enqueue one persistent launch (one workgroup per instance) on `st`
hipError_t launch_optimize(const KParams& p, bool mintime, hipStream_t st);

}  // namespace rl
