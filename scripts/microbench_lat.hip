// Latency micro-benchmarks for the B=1 (one workgroup) PGD evaluation on gfx950:
// cycles per dependent fp64 add / fma / mul, per fp64 division and sqrt, per 64-bit DPP
// wave reduction, per s_barrier (4 / 8 / 16 waves) and per LDS write -> barrier -> read
// round trip.  One workgroup, s_memtime around REPS repetitions, wave 0 reports.
// build: hipcc --offload-arch=gfx950 -O3 scripts/microbench_lat.hip -o /tmp/mb  (run on the GPU box)
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int REPS = 4096;

__device__ __forceinline__ double dpp_xor1(double x) {
    int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0xB1, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0xB1, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wsum(double x) {
    x += dpp<0xB1>(x);
    x += dpp<0x4E>(x);
    x += dpp<0x124>(x);
    x += dpp<0x128>(x);
    int lo = __double2loint(x), hi = __double2hiint(x);
    int lo2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false)[0];
    int hi2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[0];
    x += __hiloint2double(hi2, lo2);
    int lo3 = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false)[0];
    int hi3 = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false)[0];
    return x + __hiloint2double(hi3, lo3);
}

template <int which>
__global__ void k_chain(double seed, double* out, unsigned long long* cyc) {
    __shared__ double buf[2][1024];
    double x = seed + threadIdx.x * 1e-9, y = 1.0000001, z = 1e-7;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (which) {  // (one instantiation per case)
    case 0: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = x + y; } break;                    // add
    case 1: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = __builtin_fma(x, y, z); } break;   // fma
    case 2: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = 1.0 / (x + 1.5); } break;          // div (+add)
    case 3: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = sqrt(x + 1.5); } break;            // sqrt (+add)
    case 4: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = wsum(x) * 1e-3; } break;           // wave reduction (+mul)
    case 5: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { __syncthreads(); x = x + y; } break;   // barrier (+add)
    case 6:                                                                          // LDS exchange
        _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) {
            buf[i & 1][threadIdx.x] = x;
            __syncthreads();
            x = buf[i & 1][(threadIdx.x + 1) % blockDim.x] * 0.5 + y;
        }
        break;
    case 7:                                                                          // reduce + LDS + barrier
        _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) {
            double s = wsum(x);
            if ((threadIdx.x & 63) == 0) buf[i & 1][threadIdx.x >> 6] = s;
            __syncthreads();
            double t = 0.0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += buf[i & 1][w];
            x = t * 1e-3 + y;
        }
        break;
    case 8: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = (x * y < z) ? z : x * y; } break;   // mul + cmp/cndmask select
    case 9: _Pragma("unroll 8") for (int i = 0; i < REPS; ++i) { x = x * y; } break;                      // mul
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef void (*KF)(double, double*, unsigned long long*);
static void launch(int w, int T, double* out, unsigned long long* cyc) {
    static const KF ks[10] = {k_chain<0>, k_chain<1>, k_chain<2>, k_chain<3>, k_chain<4>, k_chain<5>, k_chain<6>, k_chain<7>, k_chain<8>, k_chain<9>};
    hipLaunchKernelGGL(ks[w], dim3(1), dim3(T), 0, 0, 1.0, out, cyc);
}

int main() {
    double* out; unsigned long long* cyc;
    hipMalloc(&out, 1024 * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    const char* names[] = {"fp64 add", "fp64 fma", "fp64 div", "fp64 sqrt", "wave sum (dpp+permlane)",
                           "s_barrier", "LDS write-barrier-read", "wave sum + LDS + barrier + sum", "fp64 mul + select", "fp64 mul"};
    // s_memtime rate vs wall clock: one long run timed both ways
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int T : {64, 256, 512, 1024}) {
        for (int w = 0; w < 10; ++w) {
            if (T == 64 && (w == 5 || w == 6 || w == 7)) continue;
            unsigned long long c = 0;
            float ms = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                launch(w, T, out, cyc);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
                hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
            }
            printf("T=%4d %-32s %8.1f cycles/iter  (%.3f ns/iter from events)\n", T, names[w], (double)c / REPS,
                   1e6 * ms / REPS);
        }
    }
    return 0;
}
