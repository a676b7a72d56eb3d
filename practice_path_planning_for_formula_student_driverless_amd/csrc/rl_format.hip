// rl_format.hip — the reference's CSV number format on gfx950.
// Every CSV the reference writes uses std::fixed + precision(9) (ref:1284, 1303,
// 1354, 1418, 1495): glibc's exact "%.9f" — the exact binary value rounded to 9
// fraction digits, ties to even, '-' whenever the sign bit is set ("-0.000000000"),
// "nan"/"-nan"/"inf"/"-inf".  Here: one thread per table row formats its columns
// into a staging slot (exact integer arithmetic: |x|*10^9 = m*10^9*2^e in 128 bits,
// shifted with round-half-even), a device prefix sum over the row lengths gives the
// offsets, and the rows are compacted into one contiguous buffer.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "rl_kernels.h"

namespace rl {

constexpr int FMT_NUM_MAX = 22;   // '-' + 10 integer digits + '.' + 9 digits + separator

// "%.9f" of x into p; returns the length, or -1 if |x| >= 9.2e9 (outside the fast path)
__device__ __forceinline__ int fmt_fixed9(double x, char* p) {
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    const bool neg = bits >> 63;
    const int ex = (int)((bits >> 52) & 0x7ff);
    const uint64_t fr = bits & ((1ull << 52) - 1);
    int n = 0;
    if (ex == 0x7ff) {                                 // inf / nan (glibc spelling)
        if (neg) p[n++] = '-';
        if (fr) { p[n++] = 'n'; p[n++] = 'a'; p[n++] = 'n'; }
        else { p[n++] = 'i'; p[n++] = 'n'; p[n++] = 'f'; }
        return n;
    }
    if (fabs(x) >= 9.2e9) return -1;
    // x = m * 2^e with m < 2^53
    const uint64_t m = ex ? (fr | (1ull << 52)) : fr;
    const int e = ex ? ex - 1075 : -1074;
    uint64_t N;
    if (m == 0) {
        N = 0;
    } else {
        // |x| < 9.2e9 < 2^52 implies e < 0; P = m * 10^9 < 2^83
        const unsigned __int128 P = (unsigned __int128)m * 1000000000ull;
        const int s = -e;
        if (s >= 128) {
            N = 0;
        } else {
            const unsigned __int128 q = P >> s;
            const unsigned __int128 r = P - (q << s);
            const unsigned __int128 half = (unsigned __int128)1 << (s - 1);
            uint64_t qq = (uint64_t)q;
            if (r > half || (r == half && (qq & 1))) ++qq;        // round half to even
            N = qq;
        }
    }
    if (neg) p[n++] = '-';
    uint64_t ip = N / 1000000000ull;
    uint32_t fp = (uint32_t)(N - ip * 1000000000ull);
    char tmp[20];
    int t = 0;
    do { tmp[t++] = (char)('0' + (int)(ip % 10)); ip /= 10; } while (ip);
    while (t) p[n++] = tmp[--t];
    p[n++] = '.';
    for (int d = 8; d >= 0; --d) { p[n + d] = (char)('0' + (int)(fp % 10)); fp /= 10; }
    return n + 9;
}

__global__ void fmt_rows_kernel(const double* __restrict__ table, int64_t rows, int cols, char* __restrict__ stage,
                                int stride, uint64_t* __restrict__ lens, int* __restrict__ bad) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    char* p = stage + r * (int64_t)stride;
    const double* v = table + r * (int64_t)cols;
    int n = 0;
    for (int c = 0; c < cols; ++c) {
        int k = fmt_fixed9(v[c], p + n);
        if (k < 0) { atomicExch(bad, 1); k = 0; }
        n += k;
        p[n++] = (c + 1 < cols) ? ',' : '\n';
    }
    lens[r] = (uint64_t)n;
}

__global__ void fmt_compact_kernel(const char* __restrict__ stage, int stride, const uint64_t* __restrict__ lens,
                                   const uint64_t* __restrict__ offs, int64_t rows, char* __restrict__ out) {
    // one wave per row: lanes copy the row's bytes cooperatively
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const char* src = stage + r * (int64_t)stride;
    char* dst = out + offs[r];
    const int n = (int)lens[r];
    for (int i = lane; i < n; i += 64) dst[i] = src[i];
}

// table [rows][cols] (device) -> out (device, capacity cap): returns the total length
// in *total and row offsets [rows+1] in offs (device); -1 on |x| >= 9.2e9, -2 if cap is short
int format_rows(const double* table, int64_t rows, int cols, char* out, uint64_t cap, uint64_t* offs,
                uint64_t* total, hipStream_t st) {
    const int stride = cols * FMT_NUM_MAX;
    char* stage = nullptr;
    uint64_t* lens = nullptr;
    int* bad = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int rc = 0;
    if (hipMalloc(&stage, (size_t)rows * stride) != hipSuccess || hipMalloc(&lens, (size_t)(rows + 1) * 8) != hipSuccess ||
        hipMalloc(&bad, sizeof(int)) != hipSuccess) {
        rc = -3;
    } else {
        hipMemsetAsync(bad, 0, sizeof(int), st);
        hipMemsetAsync(lens + rows, 0, 8, st);
        const int T = 256;
        hipLaunchKernelGGL(fmt_rows_kernel, dim3((unsigned)((rows + T - 1) / T)), dim3(T), 0, st, table, rows, cols,
                           stage, stride, lens, bad);
        // exclusive scan over rows+1 entries: offs[rows] = total
        hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, lens, offs, (int)(rows + 1), st);
        if (hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 8) != hipSuccess) rc = -3;
        else {
            hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, lens, offs, (int)(rows + 1), st);
            int hbad = 0;
            hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st);
            hipMemcpyAsync(total, offs + rows, 8, hipMemcpyDeviceToHost, st);
            hipStreamSynchronize(st);
            if (hbad) rc = -1;
            else if (*total > cap) rc = -2;
            else {
                const int64_t threads = rows * 64;
                hipLaunchKernelGGL(fmt_compact_kernel, dim3((unsigned)((threads + T - 1) / T)), dim3(T), 0, st, stage,
                                   stride, lens, offs, rows, out);
                if (hipStreamSynchronize(st) != hipSuccess) rc = -3;
            }
        }
    }
    if (tmp) hipFree(tmp);
    if (bad) hipFree(bad);
    if (lens) hipFree(lens);
    if (stage) hipFree(stage);
    return rc;
}

}  // namespace rl
