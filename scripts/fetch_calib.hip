// fetch_calib.hip — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 at the streaming
// kernel's own access width (MI355X_MICROARCH.md §HBM calibrates the x2
// read correction only for 16-B/lane loads).
//
// Every kernel moves a known number of bytes over a 2 GiB array (8x the 256 MiB Infinity
// Cache, so nothing is served on-die between launches):
//   read8      one double per lane, rl_stream_kernel's mapping (1024-thread workgroup per
//              contiguous slice, i = base + tid + k*1024)           bytes = n*8
//   read8nbr   the same plus the i-1 / i+1 neighbour loads of the stencil passes
//              (re-reads of lines the wave just loaded)             bytes = n*8 (unique)
//   read16     one double2 per lane (the guide's calibrated width)  bytes = n*8
//   read8buf   read8 through a buffer resource per workgroup (raw buffer loads, the
//              streaming kernel's state path since round 5)  bytes = n*8
//   read8nbrbuf  read8nbr through the same buffer resource              bytes = n*8 (unique)
//   write8     one double per lane stored, same mapping              bytes = n*8
//   write16    one double2 per lane stored                          bytes = n*8
// Each kernel writes at most one double per workgroup besides its stores.
// usage: fetch_calib <reps>      (prints one line per kernel: name bytes ms GB/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int TS = 1024;

__global__ __launch_bounds__(TS) void read8(const double* __restrict__ a, long chunk, double* out) {
    const double* s = a + (long)blockIdx.x * chunk;
    double acc = 0.0;
    for (long i = threadIdx.x; i < chunk; i += TS) acc += s[i];
    if (acc == 1.2345e300) out[blockIdx.x] = acc;     // never true: keeps the loads, no stores
}

__global__ __launch_bounds__(TS) void read8nbr(const double* __restrict__ a, long chunk, double* out) {
    const double* s = a + (long)blockIdx.x * chunk;
    double acc = 0.0;
    for (long i = threadIdx.x; i < chunk; i += TS) {
        const long im = i > 0 ? i - 1 : chunk - 1, ip = i + 1 < chunk ? i + 1 : 0;
        acc += s[im] * 0.25 + s[i] * 0.5 + s[ip] * 0.25;
    }
    if (acc == 1.2345e300) out[blockIdx.x] = acc;
}

__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, long i) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8), 0, 0));
}

__global__ __launch_bounds__(TS) void read8buf(const double* __restrict__ a, long chunk, double* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(a + (long)blockIdx.x * chunk), (short)0,
                                                                       (int)(chunk * 8), 0x00020000);
    double acc = 0.0;
    for (long i = threadIdx.x; i < chunk; i += TS) acc += bload(r, i);
    if (acc == 1.2345e300) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(TS) void read8nbrbuf(const double* __restrict__ a, long chunk, double* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(a + (long)blockIdx.x * chunk), (short)0,
                                                                       (int)(chunk * 8), 0x00020000);
    double acc = 0.0;
    for (long i = threadIdx.x; i < chunk; i += TS) {
        const long im = i > 0 ? i - 1 : chunk - 1, ip = i + 1 < chunk ? i + 1 : 0;
        acc += bload(r, im) * 0.25 + bload(r, i) * 0.5 + bload(r, ip) * 0.25;
    }
    if (acc == 1.2345e300) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(TS) void read16(const double2* __restrict__ a, long chunk2, double* out) {
    const double2* s = a + (long)blockIdx.x * chunk2;
    double acc = 0.0;
    for (long i = threadIdx.x; i < chunk2; i += TS) { const double2 v = s[i]; acc += v.x + v.y; }
    if (acc == 1.2345e300) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(TS) void write8(double* __restrict__ a, long chunk) {
    double* s = a + (long)blockIdx.x * chunk;
    for (long i = threadIdx.x; i < chunk; i += TS) s[i] = (double)i;
}

__global__ __launch_bounds__(TS) void write16(double2* __restrict__ a, long chunk2) {
    double2* s = a + (long)blockIdx.x * chunk2;
    for (long i = threadIdx.x; i < chunk2; i += TS) s[i] = make_double2((double)i, 1.0);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const long n = 1L << 28;                  // 2 GiB of doubles
    const int blocks = 1024;                  // C5's instance count per launch
    const long chunk = n / blocks;
    double *a, *out;
    CK(hipMalloc(&a, n * sizeof(double)));
    CK(hipMalloc(&out, blocks * sizeof(double)));
    CK(hipMemset(a, 0, n * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)n * 8.0;
    auto timed = [&](const char* name, auto launch) {
        launch();                             // warm-up (not in the summary: counted by name order)
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("%s bytes=%.0f ms_mean=%.4f ms_best=%.4f GBps_mean=%.1f\n", name, bytes, sum / reps, best,
               bytes / (sum / reps * 1e-3) / 1e9);
        fflush(stdout);
    };
    timed("read8", [&] { hipLaunchKernelGGL(read8, dim3(blocks), dim3(TS), 0, 0, a, chunk, out); });
    timed("read8nbr", [&] { hipLaunchKernelGGL(read8nbr, dim3(blocks), dim3(TS), 0, 0, a, chunk, out); });
    timed("read8buf", [&] { hipLaunchKernelGGL(read8buf, dim3(blocks), dim3(TS), 0, 0, a, chunk, out); });
    timed("read8nbrbuf", [&] { hipLaunchKernelGGL(read8nbrbuf, dim3(blocks), dim3(TS), 0, 0, a, chunk, out); });
    timed("read16", [&] { hipLaunchKernelGGL(read16, dim3(blocks), dim3(TS), 0, 0, (const double2*)a, chunk / 2, out); });
    timed("write8", [&] { hipLaunchKernelGGL(write8, dim3(blocks), dim3(TS), 0, 0, a, chunk); });
    timed("write16", [&] { hipLaunchKernelGGL(write16, dim3(blocks), dim3(TS), 0, 0, (double2*)a, chunk / 2); });
    CK(hipGetLastError());
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
