// Probe: gfx950 v_max_f64 / v_min_f64 on signed-zero ties and NaN, operand order fixed
// by inline asm.  Prints src0/src1/result sign bits.  (Experiment, not part of librl.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__global__ void k(const double* a, const double* b, double* mx, double* mn, int n) {
    int i = threadIdx.x;
    if (i >= n) return;
    double x = a[i], y = b[i], r1, r2;
    asm volatile("v_max_f64 %0, %1, %2" : "=v"(r1) : "v"(x), "v"(y));
    asm volatile("v_min_f64 %0, %1, %2" : "=v"(r2) : "v"(x), "v"(y));
    mx[i] = r1; mn[i] = r2;
}
int main() {
    const double nan = std::nan(""), inf = INFINITY;
    double A[] = {-0.0, 0.0, -0.0, 0.0, 1.0, nan, -1.0, 2.5, -0.0, 0.0};
    double B[] = {0.0, -0.0, -0.0, 0.0, nan, 1.0, -1.0, 2.5, -1e-300, 1e-300};
    int n = 10;
    double *da, *db, *dx, *dn;
    hipMalloc(&da, 8 * n); hipMalloc(&db, 8 * n); hipMalloc(&dx, 8 * n); hipMalloc(&dn, 8 * n);
    hipMemcpy(da, A, 8 * n, hipMemcpyHostToDevice); hipMemcpy(db, B, 8 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dx, dn, n);
    double X[10], Nn[10];
    hipMemcpy(X, dx, 8 * n, hipMemcpyDeviceToHost); hipMemcpy(Nn, dn, 8 * n, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i) {
        double smax = (A[i] < B[i]) ? B[i] : A[i];   // std::max(a, b)
        double smin = (B[i] < A[i]) ? B[i] : A[i];   // std::min(a, b)
        printf("a=%g b=%g  vmax=%g (std %g) %s  vmin=%g (std %g) %s\n", A[i], B[i], X[i], smax,
               (std::signbit(X[i]) == std::signbit(smax) && (X[i] == smax || (std::isnan(X[i]) && std::isnan(smax)))) ? "ok" : "DIFF",
               Nn[i], smin,
               (std::signbit(Nn[i]) == std::signbit(smin) && (Nn[i] == smin || (std::isnan(Nn[i]) && std::isnan(smin)))) ? "ok" : "DIFF");
    }
    (void)inf;
    return 0;
}
