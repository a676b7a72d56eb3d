// rl_math.h — host+device fp64 helpers that reproduce the reference's libm calls
// (glibc 2.35, x86-64, no FMA ifunc for hypot) using only correctly rounded
// operations (+,-,*,/,sqrt,fma), so the gfx950 results equal the CPU's.
// Pinned to the host glibc by tests/test_math_cpu.py (known-answer tests, >=10^6
// samples each: hypot bit for bit, pow15 = the correctly rounded x^1.5).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace rl {

#if defined(__HIP_DEVICE_COMPILE__)
#define RL_FMA(a, b, c) __fma_rn((a), (b), (c))
#else
#define RL_FMA(a, b, c) fma((a), (b), (c))
#endif

// std::pow(x, 1.5) for finite x > 0 (ref:617, 647: x = max(1e-12, x'^2+y'^2)).
// x*sqrt(x) carried as a double-double (exact product error + exact sqrt residual)
// and rounded once: correctly rounded except within ~1e-16 ulp of a tie.
__host__ __device__ inline double pow15(double x) {
    double s = sqrt(x);
    double p = x * s;
    double e = RL_FMA(x, s, -p);
    double r = RL_FMA(-s, s, x);
    double corr = e + x * (r / (2.0 * s));
    return p + corr;
}

// std::hypot (ref:509): glibc 2.35 __hypot (sysdeps/ieee754/dbl-64/e_hypot.c),
// the non-FMA kernel (Borges' correction step), restated.
__host__ __device__ inline double hypot_kernel(double ax, double ay) {
    double t1, t2;
    double h = sqrt(ax * ax + ay * ay);
    if (h <= 2.0 * ay) {
        double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

__host__ __device__ inline double hypot_ref(double x, double y) {
    // glibc's constants; TINY_VAL is 2^-459 (measured: glibc takes the scaled path for
    // every ay < 2^-459, tests/test_math_cpu.py), which keeps the correction terms normal
    const double SCALE = 0x1p-600, LARGE_VAL = 0x1p+511, TINY_VAL = 0x1p-459, EPS = 0x1p-54;
    if (!isfinite(x) || !isfinite(y)) {
        if (isinf(x) || isinf(y)) return INFINITY;
        return x + y;
    }
    x = fabs(x);
    y = fabs(y);
    double ax = x < y ? y : x;
    double ay = x < y ? x : y;
    if (ax > LARGE_VAL) {
        if (ay <= ax * EPS) return ax + ay;
        return hypot_kernel(ax * SCALE, ay * SCALE) / SCALE;
    }
    if (ay < TINY_VAL) {
        if (ax >= ay / EPS) return ax + ay;
        return hypot_kernel(ax / SCALE, ay / SCALE) * SCALE;
    }
    if (ay <= ax * EPS) return ax + ay;
    return hypot_kernel(ax, ay);
}

}  // namespace rl
