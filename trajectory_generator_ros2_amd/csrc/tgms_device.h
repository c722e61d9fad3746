// tgms_device.h — device-side helpers shared by the kernel translation units.
#pragma once

#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tgms.h"

namespace tgms {

constexpr int W64 = 64;  // wavefront width (gfx950)

// ---------------------------------------------------------------------------
// Septic-Hermite snap-cost matrix sub-blocks (exact integers; see
// oracle/exact.py hermite_maps() and oracle/minsnap_oracle.c KH).
// Index d, e = 0..2 stands for derivative order d+1, e+1 (v, a, j); the entry
// for a segment of duration T is scaled by r^(5-d-e), r = 1/T.
__device__ constexpr double KSS[3][3] = {{25920, 5400, 480}, {5400, 1200, 120}, {480, 120, 16}};
__device__ constexpr double KEE[3][3] = {{25920, -5400, 480}, {-5400, 1200, -120}, {480, -120, 16}};
// coupling: start derivative d (row) x end derivative e (column) of one segment
__device__ constexpr double KSE[3][3] = {{24480, -4680, 360}, {4680, -840, 60}, {360, -60, 4}};
// coupling of derivative d with the segment displacement (w1 - w0), scaled r^(6-d)
__device__ constexpr double KSP[3] = {-50400, -10080, -840};  // start derivatives
__device__ constexpr double KEP[3] = {-50400, 10080, -840};   // end derivatives

__device__ __forceinline__ void rpowers(double r, double (&p)[8]) {
    p[0] = 1.0;
    p[1] = r;
    p[2] = r * r;
    p[3] = p[2] * r;
    p[4] = p[2] * p[2];
    p[5] = p[4] * r;
    p[6] = p[3] * p[3];
    p[7] = p[6] * r;
}

// LDL^T of a 3x3 SPD block: reciprocal pivots + unit-lower multipliers.
struct Ldl3 {
    double i0, i1, i2, l10, l20, l21;
};

__device__ __forceinline__ Ldl3 ldl3(const double (&D)[3][3], bool& spd) {
    Ldl3 f;
    const double p0 = D[0][0];
    f.i0 = 1.0 / p0;
    f.l10 = D[0][1] * f.i0;
    f.l20 = D[0][2] * f.i0;
    const double p1 = D[1][1] - f.l10 * D[0][1];
    f.i1 = 1.0 / p1;
    const double t12 = D[1][2] - f.l20 * D[0][1];
    f.l21 = t12 * f.i1;
    const double p2 = D[2][2] - f.l20 * D[0][2] - f.l21 * t12;
    f.i2 = 1.0 / p2;
    spd = (p0 > 0.0) && (p1 > 0.0) && (p2 > 0.0);
    return f;
}

__device__ __forceinline__ void ldl3_solve(const Ldl3& f, double b0, double b1, double b2, double& x0,
                                           double& x1, double& x2) {
    const double y1 = b1 - f.l10 * b0;
    const double y2 = b2 - f.l20 * b0 - f.l21 * y1;
    x2 = y2 * f.i2;
    x1 = y1 * f.i1 - f.l21 * x2;
    x0 = b0 * f.i0 - f.l10 * x1 - f.l20 * x2;
}

__device__ __forceinline__ bool finite_pos(double t) { return t > 0.0 && t <= DBL_MAX; }
__device__ __forceinline__ bool finite(double v) { return v * 0.0 == 0.0; }

// 1/x to ~1 ulp: hardware reciprocal + two Newton steps (the IEEE-correct division
// sequence is ~3x longer on the dependency chain and is not needed at 1e-9).
__device__ __forceinline__ double fast_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}

// Intra-quad DPP moves (no LDS round trip, unlike __shfl*): swap lanes 2q <-> 2q+1,
// or broadcast the even / odd lane of each pair to both.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double pair_swap(double v) { return dpp_f64<0xB1>(v); }   // quad_perm [1,0,3,2]
__device__ __forceinline__ double pair_even(double v) { return dpp_f64<0xA0>(v); }   // quad_perm [0,0,2,2]
__device__ __forceinline__ double pair_odd(double v) { return dpp_f64<0xF5>(v); }    // quad_perm [1,1,3,3]

// Septic-Hermite segment -> monomial coefficients (a4 layout [axis][8]) in registers.
// g0/g1: (v, a, j) at the start / end knot, [derivative][axis].  Returns the sum of
// the coefficients (for the non-finite check).
__device__ __forceinline__ double segment_coeffs(double T, double r, const double* w0, const double* w1,
                                                 const double (&g0)[3][3], const double (&g1)[3][3],
                                                 bool zero, double (&c)[24]) {
    const double T2 = T * T, T3 = T2 * T;
    double rp[8];
    rpowers(r, rp);
    double fin = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double v0 = g0[0][a], a0 = g0[1][a], j0 = g0[2][a];
        const double v1 = g1[0][a], a1 = g1[1][a], j1 = g1[2][a];
        const double dw = w1[a] - w0[a];
        const double h1 = T * v0, h2 = T2 * a0, h3 = T3 * j0;
        const double h5 = T * v1, h6 = T2 * a1, h7 = T3 * j1;
        const double d4 = 35.0 * dw - 20.0 * h1 - 5.0 * h2 - (2.0 / 3.0) * h3 - 15.0 * h5 + 2.5 * h6 -
                          (1.0 / 6.0) * h7;
        const double d5 = -84.0 * dw + 45.0 * h1 + 10.0 * h2 + h3 + 39.0 * h5 - 7.0 * h6 + 0.5 * h7;
        const double d6 = 70.0 * dw - 36.0 * h1 - 7.5 * h2 - (2.0 / 3.0) * h3 - 34.0 * h5 + 6.5 * h6 -
                          0.5 * h7;
        const double d7 = -20.0 * dw + 10.0 * h1 + 2.0 * h2 + (1.0 / 6.0) * h3 + 10.0 * h5 - 2.0 * h6 +
                          (1.0 / 6.0) * h7;
        double* ca = c + a * 8;
        ca[0] = w0[a];
        ca[1] = v0;
        ca[2] = 0.5 * a0;
        ca[3] = j0 * (1.0 / 6.0);
        ca[4] = d4 * rp[4];
        ca[5] = d5 * rp[5];
        ca[6] = d6 * rp[6];
        ca[7] = d7 * rp[7];
        fin += ((ca[4] + ca[5]) + (ca[6] + ca[7])) + ((ca[1] + ca[2]) + ca[3]);
#pragma unroll
        for (int j = 0; j < 8; ++j) ca[j] = zero ? 0.0 : ca[j];
    }
    return fin;
}

__device__ __forceinline__ double emit_segment(double T, double r, const double* w0, const double* w1,
                                               const double (&g0)[3][3], const double (&g1)[3][3],
                                               bool zero, double* __restrict__ o) {
    double c[24];
    const double fin = segment_coeffs(T, r, w0, w1, g0, g1, zero, c);
    double2* od = reinterpret_cast<double2*>(o);
#pragma unroll
    for (int j = 0; j < 12; ++j) od[j] = make_double2(c[2 * j], c[2 * j + 1]);
    return fin;
}


// Kernel launch that reports THIS launch's error: hipLaunchKernel returns it directly,
// whereas hipLaunchKernelGGL + hipGetLastError() would also report (and clear) a
// sticky error left by an unrelated earlier HIP call on the thread.
template <class T>
struct launch_arg {
    using type = T;
};
template <class... KArgs>
__host__ hipError_t launch_kernel(void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t shmem, hipStream_t stream,
                                  typename launch_arg<KArgs>::type... args) {
    void* argv[] = {static_cast<void*>(&args)..., nullptr};
    return hipLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, argv, shmem, stream);
}
#define TGMS_LAUNCH(kernel, grid, block, shmem, stream, ...)                                       \
    do {                                                                                         \
        const hipError_t launch_e_ = ::tgms::launch_kernel(kernel, grid, block, shmem, stream, __VA_ARGS__); \
        if (launch_e_ != hipSuccess) return launch_e_;                                           \
    } while (0)

}  // namespace tgms
