// occstore.hip — the headline's store ceiling by occupancy.
//
// The lane kernel (k_lane_uniform<10>) reads 22.5 MB (waypoints + times) and writes
// 126 MB (coefficients) per launch of 65,536 trajectories at ONE wave per SIMD, every
// wave in the same phase: "read + compute prefix, then store drain".  This probe asks
// what the same bytes cost at 1 / 2 / 4 / 8 waves per SIMD and with the work cut into
// R rounds of waves (so waves finish and are replaced at different times), with and
// without a compute prefix of the lane kernel's FP64 size between the reads and the
// stores.  Occupancy is pinned with dynamic LDS (160 KiB / (4 x waves per SIMD) per
// one-wave workgroup); every configuration moves the same bytes, spread evenly over
// 1,024 x wps x R waves; 4 output sets rotate (504 MB, past the Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 -o occstore occstore.hip && ./occstore
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t B = 65536, OUT_B = B * 1920, IN_B = B * 344;
constexpr int SETS = 4;

// each wave: read its slice of `in` (16 B per lane per instruction), `fma` dependent
// FP64 FMAs on 8 independent chains, then write its slice of `out` front to back
__global__ __launch_bounds__(64) void k(const double2* __restrict__ in, double2* __restrict__ out, size_t in_per_wave,
                                       size_t out_per_wave, int fma, double seed) {
    extern __shared__ double pin_lds[];  // occupancy pin only
    const int lane = threadIdx.x;
    const size_t w = blockIdx.x;
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = seed + lane + j;
    const double2* src = in + w * in_per_wave;
    // every load of the wave's slice in flight at once (up to 24 per lane per batch),
    // as the lane kernel's LDS-DMA prologue issues them
    for (size_t i0 = 0; i0 < in_per_wave; i0 += 24 * 64) {
        double2 v[24];
#pragma unroll
        for (int q = 0; q < 24; ++q) {
            const size_t i = i0 + q * 64 + lane;
            v[q] = i < in_per_wave ? src[i] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int q = 0; q < 24; ++q) acc[q & 7] += v[q].x + v[q].y;
    }
    // 16 independent FMA chains (the lane kernel's forward sweep has ~3 x 3 x 3-deep
    // independent work per knot)
    double acc2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc2[j] = acc[j] * 0.5;
    for (int i = 0; i < fma / 2; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = __builtin_fma(acc[j], 0.999999, 1e-9);
            acc2[j] = __builtin_fma(acc2[j], 0.999999, 1e-9);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += acc2[j];
    if (seed < -1e300) pin_lds[lane] = acc[0];  // never: keeps the LDS allocation
    double2* dst = out + w * out_per_wave;
    for (size_t i = lane, q = 0; i < out_per_wave; i += 64, ++q) dst[i] = make_double2(acc[q & 7], acc[(q + 1) & 7]);
}

int main() {
    double2 *in[SETS], *out[SETS];
    for (int s = 0; s < SETS; ++s) {
        (void)hipMalloc(&in[s], IN_B);
        (void)hipMalloc(&out[s], OUT_B);
        (void)hipMemset(in[s], 0, IN_B);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // fp64 FMA wave-instructions per 64 trajectories: 0 (pure streaming) and ~3,300
    // (the lane kernel's measured FP64 work, r02_fp64pmc_summary), and twice that
    for (int pass = 0; pass < 1; ++pass)
        for (int read : {0, 1})
            for (int prefix : {0, 3328, 6656})
                for (int wps : {1, 2, 4, 8})
                    for (int rounds : {1, 2, 4, 8}) {
                        if (!read && prefix) continue;
                        const size_t waves = 1024ull * wps * rounds;
                        const size_t out_pw = OUT_B / 16 / waves, in_pw = read ? IN_B / 16 / waves : 0;
                        const int fma = (int)(prefix / 8 / (wps * rounds));
                        const size_t lds = (160 * 1024) / (4 * wps) - 256;
                        auto go = [&](int s) {
                            hipLaunchKernelGGL(k, dim3(waves), dim3(64), lds, 0, in[s], out[s], in_pw, out_pw, fma,
                                               1.0);
                        };
                        for (int i = 0; i < 4; ++i) go(i % SETS);
                        (void)hipEventRecord(e0);
                        const int N = 40;
                        for (int i = 0; i < N; ++i) go(i % SETS);
                        (void)hipEventRecord(e1);
                        (void)hipEventSynchronize(e1);
                        float ms = 0;
                        (void)hipEventElapsedTime(&ms, e0, e1);
                        const double us = ms * 1e3 / N;
                        const double bytes = (double)OUT_B + (read ? (double)IN_B : 0.0);
                        printf("{\"pass\": %d, \"read\": %d, \"fp64_per_64traj\": %d, \"waves_per_simd\": %d, "
                               "\"rounds\": %d, \"waves\": %zu, \"us\": %.2f, \"GBs\": %.0f}\n",
                               pass, read, prefix, wps, rounds, waves, us, bytes / us / 1e3);
                        fflush(stdout);
                    }
    return 0;
}
