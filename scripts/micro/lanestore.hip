// lanestore.hip — store-rate probe for the lane-per-trajectory output path:
// 64 trajectories (10 segments, 1,920 B each) per wavefront, one wavefront per SIMD
// (1,024 waves for 65,536 trajectories), whole 128-B lines, 8 lines (8 trajectories)
// per store instruction.  4 output buffers rotated (504 MB), so nothing stays in the
// Infinity Cache between launches.  `work` = dependent-free FP64 FMAs per lane between
// groups of 8 stores (the emission arithmetic), `burst` = lines per group.
//   hipcc --offload-arch=gfx950 -O3 -o lanestore lanestore.hip && ./lanestore
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int M = 10, TRAJ = M * 24, LINES = TRAJ / 16;  // 15 lines per trajectory

template <int WORK, int WAVES>
__global__ __launch_bounds__(64, WAVES) void k(double* C, double seed) {
    double* base = C + (size_t)blockIdx.x * 64 * TRAJ;
    const int lane = threadIdx.x, sub = lane & 7, grp = lane >> 3;
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = seed + lane + j;
    for (int l = LINES - 1; l >= 0; --l) {
#pragma unroll
        for (int w = 0; w < WORK / 8; ++w)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = __builtin_fma(acc[j], 1.0000001, 1e-9);
#pragma unroll
        for (int q = 0; q < 8; ++q)  // trajectories 8q..8q+7, line l
            reinterpret_cast<double2*>(base + (q * 8 + grp) * TRAJ + l * 16)[sub] = make_double2(acc[q], acc[(q + 1) & 7]);
    }
}

int main() {
    const int B = 65536, NWV = B / 64, SETS = 4;
    double* C[SETS];
    for (int s = 0; s < SETS; ++s) (void)hipMalloc(&C[s], (size_t)B * TRAJ * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name, int sets) {
        for (int w = 0; w < 4; ++w) hipLaunchKernelGGL(kern, dim3(NWV), dim3(64), 0, 0, C[w % sets], 1.0);
        (void)hipEventRecord(e0);
        for (int it = 0; it < 40; ++it) hipLaunchKernelGGL(kern, dim3(NWV), dim3(64), 0, 0, C[it % sets], 1.0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / 40;
        printf("{\"probe\": \"%s\", \"sets\": %d, \"us\": %.2f, \"GBs\": %.0f}\n", name, sets, us, (double)B * TRAJ * 8 / us / 1e3);
    };
    for (int sets : {1, 4}) {
        run(k<0, 1>, "work0 1w", sets);
        run(k<64, 1>, "work64 1w", sets);
        run(k<256, 1>, "work256 1w", sets);
        run(k<0, 2>, "work0 2wcap", sets);
    }
    return 0;
}
