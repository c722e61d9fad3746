// runstore.hip — store-pattern probe at one wavefront per SIMD (1,024 waves of 64
// trajectories x 10 segments, 1,920 B per trajectory, 4 rotated output sets = 504 MB):
//   lines8  the lane kernel's pattern: per line index, 8 instructions of 8 whole lines
//           (8 trajectories, 1,920 B apart)
//   pair384 per segment pair, every trajectory's 384 contiguous bytes (its 3 lines),
//           64 consecutive 16-B pieces per instruction (~2.7 trajectories' runs)
//   contig  the wave's 120 KB block front to back, 1 KB per instruction (the ideal)
//   hipcc --offload-arch=gfx950 -O3 -o runstore runstore.hip && ./runstore
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int M = 10, TRAJ = M * 24, LINES = TRAJ / 16;  // doubles per trajectory; 15 lines
constexpr int PIECES = 64 * TRAJ / 2;                    // 16-B pieces per wave block (7,680)

template <int PAT>
__global__ __launch_bounds__(64, 1) void k(double* C, double seed) {
    double* base = C + (size_t)blockIdx.x * 64 * TRAJ;
    double2* b2 = reinterpret_cast<double2*>(base);
    const int lane = threadIdx.x, sub = lane & 7, grp = lane >> 3;
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = seed + lane + j;
    if constexpr (PAT == 0) {
        for (int l = LINES - 1; l >= 0; --l) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
                b2[((q * 8 + grp) * TRAJ + l * 16) / 2 + sub] = make_double2(acc[q], acc[(q + 1) & 7]);
        }
    } else if constexpr (PAT == 1) {
        // segment pairs from the last down; per pair 64 x 24 pieces = 24 instructions
        for (int p = M / 2 - 1; p >= 0; --p) {
#pragma unroll
            for (int i = 0; i < 24; ++i) {
                const int j = i * 64 + lane, t = j / 24, r = j - t * 24;
                b2[(t * TRAJ + p * 48) / 2 + r] = make_double2(acc[i & 7], acc[(i + 1) & 7]);
            }
        }
    } else {
        for (int i = PIECES / 64 - 1; i >= 0; --i) b2[i * 64 + lane] = make_double2(acc[i & 7], acc[(i + 1) & 7]);
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
        printf("{\"probe\": \"%s\", \"sets\": %d, \"us\": %.2f, \"GBs\": %.0f}\n", name, sets, us,
               (double)B * TRAJ * 8 / us / 1e3);
    };
    for (int rep = 0; rep < 2; ++rep)
        for (int sets : {1, 4}) {
            run(k<0>, "lines8", sets);
            run(k<1>, "pair384", sets);
            run(k<2>, "contig", sets);
        }
    return 0;
}
