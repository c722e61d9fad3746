// storebench.hip — write-pattern micro-benchmark for the coefficient output of the
// reduced solve (65,536 trajectories x 10 segments x 24 doubles = 126 MB).
// Each wavefront owns 32 consecutive trajectories (a contiguous 61,440-B block) and
// writes it in one of several orders; only the order differs between patterns.
//   hipcc --offload-arch=gfx950 -O3 -o storebench storebench.hip && ./storebench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int M = 10, TPW = 32, B = 65536, NW = B / TPW;
constexpr int TRAJ = M * 24;  // doubles per trajectory

__device__ __forceinline__ double2 val(int a, int b) { return make_double2((double)a, (double)b); }

// P0: coalesced — consecutive lanes write consecutive 16 B of the wave's block.
__global__ __launch_bounds__(64) void p0(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
#pragma unroll 4
    for (int q = 0; q < TPW * TRAJ / 2 / 64; ++q) reinterpret_cast<double2*>(base)[q * 64 + lane] = val(q, lane);
}

// P1: per-axis staging: 16 pieces of 64 B per instruction (slot, side, axis).
__global__ __launch_bounds__(64) void p1(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
    for (int e = 0; e < M / 2; ++e)
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = lane + 64 * q, chunk = p >> 2, off = p & 3, slot = chunk >> 1, rt = chunk & 1;
                const int seg = rt ? (M - 1 - e) : e;
                reinterpret_cast<double2*>(base + slot * TRAJ + seg * 24 + a * 8)[off] = val(e, a);
            }
}

// P2: direct per-lane stores: lane (slot, side) writes its 192-B segment as 12 x 16 B.
__global__ __launch_bounds__(64) void p2(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x, slot = lane >> 1, rt = lane & 1;
    for (int e = 0; e < M / 2; ++e) {
        const int seg = rt ? (M - 1 - e) : e;
#pragma unroll
        for (int j = 0; j < 12; ++j) reinterpret_cast<double2*>(base + slot * TRAJ + seg * 24)[j] = val(e, j);
    }
}

// P3: segment staging: per side, 32 chunks of 192 B, 64 x 16 B per instruction.
__global__ __launch_bounds__(64) void p3(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
    for (int e = 0; e < M / 2; ++e)
        for (int side = 0; side < 2; ++side)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const int p = lane + 64 * q, chunk = p / 12, off = p - 12 * chunk;
                const int seg = side ? (M - 1 - e) : e;
                reinterpret_cast<double2*>(base + chunk * TRAJ + seg * 24)[off] = val(e, q);
            }
}

// P4: segment pairs: per step both sides of a trajectory are adjacent in memory
// (segment e and e+1): 32 chunks of 384 B.
__global__ __launch_bounds__(64) void p4(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
    for (int e = 0; e < M; e += 2)
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const int p = lane + 64 * q, chunk = p / 24, off = p - 24 * chunk;
            reinterpret_cast<double2*>(base + chunk * TRAJ + e * 24)[off] = val(e, q);
        }
}

int main() {
    double* C;
    hipMalloc(&C, (size_t)B * TRAJ * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    void (*ks[])(double*) = {p0, p1, p2, p3, p4};
    const char* names[] = {"P0 coalesced", "P1 axis-stage 64B", "P2 direct 16B/lane", "P3 seg-stage 192B",
                           "P4 seg-pair 384B"};
    for (int occ = 0; occ < 2; ++occ) {
        for (int k = 0; k < 5; ++k) {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(ks[k], dim3(NW), dim3(64), 0, 0, C);
            hipEventRecord(e0);
            for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(ks[k], dim3(NW), dim3(64), 0, 0, C);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 20;
            printf("{\"pattern\": \"%s\", \"us\": %.2f, \"GBs\": %.0f}\n", names[k], us,
                   (double)B * TRAJ * 8 / us / 1e3);
        }
    }
    hipFree(C);
    return 0;
}
