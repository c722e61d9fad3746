// storebench.hip — write-pattern micro-benchmark for the coefficient output of the
// reduced solve (B trajectories x 10 segments x 24 doubles; B = argv[1], default 65,536 = 126 MB).
// Each wavefront owns 32 consecutive trajectories (a contiguous 61,440-B block) and
// writes it in one of several orders; only the order differs between patterns.
//   hipcc --offload-arch=gfx950 -O3 -o storebench storebench.hip && ./storebench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int M = 10, TPW = 32;
static int B = 65536, NW = 65536 / TPW;
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

// P5: axis-outer order of the axis-sequential solve: x rows of every segment, then y, then z
// (each 128-B line holds rows of two different axes, so a line is completed a pass later).
__global__ __launch_bounds__(64) void p5(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
    for (int a = 0; a < 3; ++a)
        for (int e = 0; e < M / 2; ++e)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = lane + 64 * q, chunk = p >> 2, off = p & 3, slot = chunk >> 1, rt = chunk & 1;
                const int seg = rt ? (M - 1 - e) : e;
                reinterpret_cast<double2*>(base + slot * TRAJ + seg * 24 + a * 8)[off] = val(e, a);
            }
}

// P6: whole 128-B lines, 8 per instruction (8 lanes x 16 B each), lines of different
// trajectories (1920-B stride), every line of the block once.
__global__ __launch_bounds__(64) void p6(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x, sub = lane & 7, grp = lane >> 3;  // grp: 8 trajectories
    for (int l = 0; l < TRAJ / 16; ++l)          // 15 lines per trajectory
#pragma unroll
        for (int q = 0; q < TPW / 8; ++q)        // 4 groups of 8 trajectories
            reinterpret_cast<double2*>(base + (q * 8 + grp) * TRAJ + l * 16)[sub] = val(l, q);
}

// P7: the same lines, written as two 64-B halves by back-to-back instructions
// (16 half-lines per instruction, the second instruction completes them).
__global__ __launch_bounds__(64) void p7(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x, sub = lane & 3, grp = lane >> 2;  // grp: 16 trajectories
    for (int l = 0; l < TRAJ / 16; ++l)
#pragma unroll
        for (int q = 0; q < TPW / 16; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                reinterpret_cast<double2*>(base + (q * 16 + grp) * TRAJ + l * 16 + h * 8)[sub] = val(l, h);
}

// P8<N>: the halves of each line written N store instructions apart (the lines of the
// block in groups of 16, one instruction per half-group; other groups' halves between).
template <int N>
__global__ __launch_bounds__(64) void p8(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x, sub = lane & 3, grp = lane >> 2;
    constexpr int G = (TRAJ / 16) * (TPW / 16);  // 30 groups of 16 lines
    auto put = [&](int g, int h) {
        const int l = g >> 1, q = g & 1;
        reinterpret_cast<double2*>(base + (q * 16 + grp) * TRAJ + l * 16 + h * 8)[sub] = val(g, h);
    };
    for (int j = 0; j < G + N; ++j) {
        if (j < G) put(j, 0);
        if (j >= N) put(j - N, 1);
    }
}

// P9: P5's axis-outer order, but the first write of every 128-B line is a whole line
// (the row plus a placeholder for the partner row, back-to-back instructions), so the
// line is valid on-die before its partner half arrives a pass later as a 64-B write.
__global__ __launch_bounds__(64) void p9(double* C) {
    double* base = C + (size_t)blockIdx.x * TPW * TRAJ;
    const int lane = threadIdx.x;
    for (int a = 0; a < 3; ++a)
        for (int e = 0; e < M / 2; ++e) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = lane + 64 * q, chunk = p >> 2, off = p & 3, slot = chunk >> 1, rt = chunk & 1;
                const int seg = rt ? (M - 1 - e) : e;
                reinterpret_cast<double2*>(base + slot * TRAJ + seg * 24 + a * 8)[off] = val(e, a);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = lane + 64 * q, chunk = p >> 2, off = p & 3, slot = chunk >> 1, rt = chunk & 1;
                const int seg = rt ? (M - 1 - e) : e;
                const int r = seg * 3 + a, pr = r ^ 1, pa = pr % 3;
                if (pa > a)  // partner row not yet written: fill its half now
                    reinterpret_cast<double2*>(base + slot * TRAJ + pr * 8)[off] = val(-1, a);
            }
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

int main(int argc, char** argv) {
    if (argc > 1) { B = atoi(argv[1]); NW = B / TPW; }
    double* C;
    hipMalloc(&C, (size_t)B * TRAJ * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    void (*ks[])(double*) = {p0, p1, p2, p3, p4, p5, p6, p7, p8<1>, p8<2>, p8<4>, p8<8>, p8<16>, p9};
    const char* names[] = {"P0 coalesced", "P1 axis-stage 64B", "P2 direct 16B/lane", "P3 seg-stage 192B",
                           "P4 seg-pair 384B", "P5 axis-outer 64B", "P6 full lines 8/instr", "P7 half lines back-to-back", "P8 halves 1 apart", "P8 halves 2 apart", "P8 halves 4 apart", "P8 halves 8 apart", "P8 halves 16 apart", "P9 axis-outer, first write whole line"};
    for (int occ = 0; occ < 1; ++occ) {
        for (int k = 0; k < 14; ++k) {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(ks[k], dim3(NW), dim3(64), 0, 0, C);
            hipEventRecord(e0);
            for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(ks[k], dim3(NW), dim3(64), 0, 0, C);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 20;
            printf("{\"B\": %d, \"pattern\": \"%s\", \"us\": %.2f, \"GBs\": %.0f}\n", B, names[k], us,
                   (double)B * TRAJ * 8 / us / 1e3);
        }
    }
    hipFree(C);
    return 0;
}
