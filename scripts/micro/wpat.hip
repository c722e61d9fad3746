// Write-pattern micro-benchmark for the sampler output (2.56 GB, 16-B stores):
//   A: each workgroup streams through its own contiguous region (one trajectory per
//      workgroup, as k_sample does), 7 KB per wave step
//   B: global chunk order (consecutive 7-KB chunks go to consecutive waves), like a fill
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
typedef double double2_t __attribute__((ext_vector_type(2)));
constexpr long long BYTES = 2560LL << 20;
constexpr int CH = 7 * 1024;  // bytes per wave chunk (64 lanes x 112 B)
__global__ __launch_bounds__(256) void pat_a(double2_t* out, long long per_block, int nblk_total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int b = blockIdx.x; b < nblk_total; b += gridDim.x) {
        double2_t* base = out + (long long)b * per_block / 16;
        for (long long c = w; c * CH < per_block; c += 4) {
            double2_t* d = base + c * CH / 16;
            for (int q = 0; q < 7; ++q) d[q * 64 + lane] = double2_t{(double)q, (double)lane};
        }
    }
}
__global__ __launch_bounds__(256) void pat_b(double2_t* out, long long nchunks) {
    const int lane = threadIdx.x & 63;
    const long long wid = (long long)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (long long)gridDim.x * 4;
    for (long long c = wid; c < nchunks; c += nw) {
        double2_t* d = out + c * CH / 16;
        for (int q = 0; q < 7; ++q) d[q * 64 + lane] = double2_t{(double)q, (double)lane};
    }
}
int main() {
    double2_t* out;
    CK(hipMalloc(&out, BYTES));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int ntraj = 4096;
    const long long per = (BYTES / ntraj) / CH * CH;
    const long long nch = BYTES / CH;
    for (int grid : {768, 1024, 2048, 4096}) {
        for (int rep = 0; rep < 2; ++rep) {
            float ta, tb;
            hipEventRecord(e0); hipLaunchKernelGGL(pat_a, dim3(grid < ntraj ? grid : ntraj), dim3(256), 0, 0, out, per, ntraj);
            hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ta, e0, e1);
            hipEventRecord(e0); hipLaunchKernelGGL(pat_b, dim3(grid), dim3(256), 0, 0, out, nch);
            hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&tb, e0, e1);
            if (rep) printf("grid %d: A (per-trajectory regions) %.3f ms %.2f TB/s | B (global order) %.3f ms %.2f TB/s\n",
                            grid, ta, per * ntraj / ta / 1e9, tb, nch * CH / tb / 1e9);
        }
    }
    return 0;
}
