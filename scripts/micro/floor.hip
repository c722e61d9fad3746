// floor.hip — the headline's byte-mix floor, re-measured (round 6).
//
// Config 3 moves 22.5 MB of inputs (waypoints + times) and 126 MB of coefficients per
// launch of 65,536 trajectories.  This probe moves exactly those bytes with no solve:
// each wave reads its slice of the inputs (16 B per lane per instruction, every load in
// flight at once), optionally runs the lane kernel's FP64 work (3,328 FMA
// wave-instructions per 64 trajectories), then writes its slice of the output front to
// back, 1 KiB (eight whole 128-B lines) per wave-instruction.  Swept:
//   waves per SIMD 1..4 (pinned by LDS), rounds of waves 1/2/4 (waves finishing at
//   different times), and 1 or 4 launch streams inside one captured HIP graph of 40
//   launches (consecutive launches overlap across streams, as bench.py's headline does;
//   a direct launch loop does not overlap).
// 4 input/output sets rotate (594 MB, past the 256 MiB Infinity Cache: every launch
// reads and writes fresh lines).  One JSON line per configuration.
//   hipcc --offload-arch=gfx950 -O3 -o floor floor.hip && ./floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr size_t B = 65536, OUT_B = B * 1920, IN_B = B * 344;
constexpr int SETS = 4;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(64) void k(const double2* __restrict__ in, double2* __restrict__ out, size_t in_per_wave,
                                       size_t out_per_wave, int fma, double seed) {
    extern __shared__ double pin_lds[];  // occupancy pin only
    const int lane = threadIdx.x;
    const size_t w = blockIdx.x;
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = seed + lane + j;
    const double2* src = in + w * in_per_wave;
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
        CK(hipMalloc(&in[s], IN_B));
        CK(hipMalloc(&out[s], OUT_B));
        CK(hipMemset(in[s], 0, IN_B));
        CK(hipMemset(out[s], 0, OUT_B));
    }
    constexpr int NS = 4, N = 40;
    hipStream_t st[NS];
    hipEvent_t fork, join[NS], e0, e1;
    for (int i = 0; i < NS; ++i) {
        CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&join[i], hipEventDisableTiming));
    }
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int prefix : {0, 3328})
        for (int streams : {1, 4})
            for (int wps : {1, 2, 3, 4})
                for (int rounds : {1, 2, 4}) {
                    const size_t waves = 1024ull * wps * rounds;
                    const size_t out_pw = OUT_B / 16 / waves, in_pw = IN_B / 16 / waves;
                    const int fma = (int)(prefix / 8 / (wps * rounds));
                    const size_t lds = (160 * 1024) / (4 * wps) - 256;
                    // capture N launches: launch i on stream i % streams with set i % SETS
                    hipGraph_t g;
                    hipGraphExec_t ge;
                    CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeThreadLocal));
                    CK(hipEventRecord(fork, st[0]));
                    for (int j = 1; j < streams; ++j) CK(hipStreamWaitEvent(st[j], fork, 0));
                    for (int i = 0; i < N; ++i) {
                        const int s = i % SETS;
                        hipLaunchKernelGGL(k, dim3(waves), dim3(64), lds, st[i % streams], in[s], out[s], in_pw,
                                           out_pw, fma, 1.0);
                    }
                    for (int j = 1; j < streams; ++j) {
                        CK(hipEventRecord(join[j], st[j]));
                        CK(hipStreamWaitEvent(st[0], join[j], 0));
                    }
                    CK(hipStreamEndCapture(st[0], &g));
                    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                    CK(hipGraphLaunch(ge, st[0]));  // warm (upload)
                    CK(hipStreamSynchronize(st[0]));
                    float best = 1e30f;
                    for (int rep = 0; rep < 3; ++rep) {
                        CK(hipEventRecord(e0, st[0]));
                        CK(hipGraphLaunch(ge, st[0]));
                        CK(hipEventRecord(e1, st[0]));
                        CK(hipEventSynchronize(e1));
                        float ms = 0;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        best = ms < best ? ms : best;
                    }
                    CK(hipGraphExecDestroy(ge));
                    CK(hipGraphDestroy(g));
                    const double us = best * 1e3 / N;
                    const double bytes = (double)OUT_B + (double)IN_B;
                    std::printf("{\"fp64_per_64traj\": %d, \"streams\": %d, \"waves_per_simd\": %d, \"rounds\": %d, "
                                "\"waves\": %zu, \"us_per_launch\": %.2f, \"GBs\": %.0f}\n",
                                prefix, streams, wps, rounds, waves, us, bytes / us / 1e3);
                    std::fflush(stdout);
                }
    return 0;
}
