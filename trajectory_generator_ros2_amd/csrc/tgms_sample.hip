// tgms_sample.hip — sampler on gfx950.
//
// One wavefront per trajectory (grid-stride), lanes over samples: t_k = k*dt,
// p/v/a/j by Horner on the segment's coefficients, yaw per tgms_yaw_mode, and the
// last sample pinned to the final waypoint (Line.cpp:80-82 convention).
#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

__global__ __launch_bounds__(256) void k_sample(int32_t B, const int32_t* __restrict__ seg_offsets,
                                                const double* __restrict__ W,
                                                const double* __restrict__ T,
                                                const double* __restrict__ ED,
                                                const double* __restrict__ C, double dt,
                                                int yaw_mode, double yaw_const,
                                                const int64_t* __restrict__ sample_offsets,
                                                double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int waves_per_block = blockDim.x / W64;
    const int64_t wave = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * waves_per_block;
    for (int64_t b = wave; b < B; b += n_waves) {
        const int64_t s0 = seg_offsets[b];
        const int M = seg_offsets[b + 1] - (int32_t)s0;
        const int64_t base = sample_offsets[b];
        const int64_t ns = sample_offsets[b + 1] - base;
        const double* tt = T + s0;
        const double* cc = C + s0 * 24;
        for (int64_t k = lane; k < ns - 1; k += W64) {
            const double t = (double)k * dt;
            double tau = 0.0;
            int i = 0;
            for (int q = 0; q + 1 < M; ++q) {
                const double nt = tau + tt[q];
                if (nt <= t) { tau = nt; i = q + 1; }
                else break;
            }
            const double lt = t - tau;
            double* o = out + (base + k) * TGMS_GOAL_STRIDE;
            double v[3], ac[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const double* c = cc + (i * 3 + a) * 8;
                double cv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) cv[j] = c[j];
                double p = cv[7], dv = 7.0 * cv[7], dd = 42.0 * cv[7], jj = 210.0 * cv[7];
#pragma unroll
                for (int j = 6; j >= 0; --j) p = p * lt + cv[j];
#pragma unroll
                for (int j = 6; j >= 1; --j) dv = dv * lt + (double)j * cv[j];
#pragma unroll
                for (int j = 6; j >= 2; --j) dd = dd * lt + (double)(j * (j - 1)) * cv[j];
#pragma unroll
                for (int j = 6; j >= 3; --j) jj = jj * lt + (double)(j * (j - 1) * (j - 2)) * cv[j];
                o[a] = p;
                o[3 + a] = dv;
                o[6 + a] = dd;
                o[9 + a] = jj;
                v[a] = dv;
                ac[a] = dd;
            }
            const double s2 = v[0] * v[0] + v[1] * v[1];
            const bool yv = (yaw_mode == TGMS_YAW_VELOCITY) && (s2 > 1e-6);
            o[12] = yv ? atan2(v[1], v[0]) : yaw_const;
            o[13] = yv ? (v[0] * ac[1] - v[1] * ac[0]) / s2 : 0.0;
        }
        if (lane == 0 && ns >= 1) {
            double* o = out + (base + ns - 1) * TGMS_GOAL_STRIDE;
            const double* wl = W + (s0 + b + M) * 3;
            const double* ed = ED ? ED + b * 18 + 9 : nullptr;
            double v[3], ac[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                o[a] = wl[a];
                v[a] = ed ? ed[a] : 0.0;
                ac[a] = ed ? ed[3 + a] : 0.0;
                o[3 + a] = v[a];
                o[6 + a] = ac[a];
                o[9 + a] = ed ? ed[6 + a] : 0.0;
            }
            const double s2 = v[0] * v[0] + v[1] * v[1];
            const bool yv = (yaw_mode == TGMS_YAW_VELOCITY) && (s2 > 1e-6);
            o[12] = yv ? atan2(v[1], v[0]) : yaw_const;
            o[13] = yv ? (v[0] * ac[1] - v[1] * ac[0]) / s2 : 0.0;
        }
    }
}

}  // namespace

hipError_t launch_sample(int32_t B, const int32_t* seg_offsets, const double* W, const double* T,
                         const double* ED, const double* C, double dt, int yaw_mode,
                         double yaw_const, const int64_t* sample_offsets, double* out,
                         hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int waves = 4;
    int64_t blocks = (B + waves - 1) / waves;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_sample, dim3((unsigned)blocks), dim3(W64 * waves), 0, stream, B, seg_offsets, W, T,
                       ED, C, dt, yaw_mode, yaw_const, sample_offsets, out);
    return hipGetLastError();
}

}  // namespace tgms
