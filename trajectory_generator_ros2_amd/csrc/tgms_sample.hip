// tgms_sample.hip — sampler on gfx950.
//
// Goal-layout p/v/a/j/psi/dpsi at t_k = k*dt per trajectory, the last sample pinned
// to the final waypoint and end derivatives (Line.cpp:80-82 convention); yaw per
// tgms_yaw_mode (atan2(v_y, v_x), Figure8.cpp:123).  The output (112 B per sample)
// dominates the traffic, so the kernel is built around the store stream:
//   - one 256-thread workgroup per (trajectory, piece): a trajectory's 64-sample
//     chunks are split into `pieces` contiguous runs, so a small batch of long
//     trajectories still fills the GPU in many short rounds instead of a few long
//     ones with a ragged last round (grid-stride over the items);
//   - the workgroup's trajectory coefficients and
//     their derivative forms (j c_j, j(j-1) c_j, ...) plus the segment start times
//     sit in LDS, so p/v/a/j are four pure FMA Horner chains per axis;
//   - each wavefront evaluates 64 consecutive samples, stages them in LDS, and
//     writes the 64 x 112 B = 7 KiB run with seven fully coalesced 16-B-per-lane
//     stores.
#include <algorithm>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

#ifndef TGMS_SAMPLE_NT
#define TGMS_SAMPLE_NT 0
#endif
constexpr int SW = 4;                  // wavefronts per workgroup
constexpr int G = TGMS_GOAL_STRIDE;    // 14 doubles per sample
constexpr int CH = W64 * G / 2;        // double2 per wave chunk (448)

// atan2 for the heading (|v_xy| > 1e-3 guaranteed by the caller): octant
// reduction to u in [-tan(pi/8), tan(pi/8)], then the atan series to u^43
// (truncation < 1e-17), all in registers the caller already has free.
__device__ __forceinline__ double atan2_f64(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const double mx = fmax(ax, ay), mn = fmin(ax, ay);
    const double a = mn * fast_rcp(mx);                     // [0, 1]
    const bool hi = a > 0.41421356237309503;                // tan(pi/8)
    const double u = hi ? (a - 1.0) * fast_rcp(a + 1.0) : a;  // atan(a) = pi/4 + atan(u)
    const double u2 = u * u;
    double s = 1.0 / 43.0;
#pragma unroll
    for (int n = 20; n >= 0; --n) s = __builtin_fma(s, -u2, 1.0 / (2 * n + 1));
    double r = u * s + (hi ? 0.78539816339744828 : 0.0);
    r = ay > ax ? 1.5707963267948966 - r : r;
    r = x < 0.0 ? 3.1415926535897931 - r : r;
    return y < 0.0 ? -r : r;
}

__device__ __forceinline__ void yaw_of(int yaw_mode, double yaw_const, const double* v, const double* acc,
                                       double& psi, double& dpsi) {
    const double s2 = v[0] * v[0] + v[1] * v[1];
    const bool yv = (yaw_mode == TGMS_YAW_VELOCITY) && (s2 > 1e-6);
    const double num = v[0] * acc[1] - v[1] * acc[0];
    psi = yv ? atan2_f64(v[1], v[0]) : yaw_const;
    dpsi = yv ? num / s2 : 0.0;
}

__global__ __launch_bounds__(W64 * SW) void k_sample(int32_t B, const int32_t* __restrict__ seg_offsets,
                                                      const double* __restrict__ W,
                                                      const double* __restrict__ T,
                                                      const double* __restrict__ ED,
                                                      const double* __restrict__ C, double dt, int yaw_mode,
                                                      double yaw_const,
                                                      const int64_t* __restrict__ sample_offsets,
                                                      double* __restrict__ out, int pieces) {
    // per (segment, axis): [derivative order k][8] = d^k/dt^k coefficient of t^(j-k) at slot j
    __shared__ double cf[TGMS_MAX_SEGMENTS * 3 * 4 * 8];
    __shared__ double tau[TGMS_MAX_SEGMENTS + 1];
    __shared__ alignas(16) double stage[SW][W64 * G];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double2* st2 = reinterpret_cast<double2*>(stage[wave]);
    const int64_t n_items = (int64_t)B * pieces;
    for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
        const int64_t b = item / pieces;
        const int piece = (int)(item - b * pieces);
        const int64_t base = sample_offsets[b];
        const int64_t ns = sample_offsets[b + 1] - base;
        // this trajectory's pieces: at least 6 chunks per wave each (shorter pieces
        // cost more in start-up than they save in balance)
        const int64_t nch = (ns + W64 - 1) / W64;
        const int np = (int)std::max<int64_t>(1, std::min<int64_t>(pieces, nch / (6 * SW)));
        if (piece >= np) continue;  // workgroup-uniform
        const int64_t s0 = seg_offsets[b];
        const int M = seg_offsets[b + 1] - (int32_t)s0;
        __syncthreads();  // the previous trajectory's readers are done with cf / tau
        for (int e = tid; e < M * 24; e += W64 * SW) {  // e = (segment*3 + axis)*8 + j
            const int j = e & 7;
            const double c = C[s0 * 24 + e];
            double* f = cf + (e >> 3) * 32;
            f[j] = c;
            f[8 + j] = (double)j * c;
            f[16 + j] = (double)(j * (j - 1)) * c;
            f[24 + j] = (double)(j * (j - 1) * (j - 2)) * c;
        }
        if (tid < M) tau[tid + 1] = T[s0 + tid];  // all loads in flight at once
        __syncthreads();
        if (tid == 0) {  // prefix sums in the same order as tgms_sample_offsets / the oracle
            double acc = 0.0;
            tau[0] = 0.0;
            for (int i = 1; i <= M; ++i) {
                acc += tau[i];
                tau[i] = acc;
            }
        }
        __syncthreads();
        const double* wl = W + (s0 + b + M) * 3;
        const double* edf = ED ? ED + b * 18 + 9 : nullptr;
        // each lane's sample times only grow: carry its segment index across chunks
        int i = 0;
        double t_next = M > 1 ? tau[1] : 0.0, t_cur = 0.0;
        // this piece: a contiguous run of chunks, dealt round-robin to the waves
        const int64_t per = (nch + np - 1) / np;
        const int64_t kend = std::min<int64_t>(ns, (int64_t)(piece + 1) * per * W64);
        for (int64_t k0 = ((int64_t)piece * per + wave) * W64; k0 < kend; k0 += (int64_t)W64 * SW) {
            const int64_t k = k0 + lane;
            // each value goes to the LDS stage as soon as it exists (few live registers
            // across the atan2 below, which keeps three waves per SIMD resident)
            double* so = stage[wave] + lane * G;
            double v[2], ac[2];
            if (k < ns - 1) {
                const double t = (double)k * dt;
                while (i + 1 < M && t_next <= t) {  // same test as the oracle's scan
                    ++i;
                    t_cur = t_next;
                    t_next = tau[i + 1 < M ? i + 1 : M];
                }
                const double lt = t - t_cur;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    __builtin_amdgcn_sched_barrier(0);
                    const double* f = cf + (i * 3 + a) * 32;
                    double d[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        double s = f[q * 8 + 7];
#pragma unroll
                        for (int j = 6; j >= q; --j) s = __builtin_fma(s, lt, f[q * 8 + j]);
                        d[q] = s;
                    }
                    so[a] = d[0];
                    so[3 + a] = d[1];
                    so[6 + a] = d[2];
                    so[9 + a] = d[3];
                    if (a < 2) {
                        v[a] = d[1];
                        ac[a] = d[2];
                    }
                }
            } else {  // the pinned final sample (and lanes past the end, never stored)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const double va = edf ? edf[a] : 0.0, aa = edf ? edf[3 + a] : 0.0;
                    so[a] = wl[a];
                    so[3 + a] = va;
                    so[6 + a] = aa;
                    so[9 + a] = edf ? edf[6 + a] : 0.0;
                    if (a < 2) {
                        v[a] = va;
                        ac[a] = aa;
                    }
                }
            }
            yaw_of(yaw_mode, yaw_const, v, ac, so[12], so[13]);
            // 7 coalesced 16-B stores per lane of the wave's 64 staged samples
            __builtin_amdgcn_wave_barrier();
            const int64_t n2 = (ns - k0) * (G / 2);  // double2 of this chunk inside the trajectory
            double2* dst = reinterpret_cast<double2*>(out + (base + k0) * G);
#pragma unroll
            for (int q = 0; q < G / 2; ++q) {
                const int idx = q * W64 + lane;
#if TGMS_SAMPLE_NT  // nontemporal stores: 0.61 against 0.50 ms (profiles/r05_sampler_nt_ab.jsonl), off
                if (idx < n2) {
                    typedef double d2v __attribute__((ext_vector_type(2)));
                    const double2 x = st2[idx];
                    __builtin_nontemporal_store(d2v{x.x, x.y}, reinterpret_cast<d2v*>(&dst[idx]));
                }
#else
                if (idx < n2) dst[idx] = st2[idx];
#endif
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace

hipError_t launch_sample(int32_t B, const int32_t* seg_offsets, const double* W, const double* T,
                         const double* ED, const double* C, double dt, int yaw_mode,
                         double yaw_const, const int64_t* sample_offsets, double* out,
                         hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    // at most `pieces` per trajectory: up to ~16 rounds of the resident workgroups
    // (256 CUs x 3), so the last round's raggedness costs a few percent; the kernel
    // lowers it per trajectory for short ones.  Measured (4,096 x M = 10 at 100 Hz,
    // 22.8 M samples): 1 piece 0.55 ms, 3 pieces 0.50 ms, 12 pieces 0.61 ms.
    constexpr int64_t kItems = 16 * 256 * 3;
    const int pieces = (int)std::min<int64_t>(4, std::max<int64_t>(1, (kItems + B - 1) / B));
    const int64_t items = (int64_t)B * pieces;
    const int64_t blocks = items < 65536 ? items : 65536;
    TGMS_LAUNCH(k_sample, dim3((unsigned)blocks), dim3(W64 * SW), 0, stream, B, seg_offsets, W, T, ED, C,
                       dt, yaw_mode, yaw_const, sample_offsets, out, pieces);
    return hipSuccess;
}

}  // namespace tgms
