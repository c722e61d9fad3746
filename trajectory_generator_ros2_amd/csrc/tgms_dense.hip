// tgms_dense.hip — TGMS_METHOD_DENSE_KKT: the survey's literal a1-a3 on gfx950.
//
// One WAVEFRONT per trajectory; [[2Q, A^T],[A, 0]] (snap
// Hessian Q, a2: endpoint/continuity rows A with right-hand side b) is assembled
// in LDS (N = 14M+2, N^2*8 B = 161,312 B at M = 10); LU with partial pivoting,
// lanes over rows for the pivot search / multipliers and over columns for the
// rank-1 update; the 3 right-hand sides live in registers of the row-owner lanes.
#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {


__device__ __forceinline__ double dfac(int j, int k) {
    double r = 1.0;
    for (int q = 0; q < k; ++q) r *= (double)(j - q);
    return (k > j) ? 0.0 : r;
}

__device__ __forceinline__ double ipow(double t, int e) {
    double p = 1.0;
    for (int q = 0; q < e; ++q) p *= t;
    return p;
}

__device__ __forceinline__ double bcast(double v, int src) { return __shfl(v, src, W64); }

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64) void k_dense_kkt(int32_t n_traj, const int32_t* __restrict__ ids,
                                                  const int32_t* __restrict__ seg_offsets,
                                                  const double* __restrict__ W,
                                                  const double* __restrict__ T,
                                                  const double* __restrict__ ED,
                                                  double* __restrict__ C,
                                                  int32_t* __restrict__ status) {
    constexpr int n = 8 * M;
    constexpr int m = 8 + 6 * (M - 1);
    constexpr int N = n + m;
    constexpr int S = (N + W64 - 1) / W64;  // rows (and columns) per lane
    extern __shared__ double smem[];
    double* A = smem;          // N x N row-major KKT
    double* lcol = smem + N * N;  // multipliers of the current column

    const int lane = threadIdx.x;
    const int32_t bi = blockIdx.x;
    if (bi >= n_traj) return;
    const int32_t b = ids ? ids[bi] : bi;
    const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;
    const double* w = W + (s0 + b) * 3;
    const double* tt = T + s0;
    const double* ed = HAS_ED ? ED + (int64_t)b * 18 : nullptr;

    bool valid = true;
    for (int i = 0; i < M; ++i) valid = valid && finite_pos(tt[i]);
    {
        double s = 0.0;
        for (int q = 0; q < (M + 1) * 3; ++q) s += w[q] * 0.0;
        if (HAS_ED)
            for (int q = 0; q < 18; ++q) s += ed[q] * 0.0;
        valid = valid && (s == 0.0);
    }

    for (int e = lane; e < N * N; e += W64) A[e] = 0.0;
    __syncthreads();
    // a1: 2Q blocks
    for (int e = lane; e < M * 16; e += W64) {
        const int i = e >> 4, j = 4 + ((e >> 2) & 3), k = 4 + (e & 3);
        const int ex = j + k - 7;
        A[(8 * i + j) * N + 8 * i + k] = 2.0 * dfac(j, 4) * dfac(k, 4) * ipow(tt[i], ex) / (double)ex;
    }
    // a2: constraint rows (and their transposes), one lane per row
    for (int r = lane; r < m; r += W64) {
        double* rowp = A + (n + r) * N;
        auto put = [&](int col, double v) {
            rowp[col] = v;
            A[col * N + n + r] = v;
        };
        if (r < 4) {
            put(r, dfac(r, r));
        } else if (r < 8) {
            const int k = r - 4;
            const double t = tt[M - 1];
            for (int j = k; j < 8; ++j) put(8 * (M - 1) + j, dfac(j, k) * ipow(t, j - k));
        } else {
            const int i = 1 + (r - 8) / 6, q = (r - 8) % 6;
            const double t = tt[i - 1];
            if (q == 0) {
                for (int j = 0; j < 8; ++j) put(8 * (i - 1) + j, ipow(t, j));
            } else if (q == 1) {
                put(8 * i, 1.0);
            } else {
                const int k = q - 1;
                for (int j = k; j < 8; ++j) put(8 * (i - 1) + j, dfac(j, k) * ipow(t, j - k));
                put(8 * i + k, -dfac(k, k));
            }
        }
    }
    // right-hand sides in registers: lane owns rows lane + 64*s
    double rhs[S][3];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int v = lane + W64 * s;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double val = 0.0;
            if (v >= n && v < N) {
                const int r = v - n;
                if (r < 4) val = (r == 0) ? w[a] : (HAS_ED ? ed[(r - 1) * 3 + a] : 0.0);
                else if (r < 8) val = (r == 4) ? w[3 * M + a] : (HAS_ED ? ed[9 + (r - 5) * 3 + a] : 0.0);
                else {
                    const int i = 1 + (r - 8) / 6, q = (r - 8) % 6;
                    val = (q < 2) ? w[3 * i + a] : 0.0;
                }
            }
            rhs[s][a] = val;
        }
    }
    __syncthreads();

    // a3: LU with partial pivoting
    bool singular = false;
    for (int k = 0; k < N; ++k) {
        double best = -1.0;
        int bidx = N;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int i = lane + W64 * s;
            if (i >= k && i < N) {
                const double v = fabs(A[i * N + k]);
                if (v > best) { best = v; bidx = i; }
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double ov = __shfl_xor(best, off, W64);
            const int oi = __shfl_xor(bidx, off, W64);
            if (ov > best || (ov == best && oi < bidx)) { best = ov; bidx = oi; }
        }
        if (!(best > 0.0)) { singular = true; break; }
        const int p = bidx;
        const int ks = k / W64, kl = k % W64, ps = p / W64, pl = p % W64;
        if (p != k) {
            for (int j = k + lane; j < N; j += W64) {
                const double t = A[k * N + j];
                A[k * N + j] = A[p * N + j];
                A[p * N + j] = t;
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double vk = 0.0, vp = 0.0;
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    if (s == ks) vk = rhs[s][a];
                    if (s == ps) vp = rhs[s][a];
                }
                vk = bcast(vk, kl);
                vp = bcast(vp, pl);
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    if (s == ks && lane == kl) rhs[s][a] = vp;
                    if (s == ps && lane == pl) rhs[s][a] = vk;
                }
            }
        }
        __syncthreads();
        const double ipiv = 1.0 / A[k * N + k];
        double rk[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < S; ++s)
                if (s == ks) v = rhs[s][a];
            rk[a] = bcast(v, kl);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int i = lane + W64 * s;
            if (i > k && i < N) {
                const double l = A[i * N + k] * ipiv;
                lcol[i] = l;
#pragma unroll
                for (int a = 0; a < 3; ++a) rhs[s][a] -= l * rk[a];
            }
        }
        __syncthreads();
        double u[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int j = k + 1 + lane + W64 * s;
            u[s] = (j < N) ? A[k * N + j] : 0.0;
        }
        for (int i = k + 1; i < N; ++i) {
            const double l = lcol[i];
            if (l == 0.0) continue;  // wave-uniform: the KKT stays sparse for many steps
            double* rowi = A + i * N + k + 1 + lane;
#pragma unroll
            for (int s = 0; s < S; ++s)
                if (k + 1 + lane + W64 * s < N) rowi[W64 * s] -= l * u[s];
        }
        __syncthreads();
    }
    // back substitution (column oriented); x overwrites rhs
    if (!singular) {
        for (int k = N - 1; k >= 0; --k) {
            const int ks = k / W64, kl = k % W64;
            const double ipiv = 1.0 / A[k * N + k];
            double xk[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double v = 0.0;
#pragma unroll
                for (int s = 0; s < S; ++s)
                    if (s == ks) v = rhs[s][a];
                xk[a] = bcast(v, kl) * ipiv;
            }
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int i = lane + W64 * s;
                if (i == k) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) rhs[s][a] = xk[a];
                } else if (i < k) {
                    const double aik = A[i * N + k];
#pragma unroll
                    for (int a = 0; a < 3; ++a) rhs[s][a] -= aik * xk[a];
                }
            }
        }
    }
    // a4: coefficients [seg][axis][8]
    double fin = 0.0;
    double* out = C + s0 * 24;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int v = lane + W64 * s;
        if (v < n) {
            const int i = v >> 3, j = v & 7;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const double c = (valid && !singular) ? rhs[s][a] : 0.0;
                fin += rhs[s][a];
                out[(i * 3 + a) * 8 + j] = c;
            }
        }
    }
    // any lane non-finite -> NONFINITE
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) fin += __shfl_xor(fin, off, W64);
    if (lane == 0 && status) {
        int32_t st = TGMS_OK;
        if (!valid) st = TGMS_ERR_INVALID_ARG;
        else if (singular) st = TGMS_ERR_SINGULAR;
        else if (!(fin * 0.0 == 0.0)) st = TGMS_ERR_NONFINITE;
        status[b] = st;
    }
}

template <int M>
hipError_t dense_M(int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W,
                   const double* T, const double* ED, double* C, int32_t* status,
                   hipStream_t stream) {
    constexpr int N = 14 * M + 2;
    const size_t lds = sizeof(double) * (size_t)(N * N + N);
    if (n_traj <= 0) return hipSuccess;
    hipError_t e;
    if (ED) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dense_kkt<M, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_dense_kkt<M, true>), dim3(n_traj), dim3(W64), lds, stream, n_traj, ids, so, W, T, ED, C, status);
    } else {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dense_kkt<M, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_dense_kkt<M, false>), dim3(n_traj), dim3(W64), lds, stream, n_traj, ids, so, W, T, ED, C, status);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_dense_kkt(int M, int32_t n_traj, const int32_t* ids, const int32_t* so,
                            const double* W, const double* T, const double* ED, double* C,
                            int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return dense_M<m>(n_traj, ids, so, W, T, ED, C, status, stream);
        X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10)
#undef X
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tgms
