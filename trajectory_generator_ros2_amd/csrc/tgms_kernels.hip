// tgms_kernels.hip — CDNA4 (gfx950) kernels of the batched minimum-snap solver.
//
// Problem: per trajectory, M order-7 segments through M+1
// waypoints, 3 axes sharing segment times, minimum integrated squared snap,
// rest-to-rest (or given) end derivatives, continuity at interior knots.
//
// Kernel 1 — reduced-Hessian solve (default, TGMS_METHOD_REDUCED).
//   Eliminating the equality constraints of the survey's KKT (a2) by the
//   septic-Hermite parametrisation leaves, per axis, an SPD block-tridiagonal
//   system over the free knot derivatives u_k = (v_k, a_k, j_k), k = 1..M-1:
//       H_kk     = KEE * r_{k-1}^(5-d-e) + KSS * r_k^(5-d-e)
//       H_k,k+1  = C_k = KSE * r_k^(5-d-e)            (r_i = 1/T_i)
//   i.e. the Schur complement of the KKT onto the constraint null space, with the
//   snap Hessian (a1) folded into the integer matrix KH (oracle/exact.py derives
//   it exactly; tests prove the exact rational solutions of both systems equal).
//   One LANE per trajectory; block LDL^T (3x3 blocks, the 3 axes are 3 RHS of one
//   factorisation); every intermediate lives in registers (fully unrolled over M).
//   Inputs are staged through LDS transposed [field][lane] so per-lane reads are
//   bank-conflict-free while the global loads are coalesced across the wave.
//
// Kernel 2 — dense KKT (TGMS_METHOD_DENSE_KKT): the survey's literal a1-a3.
//   One WAVEFRONT per trajectory; [[2Q, A^T],[A, 0]] assembled in LDS
//   (N = 14M+2, N^2*8 B = 161,312 B at M = 10); LU with partial pivoting, lanes
//   over rows for the pivot search/multipliers and over columns for the rank-1
//   update; the 3 right-hand sides live in registers of the row-owner lanes.
//
// Kernel 3 — sampler: one wavefront per trajectory,
//   lanes over samples, p/v/a/j + yaw per sample, last sample pinned.
#include "tgms_internal.h"
#include "tgms.h"

#include <float.h>

namespace tgms {
namespace {

constexpr int W64 = 64;      // wavefront width (gfx950)
constexpr int LDS_STRIDE = 65;  // padded [field][lane] rows: conflict-free staging writes

// ---------------------------------------------------------------------------
// Septic-Hermite snap-cost matrix sub-blocks (exact integers; see
// oracle/exact.py hermite_maps() and oracle/minsnap_oracle.c KH).
// Index d, e = 0..2 stands for derivative order d+1, e+1 (v, a, j); the entry
// for a segment of duration T is scaled by r^(5-d-e), r = 1/T.
__device__ constexpr double KSS[3][3] = {{25920, 5400, 480}, {5400, 1200, 120}, {480, 120, 16}};
__device__ constexpr double KEE[3][3] = {{25920, -5400, 480}, {-5400, 1200, -120}, {480, -120, 16}};
// coupling: start derivative d (row) x end derivative e (column)
__device__ constexpr double KSE[3][3] = {{24480, -4680, 360}, {4680, -840, 60}, {360, -60, 4}};
// coupling of derivative d with the segment displacement (w1 - w0), scaled r^(6-d)
__device__ constexpr double KSP[3] = {-50400, -10080, -840};  // start derivatives
__device__ constexpr double KEP[3] = {-50400, 10080, -840};   // end derivatives

__device__ __forceinline__ void rpowers(double r, double (&p)[8]) {
    p[0] = 1.0;
    p[1] = r;
    p[2] = r * r;
    p[3] = p[2] * r;
    p[4] = p[2] * p[2];
    p[5] = p[4] * r;
    p[6] = p[3] * p[3];
    p[7] = p[6] * r;
}

// LDL^T of a 3x3 SPD block, stored as reciprocal pivots + unit-lower multipliers.
struct Ldl3 {
    double i0, i1, i2, l10, l20, l21;
};

__device__ __forceinline__ Ldl3 ldl3(const double (&D)[3][3], bool& spd) {
    Ldl3 f;
    const double p0 = D[0][0];
    f.i0 = 1.0 / p0;
    f.l10 = D[0][1] * f.i0;
    f.l20 = D[0][2] * f.i0;
    const double p1 = D[1][1] - f.l10 * D[0][1];
    f.i1 = 1.0 / p1;
    const double t12 = D[1][2] - f.l20 * D[0][1];
    f.l21 = t12 * f.i1;
    const double p2 = D[2][2] - f.l20 * D[0][2] - f.l21 * t12;
    f.i2 = 1.0 / p2;
    spd = spd && (p0 > 0.0) && (p1 > 0.0) && (p2 > 0.0);
    return f;
}

__device__ __forceinline__ void ldl3_solve(const Ldl3& f, double b0, double b1, double b2,
                                           double& x0, double& x1, double& x2) {
    const double y1 = b1 - f.l10 * b0;
    const double y2 = b2 - f.l20 * b0 - f.l21 * y1;
    x2 = y2 * f.i2;
    x1 = y1 * f.i1 - f.l21 * x2;
    x0 = b0 * f.i0 - f.l10 * x1 - f.l20 * x2;
}

__device__ __forceinline__ bool finite_pos(double t) { return t > 0.0 && t <= DBL_MAX; }

// ---------------------------------------------------------------------------
// Kernel 1 core: solve one trajectory on one lane.
//   sW: LDS [ (M+1)*3 ][LDS_STRIDE] waypoints (row q = knot*3 + axis)
//   sT: LDS [ M ][LDS_STRIDE] segment times
//   ed: 18 end derivatives of this trajectory (HAS_ED) = [start|final][v,a,j][x,y,z]
//   out: 24*M coefficients of this trajectory ([seg][axis][8])
template <int M, bool HAS_ED>
__device__ __forceinline__ int32_t reduced_solve_lane(const double* __restrict__ sW,
                                                      const double* __restrict__ sT, int lane,
                                                      const double* __restrict__ ed,
                                                      double* __restrict__ out) {
    constexpr int NG = (M > 2) ? (M - 2) : 1;  // G_k, k = 1..M-2
    constexpr int NZ = (M > 1) ? (M - 1) : 1;  // z_k / x_k, k = 1..M-1
    auto w = [&](int knot, int a) -> double { return sW[(knot * 3 + a) * LDS_STRIDE + lane]; };

    bool valid = true;
    double r[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const double t = sT[i * LDS_STRIDE + lane];
        valid = valid && finite_pos(t);
        r[i] = 1.0 / t;
    }
    double wsum = 0.0;
#pragma unroll
    for (int q = 0; q < (M + 1) * 3; ++q) wsum += sW[q * LDS_STRIDE + lane] * 0.0;
    valid = valid && (wsum == 0.0);

    double u0[3][3], uM[3][3];  // [derivative][axis]
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            u0[d][a] = HAS_ED ? ed[d * 3 + a] : 0.0;
            uM[d][a] = HAS_ED ? ed[9 + d * 3 + a] : 0.0;
        }
    if (HAS_ED) {
        double es = 0.0;
#pragma unroll
        for (int q = 0; q < 18; ++q) es += ed[q] * 0.0;
        valid = valid && (es == 0.0);
    }

    // ---- forward block elimination over interior knots k = 1..M-1 ----
    double G[NG][3][3];  // G_k = D_k^{-1} C_k
    double Z[NZ][3][3];  // z_k = D_k^{-1} y_k, later x_k;  [derivative][axis]
    bool spd = true;
#pragma unroll
    for (int k = 1; k < M; ++k) {
        double pp[8], pn[8];
        rpowers(r[k - 1], pp);
        rpowers(r[k], pn);
        double D[3][3];
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) D[d][e] = KEE[d][e] * pp[5 - d - e] + KSS[d][e] * pn[5 - d - e];
        double y[3][3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double wk = w(k, a);
            const double dp = wk - w(k - 1, a);
            const double dn = w(k + 1, a) - wk;
#pragma unroll
            for (int d = 0; d < 3; ++d) y[d][a] = -KEP[d] * pp[6 - d] * dp - KSP[d] * pn[6 - d] * dn;
        }
        if (HAS_ED && k == 1) {  // known start derivatives couple through C_0^T
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    const double c = KSE[e][d] * pp[5 - d - e];
#pragma unroll
                    for (int a = 0; a < 3; ++a) y[d][a] -= c * u0[e][a];
                }
        }
        if (HAS_ED && k == M - 1) {  // known final derivatives couple through C_{M-1}
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    const double c = KSE[d][e] * pn[5 - d - e];
#pragma unroll
                    for (int a = 0; a < 3; ++a) y[d][a] -= c * uM[e][a];
                }
        }
        if (k >= 2) {  // Schur update with the previous knot: D -= C^T G, y -= C^T z
            double Cp[3][3];
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
                for (int e = 0; e < 3; ++e) Cp[q][e] = KSE[q][e] * pp[5 - q - e];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    double s = D[d][e];
#pragma unroll
                    for (int q = 0; q < 3; ++q) s -= Cp[q][d] * G[k - 2][q][e];
                    D[d][e] = s;
                }
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double s = y[d][a];
#pragma unroll
                    for (int q = 0; q < 3; ++q) s -= Cp[q][d] * Z[k - 2][q][a];
                    y[d][a] = s;
                }
            }
        }
        const Ldl3 f = ldl3(D, spd);
        if (k <= M - 2) {
#pragma unroll
            for (int e = 0; e < 3; ++e)
                ldl3_solve(f, KSE[0][e] * pn[5 - e], KSE[1][e] * pn[4 - e], KSE[2][e] * pn[3 - e],
                           G[k - 1][0][e], G[k - 1][1][e], G[k - 1][2][e]);
        }
#pragma unroll
        for (int a = 0; a < 3; ++a)
            ldl3_solve(f, y[0][a], y[1][a], y[2][a], Z[k - 1][0][a], Z[k - 1][1][a], Z[k - 1][2][a]);
    }

    // ---- back substitution: x_k = z_k - G_k x_{k+1} ----
#pragma unroll
    for (int k = M - 2; k >= 1; --k)
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double s = Z[k - 1][d][a];
#pragma unroll
                for (int e = 0; e < 3; ++e) s -= G[k - 1][d][e] * Z[k][e][a];
                Z[k - 1][d][a] = s;
            }

    // ---- septic-Hermite coefficients per segment (a4 layout [seg][axis][8]) ----
    double fin = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const double T = sT[i * LDS_STRIDE + lane];
        const double T2 = T * T, T3 = T2 * T;
        double rp[8];
        rpowers(r[i], rp);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double v0 = (i == 0) ? u0[0][a] : Z[(i > 0 ? i : 1) - 1][0][a];
            const double a0 = (i == 0) ? u0[1][a] : Z[(i > 0 ? i : 1) - 1][1][a];
            const double j0 = (i == 0) ? u0[2][a] : Z[(i > 0 ? i : 1) - 1][2][a];
            const double v1 = (i == M - 1) ? uM[0][a] : Z[(i < M - 1 ? i : 0)][0][a];
            const double a1 = (i == M - 1) ? uM[1][a] : Z[(i < M - 1 ? i : 0)][1][a];
            const double j1 = (i == M - 1) ? uM[2][a] : Z[(i < M - 1 ? i : 0)][2][a];
            const double w0 = w(i, a);
            const double dw = w(i + 1, a) - w0;
            const double h1 = T * v0, h2 = T2 * a0, h3 = T3 * j0;
            const double h5 = T * v1, h6 = T2 * a1, h7 = T3 * j1;
            const double d4 = 35.0 * dw - 20.0 * h1 - 5.0 * h2 - (2.0 / 3.0) * h3 - 15.0 * h5 +
                              2.5 * h6 - (1.0 / 6.0) * h7;
            const double d5 = -84.0 * dw + 45.0 * h1 + 10.0 * h2 + h3 + 39.0 * h5 - 7.0 * h6 + 0.5 * h7;
            const double d6 = 70.0 * dw - 36.0 * h1 - 7.5 * h2 - (2.0 / 3.0) * h3 - 34.0 * h5 +
                              6.5 * h6 - 0.5 * h7;
            const double d7 = -20.0 * dw + 10.0 * h1 + 2.0 * h2 + (1.0 / 6.0) * h3 + 10.0 * h5 -
                              2.0 * h6 + (1.0 / 6.0) * h7;
            double c[8] = {w0, v0, 0.5 * a0, j0 * (1.0 / 6.0), d4 * rp[4], d5 * rp[5], d6 * rp[6], d7 * rp[7]};
            fin += (c[4] + c[5]) + (c[6] + c[7]) + (c[1] + c[2] + c[3]);
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = valid ? c[j] : 0.0;
            double2* o = reinterpret_cast<double2*>(out + (i * 3 + a) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = make_double2(c[2 * j], c[2 * j + 1]);
        }
    }
    if (!valid) return TGMS_ERR_INVALID_ARG;
    if (!spd) return TGMS_ERR_SINGULAR;
    if (!(fin * 0.0 == 0.0)) return TGMS_ERR_NONFINITE;
    return TGMS_OK;
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64) void k_reduced_uniform(int32_t B, const double* __restrict__ W,
                                                        const double* __restrict__ T,
                                                        const double* __restrict__ ED,
                                                        double* __restrict__ C,
                                                        int32_t* __restrict__ status) {
    constexpr int NW = (M + 1) * 3;
    __shared__ double sW[NW * LDS_STRIDE];
    __shared__ double sT[M * LDS_STRIDE];
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * W64;
    const int nb = (int)((B - b0) < W64 ? (B - b0) : W64);
    // coalesced wave-wide loads of the wave's contiguous input block, transposed into LDS
    const double* gW = W + b0 * NW;
    for (int e = lane; e < nb * NW; e += W64) {
        const int t = e / NW, q = e - t * NW;
        sW[q * LDS_STRIDE + t] = gW[e];
    }
    const double* gT = T + b0 * M;
    for (int e = lane; e < nb * M; e += W64) {
        const int t = e / M, q = e - t * M;
        sT[q * LDS_STRIDE + t] = gT[e];
    }
    __syncthreads();
    if (lane >= nb) return;
    const int64_t b = b0 + lane;
    const int32_t st = reduced_solve_lane<M, HAS_ED>(sW, sT, lane, HAS_ED ? ED + b * 18 : nullptr,
                                                     C + b * (24 * M));
    if (status) status[b] = st;
}

// Ragged batches: one launch per segment count M over the trajectories `perm`
// (host-grouped so every wavefront runs a single M).
template <int M, bool HAS_ED>
__global__ __launch_bounds__(64) void k_reduced_ragged(int32_t n, const int32_t* __restrict__ perm,
                                                       const int32_t* __restrict__ seg_offsets,
                                                       const double* __restrict__ W,
                                                       const double* __restrict__ T,
                                                       const double* __restrict__ ED,
                                                       double* __restrict__ C,
                                                       int32_t* __restrict__ status) {
    constexpr int NW = (M + 1) * 3;
    __shared__ double sW[NW * LDS_STRIDE];
    __shared__ double sT[M * LDS_STRIDE];
    const int lane = threadIdx.x;
    const int64_t idx = (int64_t)blockIdx.x * W64 + lane;
    const bool active = idx < n;
    int32_t b = 0;
    int64_t s0 = 0;
    if (active) {
        b = perm[idx];
        s0 = seg_offsets[b];
        const double* gW = W + (s0 + b) * 3;
#pragma unroll
        for (int q = 0; q < NW; ++q) sW[q * LDS_STRIDE + lane] = gW[q];
#pragma unroll
        for (int q = 0; q < M; ++q) sT[q * LDS_STRIDE + lane] = T[s0 + q];
    }
    __syncthreads();
    if (!active) return;
    const int32_t st = reduced_solve_lane<M, HAS_ED>(sW, sT, lane, HAS_ED ? ED + (int64_t)b * 18 : nullptr,
                                                     C + s0 * 24);
    if (status) status[b] = st;
}

// ---------------------------------------------------------------------------
// Kernel 2: dense KKT, one wavefront per trajectory.

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

// ---------------------------------------------------------------------------
// Kernel 3: sampler.
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

// ---------------------------------------------------------------------------
// dispatch tables (M = 1..TGMS_MAX_SEGMENTS)

template <int M>
hipError_t reduced_uniform_M(int32_t B, const double* W, const double* T, const double* ED,
                             double* C, int32_t* status, hipStream_t stream) {
    const unsigned grid = (unsigned)((B + W64 - 1) / W64);
    if (grid == 0) return hipSuccess;
    if (ED)
        hipLaunchKernelGGL((k_reduced_uniform<M, true>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status);
    else
        hipLaunchKernelGGL((k_reduced_uniform<M, false>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status);
    return hipGetLastError();
}

template <int M>
hipError_t reduced_ragged_M(int32_t n, const int32_t* perm, const int32_t* so, const double* W,
                            const double* T, const double* ED, double* C, int32_t* status,
                            hipStream_t stream) {
    const unsigned grid = (unsigned)((n + W64 - 1) / W64);
    if (grid == 0) return hipSuccess;
    if (ED)
        hipLaunchKernelGGL((k_reduced_ragged<M, true>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C, status);
    else
        hipLaunchKernelGGL((k_reduced_ragged<M, false>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C, status);
    return hipGetLastError();
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

#define TGMS_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

hipError_t launch_reduced_uniform(int M, int32_t B, const double* W, const double* T,
                                  const double* ED, double* C, int32_t* status,
                                  hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return reduced_uniform_M<m>(B, W, T, ED, C, status, stream);
        TGMS_CASES(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_reduced_ragged_group(int M, int32_t n, const int32_t* perm, const int32_t* so,
                                       const double* W, const double* T, const double* ED,
                                       double* C, int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return reduced_ragged_M<m>(n, perm, so, W, T, ED, C, status, stream);
        TGMS_CASES(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

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
