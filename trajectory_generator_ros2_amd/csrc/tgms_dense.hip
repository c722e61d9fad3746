// tgms_dense.hip — TGMS_METHOD_DENSE_KKT: the survey's literal a1-a3 on gfx950 as a
// dense solve (the cross-check of the reduced and band formulations).
//
// [[2Q, A^T],[A, 0]] (snap Hessian Q, a2: endpoint/continuity rows A
// with right-hand side b; N = 14M+2) with its 3 right-hand sides, eliminated by
// Gauss-Jordan with partial pivoting, the matrix resident in the registers of a
// 256-thread workgroup (k_dense_gj below).  Round 1's kernel kept the matrix in LDS
// (161 KB at M = 10: one trajectory per CU) and was bound by dependent LDS round trips
// (122 ms per 65,536); this one holds two trajectories per CU in registers (45 ms).
#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

// ---------------------------------------------------------------------------
// Register-resident Gauss-Jordan elimination with partial pivoting (round 2).
//
// The KKT (N = 14M+2, plus the 3 right-hand sides as columns N..N+2) is spread over
// a 256-thread workgroup as a 16 x 16 thread grid: thread (tr, tc) = (tid % 16, tid / 16)
// owns rows r = tr + 16 i and columns c = tc + 16 j, at most 9 x 10 doubles at M = 10,
// in registers.  Two workgroups (trajectories) per CU.  Step k: the pivot of column k
// is the largest |a| over the rows not yet pivoted, found by the column's 16 owners (one
// 16-lane row of one wave, reduced by DPP) at the end of step k-1, so the other three
// waves skip that search; the pivot row's entries right of k and the column's multipliers go through
// LDS; every thread updates its block (column blocks left of k skipped: they are
// done).  Gauss-Jordan eliminates column k from EVERY other row, so after N steps the
// solution is x_k = b'_{p_k} / a_{p_k k}: no back substitution, which in registers
// would serialise on one row group per position.  Rows never move (the pivot order is
// recorded), so a step needs two workgroup barriers and no data movement.
constexpr int GJ_G = 16;                  // thread grid: row groups
constexpr int GJ_C = 16;                  // thread grid: column groups (32: 1.8x slower, 3 waves per SIMD)
constexpr int GJ_T = GJ_G * GJ_C;         // threads per trajectory

template <int M>
struct GJShape {
    static constexpr int n = 8 * M, m = 8 + 6 * (M - 1), N = n + m;
    static constexpr int RI = (N + GJ_G - 1) / GJ_G;      // rows per thread
    static constexpr int CJ = (N + 3 + GJ_C - 1) / GJ_C;  // columns per thread (incl. right-hand sides)
};

// Entry (r, c) of [[2Q, A^T, 0],[A, 0, b]] in the oracle's KKT_C4 order (coefficients
// [seg][power], then the constraint rows: 4 start, 4 end, 6 per interior knot);
// pw[seg][e] = T_seg^e, fc(j, k) = j!/(j-k)!.
template <int M, bool HAS_ED>
__device__ __forceinline__ double gj_entry(int r, int c, const double (*pw)[8], const double* w, const double* ed) {
    using S = GJShape<M>;
    constexpr int n = S::n, N = S::N;
    auto fc = [](int j, int k) -> double {  // j!/(j-k)!, 0 when k > j
        double f = 1.0;
        for (int q = 0; q < k; ++q) f *= (double)(j - q);
        return k > j ? 0.0 : f;
    };
    // constraint row q on coefficient col (A_eq)
    auto aeq = [&](int q, int col) -> double {
        const int seg = col >> 3, j = col & 7;
        if (q < 4) return col == q ? fc(q, q) : 0.0;
        if (q < 8) {
            const int k = q - 4;
            return (seg == M - 1 && j >= k) ? fc(j, k) * pw[M - 1][j - k] : 0.0;
        }
        const int i = 1 + (q - 8) / 6, qq = (q - 8) % 6;
        if (qq == 0) return seg == i - 1 ? pw[i - 1][j] : 0.0;
        if (qq == 1) return col == 8 * i ? 1.0 : 0.0;
        const int k = qq - 1;
        if (seg == i - 1 && j >= k) return fc(j, k) * pw[i - 1][j - k];
        return col == 8 * i + k ? -fc(k, k) : 0.0;
    };
    if (r >= N || c >= N + 3) return 0.0;
    if (c >= N) {  // right-hand side of axis c - N
        if (r < n) return 0.0;
        const int q = r - n, a = c - N;
        if (q < 4) return q == 0 ? w[a] : (HAS_ED ? ed[(q - 1) * 3 + a] : 0.0);
        if (q < 8) return q == 4 ? w[3 * M + a] : (HAS_ED ? ed[9 + (q - 5) * 3 + a] : 0.0);
        const int i = 1 + (q - 8) / 6, qq = (q - 8) % 6;
        return qq < 2 ? w[3 * i + a] : 0.0;
    }
    if (r < n && c < n) {  // 2 Q_i
        const int j = r & 7, k = c & 7;
        if ((r >> 3) != (c >> 3) || j < 4 || k < 4) return 0.0;
        const int ex = j + k - 7;
        return 2.0 * fc(j, 4) * fc(k, 4) * pw[r >> 3][ex] / (double)ex;
    }
    if (r < n) return aeq(c - n, r);
    if (c < n) return aeq(r - n, c);
    return 0.0;
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(GJ_T, 2) void k_dense_gj(int32_t n_traj, const int32_t* __restrict__ ids,
                                                      const int32_t* __restrict__ seg_offsets,
                                                      const double* __restrict__ W, const double* __restrict__ T,
                                                      const double* __restrict__ ED, double* __restrict__ C,
                                                      int32_t* __restrict__ status) {
    using S = GJShape<M>;
    constexpr int n = S::n, N = S::N, RI = S::RI, CJ = S::CJ;
    __shared__ double s_pw[M][8];
    __shared__ double s_w[(M + 1) * 3];
    __shared__ double s_ed[18];
    // pivot row and multipliers, one padded run per owner thread so the update reads
    // them 16 B at a time: s_u[tc * US + j] = column tc + 16 j, s_l[tr * LS + i] = row tr + 16 i
    constexpr int US = (CJ + 1) & ~1, LS = (RI + 1) & ~1;
    __shared__ alignas(16) double s_u[GJ_C * US];  // pivot row (columns <= k stale: never read again)
    __shared__ alignas(16) double s_l[GJ_G * LS];  // multipliers (0 for the pivot row)
    __shared__ double s_cs[2];              // pivot of the next column: a, row (double-buffered)
    __shared__ int s_ci[2];
    __shared__ double s_ipiv[N];
    __shared__ int s_bad;

    // column-major grid: a column group's 16 threads are one 16-lane row of one wave, so
    // the per-column work of a step (pivot candidates, multipliers) runs in one wave and
    // the other three skip it (exec-mask branch), and its reduction stays in the row (DPP)
    const int tid = threadIdx.x, lane = tid & 63;
    const int tr = tid % GJ_G, tc = tid / GJ_G;
    const int32_t bi = blockIdx.x;
    const int32_t b = ids ? ids[bi] : bi;
    const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;

    // ---- inputs (validated; an invalid trajectory is solved with unit times, zero
    // waypoints and end derivatives and comes out as zeros) ----
    if (tid == 0) s_bad = 0;
    __syncthreads();
    {
        int bad = 0;
        if (tid < M) {
            const double t = T[s0 + tid];
            bad |= !finite_pos(t);
            double p = 1.0;
            for (int e = 0; e < 8; ++e) {
                s_pw[tid][e] = p;
                p *= t;
            }
        }
        if (tid < (M + 1) * 3) {
            const double v = W[(s0 + b) * 3 + tid];
            bad |= !finite(v);
            s_w[tid] = v;
        }
        if (HAS_ED && tid < 18) {
            const double v = ED[(int64_t)b * 18 + tid];
            bad |= !finite(v);
            s_ed[tid] = v;
        }
        if (bad) atomicOr(&s_bad, 1);
    }
    __syncthreads();
    const bool valid = s_bad == 0;
    if (!valid) {
        if (tid < M)
            for (int e = 0; e < 8; ++e) s_pw[tid][e] = 1.0;
        if (tid < (M + 1) * 3) s_w[tid] = 0.0;
        if (tid < 18) s_ed[tid] = 0.0;
        __syncthreads();
    }

    // ---- the thread's block of the augmented KKT ----
    double a[RI][CJ];
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
        for (int j = 0; j < CJ; ++j) a[i][j] = gj_entry<M, HAS_ED>(tr + GJ_G * i, tc + GJ_C * j, s_pw, s_w, s_ed);
    unsigned act = 0;  // rows not yet pivoted (bit i: row tr + 16 i)
#pragma unroll
    for (int i = 0; i < RI; ++i) act |= (tr + GJ_G * i < N) ? (1u << i) : 0u;
    int pos[RI];  // elimination position of each row (set when it becomes a pivot)
#pragma unroll
    for (int i = 0; i < RI; ++i) pos[i] = N;

    // pivot of column c (its owners: tc == c % 16, one 16-lane row): the largest |a|
    // over the rows not yet pivoted, ties to the lowest row, reduced within the row by
    // DPP (quad swaps, then half-row and row mirrors: every lane ends with the row's
    // result) and left in slot `buf`
    auto candidates = [&](int c, int buf) {
        if (tc != c % GJ_C) return;
        // only the signed candidate travels; magnitudes are compared through abs
        // modifiers.  No active row with a nonzero entry leaves brow = N and sv = 0: the
        // pivot magnitude 0 then flags the matrix singular, as the first zero would.
        double sv = 0.0;
        int brow = N;
        const int jc = c / GJ_C;
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            if (j == jc) {
#pragma unroll
                for (int i = 0; i < RI; ++i) {
                    const bool take = ((act >> i) & 1u) && fabs(a[i][j]) > fabs(sv);
                    sv = take ? a[i][j] : sv;
                    brow = take ? tr + GJ_G * i : brow;
                }
            }
        }
        auto merge = [&](double osv, int orow) {
            const bool take = (fabs(osv) > fabs(sv)) || (fabs(osv) == fabs(sv) && orow < brow);
            sv = take ? osv : sv;
            brow = take ? orow : brow;
        };
        static_assert(GJ_G == 16, "a column group is one DPP row");
        merge(dpp_f64<0xB1>(sv), __builtin_amdgcn_mov_dpp(brow, 0xB1, 0xF, 0xF, false));
        merge(dpp_f64<0x4E>(sv), __builtin_amdgcn_mov_dpp(brow, 0x4E, 0xF, 0xF, false));
        merge(dpp_f64<0x141>(sv), __builtin_amdgcn_mov_dpp(brow, 0x141, 0xF, 0xF, false));
        merge(dpp_f64<0x140>(sv), __builtin_amdgcn_mov_dpp(brow, 0x140, 0xF, 0xF, false));
        if (tr == 0) {
            s_cs[buf] = sv;
            s_ci[buf] = brow;
        }
    };
    candidates(0, 0);
    __syncthreads();

    bool singular = false;
    for (int k = 0; k < N; ++k) {
        const int buf = k & 1;
        // ---- the pivot (found by column k's owners at the end of step k-1) ----
        const double ps = s_cs[buf], pv = fabs(ps);
        const int p = __builtin_amdgcn_readfirstlane(s_ci[buf]);
        if (!(pv > 0.0)) {  // identical in every thread
            singular = true;
            break;
        }
        const double ip = fast_rcp(ps);  // within an ulp of 1 / ps
        if (tid == 0) s_ipiv[k] = ip;
        const int pg = p % GJ_G, pi = p / GJ_G;  // the pivot row's owners and their local row
        const int jk = k / GJ_C, kg = k % GJ_C;  // column k's owners and their local column
        // the pivot row -> s_u (its owners: tr == pg).  Only its columns right of k matter:
        // the update then also changes columns <= k of block k / 16, which no later step
        // and no output reads (candidates look right of k, the solution at the
        // right-hand-side columns), so the row goes over whole.
        if (tr == pg) {
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (i == pi) {
#pragma unroll
                    for (int j = 0; j < CJ; ++j) s_u[tc * US + j] = a[i][j];
                    pos[i] = k;
                }
            }
            act &= ~(1u << pi);
        }
        // the multipliers of column k -> s_l (its owners: tc == kg); 0 for the pivot row
        if (tc == kg) {
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                if (j == jk) {
#pragma unroll
                    for (int i = 0; i < RI; ++i) {
                        const int r = tr + GJ_G * i;
                        s_l[tr * LS + i] = (r == p) ? 0.0 : a[i][j] * ip;
                    }
                }
            }
        }
        __syncthreads();
        // ---- update: a -= l u over the thread's block (column blocks left of k are done) ----
        double l[LS], u[US];
#pragma unroll
        for (int q = 0; q < LS / 2; ++q) {
            const double2 v = reinterpret_cast<const double2*>(s_l + tr * LS)[q];
            l[2 * q] = v.x;
            l[2 * q + 1] = v.y;
        }
#pragma unroll
        for (int q = 0; q < US / 2; ++q) {
            if (GJ_C * (2 * q + 1) + GJ_C - 1 > k) {  // uniform: a pair with a live column block
                const double2 v = reinterpret_cast<const double2*>(s_u + tc * US)[q];
                u[2 * q] = v.x;
                u[2 * q + 1] = v.y;
            }
        }
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            if (GJ_C * j + GJ_C - 1 > k) {  // uniform
#pragma unroll
                for (int i = 0; i < RI; ++i) a[i][j] = __builtin_fma(-l[i], u[j], a[i][j]);
            }
        }
        if (k + 1 < N) candidates(k + 1, buf ^ 1);
        __syncthreads();
    }

    // ---- x_k = b'_{p_k} / a_{p_k k}: the right-hand-side owners write the coefficients ----
    // A singular matrix stopped the elimination early (uniformly: every thread read the
    // same pivot), so rows never pivoted hold no position: the whole trajectory is
    // written as exact zeros instead, as the band and lane kernels do on failure.
    if (singular) {
        for (int e = tid; e < 24 * M; e += GJ_T) C[s0 * 24 + e] = 0.0;
    }
    double fin = 0.0;
#pragma unroll
    for (int j = 0; j < CJ; ++j) {
        const int c = tc + GJ_C * j;
        if (c >= N && c < N + 3) {
            const int ax = c - N;
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const int k = pos[i];
                if (k < n && !singular) {
                    const double x = singular ? 0.0 : a[i][j] * s_ipiv[k];
                    fin += x;
                    C[s0 * 24 + ((k >> 3) * 3 + ax) * 8 + (k & 7)] = valid ? x : 0.0;
                }
            }
        }
    }
    // status: any non-finite coefficient anywhere in the workgroup
    if (!(fin * 0.0 == 0.0)) atomicOr(&s_bad, 2);
    __syncthreads();
    // a non-finite solution is rewritten as exact zeros, like every other failure (the
    // barrier above waited for every thread's coefficient stores)
    if ((s_bad & 2) && valid && !singular)
        for (int e = tid; e < 24 * M; e += GJ_T) C[s0 * 24 + e] = 0.0;
    if (tid == 0 && status) {
        int32_t st = TGMS_OK;
        if (!valid) st = TGMS_ERR_INVALID_ARG;
        else if (singular) st = TGMS_ERR_SINGULAR;
        else if (s_bad & 2) st = TGMS_ERR_NONFINITE;
        status[b] = st;
    }
}

template <int M>
hipError_t dense_M(int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W,
                   const double* T, const double* ED, double* C, int32_t* status,
                   hipStream_t stream) {
    if (n_traj <= 0) return hipSuccess;
    if (ED)
        TGMS_LAUNCH((k_dense_gj<M, true>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
    else
        TGMS_LAUNCH((k_dense_gj<M, false>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
    return hipSuccess;
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

