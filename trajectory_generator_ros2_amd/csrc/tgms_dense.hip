// tgms_dense.hip — TGMS_METHOD_DENSE_KKT: the survey's literal a1-a3 on gfx950 as a
// dense solve (the cross-check of the reduced and band formulations).
//
// [[2Q, A^T],[A, 0]] (snap Hessian Q, a2: endpoint/continuity rows A
// with right-hand side b; N = 14M+2) with its 3 right-hand sides, eliminated by
// Gauss-Jordan with partial pivoting, the matrix resident in the registers of a
// 256-thread workgroup (k_dense_gj below).  Round 1's kernel kept the matrix in LDS
// (161 KB at M = 10: one trajectory per CU) and was bound by dependent LDS round trips
// (122 ms per 65,536); this one holds two trajectories per CU in registers (45 ms).
#include <type_traits>

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

// ---------------------------------------------------------------------------
// Two columns per barrier pair (round 4).  The same Gauss-Jordan
// elimination, bit for bit (the same pivots, the same fma sequence per entry), with the
// columns taken in pairs (k, k+1) (N = 14M+2 is even):
//   lookahead (one wave: the one owning column groups k % 16 and k % 16 + 1, which are
//   two 16-lane rows of it since k is even): the pivot p_k of column k and its multipliers
//   l_k; column k+1 after step k, c' = fma(-l_k, a[p_k][k+1], c) (a[p_k][k+1] read from the
//   owner lane by readlane); the pivot p_{k+1} of c' over the rows still active without
//   p_k, and the multipliers l_{k+1} = c' / c'[p_{k+1}] (0 for p_{k+1});      barrier A
//   pivot rows: row p_k's owners publish u_k = row p_k; row p_{k+1}'s owners publish
//   u'_{k+1} = fma(-l_k[p_{k+1}], u_k, row p_{k+1}) (u_k read back from LDS inside the
//   wave: the same column group is one 16-lane row of one wave);            barrier B
//   rank-2 update: a = fma(-l_{k+1}, u'_{k+1}, fma(-l_k, u_k, a)), then the next pair's
//   lookahead.
// Two workgroup barriers per two columns instead of per column; the multipliers and the
// pivot record are double-buffered (the next pair's lookahead writes them while slower
// waves still update with the current ones).
#ifndef TGMS_DENSE_PANEL
#define TGMS_DENSE_PANEL 0  // 1 after GPU validation (scripts/dense_ab.py)
#endif

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(GJ_T, 2) void k_dense_gj2(int32_t n_traj, const int32_t* __restrict__ ids,
                                                       const int32_t* __restrict__ seg_offsets,
                                                       const double* __restrict__ W, const double* __restrict__ T,
                                                       const double* __restrict__ ED, double* __restrict__ C,
                                                       int32_t* __restrict__ status) {
    using S = GJShape<M>;
    constexpr int n = S::n, N = S::N, RI = S::RI, CJ = S::CJ;
    static_assert(N % 2 == 0, "columns are eliminated in pairs");
    static_assert(GJ_G == 16 && GJ_C == 16, "a column group is one DPP row; four per wave");
    __shared__ double s_pw[M][8];
    __shared__ double s_w[(M + 1) * 3];
    __shared__ double s_ed[18];
    constexpr int US = CJ, LS = (RI + 1) & ~1;
    __shared__ double s_u[2][GJ_C * US];          // u_k, u'_{k+1} (columns <= k+1 stale: never read again)
    __shared__ alignas(16) double s_l[2][2][GJ_G * LS];  // [pair parity][column of the pair][multipliers]
    __shared__ double s_pd[2][2];                 // [parity][column]: signed pivot
    __shared__ int s_pr[2][2];                    // [parity][column]: pivot row
    __shared__ double s_ipiv[N];
    __shared__ int s_rowpos[N];  // elimination position of each row (N: never pivoted)
    __shared__ int s_bad;

    const int tid = threadIdx.x;
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

    double a[RI][CJ];
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
        for (int j = 0; j < CJ; ++j) a[i][j] = gj_entry<M, HAS_ED>(tr + GJ_G * i, tc + GJ_C * j, s_pw, s_w, s_ed);
    unsigned act = 0;  // rows not yet pivoted (bit i: row tr + 16 i)
#pragma unroll
    for (int i = 0; i < RI; ++i) act |= (tr + GJ_G * i < N) ? (1u << i) : 0u;
    for (int r = tid; r < N; r += GJ_T) s_rowpos[r] = N;  // (ordered by the first barrier below)

    // the largest |v_i| over the rows in `msk`, ties to the lowest row, reduced over the
    // 16-lane row by DPP (every lane ends with the row's result)
    auto pick = [&](auto get, unsigned msk, double& sv, int& brow) {
        sv = 0.0;
        brow = N;
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const double vi = get(i);
            const bool take = ((msk >> i) & 1u) && fabs(vi) > fabs(sv);
            sv = take ? vi : sv;
            brow = take ? tr + GJ_G * i : brow;
        }
        auto merge = [&](double osv, int orow) {
            const bool take = (fabs(osv) > fabs(sv)) || (fabs(osv) == fabs(sv) && orow < brow);
            sv = take ? osv : sv;
            brow = take ? orow : brow;
        };
        merge(dpp_f64<0xB1>(sv), __builtin_amdgcn_mov_dpp(brow, 0xB1, 0xF, 0xF, false));
        merge(dpp_f64<0x4E>(sv), __builtin_amdgcn_mov_dpp(brow, 0x4E, 0xF, 0xF, false));
        merge(dpp_f64<0x141>(sv), __builtin_amdgcn_mov_dpp(brow, 0x141, 0xF, 0xF, false));
        merge(dpp_f64<0x140>(sv), __builtin_amdgcn_mov_dpp(brow, 0x140, 0xF, 0xF, false));
    };

    // lookahead of pair (k, k+1), k even: run by the wave holding column groups kg, kg+1.
    // Both columns sit in register column j0 = k / 16 of their owners; the body is
    // instantiated per j0 (a uniform branch) so it works on a[i][j0] in place.
    auto lookahead_j = [&](auto J, int k, int par) {
        constexpr int j0 = decltype(J)::value;
        const int kg = k % GJ_C;
        const bool own0 = tc == kg, own1 = tc == kg + 1;
        double sv0 = 0.0;
        int br0 = N;
        if (own0) pick([&](int i) { return a[i][j0]; }, act, sv0, br0);
        const int l0 = GJ_G * (kg & 3);
        const double ps0 = readlane_f64(sv0, l0);
        const int p0 = __builtin_amdgcn_readlane(br0, l0);
        const double ip0 = fast_rcp(ps0);
        const int pg0 = p0 % GJ_G, pi0 = p0 / GJ_G;
        if (own0) {
#pragma unroll
            for (int i = 0; i < RI; ++i) s_l[par][0][tr * LS + i] = (tr + GJ_G * i == p0) ? 0.0 : a[i][j0] * ip0;
            if (tr == 0) {
                s_pd[par][0] = ps0;
                s_pr[par][0] = p0;
            }
        }
        // a[p_k][k+1]: lane (row kg+1, tr = pg0), register (pi0, j0)
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < RI; ++i) v = (i == pi0) ? a[i][j0] : v;
        const double uk1 = readlane_f64(v, GJ_G * ((kg + 1) & 3) + pg0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // l_k written (this wave's own LDS order)
        __builtin_amdgcn_wave_barrier();
        if (own1) {
            // column k+1 after step k, in place: the column is dead once the pair is done
            // (the rank-2 update's second touch of it, and u'_{k+1}[k+1], are never read)
#pragma unroll
            for (int i = 0; i < RI; ++i) a[i][j0] = __builtin_fma(-s_l[par][0][tr * LS + i], uk1, a[i][j0]);
            const unsigned msk = act & ~((tr == pg0) ? (1u << pi0) : 0u);
            double sv1;
            int br1;
            pick([&](int i) { return a[i][j0]; }, msk, sv1, br1);
            const double ip1 = fast_rcp(sv1);
#pragma unroll
            for (int i = 0; i < RI; ++i) s_l[par][1][tr * LS + i] = (tr + GJ_G * i == br1) ? 0.0 : a[i][j0] * ip1;
            if (tr == 0) {
                s_pd[par][1] = sv1;
                s_pr[par][1] = br1;
            }
        }
    };
    auto lookahead = [&](int k, int par) {
        if ((tc >> 2) != ((k % GJ_C) >> 2)) return;  // wave-uniform: only the owner wave
        const int j0 = k / GJ_C;
#define TGMS_LA(jj) \
    if constexpr (jj < CJ) if (j0 == jj) lookahead_j(std::integral_constant<int, jj>{}, k, par);
        TGMS_LA(0) TGMS_LA(1) TGMS_LA(2) TGMS_LA(3) TGMS_LA(4) TGMS_LA(5) TGMS_LA(6) TGMS_LA(7) TGMS_LA(8)
        TGMS_LA(9) TGMS_LA(10) TGMS_LA(11) TGMS_LA(12) TGMS_LA(13) TGMS_LA(14) TGMS_LA(15)
#undef TGMS_LA
    };

    lookahead(0, 0);
    __syncthreads();

    bool singular = false;
    for (int k = 0; k < N; k += 2) {
        const int par = (k >> 1) & 1;
        // ---- the pair's pivots (found by the lookahead) ----
        const double ps0 = s_pd[par][0], ps1 = s_pd[par][1];
        const int p0 = __builtin_amdgcn_readfirstlane(s_pr[par][0]);
        const int p1 = __builtin_amdgcn_readfirstlane(s_pr[par][1]);
        if (!(fabs(ps0) > 0.0) || !(fabs(ps1) > 0.0)) {  // identical in every thread
            singular = true;
            break;
        }
        if (tid == 0) {
            s_ipiv[k] = fast_rcp(ps0);
            s_ipiv[k + 1] = fast_rcp(ps1);
            s_rowpos[p0] = k;
            s_rowpos[p1] = k + 1;
        }
        const int pg0 = p0 % GJ_G, pi0 = p0 / GJ_G, pg1 = p1 % GJ_G, pi1 = p1 / GJ_G;
        // ---- pivot rows: u_k, then u'_{k+1} from it (the same column group: one wave) ----
        if (tr == pg0) {
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (i == pi0) {
#pragma unroll
                    for (int j = 0; j < CJ; ++j) s_u[0][tc * US + j] = a[i][j];
                }
            }
            act &= ~(1u << pi0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (tr == pg1) {
            const double lp = s_l[par][0][pg1 * LS + pi1];
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (i == pi1) {
#pragma unroll
                    for (int j = 0; j < CJ; ++j) s_u[1][tc * US + j] = __builtin_fma(-lp, s_u[0][tc * US + j], a[i][j]);
                }
            }
            act &= ~(1u << pi1);
        }
        __syncthreads();
        // ---- rank-2 update (column blocks left of k are done), in two halves of the
        // thread's rows so only half of the multipliers are live at a time ----
        constexpr int RH = (RI + 1) / 2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            double la[RH], lb[RH];
#pragma unroll
            for (int q = 0; q < RH; ++q) {
                const int i = h * RH + q;
                if (i < RI) {
                    la[q] = s_l[par][0][tr * LS + i];
                    lb[q] = s_l[par][1][tr * LS + i];
                }
            }
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                if (GJ_C * j + GJ_C - 1 > k) {  // uniform
                    const double u0 = s_u[0][tc * US + j], u1 = s_u[1][tc * US + j];
#pragma unroll
                    for (int q = 0; q < RH; ++q) {
                        const int i = h * RH + q;
                        if (i < RI) a[i][j] = __builtin_fma(-lb[q], u1, __builtin_fma(-la[q], u0, a[i][j]));
                    }
                }
            }
        }
        if (k + 2 < N) lookahead(k + 2, par ^ 1);
        __syncthreads();
    }

    // ---- x_k = b'_{p_k} / a_{p_k k} (as k_dense_gj) ----
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
                const int r = tr + GJ_G * i;
                const int k = r < N ? s_rowpos[r] : N;
                if (k < n && !singular) {
                    const double x = a[i][j] * s_ipiv[k];
                    fin += x;
                    C[s0 * 24 + ((k >> 3) * 3 + ax) * 8 + (k & 7)] = valid ? x : 0.0;
                }
            }
        }
    }
    if (!(fin * 0.0 == 0.0)) atomicOr(&s_bad, 2);
    __syncthreads();
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
#if TGMS_DENSE_PANEL
    if (ED)
        TGMS_LAUNCH((k_dense_gj2<M, true>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
    else
        TGMS_LAUNCH((k_dense_gj2<M, false>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
#else
    if (ED)
        TGMS_LAUNCH((k_dense_gj<M, true>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
    else
        TGMS_LAUNCH((k_dense_gj<M, false>), dim3(n_traj), dim3(GJ_T), 0, stream, n_traj, ids, so, W, T, ED, C, status);
#endif
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

