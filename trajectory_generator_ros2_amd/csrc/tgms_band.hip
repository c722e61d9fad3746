// tgms_band.hip — TGMS_METHOD_BAND_KKT: the survey's literal KKT,
// LU with partial pivoting, one half-wavefront per trajectory.
//
// The KKT [[2Q, A^T],[A, 0]] (N = 14M+2) is ordered segment-interleaved:
//   [start rows (4) | c_0 (8) | knot-1 rows (6) | c_1 (8) | ... | c_{M-1} (8) | end rows (4)]
// In that order every nonzero lies within 9 of the diagonal (kl = ku = 9), because a
// coefficient only meets the constraint rows of its own two knots.  LU with partial
// pivoting keeps L inside kl sub-diagonals and U inside kl+ku super-diagonals, so the
// elimination is EXACTLY dense GEPP on the reordered matrix with the structurally-zero
// entries skipped (the same pivots, the same nonzero updates; oracle_solve KKT_BAND is
// that dense GEPP, not a band routine).  Flops: ~2 N kl (kl+ku) ~ 50 kflop at M = 10
// against 2/3 N^3 = 1.9 MFLOP for the unordered dense LU (tgms_dense.hip).
//
// Mapping (gfx950): lanes 0..31 of a wavefront solve one trajectory, lanes 32..63 the
// next.  Within a half, lane l < 19 owns the window column c = l (mod 19), lanes 19..21
// the three right-hand sides (x, y, z share the matrix), so the active window (rows
// k..k+9 x columns k..k+18) lives in 10 registers per lane and the elimination of column
// k is 9 FMAs per lane.  The pivot column's lane picks the pivot, forms the 9
// multipliers and hands them to its half through one LDS slot (in-order within the
// wave: no barrier).  The entering row k+10 is assembled on the fly from the segment
// powers T_i^e and the 2Q blocks staged in LDS (a1/a2 never exist as a matrix).
// Each finished U row (19 entries + 3 eliminated right-hand sides, 176 B) goes to a
// per-wave scratch slab; back substitution streams the slab in reverse with loads
// issued four steps ahead, one lane per pending row, x_k broadcast through LDS.
#include <algorithm>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

constexpr int KL = 9;              // sub-diagonals (== super-diagonals) of the interleaved KKT
constexpr int WR = KL + 1;         // window rows
constexpr int WC = 2 * KL + 1;     // window columns == width of a U row (diagonal + kl+ku)
constexpr int UW = WC + 3;         // scratch row: U row + 3 eliminated right-hand sides
constexpr int HL = 32;             // lanes per trajectory
constexpr int PF = 4;              // back-substitution prefetch depth (steps)

// Position q of the interleaved order.  kind: 0 start row (idx = derivative k),
// 1 coefficient (seg, idx = power j), 2 interior-knot row after segment seg
// (idx = type: 0 p(T)=w, 1 p(0)=w, 2..5 continuity of derivative idx-1), 3 end row (k),
// 4 outside the matrix.
struct Pos {
    int kind, seg, idx;
};

template <int M>
__device__ __forceinline__ Pos decode(int q) {
    constexpr int N = 14 * M + 2;
    if (q < 4) return {0, 0, q};
    if (q >= N) return {4, 0, 0};
    const int q4 = q - 4, i = q4 / 14, o = q4 - 14 * i;
    if (o < 8) return {1, i, o};
    if (i == M - 1) return {3, M - 1, o - 8};
    return {2, i, o - 8};
}

// j!/(j-k)! for 0 <= k <= 4 (0 when k > j)
__device__ __forceinline__ double dfac(int j, int k) {
    int f = 1;
    if (k > 0) f *= j;
    if (k > 1) f *= (j - 1);
    if (k > 2) f *= (j - 2);
    if (k > 3) f *= (j - 3);
    return (k > j) ? 0.0 : (double)f;
}

// A[lam][coefficient (i, j)], tp = this trajectory's T_i^e table
template <int M>
__device__ __forceinline__ double a_entry(Pos lam, int i, int j, const double* tp) {
    if (lam.kind == 0) return (i == 0 && j == lam.idx) ? dfac(j, j) : 0.0;
    if (lam.kind == 3)
        return (i == M - 1 && j >= lam.idx) ? dfac(j, lam.idx) * tp[i * 8 + j - lam.idx] : 0.0;
    if (lam.kind != 2) return 0.0;
    const int s = lam.seg, t = lam.idx, k = t - 1;
    if (i == s) {
        if (t == 0) return tp[s * 8 + j];
        if (t == 1 || j < k) return 0.0;
        return dfac(j, k) * tp[s * 8 + j - k];
    }
    if (i == s + 1) {
        if (t == 0) return 0.0;
        if (t == 1) return (j == 0) ? 1.0 : 0.0;
        return (j == k) ? -dfac(k, k) : 0.0;
    }
    return 0.0;
}

// KKT entry K[r][c] of the interleaved order
template <int M>
__device__ __forceinline__ double kkt_entry(Pos r, Pos c, const double* tp, const double* q2) {
    if (r.kind == 4 || c.kind == 4) return 0.0;
    if (r.kind == 1 && c.kind == 1)
        return (r.seg == c.seg && r.idx >= 4 && c.idx >= 4) ? q2[r.seg * 16 + (r.idx - 4) * 4 + (c.idx - 4)] : 0.0;
    if (r.kind == 1) return a_entry<M>(c, r.seg, r.idx, tp);
    if (c.kind == 1) return a_entry<M>(r, c.seg, c.idx, tp);
    return 0.0;
}

// right-hand side of row r, axis a (0 on the stationarity rows)
template <int M, bool HAS_ED>
__device__ __forceinline__ double kkt_rhs(Pos r, int a, const double* w, const double* ed) {
    if (r.kind == 0) return r.idx == 0 ? w[a] : (HAS_ED ? ed[(r.idx - 1) * 3 + a] : 0.0);
    if (r.kind == 3) return r.idx == 0 ? w[M * 3 + a] : (HAS_ED ? ed[9 + (r.idx - 1) * 3 + a] : 0.0);
    if (r.kind == 2) return r.idx <= 1 ? w[(r.seg + 1) * 3 + a] : 0.0;
    return 0.0;
}

template <int M, bool HAS_ED>
__device__ __forceinline__ double window_entry(int hl, int row, Pos pc, const double* tp, const double* q2,
                                               const double* w, const double* ed) {
    const Pos pr = decode<M>(row);
    if (hl < WC) return kkt_entry<M>(pr, pc, tp, q2);
    if (hl < UW) return kkt_rhs<M, HAS_ED>(pr, hl - WC, w, ed);
    return 0.0;
}

// One elimination step k; logical window row i lives in a[(R0 + i) % WR].
template <int M, bool HAS_ED, int R0>
__device__ __forceinline__ void elim_step(int k, int Lk, int hl, double (&a)[WR], int& col, Pos& pc, bool& sing,
                                          double* slot, double* U, const double* tp, const double* q2,
                                          const double* w, const double* ed) {
#define A_(i) a[(R0 + (i)) % WR]
    // pivot search (meaningful on the pivot column's lane Lk)
    double best = fabs(A_(0));
    int p = 0;
#pragma unroll
    for (int i = 1; i < WR; ++i) {
        const double v = fabs(A_(i));
        if (v > best) {
            best = v;
            p = i;
        }
    }
    if (hl == Lk) {
        double piv = A_(0);
#pragma unroll
        for (int i = 1; i < WR; ++i) piv = (p == i) ? A_(i) : piv;
        sing = sing || !(best > 0.0);
        const double rp = 1.0 / piv;
        slot[0] = (double)p;
#pragma unroll
        for (int i = 1; i < WR; ++i) slot[i] = ((p == i) ? A_(0) : A_(i)) * rp;
    }
    __builtin_amdgcn_wave_barrier();
    const int P = (int)slot[0];
    double l[WR];
#pragma unroll
    for (int i = 1; i < WR; ++i) l[i] = slot[i];
    // row interchange 0 <-> P, then the rank-1 update of the window
    const double v0 = A_(0);
    double n0 = v0;
#pragma unroll
    for (int i = 1; i < WR; ++i) {
        const bool s = (P == i);
        n0 = s ? A_(i) : n0;
        A_(i) = s ? v0 : A_(i);
    }
#pragma unroll
    for (int i = 1; i < WR; ++i) A_(i) = fma(-l[i], n0, A_(i));
    // U row k: lane column c -> offset c - k; right-hand sides at WC..WC+2
    if (hl < WC)
        U[k * UW + (hl >= Lk ? hl - Lk : hl - Lk + WC)] = n0;
    else if (hl < UW)
        U[k * UW + hl] = n0;
    __builtin_amdgcn_wave_barrier();  // slot is rewritten by the next step
    // slide: the pivot column leaves, column k+19 enters (zero in rows k+1..k+9);
    // logical row 0's register becomes row k+10
    if (hl == Lk) {
        col += WC;
        pc = decode<M>(col);
#pragma unroll
        for (int i = 1; i < WR; ++i) A_(i) = 0.0;
    }
    A_(0) = window_entry<M, HAS_ED>(hl, k + WR, pc, tp, q2, w, ed);
#undef A_
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(W64) void k_band_kkt(int32_t n_traj, const int32_t* __restrict__ ids,
                                                  const int32_t* __restrict__ seg_offsets,
                                                  const double* __restrict__ W, const double* __restrict__ T,
                                                  const double* __restrict__ ED, double* __restrict__ C,
                                                  int32_t* __restrict__ status, double* __restrict__ scratch) {
    constexpr int N = 14 * M + 2;
    __shared__ double s_tp[2][M * 8];       // T_i^e, e = 0..7
    __shared__ double s_q2[2][M * 16];      // 2 Q_i, rows/cols 4..7 (a1)
    __shared__ double s_w[2][(M + 1) * 3];  // waypoints
    __shared__ double s_ed[2][18];          // end derivatives (HAS_ED)
    __shared__ double s_slot[2][WR];        // pivot index + multipliers of the current step
    __shared__ double s_x[2][4];            // back substitution: x_k broadcast

    const int lane = threadIdx.x, h = lane >> 5, hl = lane & (HL - 1);
    double* U = scratch + ((size_t)blockIdx.x * 2 + h) * (size_t)N * UW;
    double* tp = s_tp[h];
    double* q2 = s_q2[h];
    double* w = s_w[h];
    double* ed = s_ed[h];
    double* slot = s_slot[h];
    const int npairs = (n_traj + 1) >> 1;

    for (int pr = blockIdx.x; pr < npairs; pr += gridDim.x) {
        const int bi = 2 * pr + h;
        const bool live = bi < n_traj;
        const int32_t b = ids ? ids[live ? bi : 2 * pr] : (live ? bi : 2 * pr);
        const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;
        const double* gw = W + (s0 + b) * 3;
        const double* gt = T + s0;

        // ---- stage inputs, validate (T > 0 finite; W, ED finite)
        bool ok = true;
        for (int q = hl; q < (M + 1) * 3; q += HL) {
            const double v = gw[q];
            w[q] = v;
            ok = ok && (v * 0.0 == 0.0);
        }
        if (HAS_ED && hl < 18) {
            const double v = ED[(int64_t)b * 18 + hl];
            ed[hl] = v;
            ok = ok && (v * 0.0 == 0.0);
        }
        if (hl < M) {
            const double t = gt[hl];
            ok = ok && finite_pos(t);
            double p = 1.0;
            tp[hl * 8] = 1.0;
#pragma unroll
            for (int e = 1; e < 8; ++e) {
                p *= t;
                tp[hl * 8 + e] = p;
            }
        }
        const unsigned long long badm = __ballot(!ok);
        const bool valid = ((h ? (badm >> 32) : badm) & 0xffffffffull) == 0;
        __builtin_amdgcn_wave_barrier();
        for (int q = hl; q < M * 16; q += HL) {
            const int i = q >> 4, j = 4 + ((q >> 2) & 3), kk = 4 + (q & 3), ex = j + kk - 7;
            q2[q] = 2.0 * (dfac(j, 4) * dfac(kk, 4) * tp[i * 8 + ex] / (double)ex);
        }
        __builtin_amdgcn_wave_barrier();

        // ---- forward elimination (a3): window rows 0..9, columns hl
        int col = hl;
        Pos pc = decode<M>(hl < WC ? col : N);
        double a[WR];
#pragma unroll
        for (int i = 0; i < WR; ++i) a[i] = window_entry<M, HAS_ED>(hl, i, pc, tp, q2, w, ed);
        bool sing = false;
        int Lk = 0;
        for (int k0 = 0; k0 < N; k0 += WR) {
#define STEP(R)                                                                                         \
    if (k0 + R < N) {                                                                                   \
        elim_step<M, HAS_ED, R>(k0 + R, Lk, hl, a, col, pc, sing, slot, U, tp, q2, w, ed);              \
        Lk = (Lk == WC - 1) ? 0 : Lk + 1;                                                               \
    }
            STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7) STEP(8) STEP(9)
#undef STEP
        }
        const unsigned long long singm = __ballot(sing);
        const bool singular = ((h ? (singm >> 32) : singm) & 0xffffffffull) != 0;
        const bool emit = live && valid && !singular;

        // ---- back substitution, column oriented: lane hl < WC holds y for the pending
        // row r = hl (mod WC) in [k-18, k]; at step k that row needs U[r][k-r].
        // the U rows this wave stored are read back by other lanes: complete the stores and
        // drop stale L1 lines (the slab is reused by the next trajectory pair)
        __threadfence();
        double y0 = 0.0, y1 = 0.0, y2 = 0.0;
        const int kN = N - 1;
        int LkB = kN % WC;
        if (hl < WC) {
            const int d = (LkB >= hl) ? LkB - hl : LkB - hl + WC;  // row kN - d
            if (kN - d >= 0) {
                const double* ur = U + (size_t)(kN - d) * UW + WC;
                y0 = ur[0];
                y1 = ur[1];
                y2 = ur[2];
            }
        }
        // prefetch ring: ud = U[k-d][d] for this lane, yn = y of the row k-19 (Lk lane)
        double ud[PF], yn[PF][3];
        auto issue = [&](int k, int slotk, int lk) {
            ud[slotk] = 0.0;
            yn[slotk][0] = yn[slotk][1] = yn[slotk][2] = 0.0;
            if (k >= 0 && hl < WC) {
                const int d = (lk >= hl) ? lk - hl : lk - hl + WC;
                if (k - d >= 0) ud[slotk] = U[(size_t)(k - d) * UW + d];
                if (d == 0 && k - WC >= 0) {
                    const double* ur = U + (size_t)(k - WC) * UW + WC;
                    yn[slotk][0] = ur[0];
                    yn[slotk][1] = ur[1];
                    yn[slotk][2] = ur[2];
                }
            }
        };
        {
            int lk = LkB;
#pragma unroll
            for (int s = 0; s < PF; ++s) {
                issue(kN - s, s, lk);
                lk = (lk == 0) ? WC - 1 : lk - 1;
            }
        }
        double* xs = s_x[h];
        double* out = C + s0 * 24;
        double fin = 0.0;
        int lkPF = LkB;  // pivot lane of step k - PF, kept for issue()
#pragma unroll
        for (int s = 0; s < PF; ++s) lkPF = (lkPF == 0) ? WC - 1 : lkPF - 1;
        for (int k0 = kN; k0 >= 0; k0 -= PF) {
#pragma unroll
            for (int s = 0; s < PF; ++s) {
                const int k = k0 - s;
                if (k >= 0) {
                    const double u = ud[s];
                    if (hl == LkB) {
                        const double rd = 1.0 / u;  // u = U[k][0], the pivot
                        const double x0 = y0 * rd, x1 = y1 * rd, x2 = y2 * rd;
                        xs[0] = x0;
                        xs[1] = x1;
                        xs[2] = x2;
                        fin += (x0 + x1 + x2) * 0.0;
                        const Pos pk = decode<M>(k);
                        if (pk.kind == 1 && live) {
                            double* o = out + pk.seg * 24 + pk.idx;
                            o[0] = emit ? x0 : 0.0;
                            o[8] = emit ? x1 : 0.0;
                            o[16] = emit ? x2 : 0.0;
                        }
                        y0 = yn[s][0];
                        y1 = yn[s][1];
                        y2 = yn[s][2];
                    }
                    __builtin_amdgcn_wave_barrier();
                    const double x0 = xs[0], x1 = xs[1], x2 = xs[2];
                    if (hl < WC && hl != LkB) {
                        y0 = fma(-u, x0, y0);
                        y1 = fma(-u, x1, y1);
                        y2 = fma(-u, x2, y2);
                    }
                    __builtin_amdgcn_wave_barrier();
                    issue(k - PF, s, lkPF);
                    LkB = (LkB == 0) ? WC - 1 : LkB - 1;
                    lkPF = (lkPF == 0) ? WC - 1 : lkPF - 1;
                }
            }
        }
        // status; non-finite solution check over the written coefficients
        const unsigned long long nf = __ballot(!(fin == 0.0));
        const bool nonfinite = ((h ? (nf >> 32) : nf) & 0xffffffffull) != 0;
        if (live && hl == 0 && status) {
            int32_t st = TGMS_OK;
            if (!valid) st = TGMS_ERR_INVALID_ARG;
            else if (singular) st = TGMS_ERR_SINGULAR;
            else if (nonfinite) st = TGMS_ERR_NONFINITE;
            status[b] = st;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int M>
hipError_t band_M(int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W, const double* T,
                  const double* ED, double* C, int32_t* status, double* scratch, int32_t grid,
                  hipStream_t stream) {
    if (n_traj <= 0) return hipSuccess;
    const int32_t g = std::min<int32_t>(grid, (n_traj + 1) / 2);
    if (ED)
        hipLaunchKernelGGL((k_band_kkt<M, true>), dim3(g), dim3(W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                           status, scratch);
    else
        hipLaunchKernelGGL((k_band_kkt<M, false>), dim3(g), dim3(W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                           status, scratch);
    return hipGetLastError();
}

}  // namespace

size_t band_scratch_bytes(int M, int32_t grid) {
    return (size_t)grid * 2 * (size_t)(14 * M + 2) * UW * sizeof(double);
}

hipError_t launch_band_kkt(int M, int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W,
                           const double* T, const double* ED, double* C, int32_t* status, double* scratch,
                           int32_t grid, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return band_M<m>(n_traj, ids, so, W, T, ED, C, status, scratch, grid, stream);
        X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#undef X
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tgms
