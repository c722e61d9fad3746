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
// issued 16 steps ahead, one lane per pending row, x_k broadcast through LDS.
#include <algorithm>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

constexpr int KL = 9;              // sub-diagonals (== super-diagonals) of the interleaved KKT
constexpr int WR = KL + 1;         // window rows
constexpr int WC = 2 * KL + 1;     // window columns == width of a U row (diagonal + kl+ku)
constexpr int UW = WC + 3;         // scratch row: U row (19) + 3 eliminated right-hand sides (lanes
                                   // 0..21 of the half store, the rest are masked off)
constexpr int HL = 32;             // lanes per trajectory
#ifdef TGMS_BAND_STAMPS  // diagnostic build: s_memtime at phase boundaries, lane 0 of blocks < 64, first pair
constexpr int BST_BLOCKS = 64, BST_STEPS = 160, BST_PH = 8;
__device__ unsigned long long g_bstamps[BST_BLOCKS * BST_STEPS * BST_PH];
#define BSTAMP(k, i)                                                                                    \
    do {                                                                                                \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                     \
        if (blockIdx.x < BST_BLOCKS && threadIdx.x == 0 && (k) < BST_STEPS && first_pair)              \
            g_bstamps[(blockIdx.x * BST_STEPS + (k)) * BST_PH + (i)] = __builtin_amdgcn_s_memtime();     \
    } while (0)
#else
#define BSTAMP(k, i) \
    do {             \
    } while (0)
#endif
constexpr int PFB = 16;            // back-substitution prefetch depth (steps)

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

// Entries of the interleaved KKT, framed in the block of segment i: offsets 0..7 are
// c_i, 8..13 the rows of the knot after segment i (the end rows if i = M-1), -4..-1 the
// start rows (i = 0).  Every entry is coef * V_i[idx] with V_i = [1, T_i^0..T_i^7,
// 2Q_i (16)] staged per trajectory in LDS, and (coef, idx) depends only on the block
// variant (first / last segment), the row offset o and the diagonal offset d = c - r, so
// the pattern is a small table built once per wavefront: an entering row costs two LDS
// reads per lane instead of a divergent case analysis.  Same entries as oracle
// assemble_kkt_cont; tests/test_oracle.py pins the band.
constexpr int VAL = 25;               // V_i stride
constexpr int NOFF = 18;              // row offsets -4..13
constexpr int NDESC = 4 * NOFF * WC;  // variants x offsets x diagonals

__host__ __device__ constexpr int pack(int coef, int idx) { return coef * 32 + idx; }

__device__ int desc_entry(int vv, int o, int d) {
    const bool first = vv & 1, last = vv & 2;
    if (o < 0 && !first) return 0;
    const int oc = o + d;
    auto at = [](int j, int kk) { return j >= kk ? pack((int)dfac(j, kk), 1 + j - kk) : 0; };
    auto before = [](int j, int t) {  // knot row type t on the coefficients of the next segment
        if (t == 0) return 0;
        if (t == 1) return j == 0 ? pack(1, 0) : 0;
        return j == t - 1 ? pack(-(int)dfac(j, j), 0) : 0;
    };
    if (o < 0) {  // start row k: r_k(0) on segment 0 = k! at coefficient k
        const int k = o + 4;
        return oc == k ? pack((int)dfac(k, k), 0) : 0;
    }
    if (o < 8) {  // stationarity row of coefficient j of segment i
        const int j = o;
        if (oc >= 0 && oc < 8) return (j >= 4 && oc >= 4) ? pack(1, 9 + (j - 4) * 4 + (oc - 4)) : 0;
        if (oc >= 14) return 0;
        if (oc >= 8) {
            const int t = oc - 8;
            if (last) return at(j, t);
            return t == 1 ? 0 : at(j, t == 0 ? 0 : t - 1);
        }
        if (first) return (oc + 4 == j) ? pack((int)dfac(j, j), 0) : 0;
        if (oc < -6) return 0;
        return before(j, oc + 6);
    }
    const int t = o - 8;  // knot row after segment i (type t), or end row k = t
    if (oc >= 0 && oc < 8) {
        if (last) return at(oc, t);
        return t == 1 ? 0 : at(oc, t == 0 ? 0 : t - 1);
    }
    if (!last && oc >= 14 && oc < 22) return before(oc - 14, t);
    return 0;
}

// Row r (wave-uniform) at this lane's column c; lanes WC..WC+2 return the right-hand
// side b_r of axis hl - WC.  Branch-free in the lane: every lane reads its matrix entry
// and the right-hand-side candidate and selects (a divergent split costs more issue
// slots than the two extra LDS reads).
template <int M, bool HAS_ED>
__device__ __forceinline__ double row_entry(int hl, int r, int c, const int* desc, const double* val,
                                            const double* w, const double* ed) {
    constexpr int N = 14 * M + 2;
    if (r >= N) return 0.0;
    const int i = (r < 4) ? 0 : min((r - 4) / 14, M - 1);
    const int o = r - (4 + 14 * i);
    // right-hand-side source (uniform): waypoint row wr or end-derivative base eb
    int wr = -1, eb = -1;
    if (o < 0) {
        if (o == -4) wr = 0;
        else eb = (o + 3) * 3;
    } else if (o >= 8) {
        const int t = o - 8;
        if (i == M - 1) {
            if (t == 0) wr = M;
            else eb = 9 + (t - 1) * 3;
        } else if (t <= 1) {
            wr = i + 1;
        }
    }
    const int ax = min(max(hl - WC, 0), 2);
    const double rw = w[max(wr, 0) * 3 + ax];
    const double re = HAS_ED ? ed[max(eb, 0) + ax] : 0.0;
    const double rhs = (wr >= 0) ? rw : ((HAS_ED && eb >= 0) ? re : 0.0);
    const int d = c - r;
    const bool inb = (c < N) && d >= -KL && d <= KL;
    const int vv = (i == 0 ? 1 : 0) | (i == M - 1 ? 2 : 0);
    const int de = desc[(vv * NOFF + o + 4) * WC + min(max(d, -KL), KL) + KL];
    const double m = (double)(de >> 5) * val[i * VAL + (de & 31)];
    return (hl < WC) ? (inb ? m : 0.0) : ((hl < WC + 3) ? rhs : 0.0);
}

// U-slab load that misses L1 (an agent-scope relaxed atomic load: sc1)
__device__ __forceinline__ double ld_u(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 1/x: hardware reciprocal + two Newton steps (within an ulp; the pivots only scale)
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}

// One elimination step k; logical window row i lives in a[(R0 + i) % WR].
template <int M, bool HAS_ED, int R0>
__device__ __forceinline__ void elim_step(int k, int Lk, int hl, double (&a)[WR], int& col, bool& sing,
                                          double* slot, double* U, const int* desc, const double* val,
                                          const double* w, const double* ed, bool first_pair) {
#define A_(i) a[(R0 + (i)) % WR]
    BSTAMP(k, 0);
    // pivot search in every lane's own column; the pivot column's lane Lk decides
    double bv = A_(0);
    int p = 0;
#pragma unroll
    for (int i = 1; i < WR; ++i) {
        const bool g = fabs(A_(i)) > fabs(bv);
        bv = g ? A_(i) : bv;
        p = g ? i : p;
    }
    BSTAMP(k, 1);
    // the two halves' pivot rows (lanes Lk and Lk + 32) through the scalar unit
    const int p0 = __builtin_amdgcn_readlane(p, Lk), p1 = __builtin_amdgcn_readlane(p, Lk + HL);
    // row interchange 0 <-> P in every column (selects: a branch per pivot row makes the
    // register allocator copy the whole window at every join)
    const int P = (hl == threadIdx.x) ? p0 : p1;
    const double v0 = A_(0);
    double n0 = v0;
#pragma unroll
    for (int i = 1; i < WR; ++i) {
        const bool s = (P == i);
        n0 = s ? A_(i) : n0;
        A_(i) = s ? v0 : A_(i);
    }
    const double best = fabs(bv);
    BSTAMP(k, 2);
    // multipliers of the pivot column, handed to the half through LDS (in order within
    // the wavefront, so no barrier)
    // The pivot column leaves the window (its lane takes column k+19, zero in rows
    // k+1..k+9): its rows are cleared here and its update below multiplies by 0.
    double nu = n0;
    const double rp = recip(n0);
    if (hl == Lk) {
        sing = sing || !(best > 0.0);
#pragma unroll
        for (int i = 1; i < WR; ++i) {
            slot[i] = A_(i) * rp;
            A_(i) = 0.0;
        }
        nu = 0.0;
    }
    BSTAMP(k, 3);
    __builtin_amdgcn_wave_barrier();
    double l[WR];
#pragma unroll
    for (int i = 1; i < WR; ++i) l[i] = slot[i];
    // rank-1 update
#pragma unroll
    for (int i = 1; i < WR; ++i) A_(i) = fma(-l[i], nu, A_(i));
    BSTAMP(k, 4);
    // U row k: lane column c -> offset c - k (the diagonal stored inverted: back
    // substitution multiplies), right-hand sides at WC..WC+2, lanes beyond into padding
    if (hl < UW) U[k * UW + (hl < WC ? (hl >= Lk ? hl - Lk : hl - Lk + WC) : hl)] = (hl == Lk) ? rp : n0;
    __builtin_amdgcn_wave_barrier();  // slot is rewritten by the next step
    // slide: logical row 0's register becomes row k+10
    if (hl == Lk) col += WC;
    A_(0) = row_entry<M, HAS_ED>(hl, k + WR, col, desc, val, w, ed);
    BSTAMP(k, 6);
#undef A_
}

constexpr int TGMS_BAND_LB = 1;  // minimum wavefronts per SIMD the register allocation must allow

template <int M, bool HAS_ED>
__global__ __launch_bounds__(W64, TGMS_BAND_LB) void k_band_kkt(int32_t n_traj, const int32_t* __restrict__ ids,
                                                  const int32_t* __restrict__ seg_offsets,
                                                  const double* __restrict__ W, const double* __restrict__ T,
                                                  const double* __restrict__ ED, double* __restrict__ C,
                                                  int32_t* __restrict__ status, double* __restrict__ scratch) {
    constexpr int N = 14 * M + 2;
    __shared__ int s_desc[NDESC];           // entry pattern of the interleaved KKT
    __shared__ double s_val[2][M * VAL];    // V_i = [1, T_i^0..T_i^7, 2Q_i] per segment
    __shared__ double s_w[2][(M + 1) * 3];  // waypoints
    __shared__ double s_ed[2][18];          // end derivatives (HAS_ED)
    __shared__ double s_slot[2][WR];        // pivot index + multipliers of the current step
    __shared__ double s_x[2][4];            // back substitution: x_k broadcast

    const int lane = threadIdx.x, h = lane >> 5, hl = lane & (HL - 1);
    double* U = scratch + ((size_t)blockIdx.x * 2 + h) * (size_t)N * UW;
    double* val = s_val[h];
    for (int q = lane; q < NDESC; q += W64) {
        const int vv = q / (NOFF * WC), rem = q - vv * NOFF * WC, o = rem / WC - 4, d = rem % WC - KL;
        s_desc[q] = desc_entry(vv, o, d);
    }
    double* w = s_w[h];
    double* ed = s_ed[h];
    double* slot = s_slot[h];
    const int npairs = (n_traj + 1) >> 1;

    for (int pr = blockIdx.x; pr < npairs; pr += gridDim.x) {
        const bool first_pair = pr == (int)blockIdx.x;
        (void)first_pair;
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
            val[hl * VAL] = 1.0;
            val[hl * VAL + 1] = 1.0;
#pragma unroll
            for (int e = 1; e < 8; ++e) {
                p *= t;
                val[hl * VAL + 1 + e] = p;
            }
        }
        const unsigned long long badm = __ballot(!ok);
        const bool valid = ((h ? (badm >> 32) : badm) & 0xffffffffull) == 0;
        __builtin_amdgcn_wave_barrier();
        for (int q = hl; q < M * 16; q += HL) {
            const int i = q >> 4, j = 4 + ((q >> 2) & 3), kk = 4 + (q & 3), ex = j + kk - 7;
            val[i * VAL + 9 + (q & 15)] = 2.0 * (dfac(j, 4) * dfac(kk, 4) * val[i * VAL + 1 + ex] / (double)ex);
        }
        __builtin_amdgcn_wave_barrier();

        // ---- forward elimination (a3): window rows 0..9, columns hl
        int col = hl;
        double a[WR];
#pragma unroll
        for (int i = 0; i < WR; ++i) a[i] = row_entry<M, HAS_ED>(hl, i, col, s_desc, val, w, ed);
        bool sing = false;
        int Lk = 0;
        for (int k0 = 0; k0 < N; k0 += WR) {
#define STEP(R)                                                                                         \
    if (k0 + R < N) {                                                                                   \
        elim_step<M, HAS_ED, R>(k0 + R, Lk, hl, a, col, sing, slot, U, s_desc, val, w, ed, first_pair);              \
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
        // The U rows this wave stored are read back by other lanes of the wave: wait for
        // the stores to reach L2, and read them with L1-bypassing loads (ld_u: the slab is
        // reused by the next pair, so L1 may hold the previous pair's lines).  An
        // agent-scope fence here instead (buffer_wbl2: write back the XCD's L2) cost the
        // whole kernel.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // Lane hl < WC holds y of its pending row r = hl (mod WC) in [k-18, k] and, loaded
        // a full lap (19 steps) ahead, the eliminated right-hand side of its next row r-19.
        // At step k it needs U[r][k-r]: those come through a PFB-deep ring of loads.
        const int kN = N - 1;
        int LkB = kN % WC;
        double y0 = 0.0, y1 = 0.0, y2 = 0.0, yb0 = 0.0, yb1 = 0.0, yb2 = 0.0;
        if (hl < WC) {
            const int d = (LkB >= hl) ? LkB - hl : LkB - hl + WC;
            const int r = kN - d;
            if (r >= 0) {
                const double* ur = U + (size_t)r * UW + WC;
                y0 = ld_u(ur);
                y1 = ld_u(ur + 1);
                y2 = ld_u(ur + 2);
            }
            if (r - WC >= 0) {
                const double* ur = U + (size_t)(r - WC) * UW + WC;
                yb0 = ld_u(ur);
                yb1 = ld_u(ur + 1);
                yb2 = ld_u(ur + 2);
            }
        }
        double ud[PFB];
        auto issue = [&](int k, int slotk, int lk) {
            const int d = (lk >= hl) ? lk - hl : lk - hl + WC;
            ud[slotk] = (k >= 0 && hl < WC && k - d >= 0) ? ld_u(U + (size_t)(k - d) * UW + d) : 0.0;
        };
        int lkPF = LkB;
#pragma unroll
        for (int s = 0; s < PFB; ++s) {
            issue(kN - s, s, lkPF);
            lkPF = (lkPF == 0) ? WC - 1 : lkPF - 1;
        }
        double* xs = s_x[h];
        double* out = C + s0 * 24;
        double fin = 0.0;
        for (int k0 = kN; k0 >= 0; k0 -= PFB) {
#pragma unroll
            for (int s = 0; s < PFB; ++s) {
                const int k = k0 - s;
                if (k >= 0) {
                    const double u = ud[s];
                    if (hl == LkB) {  // u = 1 / U[k][k]
                        const double x0 = y0 * u, x1 = y1 * u, x2 = y2 * u;
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
                        // take row k-19 (its right-hand side arrived a lap ago), fetch the next
                        y0 = yb0;
                        y1 = yb1;
                        y2 = yb2;
                        if (k - 2 * WC >= 0) {
                            const double* ur = U + (size_t)(k - 2 * WC) * UW + WC;
                            yb0 = ld_u(ur);
                            yb1 = ld_u(ur + 1);
                            yb2 = ld_u(ur + 2);
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    const double x0 = xs[0], x1 = xs[1], x2 = xs[2];
                    if (hl < WC && hl != LkB) {
                        y0 = fma(-u, x0, y0);
                        y1 = fma(-u, x1, y1);
                        y2 = fma(-u, x2, y2);
                    }
                    __builtin_amdgcn_wave_barrier();
                    issue(k - PFB, s, lkPF);
                    LkB = (LkB == 0) ? WC - 1 : LkB - 1;
                    lkPF = (lkPF == 0) ? WC - 1 : lkPF - 1;
                }
            }
        }
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
    // persistent grid: only as many wavefronts as are resident at once (a second,
    // partial round of wavefronts would double the tail)
    static int occ[2] = {0, 0};
    int& nb = occ[ED ? 1 : 0];
    if (nb == 0) {
        hipError_t e = ED ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, true>, W64, 0)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, false>, W64, 0);
        if (e != hipSuccess || nb <= 0) nb = BAND_WAVES_PER_CU;
    }
    const int32_t resident = (grid / BAND_WAVES_PER_CU) * std::min(nb, BAND_WAVES_PER_CU);
    const int32_t g = std::min<int32_t>(std::min(grid, resident), (n_traj + 1) / 2);
    if (ED)
        TGMS_LAUNCH((k_band_kkt<M, true>), dim3(g), dim3(W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                           status, scratch);
    else
        TGMS_LAUNCH((k_band_kkt<M, false>), dim3(g), dim3(W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                           status, scratch);
    return hipSuccess;
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

#ifdef TGMS_BAND_STAMPS
extern "C" int tgms_debug_band_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tgms::g_bstamps), sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}
#endif
