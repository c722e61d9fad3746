// tgms_band.hip — TGMS_METHOD_BAND_KKT: the survey's literal KKT,
// LU with partial pivoting, a 16-lane row of a wavefront per trajectory.
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
// Mapping (gfx950): a 16-lane DPP row per trajectory, four per wavefront, four
// wavefronts per workgroup (sharing the entry table).  Forward elimination keeps one
// window row per lane (row_step below): DPP pivot search, LDS broadcast of the pivot row,
// 21 FMAs per lane and step, the entering row k+10 assembled column-parallel from the
// segment powers T_i^e and the 2Q blocks staged in LDS (a1/a2 never exist as a matrix).
// Each finished U row (1/pivot, 18 super-diagonal entries, 3 eliminated right-hand
// sides: 176 B) goes to a per-trajectory slab; back substitution (back_step) streams
// the slab in reverse, a 16-B piece of a row per lane, as a DPP dot product.
// Round 2's first mapping (a half-wavefront per trajectory, lane = window column) took
// 2.50 ms per 65,536 at M = 10; this one 1.56 ms.
#include <algorithm>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

constexpr int KL = 9;              // sub-diagonals (== super-diagonals) of the interleaved KKT
constexpr int WR = KL + 1;         // window rows
constexpr int WC = 2 * KL + 1;     // window columns == width of a U row (diagonal + kl+ku)
constexpr int UW = WC + 3;         // slab row: U row (19) + 3 eliminated right-hand sides

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

// 1/x: hardware reciprocal + two Newton steps (within an ulp; the pivots only scale)
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}

// ---------------------------------------------------------------------------
// Row-lane mapping: a 16-lane DPP row per trajectory, four trajectories per wavefront.
// Lane j < WR holds one window row: its entries at columns k..k+18 in registers
// u[c mod 19] (static register names under a 19-step unroll) and its 3 right-hand
// sides.  Rows never move between lanes: the pivot search is a DPP max over the row's
// lanes (ties to the lowest position in the permuted order, as LAPACK and the oracle),
// the interchange is a swap of two position labels, and the pivot row reaches the other
// lanes through one LDS broadcast.  The pivot lane leaves with its row (it becomes U row
// k in the slab) and takes the entering row k+10, which the group assembles
// column-parallel (two entries per lane) and hands over through LDS.  A step issues
// ~160 VALU + ~100 SALU instructions per wavefront for four trajectories (the
// column-lane mapping: ~105 VALU + ~40 SALU for two).
constexpr int QG = 16;                  // lanes per trajectory (one DPP row)
constexpr int QT = W64 / QG;            // trajectories per wavefront
constexpr int QW = 4;                   // wavefronts per workgroup (share the entry table)
constexpr int QS = UW + 2;              // LDS row stride of the pivot / entering rows (16-B aligned)
#ifndef TGMS_BAND_WAVES_PER_EU
#define TGMS_BAND_WAVES_PER_EU 2           // register budget: 256 VGPRs, no spills in the step loops
#endif

using gdouble = __attribute__((address_space(1))) double;  // global: keeps slab accesses off the flat path

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}

// Column held by register t at step k (R = k mod WC): the c = t (mod WC) in [k+1, k+WC]
// once column k has left (the entering row's columns).
template <int R>
__device__ __forceinline__ int enter_col(int k, int t) {
    int d = t - (R + 1) % WC;
    d += (d < 0) ? WC : 0;
    return k + 1 + d;
}

// Lane-dependent values re-derived inside every unrolled step: an opaque copy keeps
// LICM from hoisting 19 steps' worth of per-lane index arithmetic (and its registers)
// out of the step loops.
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ gdouble* opaque(gdouble* p) {
    asm volatile("" : "+v"(p));
    return p;
}

// Entering row k+WR from its structural nonzeros (at most NE = 10 per row of the
// interleaved KKT): lanes 0..10 zero the row's 22 slots, then lane j < NE writes
// nonzero j of the row's pattern (coef * V_i[idx] at column r + d) and lanes NE..NE+2 the
// right-hand sides.  The row's block, offset and right-hand-side source are wave-uniform
// (scalar unit).  Same entries as row_entry (the list is built from the same table).
constexpr int NE = 10;                  // structural nonzeros per row, at most
constexpr int NPAT = 4 * NOFF;          // (variant, row offset) patterns

__host__ __device__ constexpr int pack_ent(int coef, int d, int idx) { return (coef << 10) | ((d + KL) << 5) | idx; }

template <int M, bool HAS_ED, int R>
__device__ __forceinline__ void enter_row(int k, int j, const int* ents, const double* val, const double* w,
                                          const double* ed, double* E) {
    constexpr int N = 14 * M + 2;
    const int r = k + WR;
    const bool live_r = r < N;
    const int i = (r < 4) ? 0 : min((r - 4) / 14, M - 1);
    const int o = live_r ? r - (4 + 14 * i) : 0;
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
    const int vv = (i == 0 ? 1 : 0) | (i == M - 1 ? 2 : 0);
    if (j < UW / 2) reinterpret_cast<double2*>(E)[j] = make_double2(0.0, 0.0);
    const int e = ents[(vv * NOFF + o + 4) * NE + min(j, NE - 1)];
    const int d = ((e >> 5) & 31) - KL;
    const double v = (double)(e >> 10) * val[i * VAL + (e & 31)];
    int t = R + WR + d;  // register slot of column r + d (in [k+1, k+19])
    t -= (t >= WC) ? WC : 0;
    const int ax = min(max(j - NE, 0), 2);
    const double rw = w[max(wr, 0) * 3 + ax];
    const double re = HAS_ED ? ed[max(eb, 0) + ax] : 0.0;
    const double rhs = (wr >= 0) ? rw : ((HAS_ED && eb >= 0) ? re : 0.0);
    const bool put = live_r && ((j < NE) ? (e != 0) : (j < NE + 3));
    if (put) E[(j < NE) ? t : WC + ax] = (j < NE) ? v : rhs;
}

template <int M, bool HAS_ED, int R>
__device__ __forceinline__ void row_step(int k, int j0, double (&u)[WC], double (&rh)[3], int& pos, bool& sing,
                                         double* P, double* E, gdouble* U, const int* ents, const double* val,
                                         const double* w, const double* ed) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int j = opaque(j0);
    enter_row<M, HAS_ED, R>(k, j, ents, val, w, ed, E);
    // pivot search in column k (register R) over the window lanes: DPP max of |a|, then
    // the lowest position among the maxima
    const double cv = u[R];
    const bool win = j < WR;
    double m = win ? fabs(cv) : -1.0;
    m = fmax(m, dpp_f64<0xB1>(m));   // quad_perm [1,0,3,2]
    m = fmax(m, dpp_f64<0x4E>(m));   // quad_perm [2,3,0,1]
    m = fmax(m, dpp_f64<0x141>(m));  // row_half_mirror
    m = fmax(m, dpp_f64<0x140>(m));  // row_mirror
    const bool eq = win && fabs(cv) == m;
    int cp = eq ? pos : 0x7fffffff;
    cp = min(cp, dpp_i32<0xB1>(cp));
    cp = min(cp, dpp_i32<0x4E>(cp));
    cp = min(cp, dpp_i32<0x141>(cp));
    cp = min(cp, dpp_i32<0x140>(cp));
    const bool piv = eq && pos == cp;
    sing = sing || !(m > 0.0);
    // the pivot lane hands its row to the group through LDS ([1/pivot, columns
    // k+1..k+18, rhs]: U row k), one 64-bit write per entry (no register shuffles)
    if (piv) {
        P[0] = recip(cv);
#pragma unroll
        for (int d = 1; d < WC; ++d) P[d] = u[(R + d) % WC];
#pragma unroll
        for (int a = 0; a < 3; ++a) P[WC + a] = rh[a];
    }
    __builtin_amdgcn_wave_barrier();
    // U row k to the slab: lane j < 11 copies 16 B of it
    if (j < UW / 2) {
        const double2 v = reinterpret_cast<const double2*>(P)[j];
        gdouble* Uk = U + (size_t)k * UW + 2 * j;
        Uk[0] = v.x;
        Uk[1] = v.y;
    }
    // rank-1 update of the other window rows (only they read the pivot row: the LDS
    // pipe, not the VALU, is the tighter resource); column k leaves (register R becomes
    // column k+19, zero outside the entering row)
    if (win && !piv) {
        double p[UW];
        const double2* Pd = reinterpret_cast<const double2*>(P);
#pragma unroll
        for (int q = 0; q < UW / 2; ++q) {
            const double2 v = Pd[q];
            p[2 * q] = v.x;
            p[2 * q + 1] = v.y;
        }
        const double l = cv * p[0];
#pragma unroll
        for (int d = 1; d < WC; ++d) u[(R + d) % WC] = fma(-l, p[d], u[(R + d) % WC]);
#pragma unroll
        for (int a = 0; a < 3; ++a) rh[a] = fma(-l, p[WC + a], rh[a]);
    }
    u[R] = 0.0;
    if (pos == k) pos = cp;  // interchange: the row at position k takes the pivot's position
    if (piv) {               // the pivot lane takes row k+WR
#pragma unroll
        for (int t = 0; t < WC; ++t) u[t] = E[t];
#pragma unroll
        for (int a = 0; a < 3; ++a) rh[a] = E[WC + a];
        pos = k + WR;
    }
    __builtin_amdgcn_wave_barrier();  // P and E are rewritten by the next step
}

// Back substitution of one trajectory by its 16-lane row, row oriented:
//   x_k = (b'_k - sum_{d=1..18} U[k][k+d] x_{k+d}) / U[k][k].
// Lane j < 11 holds 16 B of U row k, (U[k][2j], U[k][2j+1]), and the matching window
// values (x_{k+2j}, x_{k+2j+1}) for 3 axes; the dot product is a DPP butterfly over the
// row.  The eliminated right-hand side rides in the same sum: lanes 9 and 10 hold the
// constants -e_a against U[k][19..21], and lane 0's x_k slot is 0 against 1/U[k][k].
// Lane 0 finalizes x_k = -sum * (1/U[k][k]) and the window slides one position (DPP
// row shift), so x_k never leaves the registers.  Rows come through a 19-deep ring of
// 16-B buffer loads issued one lap ahead (every ring slot its own register, every lane
// loading: no load result is read before its lap is over).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int BCPOL_SC1 = 16;  // agent-scope (L1-bypassing) load: the slab was written by this wave

template <bool BOUND_ZERO>
__device__ __forceinline__ double dpp_shr1_f64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), 0x111, 0xF, 0xF, BOUND_ZERO);  // row_shr:1
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x111, 0xF, 0xF, BOUND_ZERO);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double2 ld_row16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, BCPOL_SC1));
}

// byte offset of lane j's 16 B of row kk in the wave's slabs (out of range: 0 returned)
__device__ __forceinline__ uint32_t row_off(int g, int j, int kk, int N) {
    return (kk >= 0 && j < UW / 2) ? (uint32_t)(((g * N + kk) * UW + 2 * j) * 8) : 0xFFFFFFF0u;
}

template <int M, int S>
__device__ __forceinline__ void back_step(int k, int j0, int g, __amdgpu_buffer_rsrc_t rs, double2 (&ur)[WC],
                                          double (&xa)[3], double (&xb)[3], double* out, bool live, bool emit,
                                          double& fin) {
    constexpr int N = 14 * M + 2;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int j = opaque(j0);
    const double2 uk = ur[S];
    double sm[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) sm[a] = fma(uk.y, xb[a], uk.x * xa[a]);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        sm[a] += dpp_f64<0xB1>(sm[a]);   // quad_perm [1,0,3,2]
        sm[a] += dpp_f64<0x4E>(sm[a]);   // quad_perm [2,3,0,1]
        sm[a] += dpp_f64<0x141>(sm[a]);  // row_half_mirror
        sm[a] += dpp_f64<0x140>(sm[a]);  // row_mirror
    }
    // lane 0: uk.x = 1 / U[k][k]
    double x[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = -sm[a] * uk.x;
    if (j == 0 && k >= 0) {
        fin += (x[0] + x[1] + x[2]) * 0.0;
        const Pos pk = decode<M>(k);
        if (pk.kind == 1 && live) {
            double* o = out + pk.seg * 24 + pk.idx;
            o[0] = emit ? x[0] : 0.0;
            o[8] = emit ? x[1] : 0.0;
            o[16] = emit ? x[2] : 0.0;
        }
    }
    // slide the window: (x_{k+2j}, x_{k+2j+1}) -> (x_{k-1+2j}, x_{k+2j}); lanes 9 and 10
    // keep the right-hand-side constants
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double cur = (j == 0) ? x[a] : xa[a];
        const double nxa = dpp_shr1_f64<true>(xb[a]);
        xb[a] = (j == 9) ? (a == 0 ? -1.0 : 0.0) : ((j == 10) ? (a == 2 ? -1.0 : 0.0) : cur);
        xa[a] = (j == 10) ? (a == 1 ? -1.0 : 0.0) : nxa;
    }
    // refill the ring slot for step k-19 (same slot)
    ur[S] = ld_row16(rs, row_off(g, j, k - WC, N));
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(QW * W64) __attribute__((amdgpu_waves_per_eu(TGMS_BAND_WAVES_PER_EU))) void k_band_kkt(int32_t n_traj, const int32_t* __restrict__ ids,
                                                       const int32_t* __restrict__ seg_offsets,
                                                       const double* __restrict__ W, const double* __restrict__ T,
                                                       const double* __restrict__ ED, double* __restrict__ C,
                                                       int32_t* __restrict__ status, double* __restrict__ scratch) {
    constexpr int N = 14 * M + 2;
    __shared__ int s_desc[NDESC];                            // entry pattern of the interleaved KKT
    __shared__ int s_ents[NPAT * NE];                        // the same, as per-row nonzero lists
    __shared__ double s_val[QW][QT][M * VAL];                // V_i = [1, T_i^0..T_i^7, 2Q_i] per segment
    __shared__ double s_w[QW][QT][(M + 1) * 3];              // waypoints
    __shared__ double s_ed[QW][QT][HAS_ED ? 18 : 1];         // end derivatives
    __shared__ alignas(16) double s_piv[QW][QT][QS];         // pivot row of the current step
    __shared__ alignas(16) double s_ent[QW][QT][QS];         // entering row of the current step
    __shared__ double s_x[QW][QT][4];                        // back substitution: x_k broadcast

    const int wv = threadIdx.x / W64, lane = threadIdx.x % W64, g = lane / QG;
    for (int q = threadIdx.x; q < NDESC; q += QW * W64) {
        const int vv = q / (NOFF * WC), rem = q - vv * NOFF * WC, o = rem / WC - 4, d = rem % WC - KL;
        s_desc[q] = desc_entry(vv, o, d);
    }
    for (int q = threadIdx.x; q < NPAT; q += QW * W64) {
        const int vv = q / NOFF, o = q % NOFF - 4;
        int n = 0;
        for (int d = -KL; d <= KL; ++d) {
            const int de = desc_entry(vv, o, d);
            if (de != 0 && n < NE) s_ents[q * NE + n++] = pack_ent(de >> 5, d, de & 31);
        }
        for (; n < NE; ++n) s_ents[q * NE + n] = 0;
    }
    __syncthreads();
    const int wave_id = blockIdx.x * QW + wv;
    gdouble* const U0 = (gdouble*)scratch + ((size_t)wave_id * QT + g) * (size_t)N * UW;
    double* val = s_val[wv][g];
    double* w = s_w[wv][g];
    double* ed = s_ed[wv][g];
    double* P = s_piv[wv][g];
    double* E = s_ent[wv][g];
    double* xs = s_x[wv][g];
    const int nquads = (n_traj + QT - 1) / QT;

    for (int qd = wave_id; qd < nquads; qd += gridDim.x * QW) {
        // per-quad opaque copies: the slab addresses must not be hoisted out of this loop
        gdouble* const U = opaque(U0);
        const int j = opaque(lane % QG);
        const int bi = QT * qd + g;
        const bool live = bi < n_traj;
        const int32_t b = ids ? ids[live ? bi : QT * qd] : (live ? bi : QT * qd);
        const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;
        const double* gw = W + (s0 + b) * 3;
        const double* gt = T + s0;

        // ---- stage inputs, validate (T > 0 finite; W, ED finite)
        bool ok = true;
        for (int q = j; q < (M + 1) * 3; q += QG) {
            const double v = gw[q];
            w[q] = v;
            ok = ok && (v * 0.0 == 0.0);
        }
        if (HAS_ED) {
            for (int q = j; q < 18; q += QG) {
                const double v = ED[(int64_t)b * 18 + q];
                ed[q] = v;
                ok = ok && (v * 0.0 == 0.0);
            }
        }
        for (int i = j; i < M; i += QG) {
            const double t = gt[i];
            ok = ok && finite_pos(t);
            double p = 1.0;
            val[i * VAL] = 1.0;
            val[i * VAL + 1] = 1.0;
#pragma unroll
            for (int e = 1; e < 8; ++e) {
                p *= t;
                val[i * VAL + 1 + e] = p;
            }
        }
        const unsigned long long badm = __ballot(!ok);
        const bool valid = ((badm >> (QG * g)) & 0xffffull) == 0;
        __builtin_amdgcn_wave_barrier();
        for (int q = j; q < M * 16; q += QG) {
            const int i = q >> 4, jj = 4 + ((q >> 2) & 3), kk = 4 + (q & 3), ex = jj + kk - 7;
            val[i * VAL + 9 + (q & 15)] = 2.0 * (dfac(jj, 4) * dfac(kk, 4) * val[i * VAL + 1 + ex] / (double)ex);
        }
        __builtin_amdgcn_wave_barrier();

        // ---- forward elimination (a3): lane j < WR holds window row j
        double u[WC], rh[3];
        int pos = (j < WR) ? j : -1;  // position in the permuted order (-1: not a window lane)
#pragma unroll
        for (int t = 0; t < WC; ++t) u[t] = (j < WR) ? row_entry<M, HAS_ED>(t, j, t, s_desc, val, w, ed) : 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) rh[a] = (j < WR) ? row_entry<M, HAS_ED>(WC + a, j, 0, s_desc, val, w, ed) : 0.0;
        bool sing = false;
        for (int k0 = 0; k0 < N; k0 += WC) {
#define STEP(R) \
    if (k0 + R < N) row_step<M, HAS_ED, R>(k0 + R, j, u, rh, pos, sing, P, E, U, s_ents, val, w, ed);
            STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7) STEP(8) STEP(9)
            STEP(10) STEP(11) STEP(12) STEP(13) STEP(14) STEP(15) STEP(16) STEP(17) STEP(18)
#undef STEP
        }
        const unsigned long long singm = __ballot(sing);
        const bool singular = ((singm >> (QG * g)) & 0xffffull) != 0;
        const bool emit = live && valid && !singular;

        // ---- back substitution.  The U rows this wave stored are read back by other lanes
        // of the wave: wait for the stores to reach L2 and read them with L1-bypassing loads
        // (the slab is reused by the next quad, so L1 may hold the previous one's lines)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        constexpr int kN = N - 1;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            scratch + (size_t)wave_id * QT * N * UW, (short)0, QT * N * UW * 8, 0x00020000);
        double2 ur[WC];
#pragma unroll
        for (int S = 0; S < WC; ++S) ur[S] = ld_row16(rs, row_off(g, j, kN - S, N));
        double xa[3], xb[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            xa[a] = (j == 10) ? (a == 1 ? -1.0 : 0.0) : 0.0;
            xb[a] = (j == 9) ? (a == 0 ? -1.0 : 0.0) : ((j == 10) ? (a == 2 ? -1.0 : 0.0) : 0.0);
        }
        double* out = C + s0 * 24;
        double fin = 0.0;
#ifdef TGMS_BAND_NOBACK  // ablation build: forward elimination only
        for (int k0 = kN; k0 >= 0 && false; k0 -= WC) {
#else
        for (int k0 = kN; k0 >= 0; k0 -= WC) {
#endif
#define BSTEP(S) back_step<M, S>(k0 - S, j, g, rs, ur, xa, xb, out, live, emit, fin);
            BSTEP(0) BSTEP(1) BSTEP(2) BSTEP(3) BSTEP(4) BSTEP(5) BSTEP(6) BSTEP(7) BSTEP(8) BSTEP(9)
            BSTEP(10) BSTEP(11) BSTEP(12) BSTEP(13) BSTEP(14) BSTEP(15) BSTEP(16) BSTEP(17) BSTEP(18)
#undef BSTEP
        }
        const unsigned long long nf = __ballot(!(fin == 0.0));
        const bool nonfinite = ((nf >> (QG * g)) & 0xffffull) != 0;
        if (live && j == 0 && status) {
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
    // persistent grid of resident workgroups only (a second, partial round would double
    // the tail); `grid` counts wavefronts, each with QT slabs
    static int occ[2] = {0, 0};
    int& nb = occ[ED ? 1 : 0];
    if (nb == 0) {
        hipError_t e = ED ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, true>, QW * W64, 0)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, false>, QW * W64, 0);
        if (e != hipSuccess || nb <= 0) nb = 1;
    }
    constexpr int kMaxBlocksPerCU = BAND_WAVES_PER_CU / QW;
    const int32_t resident = (grid / BAND_WAVES_PER_CU) * std::min(nb, kMaxBlocksPerCU);
    const int32_t nquads = (n_traj + QT - 1) / QT;
    const int32_t g = std::max<int32_t>(1, std::min<int32_t>(resident, (nquads + QW - 1) / QW));
    if (ED)
        TGMS_LAUNCH((k_band_kkt<M, true>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    else
        TGMS_LAUNCH((k_band_kkt<M, false>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    return hipSuccess;
}

constexpr int SLABS_PER_WAVE = QT;


}  // namespace

size_t band_scratch_bytes(int M, int32_t grid) {
    return (size_t)grid * SLABS_PER_WAVE * (size_t)(14 * M + 2) * UW * sizeof(double);
}

hipError_t launch_band_kkt(int M, int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W,
                           const double* T, const double* ED, double* C, int32_t* status, double* scratch,
                           int32_t grid, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return band_M<m>(n_traj, ids, so, W, T, ED, C, status, scratch, grid, stream);
#ifdef TGMS_BAND_ONLY_M10  // development builds: one instantiation
        X(10)
#else
        X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#endif
#undef X
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tgms
