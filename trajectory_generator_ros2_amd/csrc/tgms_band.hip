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
// start rows (i = 0).  Every entry is coef * V_i[idx] with V_i = [1, T_i^0..T_i^7]
// staged per trajectory in LDS, or (idx = 9 + e) a 2Q_i entry 2 (coef T_i^e / e), formed
// in the order the oracle assembles it (q = dfac dfac T^e / e, K = 2 q); (coef, idx)
// depends only on the block variant (first / last segment), the row offset o and the
// diagonal offset d = c - r, so the pattern is a small table built once per workgroup:
// an entering row costs two LDS reads per lane instead of a divergent case analysis.
// Same entries as oracle assemble_kkt_cont; tests/test_oracle.py
// pins the band.
constexpr int VAL = 9;                // V_i stride: [1, T_i^0..T_i^7]
constexpr int NOFF = 18;              // row offsets -4..13

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
        if (oc >= 0 && oc < 8)  // 2Q_i: idx 9 + e stands for 2 (coef T_i^e / e), e = j + k - 7
            return (j >= 4 && oc >= 4) ? pack((int)(dfac(j, 4) * dfac(oc, 4)), 9 + (j + oc - 7)) : 0;
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

// 1/x: hardware reciprocal + two Newton steps (within an ulp; the pivots only scale)
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}

// ---------------------------------------------------------------------------
// Octet mapping (round 3): eight lanes per trajectory in the forward elimination, eight
// trajectories per wavefront.  Lane j < 5 holds TWO window rows, 2j and 2j+1: their
// entries at columns k..k+18 in registers u[c mod 19] (static names under a 19-step
// unroll) and their 3 right-hand sides.  Rows never move between lanes: the pivot search
// is a DPP max over the octet (quad swaps and the half-row mirror), then the lowest
// position among the maxima (ties to the lowest position in the permuted order, as
// LAPACK and the oracle), the interchange swaps two position labels, and the pivot row
// reaches the other lanes through one LDS broadcast that each lane reads once for both
// of its rows.  The per-step work that does not grow with the rows -- pivot search,
// pivot-row hand-over, entering row, bookkeeping -- is paid once per eight trajectories
// (round 2's row-lane mapping: once per four, a 16-lane row per trajectory with one
// window row per lane).  Back substitution keeps the 16-lane rows (four trajectories at
// a time, two passes).
constexpr int QG = 16;                  // back substitution: lanes per trajectory (one DPP row)
constexpr int QT = W64 / QG;            // back substitution: trajectories per pass
constexpr int OG = 8;                   // forward elimination: lanes per trajectory (half a DPP row)
constexpr int OT = W64 / OG;            // trajectories per wavefront
constexpr int OL = WR / 2;              // lanes holding window rows (two each)
constexpr int QW = 4;                   // wavefronts per workgroup (share the entry table)
constexpr int QS = UW + 2;              // LDS row stride of the pivot / entering rows (16-B aligned)
#ifndef TGMS_BAND_WAVES_PER_EU
#define TGMS_BAND_WAVES_PER_EU 2
#endif

using gdouble = __attribute__((address_space(1))) double;  // global: keeps slab accesses off the flat path

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
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

// A row of the interleaved KKT from its structural nonzeros (at most NE = 10 per row):
// a per-(block variant, row offset) list of (coefficient, diagonal offset, V index),
// built once per workgroup from the entry table.
constexpr int NE = 10;                  // structural nonzeros per row, at most
constexpr int NPAT = 4 * NOFF;          // (variant, row offset) patterns

__host__ __device__ constexpr int pack_ent(int coef, int d, int idx) { return (coef << 10) | ((d + KL) << 5) | idx; }

// value of a packed entry of segment block vi (V_i = [1, T_i^0..T_i^7])
__device__ __forceinline__ double ent_value(int e, const double* vi) {
    const int idx = e & 31;
    const double c = (double)(e >> 10);
    if (idx < VAL) return c * vi[idx];
    const int ex = idx - VAL;  // a 2Q_i entry: 2 (dfac dfac T^e / e), as the oracle forms it
    return 2.0 * (c * vi[1 + ex] / (double)ex);
}

// Assemble row r (wave-uniform) into the octet's LDS row E in register-slot order:
// column r + d goes to slot (base + d) mod 19 (base = r mod 19 when column c sits in
// register c mod 19), the 3 right-hand sides to slots 19..21.  The octet's 8 lanes
// zero the 22 slots (11 16-B writes), then lane j writes items j and j + 8 of the row's
// 13 (10 nonzeros, 3 right-hand sides).  LDS operations of a wave execute in order, so
// the zeros land before the items.
template <int M, bool HAS_ED>
__device__ __forceinline__ void assemble_row(int r, int base, int j, const int* ents, const double* val,
                                             const double* w, const double* ed, double* E) {
    constexpr int N = 14 * M + 2;
    const bool live_r = r < N;
    const int i = (r < 4) ? 0 : min((r - 4) / 14, M - 1);
    const int o = live_r ? r - (4 + 14 * i) : 0;
    int wr = -1, eb = -1;  // right-hand-side source (uniform): waypoint row, end-derivative base
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
    double2* E2 = reinterpret_cast<double2*>(E);
    E2[j] = make_double2(0.0, 0.0);
    if (j < UW / 2 - OG) E2[OG + j] = make_double2(0.0, 0.0);
    const int* list = ents + (vv * NOFF + o + 4) * NE;
    const double* vi = val + i * VAL;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int n = j + OG * h;  // item n of 13
        if (n < NE) {
            const int e = list[n];
            const int d = ((e >> 5) & 31) - KL;
            int t = base + d;
            t += (t < 0) ? WC : 0;
            t -= (t >= WC) ? WC : 0;
            if (live_r && e != 0) E[t] = ent_value(e, vi);
        } else if (n < NE + 3) {
            const int ax = n - NE;
            const double rw = w[max(wr, 0) * 3 + ax];
            const double re = HAS_ED ? ed[max(eb, 0) + ax] : 0.0;
            const double rhs = (wr >= 0) ? rw : ((HAS_ED && eb >= 0) ? re : 0.0);
            if (live_r) E[WC + ax] = rhs;
        }
    }
}

// Take the assembled row from E into registers (11 16-B reads).
__device__ __forceinline__ void take_row(const double* E, double (&u)[WC], double (&rh)[3]) {
    const double2* E2 = reinterpret_cast<const double2*>(E);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        const double2 v = E2[q];
        u[2 * q] = v.x;
        u[2 * q + 1] = v.y;
    }
    const double2 v9 = E2[9], v10 = E2[10];
    u[18] = v9.x;
    rh[0] = v9.y;
    rh[1] = v10.x;
    rh[2] = v10.y;
}

// Hand a window row to the octet as U row k: [1/pivot, columns k+1..k+18, rhs].
template <int R>
__device__ __forceinline__ void put_pivot_row(double* P, double cv, const double (&u)[WC], const double (&rh)[3]) {
    double2* P2 = reinterpret_cast<double2*>(P);
    P2[0] = make_double2(recip(cv), u[(R + 1) % WC]);
#pragma unroll
    for (int q = 1; q < 9; ++q) P2[q] = make_double2(u[(R + 2 * q) % WC], u[(R + 2 * q + 1) % WC]);
    P2[9] = make_double2(u[(R + 18) % WC], rh[0]);
    P2[10] = make_double2(rh[1], rh[2]);
}

template <int M, bool HAS_ED, int R>
__device__ __forceinline__ void oct_step(int k, int j0, double (&u0)[WC], double (&u1)[WC], double (&r0)[3],
                                         double (&r1)[3], int& pos0, int& pos1, bool& sing, double* P, double* E,
                                         gdouble* U, const int* ents, const double* val, const double* w,
                                         const double* ed) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int j = opaque(j0);
    assemble_row<M, HAS_ED>(k + WR, (R + WR) % WC, j, ents, val, w, ed, E);  // the entering row
    // pivot search in column k (register R) over the octet's ten window rows
    const bool win = j < OL;
    const double c0 = u0[R], c1 = u1[R];
    const double a0 = fabs(c0), a1 = fabs(c1);
    double m = win ? fmax(a0, a1) : -1.0;
    m = fmax(m, dpp_f64<0xB1>(m));   // quad_perm [1,0,3,2]
    m = fmax(m, dpp_f64<0x4E>(m));   // quad_perm [2,3,0,1]
    m = fmax(m, dpp_f64<0x141>(m));  // row_half_mirror: the octet
    const bool eq0 = win && a0 == m, eq1 = win && a1 == m;
    int cp = min(eq0 ? pos0 : 0x7fffffff, eq1 ? pos1 : 0x7fffffff);
    cp = min(cp, dpp_i32<0xB1>(cp));
    cp = min(cp, dpp_i32<0x4E>(cp));
    cp = min(cp, dpp_i32<0x141>(cp));
    const bool piv0 = eq0 && pos0 == cp, piv1 = eq1 && pos1 == cp;
    sing = sing || !(m > 0.0);
    if (piv0) put_pivot_row<R>(P, c0, u0, r0);
    if (piv1) put_pivot_row<R>(P, c1, u1, r1);
    __builtin_amdgcn_wave_barrier();
    // U row k to the slab: 11 16-B pieces over the octet's 8 lanes
    {
        const double2* P2 = reinterpret_cast<const double2*>(P);
        gdouble* Uk = U + (size_t)k * UW;
        const double2 v = P2[j];
        Uk[2 * j] = v.x;
        Uk[2 * j + 1] = v.y;
        if (j < UW / 2 - OG) {
            const double2 v2 = P2[OG + j];
            Uk[2 * (OG + j)] = v2.x;
            Uk[2 * (OG + j) + 1] = v2.y;
        }
    }
    // rank-1 update of both rows of every window lane (the pivot row with multiplier 0:
    // it is replaced by the entering row below); column k leaves (register R becomes
    // column k+19, zero outside the entering row)
    if (win) {
        double p[UW];
        const double2* Pd = reinterpret_cast<const double2*>(P);
#pragma unroll
        for (int q = 0; q < UW / 2; ++q) {
            const double2 v = Pd[q];
            p[2 * q] = v.x;
            p[2 * q + 1] = v.y;
        }
        const double l0 = piv0 ? 0.0 : c0 * p[0];
        const double l1 = piv1 ? 0.0 : c1 * p[0];
#pragma unroll
        for (int d = 1; d < WC; ++d) {
            u0[(R + d) % WC] = fma(-l0, p[d], u0[(R + d) % WC]);
            u1[(R + d) % WC] = fma(-l1, p[d], u1[(R + d) % WC]);
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            r0[a] = fma(-l0, p[WC + a], r0[a]);
            r1[a] = fma(-l1, p[WC + a], r1[a]);
        }
    }
    u0[R] = 0.0;
    u1[R] = 0.0;
    if (pos0 == k) pos0 = cp;  // interchange: the row at position k takes the pivot's position
    if (pos1 == k) pos1 = cp;
    if (piv0) {  // the pivot's lane takes row k+WR into the pivot's slot
        take_row(E, u0, r0);
        pos0 = k + WR;
    }
    if (piv1) {
        take_row(E, u1, r1);
        pos1 = k + WR;
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
__global__ __launch_bounds__(QW * W64) __attribute__((amdgpu_waves_per_eu(TGMS_BAND_WAVES_PER_EU))) void k_band_kkt(
    int32_t n_traj, const int32_t* __restrict__ ids, const int32_t* __restrict__ seg_offsets,
    const double* __restrict__ W, const double* __restrict__ T, const double* __restrict__ ED, double* __restrict__ C,
    int32_t* __restrict__ status, double* __restrict__ scratch) {
    constexpr int N = 14 * M + 2;
    __shared__ int s_ents[NPAT * NE];                        // per-row nonzero lists of the interleaved KKT
    __shared__ double s_val[QW][OT][M * VAL];                // V_i = [1, T_i^0..T_i^7] per segment
    __shared__ double s_w[QW][OT][(M + 1) * 3];              // waypoints
    __shared__ double s_ed[QW][OT][HAS_ED ? 18 : 1];         // end derivatives
    __shared__ alignas(16) double s_piv[QW][OT][QS];         // pivot row of the current step
    __shared__ alignas(16) double s_ent[QW][OT][QS];         // entering row of the current step

    const int wv = threadIdx.x / W64, lane = threadIdx.x % W64, g = lane / OG;
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
    gdouble* const U0 = (gdouble*)scratch + ((size_t)wave_id * OT + g) * (size_t)N * UW;
    double* val = s_val[wv][g];
    double* w = s_w[wv][g];
    double* ed = s_ed[wv][g];
    double* P = s_piv[wv][g];
    double* E = s_ent[wv][g];
    const int nocts = (n_traj + OT - 1) / OT;

    for (int oc = wave_id; oc < nocts; oc += gridDim.x * QW) {
        // per-octet opaque copies: the slab addresses must not be hoisted out of this loop
        gdouble* const U = opaque(U0);
        const int j = opaque(lane % OG);
        const int bi = OT * oc + g;
        const bool live = bi < n_traj;
        const int32_t b = ids ? ids[live ? bi : OT * oc] : (live ? bi : OT * oc);
        const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;
        const double* gw = W + (s0 + b) * 3;
        const double* gt = T + s0;

        // ---- stage inputs, validate (T > 0 finite; W, ED finite)
        bool ok = true;
        for (int q = j; q < (M + 1) * 3; q += OG) {
            const double v = gw[q];
            w[q] = v;
            ok = ok && (v * 0.0 == 0.0);
        }
        if (HAS_ED) {
            for (int q = j; q < 18; q += OG) {
                const double v = ED[(int64_t)b * 18 + q];
                ed[q] = v;
                ok = ok && (v * 0.0 == 0.0);
            }
        }
        for (int i = j; i < M; i += OG) {
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
        const unsigned long long badm = __ballot(!ok);  // 8 bits per octet
        __builtin_amdgcn_wave_barrier();

        // ---- the initial window: rows 0..9, assembled through E one at a time; lane
        // j < 5 takes rows 2j (u0) and 2j+1 (u1)
        double u0[WC], u1[WC], r0[3], r1[3];
#pragma unroll
        for (int rr = 0; rr < WR; ++rr) {
            assemble_row<M, HAS_ED>(rr, rr, j, s_ents, val, w, ed, E);
            __builtin_amdgcn_wave_barrier();
            if (j == rr / 2) {
                if (rr & 1)
                    take_row(E, u1, r1);
                else
                    take_row(E, u0, r0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        int pos0 = (j < OL) ? 2 * j : -1, pos1 = (j < OL) ? 2 * j + 1 : -1;  // positions in the permuted order
        bool sing = false;

        // ---- forward elimination (a3)
        for (int k0 = 0; k0 < N; k0 += WC) {
#define STEP(R) \
    if (k0 + R < N) oct_step<M, HAS_ED, R>(k0 + R, j, u0, u1, r0, r1, pos0, pos1, sing, P, E, U, s_ents, val, w, ed);
            STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7) STEP(8) STEP(9)
            STEP(10) STEP(11) STEP(12) STEP(13) STEP(14) STEP(15) STEP(16) STEP(17) STEP(18)
#undef STEP
        }
        const unsigned long long singm = __ballot(sing);

        // ---- back substitution, 16-lane rows, four trajectories per pass.  The U rows
        // this wave stored are read back by other lanes of the wave: wait for the stores to
        // reach L2 and read them with L1-bypassing loads (the slab is reused by the next
        // octet, so L1 may hold the previous one's lines)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        constexpr int kN = N - 1;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            scratch + (size_t)wave_id * OT * N * UW, (short)0, OT * N * UW * 8, 0x00020000);
        const int jq = opaque(lane % QG);
#pragma unroll 1
        for (int pass = 0; pass < OT / QT; ++pass) {
            const int slot = pass * QT + lane / QG;  // trajectory slot of this 16-lane row
            const int bq = OT * oc + slot;
            const bool liveq = bq < n_traj;
            const int32_t bb = ids ? ids[liveq ? bq : OT * oc] : (liveq ? bq : OT * oc);
            const int64_t sq = seg_offsets ? (int64_t)seg_offsets[bb] : (int64_t)bb * M;
            const bool valid = ((badm >> (OG * slot)) & 0xffull) == 0;
            const bool singular = ((singm >> (OG * slot)) & 0xffull) != 0;
            const bool emit = liveq && valid && !singular;
            double2 ur[WC];
#pragma unroll
            for (int S = 0; S < WC; ++S) ur[S] = ld_row16(rs, row_off(slot, jq, kN - S, N));
            double xa[3], xb[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                xa[a] = (jq == 10) ? (a == 1 ? -1.0 : 0.0) : 0.0;
                xb[a] = (jq == 9) ? (a == 0 ? -1.0 : 0.0) : ((jq == 10) ? (a == 2 ? -1.0 : 0.0) : 0.0);
            }
            double* out = C + sq * 24;
            double fin = 0.0;
#ifdef TGMS_BAND_NOBACK  // ablation build: forward elimination only
            for (int k0 = kN; k0 >= 0 && false; k0 -= WC) {
#else
            for (int k0 = kN; k0 >= 0; k0 -= WC) {
#endif
#define BSTEP(S) back_step<M, S>(k0 - S, jq, slot, rs, ur, xa, xb, out, liveq, emit, fin);
                BSTEP(0) BSTEP(1) BSTEP(2) BSTEP(3) BSTEP(4) BSTEP(5) BSTEP(6) BSTEP(7) BSTEP(8) BSTEP(9)
                BSTEP(10) BSTEP(11) BSTEP(12) BSTEP(13) BSTEP(14) BSTEP(15) BSTEP(16) BSTEP(17) BSTEP(18)
#undef BSTEP
            }
            const unsigned long long nf = __ballot(!(fin == 0.0));
            const bool nonfinite = ((nf >> (QG * (lane / QG))) & 0xffffull) != 0;
            if (liveq && jq == 0 && status) {
                int32_t st = TGMS_OK;
                if (!valid) st = TGMS_ERR_INVALID_ARG;
                else if (singular) st = TGMS_ERR_SINGULAR;
                else if (nonfinite) st = TGMS_ERR_NONFINITE;
                status[bb] = st;
            }
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
    const int32_t nocts = (n_traj + OT - 1) / OT;
    const int32_t g = std::max<int32_t>(1, std::min<int32_t>(resident, (nocts + QW - 1) / QW));
    if (ED)
        TGMS_LAUNCH((k_band_kkt<M, true>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    else
        TGMS_LAUNCH((k_band_kkt<M, false>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    return hipSuccess;
}

constexpr int SLABS_PER_WAVE = OT;


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
