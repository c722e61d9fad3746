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
// Mapping (gfx950, round 3): forward elimination by a quad of lanes per trajectory,
// sixteen trajectories per wavefront, the whole 10 x 22 window in registers (quad_step
// below: DPP pivot broadcast, in-register row selection by exact 0/1 masks, no LDS
// traffic for window data); each finished U row, scaled by 1/pivot, goes to a
// per-trajectory slab in slot order; back substitution (back_step) by 8-lane groups
// reads it back 16 + 8 B per lane and row.  Round 2's row-lane mapping (a 16-lane DPP row
// per trajectory, LDS pivot-row broadcast) took 1.56-1.61 ms per 65,536 at M = 10; this
// one 1.33 ms at one wavefront per SIMD, 1.22 ms at two.
#include <algorithm>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

constexpr int KL = 9;              // sub-diagonals (== super-diagonals) of the interleaved KKT
constexpr int WR = KL + 1;         // window rows
constexpr int WC = 2 * KL + 1;     // window columns == width of a U row (diagonal + kl+ku)
constexpr int SW = 22;             // slab row: 19 window slots + 3 eliminated right-hand sides (176 B)

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
// Quad mapping (round 3): four lanes per trajectory, sixteen trajectories per wavefront,
// the whole 10-row window in registers.  Lane q of a trajectory's quad holds every
// window row's entries in register slots s = 4 j + q (j = 0..5): slots 0..18 are the
// window columns (column c in slot c mod 19, so a column leaves and the next one enters
// the same slot and the 19-step unroll names every register statically), 19..21 the
// three right-hand sides, 22..23 unused zeros.  Rows never move; a position label per
// row records the interchanges.  A step k (R = k mod 19):
//   - column k (slot R, one lane's register) is broadcast over the quad by a DPP
//     quad_perm, so every lane finds the same pivot: the largest |a|, ties to the lowest
//     position (as LAPACK and the oracle's KKT_BAND);
//   - with m_r = [r is the pivot row] the pivot row is p = sum_r m_r u_r (exact: one
//     term is nonzero) and the multipliers l_r = a_rk / a_pk with l_p = 1 exactly;
//   - every row: u_r <- u_r - l_r p + m_r e, e the entering row k+10 -- the pivot row
//     cancels exactly and takes the entering row, the others are eliminated, slot R
//     restarts as column k+19 (zero outside the entering row);
//   - the U row [1/pivot, columns k+1..k+18, rhs] goes to the trajectory's slab (8 B per
//     lane and register), in the layout back_step reads.
// The entering row is assembled per lane from the pattern table (coefficient, index
// into the staged V of the row's segment) for its own slots.  No LDS traffic carries
// window data; the per-step work is ~380 VALU instructions per wavefront = ~24 per
// trajectory (round 2's row-lane mapping: ~50 VALU + ~50 SALU + 14 LDS per trajectory).
constexpr int QL = 4;                   // forward elimination: lanes per trajectory
constexpr int QTW = W64 / QL;           // trajectories per wavefront
constexpr int NJ = 6;                   // registers per window row and lane (slots 4 j + q)
#ifndef TGMS_BAND_QW
#define TGMS_BAND_QW 4
#endif
constexpr int QW = TGMS_BAND_QW;        // wavefronts per workgroup (share the pattern table)
// Two wavefronts per SIMD (two workgroups per CU, TGMS_BAND_WAVES_PER_CU = 8): the window
// (120 VGPRs), masks, multipliers, pivot and entering rows need ~290 registers, so within
// 256 the compiler spills ~37 VGPRs (144 B of scratch per lane, a few per step);
// the second wavefront hides the one-wave build's exposed step latency: 1.22 vs 1.28-1.32 ms
// per 65,536 at M = 10.  Round 3 shipped one wavefront per SIMD after
// an intermediate two-wave build returned wrong results; round 4 could not reproduce that
// with any committed source (HW_ID-tagged runs at two workgroups per CU,
// every shape that failed, three runs each, all exact), and tests/test_gpu_band.py checks
// those shapes on every GPU run.  TGMS_BAND_WAVES_PER_EU=1 with TGMS_BAND_WAVES_PER_CU=4
// builds the round-3 configuration (AGPRs as register space, no scratch).
#ifndef TGMS_BAND_WAVES_PER_EU
#define TGMS_BAND_WAVES_PER_EU 2
#endif
static_assert(TGMS_BAND_WAVES_PER_EU * 4 <= BAND_WAVES_PER_CU,  // 4 SIMDs per CU
              "the persistent grid and the slab scratch must cover every resident wavefront");

// Per-trajectory LDS block: Vc (the entering row's segment) | T | waypoints | end derivs.
// Vc = [1, T^0..T^7 (0..8), 2 T^e / e for e = 1..7 (9..15), 0, 0, 0 (16..18)]
constexpr int XV = 19;
constexpr int XZ = 16;                  // first of the three zero slots
__host__ __device__ constexpr int x_t(int) { return XV; }
__host__ __device__ constexpr int x_w(int M) { return XV + M; }
__host__ __device__ constexpr int x_e(int M) { return XV + M + 3 * (M + 1); }
__host__ __device__ constexpr int x_len(int M) { return XV + M + 3 * (M + 1) + 18; }

// pattern table entry: coefficient and Vc index of the entry at (row pattern, d + 9)
__host__ __device__ constexpr int pack_d(int coef, int idx) { return coef * 256 + idx; }
constexpr int NPAT = 4 * NOFF;          // (block variant, row offset) patterns

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

// This lane's index in its wavefront, recomputed where it is used (volatile: never hoisted
// or kept live across the sweep).  Used by the back substitution only (see the group loop).
__device__ __forceinline__ int lane_now() {
    int l = 0;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "+v"(l));
    return l;
}

// Vc of segment i from the staged T_i (one lane of the quad writes it)
__device__ __forceinline__ void set_vc(int i, int q, double* X) {
    if (q == 0) {
        const double t = X[XV + i];
        double pw = 1.0;
        X[0] = 1.0;
        X[1] = 1.0;
#pragma unroll
        for (int e = 1; e < 8; ++e) {
            pw *= t;
            X[1 + e] = pw;
            X[8 + e] = 2.0 * (pw / (double)e);
        }
    }
}

// The row pattern (offset into the table) and the right-hand-side source (index into
// X; the zero slots when the row has none) of interleaved-KKT row r (wave-uniform).
template <int M, bool HAS_ED>
__device__ __forceinline__ void row_info(int r, int& pat_off, int& rsrc, int& seg) {
    const int i = (r < 4) ? 0 : min((r - 4) / 14, M - 1);
    const int o = r - (4 + 14 * i);
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
    pat_off = (vv * NOFF + o + 4) * WC;
    rsrc = (wr >= 0) ? x_w(M) + 3 * wr : ((HAS_ED && eb >= 0) ? x_e(M) + eb : XZ);
    seg = i;
}

// This lane's register J of a row: slot s = 4 J + q.  Window slots hold the entry at
// table column ((s - R1) mod 19) + DD0 (a diagonal offset + 9; outside 0..18: zero),
// slot 19 + a the row's right-hand side a, slots 22..23 zero.
template <int J, int R1, int DD0>
__device__ __forceinline__ double row_entry(int q, int pat_off, int rsrc, const int* sd, const double* X) {
    if (J == 5) {
        const int xi = (q < 2) ? rsrc + 1 + q : XZ;
        return X[xi];
    }
    const int s = 4 * J + q;
    int tt = s - R1 + WC;
    tt -= (tt >= WC) ? WC : 0;
    const int id = tt + DD0;
    const bool ok = (DD0 == 0) || (id >= 0 && id < WC);
    int de = sd[pat_off + (ok ? id : 0)];
    de = ok ? de : pack_d(0, XZ);
    int xi = de & 255;
    double c = (double)(de >> 8);
    if (J == 4) {
        const bool rot = q < 3;
        xi = rot ? xi : rsrc;
        c = rot ? c : 1.0;
    }
    return c * X[xi];
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Row positions: in registers (default, 10 VGPRs) or in the trajectory's LDS block.
#ifndef TGMS_BAND_POS_LDS
#define TGMS_BAND_POS_LDS 0
#endif
#if TGMS_BAND_POS_LDS
typedef int* PosRef;
#else
typedef int (&PosRef)[WR];
#endif

template <int M, bool HAS_ED, int R>
__device__ __forceinline__ void quad_step(const int k, const int q0, double (&u)[WR][NJ], PosRef P,
                                          int& sing, __amdgpu_buffer_rsrc_t rs, const uint32_t vrow,
                                          const int* sd, double* X) {
    constexpr int N = 14 * M + 2;
    constexpr int JR = R / 4, O = R % 4;
    constexpr int BC = O * 0x55;        // quad_perm [O, O, O, O]
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int q = opaque(q0);
    // pivot search on this lane's register JR (meaningful in lane O, which holds column k):
    // the largest |a|, ties to the lowest position
    double m = fabs(u[0][JR]);
#pragma unroll
    for (int r = 1; r < WR; ++r) m = fmax(m, fabs(u[r][JR]));
    // row positions from the trajectory's LDS block (registers are the scarce resource at
    // two wavefronts per SIMD; the quad's lanes read the same words)
#if TGMS_BAND_POS_LDS
    int pos[WR];
    {
        const int4 pa = *reinterpret_cast<const int4*>(P), pb = *reinterpret_cast<const int4*>(P + 4);
        const int2 pc = *reinterpret_cast<const int2*>(P + 8);
        pos[0] = pa.x; pos[1] = pa.y; pos[2] = pa.z; pos[3] = pa.w;
        pos[4] = pb.x; pos[5] = pb.y; pos[6] = pb.z; pos[7] = pb.w;
        pos[8] = pc.x; pos[9] = pc.y;
    }
#else
    int(&pos)[WR] = P;
#endif
    int key = 0x7fffffff, rk = 0;  // rk: the row at position k
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        key = min(key, fabs(u[r][JR]) == m ? ((pos[r] << 4) | r) : 0x7fffffff);
        rk = (pos[r] == k) ? r : rk;
    }
    // folded in here (anchored): left to the compiler, the test sinks to the end of the
    // unrolled steps and m or its flag is spilled across them
    sing |= (q == O && !(m > 0.0)) ? 1 : 0;
    asm volatile("" : "+v"(sing));
    key = dpp_i32<BC>(key);  // lane O's pivot to the quad
    const int ps = key & 15, cp = key >> 4;
    // the pivot row by selection (exactly one row matches; no 0/1 multiplier registers)
    double pv = u[0][JR];
#pragma unroll
    for (int r = 1; r < WR; ++r) pv = (ps == r) ? u[r][JR] : pv;
    // 1/pivot, formed in lane O, to the quad
    const double inv = dpp_f64<BC>(recip(pv));
    double p[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        double a = u[0][j];
#pragma unroll
        for (int r = 1; r < WR; ++r) a = (ps == r) ? u[r][j] : a;
        p[j] = a;
    }
    // U row k, scaled by 1/pivot, to the slab in slot order, laid out for 16-B accesses on
    // both sides: slots (s, s + 8), s < 8, as a 16-B pair at 16 s; slot s + 16 (s < 6) at
    // 128 + 8 s.  This lane's registers (0, 2) and (1, 3) are pairs, 4 and 5 singles;
    // column k's own slot stores 0 (the back substitution never multiplies it)
    {
        double v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = (j == JR && q == O) ? 0.0 : p[j] * inv;
#ifndef TGMS_BAND_NOSTORE  // ablation build: no slab stores
        const int so = k * (SW * 8);
        // this lane's singles at 128 + 8 q and (register 5: the right-hand sides 1 and 2,
        // lanes 0 and 1; lanes 2 and 3 hold the unused slots 22 and 23, which the slab does
        // not keep: an out-of-range offset drops the store) 160 + 8 q, re-derived here so no
        // register holds them over the sweep.  Round 5: with the stores issued three instructions
        // after these offsets were computed, the kernel returned wrong trajectories (DPP bank 3
        // of later groups, 128-267 of 20,001 per run at M = 3); 16 wait states between the two
        // are exact in every run and shape (profiles/r05_band_lane_variants.jsonl: L / LN,
        // J0 / JG).  A standalone probe of VALU-written store offsets does not reproduce the
        // failure, so the guard stays where the kernel needs it.
        const uint32_t vrow1 = vrow + 128u - 8u * (uint32_t)q;
        const uint32_t vrow5 = (q < 2) ? vrow1 + 32u : 0x7FFFFF00u;
        asm volatile("" ::"v"(vrow1), "v"(vrow5));
        __builtin_amdgcn_sched_barrier(0);
#ifndef TGMS_BAND_NOGUARD  // diagnosis build: the unguarded form of round 5's failing builds
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#endif
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[0], v[2])), rs, vrow, so, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[1], v[3])), rs, vrow + 64u, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[4]), rs, vrow1, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[5]), rs, vrow5, so, 0);
#else
        asm volatile("" : : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]));
#endif
    }
    // the entering row k + 10
#ifdef TGMS_BAND_SB1
    __builtin_amdgcn_sched_barrier(0);
#endif
    double e[NJ];
    const int re = k + WR;
    if (re < N) {
        int pat_off, rsrc, seg;
        row_info<M, HAS_ED>(re, pat_off, rsrc, seg);
        if (seg > 0 && re == 4 + 14 * seg) {  // first row of a new segment block
            set_vc(seg, q, X);
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
        constexpr int R1 = (R + 1) % WC;
        e[0] = row_entry<0, R1, 0>(q, pat_off, rsrc, sd, X);
        e[1] = row_entry<1, R1, 0>(q, pat_off, rsrc, sd, X);
        e[2] = row_entry<2, R1, 0>(q, pat_off, rsrc, sd, X);
        e[3] = row_entry<3, R1, 0>(q, pat_off, rsrc, sd, X);
        e[4] = row_entry<4, R1, 0>(q, pat_off, rsrc, sd, X);
        e[5] = row_entry<5, R1, 0>(q, pat_off, rsrc, sd, X);
    } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) e[j] = 0.0;
    }
#ifdef TGMS_BAND_SB2
    __builtin_amdgcn_sched_barrier(0);
#endif
    // rank-1 update; the pivot row cancels exactly and takes the entering row; column k
    // (lane O, register JR) restarts as column k + 19
    const bool restart = q == O;  // column k's register restarts (as column k + 19)
    p[JR] = restart ? 0.0 : p[JR];
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        // multiplier a_rk / a_pk, formed in lane O (row r's column k is still unchanged
        // there), to the quad; the pivot row takes the entering row instead
        const double lr = dpp_f64<BC>(u[r][JR] * inv);
        const bool piv = ps == r;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const double base = (j == JR && restart) ? 0.0 : u[r][j];
            const double nv = fma(-lr, p[j], base);
            u[r][j] = piv ? e[j] : nv;
        }
    }
    // interchange: the row at position k takes the pivot's position; the pivot's slot
    // holds row k + 10 now (the second store wins when the pivot is the row at position k)
#if TGMS_BAND_POS_LDS
    P[rk] = cp;
    P[ps] = re;
#else
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        int v = pos[r];
        v = (v == k) ? cp : v;
        pos[r] = (ps == r) ? re : v;
    }
#endif
}

// Back substitution, eight lanes per trajectory, slot order.  Lane l holds slots l, l+8,
// l+16 of the scaled U row k (one 16-B and one 8-B buffer load) and of the solution
// window: x_c lives in slot c mod 19 for as long as it is in the band, the right-hand-side
// slots 19..21 hold the constants -1 of their axis, slots 22..23 zero.  Then
//   x_k = -sum_s U'[k][s] x[s]      (U' = U / pivot; slot k mod 19 stored as 0)
// is a three-FMA partial per lane and axis and a DPP butterfly over the eight lanes; the
// lane of slot k mod 19 keeps x_k (it replaces x_{k+19}, which left the band).  Rows come
// through a 19-deep ring of loads issued one lap ahead (every ring slot its own
// registers).
constexpr int BCPOL_SC1 = 16;  // agent-scope (L1-bypassing) load: the slab was written by this wave
constexpr int BL = 8;          // back substitution: lanes per trajectory
constexpr int BT = W64 / BL;   // back substitution: trajectories per pass

// byte offset of row kk of slab g (rows before 0: out of range, read as 0)
__device__ __forceinline__ uint32_t slot_off(int g, int kk, int N) {
    return (kk >= 0) ? (uint32_t)((g * N + kk) * SW * 8) : 0x7FFFFF00u;
}

// lane l's slots of a row: (l, l + 8) at 16 l, l + 16 at 128 + 8 l (slots 22, 23, lanes 6
// and 7, are not stored: read as 0 through an out-of-range offset)
__device__ __forceinline__ void ld_slots(__amdgpu_buffer_rsrc_t rs, uint32_t row, int l, double2& a, double& b) {
    a = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, row + 16u * l, 0, BCPOL_SC1));
    const uint32_t o1 = (l < 6 && row < 0x7FFFFF00u) ? row + 128u + 8u * l : 0x7FFFFF00u;
    b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, BCPOL_SC1));
}

template <int M, int S>
__device__ __forceinline__ void back_step(int k, int l0, int g, __amdgpu_buffer_rsrc_t rs, double2 (&ra)[WC],
                                          double (&rb)[WC], double (&x)[3][3], double* out, bool live, bool emit,
                                          double& fin) {
    constexpr int N = 14 * M + 2;
    constexpr int R = ((N - 1 - S) % WC + WC) % WC;  // slot of column k
    constexpr int RI = R / BL, RL = R % BL;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int l = opaque(l0);
    const double2 ua = ra[S];
    const double ub = rb[S];
    double sm[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) sm[a] = fma(ub, x[2][a], fma(ua.y, x[1][a], ua.x * x[0][a]));
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        sm[a] += dpp_f64<0xB1>(sm[a]);   // quad_perm [1,0,3,2]
        sm[a] += dpp_f64<0x4E>(sm[a]);   // quad_perm [2,3,0,1]
        sm[a] += dpp_f64<0x141>(sm[a]);  // row_half_mirror: the eight lanes
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) x[RI][a] = (l == RL) ? -sm[a] : x[RI][a];
    if (l == 0 && k >= 0) {
        fin += (sm[0] + sm[1] + sm[2]) * 0.0;
        const Pos pk = decode<M>(k);
        if (pk.kind == 1 && live) {
            double* o = out + pk.seg * 24 + pk.idx;
            // the same guard as quad_step's slab stores: the address is not a fresh VALU result
            asm volatile("" ::"v"(o));
            __builtin_amdgcn_sched_barrier(0);
#ifndef TGMS_BAND_NOGUARD
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#endif
            __builtin_amdgcn_sched_barrier(0);
            o[0] = emit ? -sm[0] : 0.0;
            o[8] = emit ? -sm[1] : 0.0;
            o[16] = emit ? -sm[2] : 0.0;
        }
    }
    // refill the ring slot for step k-19 (same slot)
    ld_slots(rs, slot_off(g, k - WC, N), l, ra[S], rb[S]);
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(QW * W64) __attribute__((amdgpu_waves_per_eu(TGMS_BAND_WAVES_PER_EU))) void k_band_kkt(
    int32_t n_traj, const int32_t* __restrict__ ids, const int32_t* __restrict__ seg_offsets,
    const double* __restrict__ W, const double* __restrict__ T, const double* __restrict__ ED, double* __restrict__ C,
    int32_t* __restrict__ status, double* __restrict__ scratch) {
    constexpr int N = 14 * M + 2;
    constexpr int XL = x_len(M);
    __shared__ int s_desc[NPAT * WC];                  // pattern table of the interleaved KKT
    __shared__ double s_x[QW][QTW][XL];                // per-trajectory Vc | T | W | ED
    __shared__ alignas(16) int s_pos[QW][QTW][12];     // per-trajectory row positions (10 used)

    for (int n = threadIdx.x; n < NPAT * WC; n += QW * W64) {
        const int pat = n / WC, d = n % WC - KL;
        const int vv = pat / NOFF, o = pat % NOFF - 4;
        const int de = desc_entry(vv, o, d);
        const int idx = de & 31;
        s_desc[n] = (de == 0) ? pack_d(0, XZ) : pack_d(de >> 5, idx < VAL ? idx : idx - 1);
    }
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / W64);
    const int wave_id = blockIdx.x * QW + wv;  // wave-uniform (SGPR): the slab resource stays scalar
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        scratch + (size_t)wave_id * QTW * N * SW, (short)0, QTW * N * SW * 8, 0x00020000);
    const int ngroups = (n_traj + QTW - 1) / QTW;

    // The lane index is recomputed at the top of every group (the mbcnt builtins on an
    // accumulator the compiler cannot hoist), so nothing lane-derived stays live across the
    // group loop: no scratch at any M (held in a register from threadIdx.x instead, 11 of 32
    // instantiations spilled 1-17 VGPRs).  Round 5: builds like this one returned wrong
    // trajectories with status OK (quads 3, 7, 11, 15 of a third of a wave's later groups --
    // round 3's unexplained signature) until the stores were guarded: the compiler re-derived
    // the lane-dependent slab offsets next to their buffer stores, three instructions before
    // the store read them (quad_step).
    for (int grp = wave_id; grp < ngroups; grp += gridDim.x * QW) {
        const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, (unsigned)opaque(0)));
        const int g = lane / QL;
        const int q = opaque(lane % QL);
        double* const X = s_x[wv][g];
        // this lane's place in a slab row: its pairs at 16 q (+ 64) (its singles: quad_step)
        const uint32_t vrow = (uint32_t)(g * N * SW * 8 + 16 * q);
        const int bi = QTW * grp + g;
        const bool live = bi < n_traj;
        const int32_t b = ids ? ids[live ? bi : QTW * grp] : (live ? bi : QTW * grp);
        const int64_t s0 = seg_offsets ? (int64_t)seg_offsets[b] : (int64_t)b * M;
        const double* gw = W + (s0 + b) * 3;
        const double* gt = T + s0;

        // ---- stage inputs, validate (T > 0 finite; W, ED finite)
        bool ok = true;
        for (int n = q; n < (M + 1) * 3; n += QL) {
            const double v = gw[n];
            X[x_w(M) + n] = v;
            ok = ok && (v * 0.0 == 0.0);
        }
        if (HAS_ED) {
            for (int n = q; n < 18; n += QL) {
                const double v = ED[(int64_t)b * 18 + n];
                X[x_e(M) + n] = v;
                ok = ok && (v * 0.0 == 0.0);
            }
        }
        for (int i = q; i < M; i += QL) {
            const double t = gt[i];
            ok = ok && finite_pos(t);
            X[x_t(M) + i] = t;
        }
        if (q < 3) X[XZ + q] = 0.0;
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        set_vc(0, q, X);
        const unsigned long long badm = __ballot(!ok);  // 4 bits per trajectory
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();

        // ---- the initial window: rows 0..9 over columns 0..18 (slot s = column s)
        double u[WR][NJ];
#if TGMS_BAND_POS_LDS
        int* const P = &s_pos[0][0][0] + (wv * QTW + g) * 12;
#else
        int P[WR];
#endif
#define IROW(RR)                                                                      \
    {                                                                                 \
        int pat_off, rsrc, seg;                                                       \
        row_info<M, HAS_ED>(RR, pat_off, rsrc, seg);                                  \
        u[RR][0] = row_entry<0, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        u[RR][1] = row_entry<1, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        u[RR][2] = row_entry<2, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        u[RR][3] = row_entry<3, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        u[RR][4] = row_entry<4, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        u[RR][5] = row_entry<5, 0, 9 - RR>(q, pat_off, rsrc, s_desc, X);              \
        P[RR] = pos0 + RR;                                                            \
    }
        const int pos0 = opaque(0);  // (a hoisted constant pair would be spilled over the sweep)
        IROW(0) IROW(1) IROW(2) IROW(3) IROW(4) IROW(5) IROW(6) IROW(7) IROW(8) IROW(9)
#undef IROW
        int sing = 0;

        // ---- forward elimination (a3)
        for (int k0 = 0; k0 < N; k0 += WC) {
#define STEP(R) \
    if (k0 + R < N) quad_step<M, HAS_ED, R>(k0 + R, q, u, P, sing, rs, vrow, s_desc, X);
            STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7) STEP(8) STEP(9)
            STEP(10) STEP(11) STEP(12) STEP(13) STEP(14) STEP(15) STEP(16) STEP(17) STEP(18)
#undef STEP
        }
        const unsigned long long singm = __ballot(sing != 0);

        // ---- back substitution (round 3), 8-lane groups, eight trajectories per pass.  The U rows
        // this wave stored are read back by other lanes of the wave: wait for the stores to
        // reach L2 and read them with L1-bypassing loads (the slab is reused by the next
        // group, so L1 may hold the previous one's lines)
#ifdef TGMS_BAND_FENCE  // diagnosis build: a full agent-scope acquire/release at the hand-off
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        constexpr int kN = N - 1;
        const int lane_b = lane_now(), lb = lane_b % BL;
#pragma unroll 1
        for (int pass = 0; pass < QTW / BT; ++pass) {
            const int slot = pass * BT + lane_b / BL;  // trajectory slot of this 8-lane group
            const int bq = QTW * grp + slot;
            const bool liveq = bq < n_traj;
            const int32_t bb = ids ? ids[liveq ? bq : QTW * grp] : (liveq ? bq : QTW * grp);
            const int64_t sq = seg_offsets ? (int64_t)seg_offsets[bb] : (int64_t)bb * M;
            const bool valid = ((badm >> (QL * slot)) & 0xfull) == 0;
            const bool singular = ((singm >> (QL * slot)) & 0xfull) != 0;
            const bool emit = liveq && valid && !singular;
            double2 ra[WC];
            double rb[WC];
#pragma unroll
            for (int S = 0; S < WC; ++S) ld_slots(rs, slot_off(slot, kN - S, N), lb, ra[S], rb[S]);
            double x[3][3];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int a = 0; a < 3; ++a) x[i][a] = (i == 2 && lb == 3 + a) ? -1.0 : 0.0;
            double* out = C + sq * 24;
            double fin = 0.0;
#ifdef TGMS_BAND_NOBACK  // ablation build: forward elimination only
            for (int k0 = kN; k0 >= 0 && false; k0 -= WC) {
#else
            for (int k0 = kN; k0 >= 0; k0 -= WC) {
#endif
#define BSTEP(S) back_step<M, S>(k0 - S, lb, slot, rs, ra, rb, x, out, liveq, emit, fin);
                BSTEP(0) BSTEP(1) BSTEP(2) BSTEP(3) BSTEP(4) BSTEP(5) BSTEP(6) BSTEP(7) BSTEP(8) BSTEP(9)
                BSTEP(10) BSTEP(11) BSTEP(12) BSTEP(13) BSTEP(14) BSTEP(15) BSTEP(16) BSTEP(17) BSTEP(18)
#undef BSTEP
            }
            const unsigned long long nf = __ballot(!(fin == 0.0));
            const bool nonfinite = ((nf >> (BL * (lane_b / BL))) & 0xffull) != 0;
            if (liveq && lb == 0 && status) {
                int32_t st = TGMS_OK;
                if (!valid) st = TGMS_ERR_INVALID_ARG;
                else if (singular) st = TGMS_ERR_SINGULAR;
                else if (nonfinite) st = TGMS_ERR_NONFINITE;
#ifdef TGMS_BAND_HWID  // diagnosis build (scripts/band_hwdiag.py): where the trajectory ran
                uint32_t hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                st = (int32_t)((hw & 0x000FFFFFu) | ((xcc & 0xFu) << 20) | ((uint32_t)(st & 0xF) << 24));
#endif
                status[bb] = st;
            }
            // a non-finite solution is rewritten as exact zeros, like every other failure
            // (its coefficients were stored during the sweep): rare path, after this
            // wave's own stores to the range have completed
            if (liveq && valid && !singular && nonfinite) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int64_t mq = seg_offsets ? (int64_t)seg_offsets[bb + 1] - sq : M;
                for (int64_t e = lb; e < mq * 24; e += BL) out[e] = 0.0;
            }
        }
#ifdef TGMS_BAND_FENCE
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
#endif
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
}

template <int M>
hipError_t band_M(int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W, const double* T,
                  const double* ED, double* C, int32_t* status, double* scratch, int32_t grid,
                  hipStream_t stream) {
    if (n_traj <= 0) return hipSuccess;
    // persistent grid of resident workgroups only (a second, partial round would double
    // the tail); `grid` counts wavefronts, each with QTW slabs
    static int occ[2] = {0, 0};
    int& nb = occ[ED ? 1 : 0];
    if (nb == 0) {
        hipError_t e = ED ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, true>, QW * W64, 0)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_band_kkt<M, false>, QW * W64, 0);
        if (e != hipSuccess || nb <= 0) nb = 1;
    }
    constexpr int kMaxBlocksPerCU = BAND_WAVES_PER_CU / QW;
    const int32_t resident = (grid / BAND_WAVES_PER_CU) * std::min(nb, kMaxBlocksPerCU);
    const int32_t ngroups = (n_traj + QTW - 1) / QTW;
    const int32_t g = std::max<int32_t>(1, std::min<int32_t>(resident, (ngroups + QW - 1) / QW));
    if (ED)
        TGMS_LAUNCH((k_band_kkt<M, true>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    else
        TGMS_LAUNCH((k_band_kkt<M, false>), dim3(g), dim3(QW * W64), 0, stream, n_traj, ids, so, W, T, ED, C,
                    status, scratch);
    return hipSuccess;
}

}  // namespace

size_t band_scratch_bytes(int M, int32_t grid) {
    return (size_t)grid * QTW * (size_t)(14 * M + 2) * SW * sizeof(double);
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
