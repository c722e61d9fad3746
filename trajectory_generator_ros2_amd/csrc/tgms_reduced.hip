// tgms_reduced.hip — default solve path (TGMS_METHOD_REDUCED), gfx950.
//
// Eliminating the equality constraints of the survey's KKT
// with the septic-Hermite parametrisation leaves, per axis, an SPD
// block-tridiagonal system over the free knot derivatives u_k = (v_k, a_k, j_k),
// k = 1..M-1 (the Schur complement of the KKT onto the constraint null space; the
// snap Hessian a1 is folded into the integer matrix KH):
//     H_kk    = KEE * r_{k-1}^(5-d-e) + KSS * r_k^(5-d-e)          (r_i = 1/T_i)
//     H_k,k+1 = C_k = KSE * r_k^(5-d-e),   H_k+1,k = C_k^T
//     rhs_k   = -KEP r_{k-1}^(6-d) (w_k - w_{k-1}) - KSP r_k^(6-d) (w_{k+1} - w_k)
// The 3 axes are 3 right-hand sides of one factorisation.  tests/test_oracle.py
// proves with exact rational arithmetic that this system and the KKT of a1-a3
// have identical solutions.
//
// Mapping: a LANE PAIR per trajectory (32 trajectories per wavefront, one
// wavefront per workgroup).  Block LDL^T runs from both ends ("twisted"): the
// even lane eliminates knots 1..c, the odd lane knots M-1..c+1.  The odd lane
// works on the TIME-REVERSED trajectory (min-snap is invariant under t -> T-t,
// knot derivatives map by P = diag(-1, +1, -1)), so both lanes execute the same
// left-to-right instruction stream on their own "virtual" frame.  The chains meet
// at the coupled knots (c, c+1): both lanes broadcast their last pivot block and
// right-hand side in the physical frame (DPP quad_perm), solve the same 6x6
// interface bit-identically, and back-substitute outwards.
//
// Memory path: the wave's 32 input trajectories are one contiguous HBM block,
// loaded with 16-B loads all in flight at once and transposed into LDS
// ([field][trajectory], padded); coefficients leave through a 16-B-aligned LDS
// stage so each store instruction writes whole 64-B (segment, axis) rows.
#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

#ifndef TGMS_MIN_WAVES
#define TGMS_MIN_WAVES 1  // waves per SIMD the register allocation must allow
#endif

// Scheduling fence between unrolled chain / emission steps.  The compiler-level
// memory clobber also stops CSE of LDS reads across steps: re-reading LDS is far
// cheaper than keeping values live.
#ifndef TGMS_NO_SCHED_FENCE
#define SCHED_FENCE()                      \
    do {                                   \
        asm volatile("" ::: "memory");     \
        __builtin_amdgcn_sched_barrier(0); \
    } while (0)
#else
#define SCHED_FENCE() ((void)0)
#endif
#ifdef TGMS_MARKS  // phase markers in the ISA (register-pressure investigations)
#define MARK(x) asm volatile(";MARK " #x ::: "memory")
#else
#define MARK(x) ((void)0)
#endif

constexpr int TPW = 32;      // trajectories per wavefront
constexpr int PSTRIDE = 33;  // LDS row stride (doubles) of the [field][trajectory] staging
// Staged output row: one axis of one segment (8 doubles, 64 B) padded to 80 B so
// the 8 lanes of each ds_write_b128 group hit 8 distinct 4-bank slots.
constexpr int OSTRIDE = 10;

template <int M>
struct alignas(16) Stage {
    // First and 16-B aligned: every ds_*_b128 on it must be naturally aligned, or
    // the LDS replays it (SQ_LDS_UNALIGNED_STALL; cdna_hip_programming.md G17).
    alignas(16) double O[W64 * OSTRIDE];  // one axis of one emission step, every lane
    double W[(M + 1) * 3 * PSTRIDE];
    double T[M * PSTRIDE];
    double R[M * PSTRIDE];  // 1/T, computed once while staging
    int64_t base[TPW];      // coefficient offset (doubles) of each slot's trajectory
    int bad[TPW];
};
static_assert(OSTRIDE % 2 == 0, "staged rows must keep 16-B alignment");

// Per-lane view of the staged inputs in the lane's VIRTUAL frame: the even lane
// sees the trajectory as is, the odd lane time-reversed (virtual knot j = physical
// knot M-j, virtual segment i = physical segment M-1-i).
struct LaneView {
    const double* Wb;  // &W[phys knot of virtual knot 0][axis 0][slot]
    const double* Tb;  // &T[phys segment of virtual segment 0][slot]
    const double* Rb;  // &R[...]
    int kstep;         // +-3*PSTRIDE doubles per virtual knot
    int sstep;         // +-PSTRIDE doubles per virtual segment
    __device__ __forceinline__ double w(int j, int a) const { return Wb[j * kstep + a * PSTRIDE]; }
    __device__ __forceinline__ double t(int i) const { return Tb[i * sstep]; }
    __device__ __forceinline__ double r(int i) const { return Rb[i * sstep]; }
};

template <int M>
__device__ __forceinline__ LaneView make_view(const Stage<M>& sm, int slot, bool right) {
    LaneView L;
    L.Wb = sm.W + (right ? M * 3 * PSTRIDE : 0) + slot;
    L.Tb = sm.T + (right ? (M - 1) * PSTRIDE : 0) + slot;
    L.Rb = sm.R + (right ? (M - 1) * PSTRIDE : 0) + slot;
    L.kstep = right ? -3 * PSTRIDE : 3 * PSTRIDE;
    L.sstep = right ? -PSTRIDE : PSTRIDE;
    return L;
}

// ---------------------------------------------------------------------------
// Output path.  Piece q (0..3) of a lane's write-out is 16 B #(p & 3) of the row
// staged by source lane p >> 2, p = lane + 64 q; its destination depends on the
// step only through a uniform offset, so addresses are formed once per kernel.
struct OutCtx {
    double* stage;   // LDS [W64][OSTRIDE]
    double* dst[4];  // global address of piece q for segment 0, axis 0
    bool live[4];    // piece q belongs to a live trajectory
    bool rt[4];      // piece q was staged by an odd (right) lane
    int lane;
};

__device__ __forceinline__ OutCtx make_out(double* stage, const int64_t* base, double* C, int nb, int lane) {
    OutCtx o;
    o.stage = stage;
    o.lane = lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int p = lane + W64 * q;
        const int chunk = p >> 2, slot = chunk >> 1;
        o.live[q] = slot < nb;
        o.rt[q] = chunk & 1;
        o.dst[q] = C + base[slot < nb ? slot : 0] + (p & 3) * 2;
    }
    return o;
}

// LDS hand-off inside ONE wavefront: DS instructions of a wave execute in order,
// so waiting for this wave's own LDS ops and pinning the compiler's order is
// enough.  (__syncthreads() would also fence global memory: vmcnt(0) on every
// in-flight store.)
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Stage one axis (8 coefficients) of every lane's current segment, then store.
// Even lanes hold segment segL, odd lanes segment segR (odd lanes are idle when
// !has_r, a compile-time property of the step).
__device__ __forceinline__ void stage_axis(const OutCtx& o, const double (&c)[8], int a, int segL, int segR,
                                           bool has_r) {
    wave_lds_sync();  // previous readers are done with the stage
    double2* d = reinterpret_cast<double2*>(o.stage + o.lane * OSTRIDE);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = make_double2(c[2 * j], c[2 * j + 1]);
    wave_lds_sync();
    // all LDS reads first, then the stores (written out by hand: an array of the
    // four pieces ends up in scratch memory)
    auto piece = [&](int q) {
        const int p = o.lane + W64 * q;
        return *reinterpret_cast<const double2*>(o.stage + (p >> 2) * OSTRIDE + (p & 3) * 2);
    };
    const double2 v0 = piece(0), v1 = piece(1), v2 = piece(2), v3 = piece(3);
    const int offL = segL * 24 + a * 8, offR = segR * 24 + a * 8;
    auto put = [&](int q, const double2& v) {
        if (o.live[q] && (has_r || !o.rt[q])) {
#ifdef TGMS_ABL_NOSTORE  // ablation: everything but the global stores
            asm volatile("" ::"v"(v.x), "v"(v.y));
#else
            *reinterpret_cast<double2*>(o.dst[q] + (o.rt[q] ? offR : offL)) = v;
#endif
        }
    };
    put(0, v0);
    put(1, v1);
    put(2, v2);
    put(3, v3);
}

// Coefficients of one physical segment (a4 layout [axis][8]) from its end data:
// physical start knot (w0, g0) and end knot (w1, g1), g = (v, a, j) x axis.
__device__ __forceinline__ void emit_step(const OutCtx& o, double T, double r, const double* w0, const double* w1,
                                          const double (&g0)[3][3], const double (&g1)[3][3], int segL, int segR,
                                          bool has_r) {
    const double T2 = T * T, T3 = T2 * T;
    double rp[8];
    rpowers(r, rp);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double dw = w1[a] - w0[a];
        const double v0 = g0[0][a], a0 = g0[1][a], j0 = g0[2][a];
        const double v1 = g1[0][a], a1 = g1[1][a], j1 = g1[2][a];
        const double h1 = T * v0, h2 = T2 * a0, h3 = T3 * j0;
        const double h5 = T * v1, h6 = T2 * a1, h7 = T3 * j1;
        const double d4 = 35.0 * dw - 20.0 * h1 - 5.0 * h2 - (2.0 / 3.0) * h3 - 15.0 * h5 + 2.5 * h6 -
                          (1.0 / 6.0) * h7;
        const double d5 = -84.0 * dw + 45.0 * h1 + 10.0 * h2 + h3 + 39.0 * h5 - 7.0 * h6 + 0.5 * h7;
        const double d6 = 70.0 * dw - 36.0 * h1 - 7.5 * h2 - (2.0 / 3.0) * h3 - 34.0 * h5 + 6.5 * h6 -
                          0.5 * h7;
        const double d7 = -20.0 * dw + 10.0 * h1 + 2.0 * h2 + (1.0 / 6.0) * h3 + 10.0 * h5 - 2.0 * h6 +
                          (1.0 / 6.0) * h7;
        const double c[8] = {w0[a], v0, 0.5 * a0, j0 * (1.0 / 6.0), d4 * rp[4], d5 * rp[5], d6 * rp[6], d7 * rp[7]};
        stage_axis(o, c, a, segL, segR, has_r);
    }
}

// Emit virtual segment e (virtual knots e .. e+1, derivatives xs / xe).  The even
// lane's virtual segment e is physical segment e; the odd lane's is physical
// segment M-1-e traversed backwards (physical start = virtual knot e+1, with P).
template <int M>
__device__ __forceinline__ void emit_virtual(const OutCtx& o, const LaneView& L, bool right, int e,
                                             const double (&xs)[3][3], const double (&xe)[3][3], bool has_r) {
    const double sg = right ? -1.0 : 1.0;
    double g0[3][3], g1[3][3], w0[3], w1[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double ws = L.w(e, a), we = L.w(e + 1, a);
        w0[a] = right ? we : ws;
        w1[a] = right ? ws : we;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double f = (d == 1) ? 1.0 : sg;
            g0[d][a] = right ? f * xe[d][a] : xs[d][a];
            g1[d][a] = right ? f * xs[d][a] : xe[d][a];
        }
    }
    emit_step(o, L.t(e), L.r(e), w0, w1, g0, g1, e, M - 1 - e, has_r);
}

// ---------------------------------------------------------------------------
// Block algebra.

struct Sym3 {  // symmetric 3x3 block (upper triangle)
    double a00, a01, a02, a11, a12, a22;
};

__device__ __forceinline__ Ldl3 ldl3s(const Sym3& D, bool& spd) {
    Ldl3 f;
    f.i0 = fast_rcp(D.a00);
    f.l10 = D.a01 * f.i0;
    f.l20 = D.a02 * f.i0;
    const double p1 = D.a11 - f.l10 * D.a01;
    f.i1 = fast_rcp(p1);
    const double t12 = D.a12 - f.l20 * D.a01;
    f.l21 = t12 * f.i1;
    const double p2 = D.a22 - f.l20 * D.a02 - f.l21 * t12;
    f.i2 = fast_rcp(p2);
    spd = (D.a00 > 0.0) && (p1 > 0.0) && (p2 > 0.0);
    return f;
}

__device__ __forceinline__ void sym_sub_btw(Sym3& D, const double (&B)[3][3], const double (&Wc)[3][3]) {
    // D -= B^T Wc (the product is symmetric: Wc = D_prev^{-1} B)
    D.a00 -= B[0][0] * Wc[0][0] + B[1][0] * Wc[1][0] + B[2][0] * Wc[2][0];
    D.a01 -= B[0][0] * Wc[0][1] + B[1][0] * Wc[1][1] + B[2][0] * Wc[2][1];
    D.a02 -= B[0][0] * Wc[0][2] + B[1][0] * Wc[1][2] + B[2][0] * Wc[2][2];
    D.a11 -= B[0][1] * Wc[0][1] + B[1][1] * Wc[1][1] + B[2][1] * Wc[2][1];
    D.a12 -= B[0][1] * Wc[0][2] + B[1][1] * Wc[1][2] + B[2][1] * Wc[2][2];
    D.a22 -= B[0][2] * Wc[0][2] + B[1][2] * Wc[1][2] + B[2][2] * Wc[2][2];
}

// Diagonal block of a knot from the powers of its left (pp) and right (pn) segments.
__device__ __forceinline__ Sym3 knot_diag(const double (&pp)[8], const double (&pn)[8]) {
    Sym3 D;
    D.a00 = KEE[0][0] * pp[5] + KSS[0][0] * pn[5];
    D.a01 = KEE[0][1] * pp[4] + KSS[0][1] * pn[4];
    D.a02 = KEE[0][2] * pp[3] + KSS[0][2] * pn[3];
    D.a11 = KEE[1][1] * pp[3] + KSS[1][1] * pn[3];
    D.a12 = KEE[1][2] * pp[2] + KSS[1][2] * pn[2];
    D.a22 = KEE[2][2] * pp[1] + KSS[2][2] * pn[1];
    return D;
}

// Right-hand side of (virtual) knot k, [derivative][axis]; start derivatives u0
// enter at k == 1 through C_0^T.  (For M >= 3 no chain reaches knot M-1, so the
// final derivatives never enter a chain.)
template <bool HAS_ED>
__device__ __forceinline__ void knot_rhs(const LaneView& L, int k, const double (&pp)[8], const double (&pn)[8],
                                         const double (&u0)[3][3], double (&y)[3][3]) {
    const double fp[3] = {-KEP[0] * pp[6], -KEP[1] * pp[5], -KEP[2] * pp[4]};
    const double fn[3] = {-KSP[0] * pn[6], -KSP[1] * pn[5], -KSP[2] * pn[4]};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double wk = L.w(k, a);
        const double dp = wk - L.w(k - 1, a);
        const double dn = L.w(k + 1, a) - wk;
#pragma unroll
        for (int d = 0; d < 3; ++d) y[d][a] = fp[d] * dp + fn[d] * dn;
    }
    if (HAS_ED && k == 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                const double c0 = KSE[e][d] * pp[5 - d - e];
#pragma unroll
                for (int a = 0; a < 3; ++a) y[d][a] -= c0 * u0[e][a];
            }
    }
}

// C_i = H_{i, i+1} = KSE r_i^(5-d-e) (start derivative d of segment i x end derivative e).
__device__ __forceinline__ void coupling(const double (&p)[8], double (&B)[3][3]) {
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int e = 0; e < 3; ++e) B[d][e] = KSE[d][e] * p[5 - d - e];
}

// ---------------------------------------------------------------------------
// One trajectory on a lane pair.  Invalid trajectories were replaced by an
// all-zero, unit-time one during staging, so they come out as exact zeros.
// Returns the status (meaningful on both lanes).
template <int M, bool HAS_ED>
__device__ __forceinline__ int32_t pair_solve(const LaneView& L, bool right, bool valid,
                                              const double* __restrict__ ed, const OutCtx& O) {
    // virtual-frame end derivatives: even lane (u0, uM); odd lane (P uM, P u0)
    double u0[3][3], uM[3][3];  // [derivative][axis]
    const double sg = right ? -1.0 : 1.0;
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double s0 = (HAS_ED && valid) ? ed[d * 3 + a] : 0.0;
            const double s1 = (HAS_ED && valid) ? ed[9 + d * 3 + a] : 0.0;
            const double f = (d == 1) ? 1.0 : sg;
            u0[d][a] = right ? f * s1 : s0;
            uM[d][a] = right ? f * s0 : s1;
        }
    bool spd = true;
    double fin = 0.0;  // sum of the solved knot derivatives (non-finite check)

#ifdef TGMS_ABL_NOCOMPUTE  // ablation: staging + emission only, knot derivatives = 0
    if constexpr (true) {
#pragma unroll
        for (int e = 0; e < (M + 1) / 2; ++e) emit_virtual<M>(O, L, right, e, u0, uM, e < M / 2);
    } else
#endif
    if constexpr (M == 1) {
        emit_virtual<M>(O, L, right, 0, u0, uM, false);
    } else if constexpr (M == 2) {
        // one interior knot: virtual knot 1 on both lanes (physical 1 for both)
        double pp[8], pn[8], y[3][3], x[3][3];
        rpowers(L.r(0), pp);
        rpowers(L.r(1), pn);
        const Sym3 D = knot_diag(pp, pn);
        knot_rhs<HAS_ED>(L, 1, pp, pn, u0, y);
        if (HAS_ED) {  // final derivatives through C_1 (virtual segment 1)
            double C1[3][3];
            coupling(pn, C1);
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) y[d][a] -= C1[d][0] * uM[0][a] + C1[d][1] * uM[1][a] + C1[d][2] * uM[2][a];
        }
        const Ldl3 f = ldl3s(D, spd);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            ldl3_solve(f, y[0][a], y[1][a], y[2][a], x[0][a], x[1][a], x[2][a]);
            fin += (x[0][a] + x[1][a]) + x[2][a];
        }
        emit_virtual<M>(O, L, right, 0, u0, x, true);
    } else {
        constexpr int c = (M - 1) / 2;  // even chain: knots 1..c, odd chain: M-1..c+1
        constexpr int nL = c, nR = M - 1 - c, NS = nR;
        const int nl = right ? nR : nL;
        Ldl3 F[NS];
        double Y[NS + 1][3][3];  // chain right-hand sides, then knot derivatives; Y[nl] = other interface knot
        Sym3 Dl;
        MARK(chain);
        // ---- elimination along the lane's virtual chain, knots 1..nl ----
        double pp[8], pn[8];  // powers of r of the segments left / right of the current knot
        rpowers(L.r(0), pp);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            SCHED_FENCE();
            const int k = s + 1;
            rpowers(L.r(k), pn);
            Sym3 D = knot_diag(pp, pn);
            double y[3][3];
            knot_rhs<HAS_ED>(L, k, pp, pn, u0, y);
            if (s >= 1) {
                double B[3][3], Wc[3][3];
                coupling(pp, B);  // H_{k-1, k}
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double v0, v1, v2;
                    ldl3_solve(F[s - 1], Y[s - 1][0][a], Y[s - 1][1][a], Y[s - 1][2][a], v0, v1, v2);
#pragma unroll
                    for (int d = 0; d < 3; ++d) y[d][a] -= B[0][d] * v0 + B[1][d] * v1 + B[2][d] * v2;
                }
#pragma unroll
                for (int e = 0; e < 3; ++e) ldl3_solve(F[s - 1], B[0][e], B[1][e], B[2][e], Wc[0][e], Wc[1][e], Wc[2][e]);
                sym_sub_btw(D, B, Wc);
            }
            bool ok;
            F[s] = ldl3s(D, ok);
            spd = spd && (ok || s >= nl);
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) Y[s][d][a] = y[d][a];
            if (s == nL - 1) Dl = D;
            if (nR > nL && s == nR - 1) {
                Dl.a00 = right ? D.a00 : Dl.a00;
                Dl.a01 = right ? D.a01 : Dl.a01;
                Dl.a02 = right ? D.a02 : Dl.a02;
                Dl.a11 = right ? D.a11 : Dl.a11;
                Dl.a12 = right ? D.a12 : Dl.a12;
                Dl.a22 = right ? D.a22 : Dl.a22;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) pp[q] = pn[q];
        }
        MARK(interface);
        SCHED_FENCE();
        // ---- interface: physical knots c (even chain's last) and c+1 (odd's) ----
        // Each lane maps its last pivot block / right-hand side to the physical frame
        // (P flips exactly), the even and odd lane broadcast theirs, and both lanes
        // solve the same 6x6 system with bit-identical operations: x_c by the Schur
        // complement onto knot c, then x_{c+1} back-solved from it.  (Two independent
        // Schur solves leave x_c / x_{c+1} mutually inconsistent: ~70x less accurate.)
        double xm[3][3];
        {
            Sym3 DL, DR;
            {
                const double p01 = sg * Dl.a01, p12 = sg * Dl.a12;
                DL = Sym3{pair_even(Dl.a00), pair_even(p01), pair_even(Dl.a02),
                          pair_even(Dl.a11), pair_even(p12), pair_even(Dl.a22)};
                DR = Sym3{pair_odd(Dl.a00), pair_odd(p01), pair_odd(Dl.a02),
                          pair_odd(Dl.a11), pair_odd(p12), pair_odd(Dl.a22)};
            }
            double Cc[3][3];  // H_{c, c+1}: physical segment c = virtual segment nl on both lanes
            {
                double pc[8];
                rpowers(L.r(nl), pc);
                coupling(pc, Cc);
            }
            bool ok1, ok2;
            const Ldl3 FR = ldl3s(DR, ok1);
            {
                double Wm[3][3];
#pragma unroll
                for (int e = 0; e < 3; ++e) ldl3_solve(FR, Cc[e][0], Cc[e][1], Cc[e][2], Wm[0][e], Wm[1][e], Wm[2][e]);
                DL.a00 -= Cc[0][0] * Wm[0][0] + Cc[0][1] * Wm[1][0] + Cc[0][2] * Wm[2][0];
                DL.a01 -= Cc[0][0] * Wm[0][1] + Cc[0][1] * Wm[1][1] + Cc[0][2] * Wm[2][1];
                DL.a02 -= Cc[0][0] * Wm[0][2] + Cc[0][1] * Wm[1][2] + Cc[0][2] * Wm[2][2];
                DL.a11 -= Cc[1][0] * Wm[0][1] + Cc[1][1] * Wm[1][1] + Cc[1][2] * Wm[2][1];
                DL.a12 -= Cc[1][0] * Wm[0][2] + Cc[1][1] * Wm[1][2] + Cc[1][2] * Wm[2][2];
                DL.a22 -= Cc[2][0] * Wm[0][2] + Cc[2][1] * Wm[1][2] + Cc[2][2] * Wm[2][2];
            }
            const Ldl3 FS = ldl3s(DL, ok2);
            spd = spd && ok1 && ok2;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double yL[3], yR[3];
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    // this lane's last chain right-hand side Y[nl-1], in the physical frame
                    const double yv = (nR > nL) ? (right ? Y[NS - 1][d][a] : Y[nL - 1][d][a]) : Y[nL - 1][d][a];
                    const double yp = (d == 1) ? yv : sg * yv;
                    yL[d] = pair_even(yp);
                    yR[d] = pair_odd(yp);
                }
                double g0, g1, g2;
                ldl3_solve(FR, yR[0], yR[1], yR[2], g0, g1, g2);
#pragma unroll
                for (int d = 0; d < 3; ++d) yL[d] -= Cc[d][0] * g0 + Cc[d][1] * g1 + Cc[d][2] * g2;
                double xc0, xc1, xc2, x10, x11, x12;
                ldl3_solve(FS, yL[0], yL[1], yL[2], xc0, xc1, xc2);
                const double b0 = yR[0] - (Cc[0][0] * xc0 + Cc[1][0] * xc1 + Cc[2][0] * xc2);
                const double b1 = yR[1] - (Cc[0][1] * xc0 + Cc[1][1] * xc1 + Cc[2][1] * xc2);
                const double b2 = yR[2] - (Cc[0][2] * xc0 + Cc[1][2] * xc1 + Cc[2][2] * xc2);
                ldl3_solve(FR, b0, b1, b2, x10, x11, x12);
                // own / other interface knot in the lane's virtual frame
                xm[0][a] = right ? -x10 : xc0;
                xm[1][a] = right ? x11 : xc1;
                xm[2][a] = right ? -x12 : xc2;
                const double o0 = right ? -xc0 : x10, o1 = right ? xc1 : x11, o2 = right ? -xc2 : x12;
                if (nR > nL) {  // the other knot goes to slot nl: nL (even) / nR (odd)
                    Y[nL][0][a] = right ? Y[nL][0][a] : o0;
                    Y[nL][1][a] = right ? Y[nL][1][a] : o1;
                    Y[nL][2][a] = right ? Y[nL][2][a] : o2;
                    Y[nR][0][a] = right ? o0 : Y[nR][0][a];
                    Y[nR][1][a] = right ? o1 : Y[nR][1][a];
                    Y[nR][2][a] = right ? o2 : Y[nR][2][a];
                } else {
                    Y[nL][0][a] = o0;
                    Y[nL][1][a] = o1;
                    Y[nL][2][a] = o2;
                }
                fin += (xc0 + xc1) + (xc2 + x10) + (x11 + x12);
            }
        }
        MARK(backsub);
        // ---- back substitution along the virtual chain: x_s = F_s^{-1}(y_s - C_{s+1} x_{s+1}) ----
#pragma unroll
        for (int s = NS - 1; s >= 0; --s) {
            SCHED_FENCE();
            const bool at_end = (s == nl - 1);
            const bool inside = (s < nl - 1);
            if (s + 1 < NS) {
                double B[3][3];
                {
                    double pb[8];
                    rpowers(L.r(s + 1), pb);
                    coupling(pb, B);  // H_{s+1, s+2} (virtual knots)
                }
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double b[3], x0, x1, x2;
#pragma unroll
                    for (int d = 0; d < 3; ++d)
                        b[d] = Y[s][d][a] - (B[d][0] * Y[s + 1][0][a] + B[d][1] * Y[s + 1][1][a] + B[d][2] * Y[s + 1][2][a]);
                    ldl3_solve(F[s], b[0], b[1], b[2], x0, x1, x2);
                    Y[s][0][a] = at_end ? xm[0][a] : (inside ? x0 : Y[s][0][a]);
                    Y[s][1][a] = at_end ? xm[1][a] : (inside ? x1 : Y[s][1][a]);
                    Y[s][2][a] = at_end ? xm[2][a] : (inside ? x2 : Y[s][2][a]);
                    fin += inside ? (x0 + x1) + x2 : 0.0;
                }
            } else {
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int a = 0; a < 3; ++a) Y[s][d][a] = at_end ? xm[d][a] : Y[s][d][a];
            }
        }
        MARK(emission);
#ifdef TGMS_ABL_NOEMIT  // ablation (register study): consume the knot derivatives, emit nothing
#pragma unroll
        for (int e = 0; e <= NS; ++e)
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) asm volatile("" ::"v"(Y[e][d][a]));
#else
        // ---- coefficients: virtual segment e = virtual knots e..e+1 ----
        constexpr int NE = nL + 1;  // even lane: nL+1 segments; odd lane: nR (<= nL+1)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            SCHED_FENCE();
            double xs[3][3];
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) xs[d][a] = (e == 0) ? u0[d][a] : Y[e >= 1 ? e - 1 : 0][d][a];
            emit_virtual<M>(O, L, right, e, xs, Y[e], e < nR);
        }
#endif
    }
    // combine the pair's flags
    const bool spd_pair = spd && (pair_swap(spd ? 1.0 : 0.0) != 0.0);
    const double fin_pair = fin + pair_swap(fin);
    if (!valid) return TGMS_ERR_INVALID_ARG;
    if (!spd_pair) return TGMS_ERR_SINGULAR;
    if (!finite(fin_pair)) return TGMS_ERR_NONFINITE;
    return TGMS_OK;
}

// ---------------------------------------------------------------------------
// Staging.

template <int M>
__device__ __forceinline__ void stage_row_w(Stage<M>& sm, int t, int q, double v) {
    sm.W[q * PSTRIDE + t] = v;
    if (!finite(v)) atomicOr(&sm.bad[t], 1);
}
template <int M>
__device__ __forceinline__ void stage_row_t(Stage<M>& sm, int t, int q, double v) {
    sm.T[q * PSTRIDE + t] = v;
    sm.R[q * PSTRIDE + t] = fast_rcp(v);
    if (!finite_pos(v)) atomicOr(&sm.bad[t], 1);
}

// Invalid trajectories are replaced by an all-zero, unit-time one (whose solution
// is exactly zero), so the solver needs no per-coefficient masking.  Rare path.
template <int M>
__device__ __forceinline__ void sanitize(Stage<M>& sm, int lane) {
    if (lane < TPW && sm.bad[lane]) {
        for (int q = 0; q < (M + 1) * 3; ++q) sm.W[q * PSTRIDE + lane] = 0.0;
        for (int q = 0; q < M; ++q) {
            sm.T[q * PSTRIDE + lane] = 1.0;
            sm.R[q * PSTRIDE + lane] = 1.0;
        }
    }
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_MIN_WAVES) void k_reduced_uniform(int32_t B, const double* __restrict__ W,
                                                                        const double* __restrict__ T,
                                                                        const double* __restrict__ ED,
                                                                        double* __restrict__ C,
                                                                        int32_t* __restrict__ status) {
    constexpr int NW = (M + 1) * 3;
    __shared__ Stage<M> sm;
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * TPW;
    const int nb = (int)((B - b0) < TPW ? (B - b0) : TPW);
    if (lane < TPW) {
        sm.bad[lane] = 0;
        sm.base[lane] = (b0 + lane) * (24 * M);
    }
    __syncthreads();
#ifndef TGMS_ABL_NOLOAD  // ablation: skip the input loads (LDS holds garbage)
    // The wave's trajectories are contiguous in HBM: 16-B loads across the wave, all
    // issued before the first use (one memory round trip), then transposed into LDS.
    constexpr int NW2 = (TPW * NW / 2 + W64 - 1) / W64;  // double2 loads per lane, waypoints
    constexpr int NT2 = (TPW * M / 2 + W64 - 1) / W64;   // double2 loads per lane, times
    const double2* gW2 = reinterpret_cast<const double2*>(W + b0 * NW);
    const double2* gT2 = reinterpret_cast<const double2*>(T + b0 * M);
    const int nw = nb * NW, nt = nb * M;  // doubles present in this wave's block
    double2 wv[NW2], tv[NT2];
    if (nb == TPW) {
#pragma unroll
        for (int i = 0; i < NW2; ++i)
            if ((TPW * NW) % 128 == 0 || 2 * (lane + W64 * i) < TPW * NW) wv[i] = gW2[lane + W64 * i];
#pragma unroll
        for (int i = 0; i < NT2; ++i)
            if ((TPW * M) % 128 == 0 || 2 * (lane + W64 * i) < TPW * M) tv[i] = gT2[lane + W64 * i];
    } else {  // tail block: element-wise bounds
        const double* gW = W + b0 * NW;
        const double* gT = T + b0 * M;
#pragma unroll
        for (int i = 0; i < NW2; ++i) {
            const int e = 2 * (lane + W64 * i);
            wv[i].x = (e < nw) ? gW[e] : 0.0;
            wv[i].y = (e + 1 < nw) ? gW[e + 1] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NT2; ++i) {
            const int e = 2 * (lane + W64 * i);
            tv[i].x = (e < nt) ? gT[e] : 1.0;
            tv[i].y = (e + 1 < nt) ? gT[e + 1] : 1.0;
        }
    }
#pragma unroll
    for (int i = 0; i < NW2; ++i) {
        const int e = 2 * (lane + W64 * i);
        if (e < nw) {
            const int t0 = e / NW, q0 = e - t0 * NW;
            stage_row_w(sm, t0, q0, wv[i].x);
            const int t1 = (e + 1) / NW, q1 = e + 1 - t1 * NW;
            if (e + 1 < nw) stage_row_w(sm, t1, q1, wv[i].y);
        }
    }
#pragma unroll
    for (int i = 0; i < NT2; ++i) {
        const int e = 2 * (lane + W64 * i);
        if (e < nt) {
            stage_row_t(sm, e / M, e % M, tv[i].x);
            if (e + 1 < nt) stage_row_t(sm, (e + 1) / M, (e + 1) % M, tv[i].y);
        }
    }
#endif
    __syncthreads();
    sanitize(sm, lane);
    __syncthreads();
    // Every lane runs to the end (the output stage needs the whole wave); pairs
    // beyond nb compute on stale LDS and store nothing.
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const bool live = slot < nb;
    const int64_t b = b0 + slot;
    const bool valid = sm.bad[slot] == 0;
    const LaneView L = make_view<M>(sm, slot, right);
    const OutCtx O = make_out(sm.O, sm.base, C, nb, lane);
    const int32_t st = pair_solve<M, HAS_ED>(L, right, valid, (HAS_ED && live) ? ED + b * 18 : ED, O);
    if (live && !right && status) status[b] = st;
}

// Ragged batches: one launch per segment count M over the trajectories `perm`.
template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_MIN_WAVES) void k_reduced_ragged(int32_t n, const int32_t* __restrict__ perm,
                                                                       const int32_t* __restrict__ seg_offsets,
                                                                       const double* __restrict__ W,
                                                                       const double* __restrict__ T,
                                                                       const double* __restrict__ ED,
                                                                       double* __restrict__ C,
                                                                       int32_t* __restrict__ status) {
    constexpr int NW = (M + 1) * 3;
    __shared__ Stage<M> sm;
    const int lane = threadIdx.x;
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const int64_t i0 = (int64_t)blockIdx.x * TPW;
    const int nb = (int)((n - i0) < TPW ? (n - i0) : TPW);
    const bool live = slot < nb;
    if (lane < TPW) {
        sm.bad[lane] = 0;
        sm.base[lane] = 0;
    }
    __syncthreads();
    int32_t b = 0;
    if (live) {
        b = perm[i0 + slot];
        const int64_t s0 = seg_offsets[b];
        if (!right) sm.base[slot] = s0 * 24;
        const double* gW = W + (s0 + b) * 3;
        // the two lanes of a pair split the trajectory's rows
        for (int q = right; q < NW; q += 2) stage_row_w(sm, slot, q, gW[q]);
        for (int q = right; q < M; q += 2) stage_row_t(sm, slot, q, T[s0 + q]);
    }
    __syncthreads();
    sanitize(sm, lane);
    __syncthreads();
    const bool valid = sm.bad[slot] == 0;
    const LaneView L = make_view<M>(sm, slot, right);
    const OutCtx O = make_out(sm.O, sm.base, C, nb, lane);
    const int32_t st = pair_solve<M, HAS_ED>(L, right, valid, (HAS_ED && live) ? ED + (int64_t)b * 18 : ED, O);
    if (live && !right && status) status[b] = st;
}

template <int M>
hipError_t uniform_M(int32_t B, const double* W, const double* T, const double* ED, double* C, int32_t* status,
                     hipStream_t stream) {
    const unsigned grid = (unsigned)((B + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    if (ED)
        hipLaunchKernelGGL((k_reduced_uniform<M, true>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status);
    else
        hipLaunchKernelGGL((k_reduced_uniform<M, false>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status);
    return hipGetLastError();
}

template <int M>
hipError_t ragged_M(int32_t n, const int32_t* perm, const int32_t* so, const double* W, const double* T,
                    const double* ED, double* C, int32_t* status, hipStream_t stream) {
    const unsigned grid = (unsigned)((n + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    if (ED)
        hipLaunchKernelGGL((k_reduced_ragged<M, true>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C,
                           status);
    else
        hipLaunchKernelGGL((k_reduced_ragged<M, false>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C,
                           status);
    return hipGetLastError();
}

}  // namespace

#ifdef TGMS_ONLY_M  // compile-only experiments: instantiate a single M
#define TGMS_CASES(X) X(TGMS_ONLY_M)
#else
#define TGMS_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#endif

hipError_t launch_reduced_uniform(int M, int32_t B, const double* W, const double* T, const double* ED,
                                  double* C, int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return uniform_M<m>(B, W, T, ED, C, status, stream);
        TGMS_CASES(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_reduced_ragged_group(int M, int32_t n, const int32_t* perm, const int32_t* so,
                                       const double* W, const double* T, const double* ED, double* C,
                                       int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return ragged_M<m>(n, perm, so, W, T, ED, C, status, stream);
        TGMS_CASES(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tgms
