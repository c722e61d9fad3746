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
#include <type_traits>

#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {

// Waves per SIMD the register allocation must allow: two for the axis-sequential
// solve while its state fits 256 registers without spilling (M <= 11), else one.
#define TGMS_WAVES(M) ((M) <= TGMS_TWO_WAVE_MAX_M ? 2 : 1)
// The refinement loop's one-wave class as persistent waves sized from the plan (round 6,
// k_refine_loop_dev); TGMS_C5_W1: SIMD time per unit of work of a one-wave tile against a
// two-wave tile (x 100), TGMS_C5_BIAS: the share's bias (%)
#ifndef TGMS_C5_PERSIST
#define TGMS_C5_PERSIST 1
#endif
#ifndef TGMS_C5_W1
#define TGMS_C5_W1 157
#endif
#ifndef TGMS_C5_BIAS
#define TGMS_C5_BIAS 110
#endif
// One-wave-per-SIMD kernels solve the three axes side by side (pair_solve_joint).
// The axis-sequential lane-pair solve reads the next knot's waypoints and 1/T from the
// LDS stage one step ahead (the per-step SCHED_FENCE otherwise exposes the LDS latency at
// every step): config 5 0.477-0.488 -> 0.462-0.473 ms, uniform M = 3/5 -2-3 % (round 4).
// The joint solve does the same (TGMS_JOINT_PREFETCH): the one-wave class timed alone
// 0.232-0.233 -> 0.216-0.220 ms, the whole config-5 call 0.486-0.492 -> 0.477-0.485 ms,
// three alternating runs (round 5, profiles/r05_c5_joint_prefetch_ab.jsonl).
#ifndef TGMS_PAIR_PREFETCH
#define TGMS_PAIR_PREFETCH 1
#endif
#ifndef TGMS_JOINT_PREFETCH
#define TGMS_JOINT_PREFETCH 1
#endif
#ifndef TGMS_JOINT_AXES
#define TGMS_JOINT_AXES 1
#endif
// The refinement gradient in the Legendre basis of the snap (seg_grad_u, round 6); 0: round
// 5's P4..P7 + seg_cost_p form (A/B builds).
#ifndef TGMS_GRAD_LEGENDRE
#define TGMS_GRAD_LEGENDRE 1
#endif

// Scheduling fence between unrolled chain / emission steps.  The compiler-level
// memory clobber also stops CSE of LDS reads across steps: re-reading LDS is far
// cheaper than keeping values live.
#define SCHED_FENCE()                      \
    do {                                   \
        asm volatile("" ::: "memory");     \
        __builtin_amdgcn_sched_barrier(0); \
    } while (0)
#ifdef TGMS_STAMPS  // diagnostic build: per-wave phase timestamps (s_memtime), lane 0
__device__ unsigned long long g_stamps[8192 * 16];
#define STAMP(i)                                                                              \
    do {                                                                                      \
        asm volatile("" ::: "memory");                                                        \
        if (threadIdx.x == 0) g_stamps[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define STAMP_RT(i)                                                                                  \
    do {                                                                                             \
        if (threadIdx.x == 0) {                                                                      \
            g_stamps[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime();            \
            g_stamps[(size_t)blockIdx.x * 16 + 8] = __builtin_amdgcn_s_getreg((3 << 11) | 20);     \
            g_stamps[(size_t)blockIdx.x * 16 + 9] = __builtin_amdgcn_s_getreg((31 << 11) | 4);     \
        }                                                                                            \
    } while (0)
#else
#define STAMP(i) ((void)0)
#define STAMP_RT(i) ((void)0)
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

// The one-wave (joint-axes, M > TGMS_TWO_WAVE_MAX_M) kernels read the stage with no second
// wavefront to hide LDS time, and with the padded stride the two lanes of a pair collide:
// a ds_read_b64 serves lanes 0-31 and 32-63 in one LDS cycle each, i.e. 16 trajectories
// whose even lanes read knot j and odd lanes knot M-j, two 32-bank windows at a distance
// of 2 (F_e - F_o) banks that overlap for almost every j (PMC of the one-wave class alone:
// SQ_LDS_BANK_CONFLICT 2.1x SQ_ACTIVE_INST_LDS).  Swizzled: rows of exactly 32 doubles, and
// the rows of the second half of the trajectory (knot k with 2k > M, segment i with
// 2i + 1 > M) hold trajectory t at column t ^ 16, so in every read the pair's two lanes
// land in opposite bank halves (the middle knot / segment both read is one address).
// Measured (round 5, profiles/r05_c5_swizzle_ab.jsonl): the conflict cycles of the one-wave
// class halve (4.23 M -> 2.15 M per call) but its time does not move (0.213-0.216 ms both
// ways; the whole call 0.481-0.488 vs 0.482-0.493 ms; for every M, where the two-wave
// class spills 2 VGPRs, 0.480-0.490), so it is off.
#ifndef TGMS_PAIR_SWIZZLE
#define TGMS_PAIR_SWIZZLE 0
#endif
#ifndef TGMS_PAIR_SWIZZLE_MIN_M
#define TGMS_PAIR_SWIZZLE_MIN_M (TGMS_TWO_WAVE_MAX_M + 1)
#endif
template <int M>
constexpr bool pair_swz() { return TGMS_PAIR_SWIZZLE && M >= TGMS_PAIR_SWIZZLE_MIN_M; }
template <int M>
constexpr int pstride() { return pair_swz<M>() ? TPW : PSTRIDE; }
template <int M>
__device__ __forceinline__ int w_at(int q, int t) {  // field q = 3 knot + axis, trajectory t
    if constexpr (pair_swz<M>()) return q * TPW + ((2 * (q / 3) > M) ? (t ^ 16) : t);
    else return q * PSTRIDE + t;
}
template <int M>
__device__ __forceinline__ int r_at(int i, int t) {  // segment i, trajectory t
    if constexpr (pair_swz<M>()) return i * TPW + ((2 * i + 1 > M) ? (t ^ 16) : t);
    else return i * PSTRIDE + t;
}

// One group's staged inputs, [field][trajectory] with a padded trajectory stride.
template <int M>
struct In {
    double W[(M + 1) * 3 * pstride<M>()];
    double R[M * pstride<M>()];  // 1/T, computed once while staging (T itself is not staged:
                            // at 2.9 KB for M = 11 it cost the 2-wave kernels their 8th wave per CU)
    int64_t base[TPW];      // coefficient offset (doubles) of each slot's trajectory
    int bad[TPW];
};

template <int M>
struct alignas(16) Stage {
    // First and 16-B aligned: every ds_*_b128 on it must be naturally aligned, or
    // the LDS replays it (SQ_LDS_UNALIGNED_STALL; cdna_hip_programming.md G17).
    alignas(16) double O[W64 * OSTRIDE];  // one axis of one emission step, every lane
    In<M> in;
};

static_assert(OSTRIDE % 2 == 0, "staged rows must keep 16-B alignment");

// Per-lane view of the staged inputs in the lane's VIRTUAL frame: the even lane
// sees the trajectory as is, the odd lane time-reversed (virtual knot j = physical
// knot M-j, virtual segment i = physical segment M-1-i).
struct LaneView {
    const double* Wb;  // &W[phys knot of virtual knot 0][axis 0][slot] for virtual knots 2j < M
    const double* Wf;  // the same for 2j > M and
    const double* Wm;  // 2j == M (all three equal unless the stage is swizzled)
    const double* Rb;  // &R[...], virtual segments 2i + 1 < M,
    const double* Rf;  // > M and
    const double* Rm;  // == M
    int kstep;         // +-3 fields per virtual knot (x the field stride)
    int sstep;         // +-1 segment per virtual segment (x the field stride)
    int astep;         // doubles between the axes of one knot: the field stride (transposed) or 1 (raw)
    int m;             // M
    __device__ __forceinline__ double w(int j, int a) const {
        const double* p = (2 * j < m) ? Wb : ((2 * j > m) ? Wf : Wm);
        return p[j * kstep + a * astep];
    }
    __device__ __forceinline__ double r(int i) const {
        const double* p = (2 * i + 1 < m) ? Rb : ((2 * i + 1 > m) ? Rf : Rm);
        return p[i * sstep];
    }
};

template <int M>
__device__ __forceinline__ LaneView make_view(const In<M>& sm, int slot, bool right) {
    constexpr int S = pstride<M>();
    LaneView L;
    const double* w0 = sm.W + (right ? M * 3 * S : 0);
    const double* r0 = sm.R + (right ? (M - 1) * S : 0);
    // swizzled: the even lane's near half (virtual = physical) is unswizzled, its far half
    // swizzled; the odd lane (virtual knot j = physical M - j) the other way round
    const int sx = pair_swz<M>() ? (slot ^ 16) : slot;
    L.Wb = w0 + (right ? sx : slot);
    L.Wf = w0 + (right ? slot : sx);
    L.Wm = w0 + slot;
    L.Rb = r0 + (right ? sx : slot);
    L.Rf = r0 + (right ? slot : sx);
    L.Rm = r0 + slot;
    L.kstep = right ? -3 * S : 3 * S;
    L.sstep = right ? -S : S;
    L.astep = S;
    L.m = M;
    return L;
}

// Raw layout (uniform batches): the group's inputs exactly as they sit in HBM,
// [trajectory][knot][axis] and [trajectory][segment], copied 16 B per lane with no
// index arithmetic; 1/T replaces T.  Column reads across the 32 slots are
// conflict-free for W (66-dword stride) and at most 2-way for R (20-dword stride).
template <int M, int NT = TPW>
struct RawIn {
    static constexpr int NW = (M + 1) * 3;
    double W[NT * NW];
    double R[NT * M];
    int bad[NT];
};

template <int M>
struct alignas(16) RawStage {
    alignas(16) double O[W64 * OSTRIDE];
    RawIn<M> in;
};

template <int M>
__device__ __forceinline__ LaneView make_view_raw(const RawIn<M>& sm, int slot, bool right) {
    LaneView L;
    L.Wb = L.Wf = L.Wm = sm.W + slot * RawIn<M>::NW + (right ? M * 3 : 0);
    L.Rb = L.Rf = L.Rm = sm.R + slot * M + (right ? M - 1 : 0);
    L.kstep = right ? -3 : 3;
    L.sstep = right ? -1 : 1;
    L.astep = 1;
    L.m = M;
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
            *reinterpret_cast<double2*>(o.dst[q] + (o.rt[q] ? offR : offL)) = v;
        }
    };
    put(0, v0);
    put(1, v1);
    put(2, v2);
    put(3, v3);
}

// Uniform batches: the wave's 32 trajectories are one contiguous block of C, so
// the four pieces a lane stores sit at fixed distances (8 trajectories apart) and
// each gets its own buffer resource over the block.  One 32-bit offset per lane
// then addresses every store, and the resources' range check drops the pieces of
// trajectories beyond the batch (tail group) without any branch.
struct OutBuf {
    double* stage;                  // LDS [W64][OSTRIDE]
    __amdgpu_buffer_rsrc_t rs[4];   // piece q: trajectories 8q .. of the wave's block
    uint32_t voff0;                 // byte offset of the lane's piece, emission step 0, axis 0
    int32_t estep;                  // +-1 segment (192 B) per emission step
    bool rt;                        // the lane's pieces were staged by odd (right) lanes
    bool nt;                        // streaming stores (the batch's output exceeds the Infinity Cache)
    int lane;
};

template <int M>
__device__ __forceinline__ OutBuf make_out_buf(double* stage, double* C, int64_t b0, int nb, int lane,
                                               bool nt = false) {
    constexpr int TRAJ_B = M * 24 * 8;  // bytes per trajectory
    OutBuf o;
    o.stage = stage;
    o.lane = lane;
    o.nt = nt;
    double* base = C + b0 * (M * 24);
    const int block = nb * TRAJ_B;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int lim = block - q * 8 * TRAJ_B;
        o.rs[q] = __builtin_amdgcn_make_buffer_rsrc(base + (int64_t)q * 8 * M * 24, (short)0, lim > 0 ? lim : 0,
                                                    0x00020000);
    }
    o.rt = (lane >> 2) & 1;
    o.voff0 = (uint32_t)((lane >> 3) * TRAJ_B + (o.rt ? (M - 1) * 192 : 0) + (lane & 3) * 16);
    o.estep = o.rt ? -192 : 192;
    return o;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Cache policy of the coefficient stores (gfx950: sc0 = 1, nt = 2, sc1 = 16).  A batch
// whose output stays in the 256 MB Infinity Cache (config 3: 126 MB) wants sc1
// (28.2 -> 26.9 us; nt 41 us there); one whose output does not (config 4's 131,072
// per GPU: 252 MB) wants sc1|nt (92 -> 74 us with a fresh batch every launch).
#ifndef TGMS_STORE_CPOL
#define TGMS_STORE_CPOL 16
#endif
#ifndef TGMS_STORE_CPOL_NT
#define TGMS_STORE_CPOL_NT 18
#endif
constexpr int64_t kStreamingOutputBytes = 192ll << 20;

// Stage one axis of every lane's current segment, then store it (OutBuf version;
// `voff` is the lane's piece offset at this emission step).
__device__ __forceinline__ void stage_axis(const OutBuf& o, const double (&c)[8], int a, uint32_t voff,
                                           bool has_r) {
    wave_lds_sync();  // previous readers are done with the stage
    double2* d = reinterpret_cast<double2*>(o.stage + o.lane * OSTRIDE);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = make_double2(c[2 * j], c[2 * j + 1]);
    wave_lds_sync();
    auto piece = [&](int q) {
        const int p = o.lane + W64 * q;
        return *reinterpret_cast<const double2*>(o.stage + (p >> 2) * OSTRIDE + (p & 3) * 2);
    };
    const double2 v0 = piece(0), v1 = piece(1), v2 = piece(2), v3 = piece(3);
    const uint32_t off = (has_r || !o.rt) ? voff : 0x80000000u;  // idle odd rows: out of range
    if (o.nt) {  // wave-uniform
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), o.rs[0], off, a * 64, TGMS_STORE_CPOL_NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v1), o.rs[1], off, a * 64, TGMS_STORE_CPOL_NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v2), o.rs[2], off, a * 64, TGMS_STORE_CPOL_NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v3), o.rs[3], off, a * 64, TGMS_STORE_CPOL_NT);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), o.rs[0], off, a * 64, TGMS_STORE_CPOL);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v1), o.rs[1], off, a * 64, TGMS_STORE_CPOL);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v2), o.rs[2], off, a * 64, TGMS_STORE_CPOL);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v3), o.rs[3], off, a * 64, TGMS_STORE_CPOL);
    }
}

// Output address of emission step e for either output context.
__device__ __forceinline__ uint32_t out_step(const OutBuf& o, int e) { return o.voff0 + e * o.estep; }
__device__ __forceinline__ int out_step(const OutCtx&, int e) { return e; }

// ---------------------------------------------------------------------------
// Block algebra.

// ---------------------------------------------------------------------------
// The lane-pair kernels solve the reduced system in scaled knot unknowns x' = S^-1 x,
// S = diag(21, 3, 1) on (v, a, j) (round 6): every block becomes S H S.  KSE factors as
// a_d b_e c_(d+e) with a = (1, 1, 3/7), b = (1, -1, 3/7), so the scaled coupling
// S C_i S is the signed Hankel matrix [sigma_e q_(d+e)], sigma = (+, -, +), of the five
// numbers q_k = HNK_k r_i^(5-k): 5 multiplies per coupling instead of 9 (the signs fold into
// the consuming FMAs), integer constants throughout.  Factorisation, substitutions and the
// interface keep their form; the emission and the gradient fold 21 and 3 into their
// constants, and the given end derivatives are scaled once on load.  TGMS_PAIR_SCALED=0
// solves the unscaled system (A/B builds).  The lane kernel (k_lane_uniform) is unscaled.
#ifndef TGMS_PAIR_SCALED
#define TGMS_PAIR_SCALED 1
#endif
#if TGMS_PAIR_SCALED
constexpr double PSV = 21.0, PSA = 3.0;  // v = 21 v', a = 3 a', j = j'
__device__ constexpr double pKSS[3][3] = {{11430720, 340200, 10080}, {340200, 10800, 360}, {10080, 360, 16}};
__device__ constexpr double pKEE[3][3] = {{11430720, -340200, 10080}, {-340200, 10800, -360}, {10080, -360, 16}};
__device__ constexpr double pKSE[3][3] = {{10795680, -294840, 7560}, {294840, -7560, 180}, {7560, -180, 4}};
__device__ constexpr double pKSP[3] = {-1058400, -30240, -840};
__device__ constexpr double pKEP[3] = {-1058400, 30240, -840};
#else
constexpr double PSV = 1.0, PSA = 1.0;
__device__ constexpr double pKSS[3][3] = {{25920, 5400, 480}, {5400, 1200, 120}, {480, 120, 16}};
__device__ constexpr double pKEE[3][3] = {{25920, -5400, 480}, {-5400, 1200, -120}, {480, -120, 16}};
__device__ constexpr double pKSE[3][3] = {{24480, -4680, 360}, {4680, -840, 60}, {360, -60, 4}};
__device__ constexpr double pKSP[3] = {-50400, -10080, -840};
__device__ constexpr double pKEP[3] = {-50400, 10080, -840};
#endif
constexpr double PSI[3] = {1.0 / PSV, 1.0 / PSA, 1.0};  // x' = x * PSI (end derivatives on load)

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
    const double fp[3] = {-pKEP[0] * pp[6], -pKEP[1] * pp[5], -pKEP[2] * pp[4]};
    const double fn[3] = {-pKSP[0] * pn[6], -pKSP[1] * pn[5], -pKSP[2] * pn[4]};
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
                const double c0 = pKSE[e][d] * pp[5 - d - e];
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

__device__ __forceinline__ Sym3 knot_diag_p(const double (&pp)[8], const double (&pn)[8]) {
    Sym3 D;
    D.a00 = pKEE[0][0] * pp[5] + pKSS[0][0] * pn[5];
    D.a01 = pKEE[0][1] * pp[4] + pKSS[0][1] * pn[4];
    D.a02 = pKEE[0][2] * pp[3] + pKSS[0][2] * pn[3];
    D.a11 = pKEE[1][1] * pp[3] + pKSS[1][1] * pn[3];
    D.a12 = pKEE[1][2] * pp[2] + pKSS[1][2] * pn[2];
    D.a22 = pKEE[2][2] * pp[1] + pKSS[2][2] * pn[1];
    return D;
}

__device__ __forceinline__ void coupling_p(const double (&p)[8], double (&B)[3][3]) {
#if TGMS_PAIR_SCALED
    const double q0 = 10795680.0 * p[5], q1 = 294840.0 * p[4], q2 = 7560.0 * p[3], q3 = 180.0 * p[2];
    const double q4 = 4.0 * p[1];
    B[0][0] = q0;
    B[0][1] = -q1;
    B[0][2] = q2;
    B[1][0] = q1;
    B[1][1] = -q2;
    B[1][2] = q3;
    B[2][0] = q2;
    B[2][1] = -q3;
    B[2][2] = q4;
#else
    coupling(p, B);
#endif
}

// ---------------------------------------------------------------------------
// One trajectory on a lane pair.  Invalid trajectories were replaced by an
// all-zero, unit-time one during staging, so they come out as exact zeros.
template <int M>
struct Chain {
    static constexpr int c = (M - 1) / 2;  // even chain: knots 1..c, odd chain: M-1..c+1
    static constexpr int nL = c, nR = M - 1 - c, NS = nR;
    static constexpr int NE = nL + 1;      // emission steps (even lane: nL+1 segments, odd: nR)
};

// ---------------------------------------------------------------------------
// Axis-sequential solve (default for M >= 3).  The 3x3 block factorisation is
// shared by the three axes, but the right-hand sides are not: factor once, then
// run forward substitution, interface, back substitution and emission one axis at
// a time.  Only the factors and ONE axis' knot derivatives are live at once
// (~100 doubles per lane instead of ~160), which lets two waves share a SIMD:
// one wave's FP64 dependency chains, LDS round trips and store stalls are hidden
// behind the other's work.  Same arithmetic, in the same order per axis, as the
// joint solve above.
template <int M>
struct AxFactors {
    Ldl3 F[Chain<M>::NS];
    Ldl3 FR, FS;       // interface: odd-side pivot block, Schur complement onto knot c
    double Cc[3][3];   // H_{c, c+1}
    bool spd;
};

template <int M>
__device__ __forceinline__ void ax_factor(AxFactors<M>& Fa, const LaneView& L, bool right) {
    using CH = Chain<M>;
    constexpr int nL = CH::nL, nR = CH::nR, NS = CH::NS;
    const int nl = right ? nR : nL;
    const double sg = right ? -1.0 : 1.0;
    Fa.spd = true;
    Sym3 Dl;
    double pp[8];
    rpowers(L.r(0), pp);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        SCHED_FENCE();
        const int k = s + 1;
        double pn[8];
        rpowers(L.r(k), pn);
        Sym3 D = knot_diag_p(pp, pn);
        if (s >= 1) {
            double B[3][3], Wc[3][3];
            coupling_p(pp, B);  // H_{k-1, k}
#pragma unroll
            for (int e = 0; e < 3; ++e)
                ldl3_solve(Fa.F[s - 1], B[0][e], B[1][e], B[2][e], Wc[0][e], Wc[1][e], Wc[2][e]);
            sym_sub_btw(D, B, Wc);
        }
        bool ok;
        Fa.F[s] = ldl3s(D, ok);
        Fa.spd = Fa.spd && (ok || s >= nl);
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
    SCHED_FENCE();
    // interface blocks in the physical frame, broadcast from both lanes of the pair
    Sym3 DL, DR;
    {
        const double p01 = sg * Dl.a01, p12 = sg * Dl.a12;
        DL = Sym3{pair_even(Dl.a00), pair_even(p01), pair_even(Dl.a02),
                  pair_even(Dl.a11), pair_even(p12), pair_even(Dl.a22)};
        DR = Sym3{pair_odd(Dl.a00), pair_odd(p01), pair_odd(Dl.a02),
                  pair_odd(Dl.a11), pair_odd(p12), pair_odd(Dl.a22)};
    }
    {
        double pc[8];
        rpowers(L.r(nl), pc);  // physical segment c = virtual segment nl on both lanes
        coupling_p(pc, Fa.Cc);
    }
    bool ok1, ok2;
    Fa.FR = ldl3s(DR, ok1);
    {
        double Wm[3][3];
#pragma unroll
        for (int e = 0; e < 3; ++e)
            ldl3_solve(Fa.FR, Fa.Cc[e][0], Fa.Cc[e][1], Fa.Cc[e][2], Wm[0][e], Wm[1][e], Wm[2][e]);
        const double(&Cc)[3][3] = Fa.Cc;
        DL.a00 -= Cc[0][0] * Wm[0][0] + Cc[0][1] * Wm[1][0] + Cc[0][2] * Wm[2][0];
        DL.a01 -= Cc[0][0] * Wm[0][1] + Cc[0][1] * Wm[1][1] + Cc[0][2] * Wm[2][1];
        DL.a02 -= Cc[0][0] * Wm[0][2] + Cc[0][1] * Wm[1][2] + Cc[0][2] * Wm[2][2];
        DL.a11 -= Cc[1][0] * Wm[0][1] + Cc[1][1] * Wm[1][1] + Cc[1][2] * Wm[2][1];
        DL.a12 -= Cc[1][0] * Wm[0][2] + Cc[1][1] * Wm[1][2] + Cc[1][2] * Wm[2][2];
        DL.a22 -= Cc[2][0] * Wm[0][2] + Cc[2][1] * Wm[1][2] + Cc[2][2] * Wm[2][2];
    }
    Fa.FS = ldl3s(DL, ok2);
    Fa.spd = Fa.spd && ok1 && ok2;
}

// Right-hand side of virtual knot k for axis a (see knot_rhs).
template <bool HAS_ED>
__device__ __forceinline__ void knot_rhs_axis(const LaneView& L, int k, int a, const double (&pp)[8],
                                              const double (&pn)[8], const double (&u0)[3], double (&y)[3]) {
    const double fp[3] = {-pKEP[0] * pp[6], -pKEP[1] * pp[5], -pKEP[2] * pp[4]};
    const double fn[3] = {-pKSP[0] * pn[6], -pKSP[1] * pn[5], -pKSP[2] * pn[4]};
    const double wk = L.w(k, a);
    const double dp = wk - L.w(k - 1, a);
    const double dn = L.w(k + 1, a) - wk;
#pragma unroll
    for (int d = 0; d < 3; ++d) y[d] = fp[d] * dp + fn[d] * dn;
    if (HAS_ED && k == 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) y[d] -= (pKSE[e][d] * pp[5 - d - e]) * u0[e];
    }
}

// knot_rhs_axis from waypoint values already in registers (wm, wk, wn: knots k-1, k, k+1).
template <bool HAS_ED>
__device__ __forceinline__ void knot_rhs_vals(int k, double wm, double wk, double wn, const double (&pp)[8],
                                              const double (&pn)[8], const double (&u0)[3], double (&y)[3]) {
    const double fp[3] = {-pKEP[0] * pp[6], -pKEP[1] * pp[5], -pKEP[2] * pp[4]};
    const double fn[3] = {-pKSP[0] * pn[6], -pKSP[1] * pn[5], -pKSP[2] * pn[4]};
    const double dp = wk - wm;
    const double dn = wn - wk;
#pragma unroll
    for (int d = 0; d < 3; ++d) y[d] = fp[d] * dp + fn[d] * dn;
    if (HAS_ED && k == 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) y[d] -= (pKSE[e][d] * pp[5 - d - e]) * u0[e];
    }
}

// Coefficients of axis a of virtual segment e (knots e, e+1 with derivatives xs, xe).
// ---------------------------------------------------------------------------
// Time-allocation refinement: instead of storing a
// segment's coefficients, accumulate its snap cost J_i and dJ_i/dT_i.  With the
// knot data held fixed (they are optimal, so by the envelope theorem only the
// explicit dependence on T_i counts) and u = (w r^3, v r^2, a r, j) at both ends,
//   J_i = r u^T KH u,   dJ_i/dT_i = r^2 u^T (KH o (s_a + s_b - 7)) u
// (KH: oracle/minsnap_oracle.c, s = derivative order).  The position entries of
// KH are antisymmetric between the ends, so only D = (w1 - w0) r^3 appears.
template <int NE>
struct GradAcc {
    mutable double J;       // this lane's snap cost (its segments; only the sum is used)
    mutable double dJ[NE];  // per emission step of this lane: d cost / d duration of its segment
};
template <class T>
struct is_grad : std::false_type {};
template <int NE>
struct is_grad<GradAcc<NE>> : std::true_type {};
// The refinement loop's last pass: the coefficients at the final times AND the cost there
// (the sum of this lane's J only) from one solve, instead of a cost pass and a separate
// emission pass.
template <class O>
struct CostOutT {
    O o;
    mutable double J;
};
using CostOut = CostOutT<OutCtx>;
template <class T>
struct is_cost_out : std::false_type {};
template <class O>
struct is_cost_out<CostOutT<O>> : std::true_type {};


// The same J and dJ/dT from the segment's scaled monomial data P4..P7 (c_k = r^(k-3) P_k)
// instead of the Hermite data: with s = t / T the snap is r q(s),
// q = 24 P4 + 120 P5 s + 360 P6 s^2 + 840 P7 s^3, so J = r Q with Q = P^T H P,
// H_kl = a_k a_l / (k + l + 1) for k, l = 0..3 (a = 24, 120, 360, 840; H_33 = 100800, KH's position
// entry).  P is linear in u = (D, V0, A0, J0, V1, A1, J1) whose entries carry r^3, r^2,
// r, 1, r^2, r, 1, so dQ/dr = (2/r) P^T H P' with P' the same map applied to
// (3D, 2V0, A0, 0, 2V1, A1, 0); dJ/dT = -r^2 dJ/dr = r^2 Qd with Qd = -(Q + 2 P'^T H P).
// 47 FP64 operations per axis and segment instead of ~100 for the quadratic form in u
// with KH (round 2; the P4..P7 are computed for the coefficients anyway).  The two agree
// up to rounding (tests/test_refine_oracle.py pins the gradient on the CPU side).
__device__ __forceinline__ void seg_cost_p(double D, double V0, double A0, double V1, double A1, double P4,
                                           double P5, double P6, double P7, double& Q, double& Qd) {
    const double Q4 = 105.0 * D - 40.0 * V0 - 5.0 * A0 - 30.0 * V1 + 2.5 * A1;
    const double Q5 = -252.0 * D + 90.0 * V0 + 10.0 * A0 + 78.0 * V1 - 7.0 * A1;
    const double Q6 = 210.0 * D - 72.0 * V0 - 7.5 * A0 - 68.0 * V1 + 6.5 * A1;
    const double Q7 = -60.0 * D + 20.0 * V0 + 2.0 * A0 + 20.0 * V1 - 2.0 * A1;
    const double H4 = 576.0 * P4 + 1440.0 * P5 + 2880.0 * P6 + 5040.0 * P7;
    const double H5 = 1440.0 * P4 + 4800.0 * P5 + 10800.0 * P6 + 20160.0 * P7;
    const double H6 = 2880.0 * P4 + 10800.0 * P5 + 25920.0 * P6 + 50400.0 * P7;
    const double H7 = 5040.0 * P4 + 20160.0 * P5 + 50400.0 * P6 + 100800.0 * P7;
    Q = P4 * H4 + P5 * H5 + P6 * H6 + P7 * H7;
    const double G = Q4 * H4 + Q5 * H5 + Q6 * H6 + Q7 * H7;
    Qd = -(Q + 2.0 * G);
}
// Round 6: the same Q and Qd in the Legendre basis of the snap, from the scaled end data
// directly (no P4..P7; used by the gradient passes, which need no coefficients).  The Gram
// matrix above factors as H = L L^T with L^T E = diag(1, sqrt3, sqrt5, sqrt7) x an integer
// map, so with
//   g0 = j1 - j0,  g1 = 2 (A0 - A1) + (j0 + j1),  g2 = 12 (V1 - V0) - 6 (A0 + A1) + (j1 - j0),
//   g3 = -120 D + 60 (V0 + V1) + 12 (A0 - A1) + (j0 + j1)
// (the orthonormal shifted-Legendre coefficients of the snap, up to those square roots):
//   Q = g0^2 + 3 g1^2 + 5 g2^2 + 7 g3^2,
//   G = Qv^T H P = 3 g1 d1 + 5 g2 d2 + 7 g3 d3 with d the same map of (3D, 2V0, A0, 0, 2V1, A1, 0),
//   Qd = -(Q + 2 G)
// -- exact integer identities (checked symbolically), ~33 FP64 operations
// per axis and segment instead of ~74 for P4..P7 + seg_cost_p.  V and A arrive in the pair
// kernels' scaled unknowns (V = PSV V', A = PSA A'); the factors fold into the constants.
__device__ __forceinline__ void seg_grad_u(double D, double V0, double A0, double j0, double V1, double A1,
                                           double j1, double& Q, double& Qd) {
    const double sA = A0 - A1, pA = A0 + A1, sJ = j0 + j1, dJ = j1 - j0, sV = V0 + V1, dV = V1 - V0;
    const double g0 = dJ;
    const double g1 = fma(2.0 * PSA, sA, sJ);
    const double g2 = fma(12.0 * PSV, dV, fma(-6.0 * PSA, pA, dJ));
    const double g3 = fma(-120.0, D, fma(60.0 * PSV, sV, fma(12.0 * PSA, sA, sJ)));
    const double e1 = (6.0 * PSA) * sA;                                              // 3 d1
    const double e2 = fma(120.0 * PSV, dV, (-30.0 * PSA) * pA);                      // 5 d2
    const double e3 = fma(-2520.0, D, fma(840.0 * PSV, sV, (84.0 * PSA) * sA));      // 7 d3
    Q = fma(g3, 7.0 * g3, fma(g2, 5.0 * g2, fma(g1, 3.0 * g1, g0 * g0)));
    const double G = fma(g3, e3, fma(g2, e2, g1 * e1));
    Qd = fma(-2.0, G, -Q);
}

// Q alone (the cost at the final times needs no derivative): 20 FP64 operations.
__device__ __forceinline__ double seg_cost_q(double P4, double P5, double P6, double P7) {
    const double H4 = 576.0 * P4 + 1440.0 * P5 + 2880.0 * P6 + 5040.0 * P7;
    const double H5 = 1440.0 * P4 + 4800.0 * P5 + 10800.0 * P6 + 20160.0 * P7;
    const double H6 = 2880.0 * P4 + 10800.0 * P5 + 25920.0 * P6 + 50400.0 * P7;
    const double H7 = 5040.0 * P4 + 20160.0 * P5 + 50400.0 * P6 + 100800.0 * P7;
    return P4 * H4 + P5 * H5 + P6 * H6 + P7 * H7;
}

// Where one axis of segment e goes, per output kind.
template <int M>
__device__ __forceinline__ void emit_c(const OutBuf& o, const double (&c)[8], int a, int e, bool has_r) {
    stage_axis(o, c, a, out_step(o, e), has_r);
}
template <int M>
__device__ __forceinline__ void emit_c(const OutCtx& o, const double (&c)[8], int a, int e, bool has_r) {
    stage_axis(o, c, a, e, M - 1 - e, has_r);
}

template <int M, class Out>
__device__ __forceinline__ void emit_axis_v(const Out& o, double ws, double we, double r, bool right, int e, int a,
                                            const double (&xs)[3], const double (&xe)[3], bool has_r,
                                            bool zero = false) {
#if TGMS_GRAD_LEGENDRE
    if constexpr (is_grad<Out>::value) {
        // The snap cost of a segment and its T-derivative do not change under time reversal
        // (the odd lane's virtual segment is the physical one run backwards, with
        // (D, v, a, j) -> (-D, -v, a, -j) and the ends swapped: g0, g2, d2 keep their sign,
        // g1, g3, d1, d3 flip, and only squares and products of equal parity enter Q and G),
        // so the gradient pass takes the virtual end data as they are: no frame selects.
        const double r2 = r * r, r3 = r2 * r;
        double Q, Qd;
        seg_grad_u((we - ws) * r3, xs[0] * r2, xs[1] * r, xs[2], xe[0] * r2, xe[1] * r, xe[2], Q, Qd);
        const bool mine = has_r || !right;  // the odd lane's last step may duplicate the even lane's
        o.J += mine ? r * Q : 0.0;
        o.dJ[e] += mine ? r2 * Qd : 0.0;
        // anchored here: nothing stores these sums until the step's update, so without
        // the anchor the compiler sinks every segment's cost arithmetic (and keeps all
        // knot data live for it) to the end of the solve
        asm volatile("" : "+v"(o.J), "+v"(o.dJ[e]));
        return;
    }
#endif
    const double w0 = right ? we : ws, w1 = right ? ws : we;
    // the odd lane runs the segment backwards: physical start = virtual knot e+1, with P
    const double v0 = right ? -xe[0] : xs[0], a0 = right ? xe[1] : xs[1], j0 = right ? -xe[2] : xs[2];
    const double v1 = right ? -xs[0] : xe[0], a1 = right ? xs[1] : xe[1], j1 = right ? -xs[2] : xe[2];
    // Hermite -> monomial in r = 1/T scaled variables (no T needed):
    //   c4 = r P4, c5 = r^2 P5, c6 = r^3 P6, c7 = r^4 P7 with P linear in
    //   D = (w1 - w0) r^3, V = v r^2, A = a r, J = j at both ends.
    const double r2 = r * r, r3 = r2 * r, r4 = r2 * r2;
    const double D = (w1 - w0) * r3;
    const double V0 = v0 * r2, A0 = a0 * r, V1 = v1 * r2, A1 = a1 * r;  // scaled: x PSV, x PSA
    const double P4 = 35.0 * D - (20.0 * PSV) * V0 - (5.0 * PSA) * A0 - (2.0 / 3.0) * j0 - (15.0 * PSV) * V1 +
                      (2.5 * PSA) * A1 - (1.0 / 6.0) * j1;
    const double P5 = -84.0 * D + (45.0 * PSV) * V0 + (10.0 * PSA) * A0 + j0 + (39.0 * PSV) * V1 -
                      (7.0 * PSA) * A1 + 0.5 * j1;
    const double P6 = 70.0 * D - (36.0 * PSV) * V0 - (7.5 * PSA) * A0 - (2.0 / 3.0) * j0 - (34.0 * PSV) * V1 +
                      (6.5 * PSA) * A1 - 0.5 * j1;
    const double P7 = -20.0 * D + (10.0 * PSV) * V0 + (2.0 * PSA) * A0 + (1.0 / 6.0) * j0 + (10.0 * PSV) * V1 -
                      (2.0 * PSA) * A1 + (1.0 / 6.0) * j1;
#if !TGMS_GRAD_LEGENDRE
    if constexpr (is_grad<Out>::value) {  // round 5's form (A/B builds)
        double Q, Qd;
        seg_cost_p(D, PSV * V0, PSA * A0, PSV * V1, PSA * A1, P4, P5, P6, P7, Q, Qd);
        const bool mine = has_r || !right;  // the odd lane's last step may duplicate the even lane's
        o.J += mine ? r * Q : 0.0;
        o.dJ[e] += mine ? r2 * Qd : 0.0;
        // anchored here: nothing stores these sums until the step's update, so without
        // the anchor the compiler sinks every segment's cost arithmetic (and keeps all
        // knot data live for it) to the end of the solve
        asm volatile("" : "+v"(o.J), "+v"(o.dJ[e]));
        return;
    }
#endif
    if constexpr (!is_grad<Out>::value) {
        double c[8] = {w0, PSV * v0, (0.5 * PSA) * a0, j0 * (1.0 / 6.0), P4 * r, P5 * r2, P6 * r3, P7 * r4};
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = zero ? 0.0 : c[j];  // a failed factorisation: exact zeros
        if constexpr (is_cost_out<Out>::value) {
            const bool mine = has_r || !right;  // as for GradAcc
            o.J += mine ? r * seg_cost_q(P4, P5, P6, P7) : 0.0;
            asm volatile("" : "+v"(o.J));
            emit_c<M>(o.o, c, a, e, has_r);
        } else {
            emit_c<M>(o, c, a, e, has_r);
        }
    }
}

template <int M, class Out>
__device__ __forceinline__ void emit_axis(const Out& o, const LaneView& L, bool right, int e, int a,
                                          const double (&xs)[3], const double (&xe)[3], bool has_r,
                                          bool zero = false) {
    emit_axis_v<M, Out>(o, L.w(e, a), L.w(e + 1, a), L.r(e), right, e, a, xs, xe, has_r, zero);
}

// `valid` is a bool, or a callable returning it that runs after the factorisation
// (the uniform kernel stages the waypoints there).
template <class V>
__device__ __forceinline__ bool get_valid(V&& v) {
    if constexpr (std::is_same<typename std::decay<V>::type, bool>::value)
        return v;
    else
        return v();
}

template <int M, bool HAS_ED, class Out, class V>
__device__ __forceinline__ int32_t pair_solve_ax(const LaneView& L, bool right, V&& valid_src,
                                                 const double* __restrict__ ed, const Out& O) {
    using CH = Chain<M>;
    constexpr int nL = CH::nL, nR = CH::nR, NS = CH::NS, NE = CH::NE;
    const int nl = right ? nR : nL;
    const double sg = right ? -1.0 : 1.0;
    MARK(ax_factor);
    AxFactors<M> Fa;
    ax_factor<M>(Fa, L, right);
    const bool spd_pair = Fa.spd && (pair_swap(Fa.spd ? 1.0 : 0.0) != 0.0);
    const bool valid = get_valid(valid_src);
    MARK(ax_axisloop);
    double fin = 0.0;
#pragma unroll 1
    for (int a = 0; a < 3; ++a) {
        // virtual-frame start derivatives of this axis: even lane u0, odd lane P uM
        double u0[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double s0 = (HAS_ED && valid) ? ed[d * 3 + a] : 0.0;
            const double s1 = (HAS_ED && valid) ? ed[9 + d * 3 + a] : 0.0;
            u0[d] = (right ? ((d == 1) ? s1 : -s1) : s0) * PSI[d];  // scaled unknowns
        }
        // ---- forward substitution ----
        MARK(ax_fwd);
        double Y[NS + 1][3];
        {
            double pp[8];
            rpowers(L.r(0), pp);
#if TGMS_PAIR_PREFETCH  // the next step's LDS values are read one step ahead
            double rk = L.r(1), wm = L.w(0, a), wk = L.w(1, a), wn = L.w(2, a);
#endif
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                SCHED_FENCE();
                const int k = s + 1;
                double pn[8];
                double y[3];
#if TGMS_PAIR_PREFETCH
                const double rk1 = (s + 1 < NS) ? L.r(k + 1) : 0.0;
                const double wn1 = (s + 1 < NS) ? L.w(k + 2, a) : 0.0;
                rpowers(rk, pn);
                knot_rhs_vals<HAS_ED>(k, wm, wk, wn, pp, pn, u0, y);
                rk = rk1;
                wm = wk;
                wk = wn;
                wn = wn1;
#else
                rpowers(L.r(k), pn);
                knot_rhs_axis<HAS_ED>(L, k, a, pp, pn, u0, y);
#endif
                if (s >= 1) {
                    double B[3][3], v0, v1, v2;
                    coupling_p(pp, B);
                    ldl3_solve(Fa.F[s - 1], Y[s - 1][0], Y[s - 1][1], Y[s - 1][2], v0, v1, v2);
#pragma unroll
                    for (int d = 0; d < 3; ++d) y[d] -= B[0][d] * v0 + B[1][d] * v1 + B[2][d] * v2;
                }
#pragma unroll
                for (int d = 0; d < 3; ++d) Y[s][d] = y[d];
#pragma unroll
                for (int q = 0; q < 8; ++q) pp[q] = pn[q];
            }
        }
        SCHED_FENCE();
        MARK(ax_iface);
        // ---- interface (bit-identical on both lanes, see ps_finish) ----
        double xm[3];
        {
            double yL[3], yR[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const double yv = (nR > nL) ? (right ? Y[NS - 1][d] : Y[nL - 1][d]) : Y[nL - 1][d];
                const double yp = (d == 1) ? yv : sg * yv;
                yL[d] = pair_even(yp);
                yR[d] = pair_odd(yp);
            }
            double Cc[3][3];  // recomputed per axis: 18 fewer live registers across the axis loop
            {
                double pc[8];
                rpowers(L.r(nl), pc);
                coupling_p(pc, Cc);
            }
            double g0, g1, g2;
            ldl3_solve(Fa.FR, yR[0], yR[1], yR[2], g0, g1, g2);
#pragma unroll
            for (int d = 0; d < 3; ++d) yL[d] -= Cc[d][0] * g0 + Cc[d][1] * g1 + Cc[d][2] * g2;
            double xc0, xc1, xc2, x10, x11, x12;
            ldl3_solve(Fa.FS, yL[0], yL[1], yL[2], xc0, xc1, xc2);
            const double b0 = yR[0] - (Cc[0][0] * xc0 + Cc[1][0] * xc1 + Cc[2][0] * xc2);
            const double b1 = yR[1] - (Cc[0][1] * xc0 + Cc[1][1] * xc1 + Cc[2][1] * xc2);
            const double b2 = yR[2] - (Cc[0][2] * xc0 + Cc[1][2] * xc1 + Cc[2][2] * xc2);
            ldl3_solve(Fa.FR, b0, b1, b2, x10, x11, x12);
            xm[0] = right ? -x10 : xc0;
            xm[1] = right ? x11 : xc1;
            xm[2] = right ? -x12 : xc2;
            const double o0 = right ? -xc0 : x10, o1 = right ? xc1 : x11, o2 = right ? -xc2 : x12;
            if (nR > nL) {
                Y[nL][0] = right ? Y[nL][0] : o0;
                Y[nL][1] = right ? Y[nL][1] : o1;
                Y[nL][2] = right ? Y[nL][2] : o2;
                Y[nR][0] = right ? o0 : Y[nR][0];
                Y[nR][1] = right ? o1 : Y[nR][1];
                Y[nR][2] = right ? o2 : Y[nR][2];
            } else {
                Y[nL][0] = o0;
                Y[nL][1] = o1;
                Y[nL][2] = o2;
            }
            fin += (xc0 + xc1) + (xc2 + x10) + (x11 + x12);
        }
        // ---- back substitution, each segment emitted as soon as its end knots are
        // final (segment s+1 right after knot s): the two are independent, which
        // gives the scheduler a second dependency chain to interleave ----
        MARK(ax_back);
#if TGMS_PAIR_PREFETCH  // segment s+1's waypoints and 1/T, read one step ahead
        double w_lo = L.w(NS, a), w_hi = L.w(NS + 1, a), r_n = L.r(NS);
#endif
#pragma unroll
        for (int s = NS - 1; s >= 0; --s) {
            SCHED_FENCE();
            const bool at_end = (s == nl - 1);
            const bool inside = (s < nl - 1);
#if TGMS_PAIR_PREFETCH
            const double w_next = L.w(s, a), r_next = L.r(s);
#endif
            if (s + 1 < NS) {
                double B[3][3];
                {
                    double pb[8];
#if TGMS_PAIR_PREFETCH
                    rpowers(r_n, pb);
#else
                    rpowers(L.r(s + 1), pb);
#endif
                    coupling_p(pb, B);
                }
                double b[3], x0, x1, x2;
#pragma unroll
                for (int d = 0; d < 3; ++d) b[d] = Y[s][d] - (B[d][0] * Y[s + 1][0] + B[d][1] * Y[s + 1][1] + B[d][2] * Y[s + 1][2]);
                ldl3_solve(Fa.F[s], b[0], b[1], b[2], x0, x1, x2);
                Y[s][0] = at_end ? xm[0] : (inside ? x0 : Y[s][0]);
                Y[s][1] = at_end ? xm[1] : (inside ? x1 : Y[s][1]);
                Y[s][2] = at_end ? xm[2] : (inside ? x2 : Y[s][2]);
                fin += inside ? (x0 + x1) + x2 : 0.0;
            } else {
#pragma unroll
                for (int d = 0; d < 3; ++d) Y[s][d] = at_end ? xm[d] : Y[s][d];
            }
#if TGMS_PAIR_PREFETCH
            if (s + 1 < NE)
                emit_axis_v<M, Out>(O, w_lo, w_hi, r_n, right, s + 1, a, Y[s], Y[s + 1], s + 1 < nR, !spd_pair);
            w_hi = w_lo;
            w_lo = w_next;
            r_n = r_next;
#else
            if (s + 1 < NE) emit_axis<M, Out>(O, L, right, s + 1, a, Y[s], Y[s + 1], s + 1 < nR, !spd_pair);
#endif
        }
        MARK(ax_emit);
        SCHED_FENCE();
#if TGMS_PAIR_PREFETCH
        emit_axis_v<M, Out>(O, w_lo, w_hi, r_n, right, 0, a, u0, Y[0], 0 < nR, !spd_pair);
#else
        emit_axis<M, Out>(O, L, right, 0, a, u0, Y[0], 0 < nR, !spd_pair);
#endif
    }
    MARK(ax_end);
    const double fin_pair = fin + pair_swap(fin);
    if (!valid) return TGMS_ERR_INVALID_ARG;
    if (!spd_pair) return TGMS_ERR_SINGULAR;
    if (!finite(fin_pair)) return TGMS_ERR_NONFINITE;
    return TGMS_OK;
}

// A trajectory whose solution came out non-finite is rewritten as exact zeros, like every
// other failure (its coefficients were already stored during the solve).  Rare path: the
// wave first waits for its own stores to the range, then lanes first, first + step, ...
// rewrite it.
__device__ __forceinline__ void zero_traj(double* c, int n, int first, int step) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int e = first; e < n; e += step) c[e] = 0.0;
}

// Anchor a value at this point of the instruction stream: it must be computed before
// the (volatile, ordered) statement, so IR-level sinking cannot pile every step's
// arithmetic into one block after the last scheduling fence (which only orders the
// machine scheduler).
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin_ldl3(Ldl3& f) {
    pin(f.i0);
    pin(f.i1);
    pin(f.i2);
    pin(f.l10);
    pin(f.l20);
    pin(f.l21);
}
__device__ __forceinline__ void pin33(double (&m)[3][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) pin(m[i][j]);
}

// Whole-line output of the joint solve (uniform batches, even M; PairLineOut below): the
// three axes of a segment are emitted together, as whole 128-B lines.
struct PairLineOut;
template <class T>
struct is_pair_lines : std::false_type {};
template <>
struct is_pair_lines<PairLineOut> : std::true_type {};
template <int M>
__device__ __forceinline__ void pair_emit_lines(const PairLineOut& o, int j, bool right, const double (&c)[3][8]);
template <int M>
__device__ __forceinline__ void pair_flush_lines(const PairLineOut& o);

// Monomial coefficients of one axis of a segment from its Hermite data (emit_axis_v's
// arithmetic), zeroed for a failed factorisation.
__device__ __forceinline__ void axis_coeffs(double ws, double we, double r, bool right, const double (&xs)[3],
                                            const double (&xe)[3], bool zero, double (&c)[8]) {
    const double w0 = right ? we : ws, w1 = right ? ws : we;
    const double v0 = right ? -xe[0] : xs[0], a0 = right ? xe[1] : xs[1], j0 = right ? -xe[2] : xs[2];
    const double v1 = right ? -xs[0] : xe[0], a1 = right ? xs[1] : xe[1], j1 = right ? -xs[2] : xe[2];
    const double r2 = r * r, r3 = r2 * r, r4 = r2 * r2;
    const double D = (w1 - w0) * r3;
    const double V0 = v0 * r2, A0 = a0 * r, V1 = v1 * r2, A1 = a1 * r;  // scaled: x PSV, x PSA
    const double P4 = 35.0 * D - (20.0 * PSV) * V0 - (5.0 * PSA) * A0 - (2.0 / 3.0) * j0 - (15.0 * PSV) * V1 +
                      (2.5 * PSA) * A1 - (1.0 / 6.0) * j1;
    const double P5 = -84.0 * D + (45.0 * PSV) * V0 + (10.0 * PSA) * A0 + j0 + (39.0 * PSV) * V1 -
                      (7.0 * PSA) * A1 + 0.5 * j1;
    const double P6 = 70.0 * D - (36.0 * PSV) * V0 - (7.5 * PSA) * A0 - (2.0 / 3.0) * j0 - (34.0 * PSV) * V1 +
                      (6.5 * PSA) * A1 - 0.5 * j1;
    const double P7 = -20.0 * D + (10.0 * PSV) * V0 + (2.0 * PSA) * A0 + (1.0 / 6.0) * j0 + (10.0 * PSV) * V1 -
                      (2.0 * PSA) * A1 + (1.0 / 6.0) * j1;
    c[0] = w0;
    c[1] = PSV * v0;
    c[2] = (0.5 * PSA) * a0;
    c[3] = j0 * (1.0 / 6.0);
    c[4] = P4 * r;
    c[5] = P5 * r2;
    c[6] = P6 * r3;
    c[7] = P7 * r4;
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = zero ? 0.0 : c[k];
}

// The same solve with the three axes side by side in every knot step (knot-major
// instead of axis-major), for the kernels that run at one wave per SIMD anyway
// (M > TGMS_TWO_WAVE_MAX_M): the per-knot couplings and powers are formed once
// instead of once per axis, and the three substitution chains are independent work
// for the scheduler (one wave per SIMD has no second wave to hide their latency).
// It keeps three axes' knot data live (+54 doubles); that only fits the one-wave
// budget.  Per axis the same operations in the same order as pair_solve_ax, and every
// per-segment accumulation (GradAcc) still adds the axes in order 0, 1, 2: the results
// are bit-identical.
template <int M, bool HAS_ED, class Out, class V>
__device__ __forceinline__ int32_t pair_solve_joint(const LaneView& L, bool right, V&& valid_src,
                                                    const double* __restrict__ ed, const Out& O) {
    using CH = Chain<M>;
    constexpr int nL = CH::nL, nR = CH::nR, NS = CH::NS, NE = CH::NE;
    const int nl = right ? nR : nL;
    const double sg = right ? -1.0 : 1.0;
    AxFactors<M> Fa;
    ax_factor<M>(Fa, L, right);
    const bool spd_pair = Fa.spd && (pair_swap(Fa.spd ? 1.0 : 0.0) != 0.0);
    const bool valid = get_valid(valid_src);
    double fin = 0.0;
    double u0[3][3];  // [axis][derivative], virtual-frame start derivatives
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double s0 = (HAS_ED && valid) ? ed[d * 3 + a] : 0.0;
            const double s1 = (HAS_ED && valid) ? ed[9 + d * 3 + a] : 0.0;
            u0[a][d] = (right ? ((d == 1) ? s1 : -s1) : s0) * PSI[d];  // scaled unknowns
        }
    // ---- forward substitution, three axes per knot ----
    double Y[NS + 1][3][3];  // [knot][axis][derivative]
    {
        double pp[8];
        rpowers(L.r(0), pp);
#if TGMS_JOINT_PREFETCH
        double rk = L.r(1), wm[3], wk[3], wn[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            wm[a] = L.w(0, a);
            wk[a] = L.w(1, a);
            wn[a] = L.w(2, a);
        }
#endif
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            SCHED_FENCE();
            const int k = s + 1;
            double pn[8];
#if TGMS_JOINT_PREFETCH
            const double rk1 = (s + 1 < NS) ? L.r(k + 1) : 0.0;
            double wn1[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) wn1[a] = (s + 1 < NS) ? L.w(k + 2, a) : 0.0;
            rpowers(rk, pn);
#else
            rpowers(L.r(k), pn);
#endif
            double B[3][3];
            if (s >= 1) coupling_p(pp, B);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double y[3];
#if TGMS_JOINT_PREFETCH
                knot_rhs_vals<HAS_ED>(k, wm[a], wk[a], wn[a], pp, pn, u0[a], y);
#else
                knot_rhs_axis<HAS_ED>(L, k, a, pp, pn, u0[a], y);
#endif
                if (s >= 1) {
                    double v0, v1, v2;
                    ldl3_solve(Fa.F[s - 1], Y[s - 1][a][0], Y[s - 1][a][1], Y[s - 1][a][2], v0, v1, v2);
#pragma unroll
                    for (int d = 0; d < 3; ++d) y[d] -= B[0][d] * v0 + B[1][d] * v1 + B[2][d] * v2;
                }
#pragma unroll
                for (int d = 0; d < 3; ++d) Y[s][a][d] = y[d];
            }
            pin33(Y[s]);
#pragma unroll
            for (int q = 0; q < 8; ++q) pp[q] = pn[q];
#if TGMS_JOINT_PREFETCH
            rk = rk1;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                wm[a] = wk[a];
                wk[a] = wn[a];
                wn[a] = wn1[a];
            }
#endif
        }
    }
    SCHED_FENCE();
    // ---- interface, per axis (bit-identical on both lanes) ----
    double xm[3][3];
    {
        double Cc[3][3];
        {
            double pc[8];
            rpowers(L.r(nl), pc);
            coupling_p(pc, Cc);
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double yL[3], yR[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const double yv = (nR > nL) ? (right ? Y[NS - 1][a][d] : Y[nL - 1][a][d]) : Y[nL - 1][a][d];
                const double yp = (d == 1) ? yv : sg * yv;
                yL[d] = pair_even(yp);
                yR[d] = pair_odd(yp);
            }
            double g0, g1, g2;
            ldl3_solve(Fa.FR, yR[0], yR[1], yR[2], g0, g1, g2);
#pragma unroll
            for (int d = 0; d < 3; ++d) yL[d] -= Cc[d][0] * g0 + Cc[d][1] * g1 + Cc[d][2] * g2;
            double xc0, xc1, xc2, x10, x11, x12;
            ldl3_solve(Fa.FS, yL[0], yL[1], yL[2], xc0, xc1, xc2);
            const double b0 = yR[0] - (Cc[0][0] * xc0 + Cc[1][0] * xc1 + Cc[2][0] * xc2);
            const double b1 = yR[1] - (Cc[0][1] * xc0 + Cc[1][1] * xc1 + Cc[2][1] * xc2);
            const double b2 = yR[2] - (Cc[0][2] * xc0 + Cc[1][2] * xc1 + Cc[2][2] * xc2);
            ldl3_solve(Fa.FR, b0, b1, b2, x10, x11, x12);
            xm[a][0] = right ? -x10 : xc0;
            xm[a][1] = right ? x11 : xc1;
            xm[a][2] = right ? -x12 : xc2;
            const double o0 = right ? -xc0 : x10, o1 = right ? xc1 : x11, o2 = right ? -xc2 : x12;
            if (nR > nL) {
                Y[nL][a][0] = right ? Y[nL][a][0] : o0;
                Y[nL][a][1] = right ? Y[nL][a][1] : o1;
                Y[nL][a][2] = right ? Y[nL][a][2] : o2;
                Y[nR][a][0] = right ? o0 : Y[nR][a][0];
                Y[nR][a][1] = right ? o1 : Y[nR][a][1];
                Y[nR][a][2] = right ? o2 : Y[nR][a][2];
            } else {
                Y[nL][a][0] = o0;
                Y[nL][a][1] = o1;
                Y[nL][a][2] = o2;
            }
            fin += (xc0 + xc1) + (xc2 + x10) + (x11 + x12);
        }
    }
    // ---- back substitution, three axes per knot; segment s+1 emitted right after ----
#if TGMS_JOINT_PREFETCH
    double w_lo[3], w_hi[3], r_n = L.r(NS);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w_lo[a] = L.w(NS, a);
        w_hi[a] = L.w(NS + 1, a);
    }
#endif
#pragma unroll
    for (int s = NS - 1; s >= 0; --s) {
        SCHED_FENCE();
        const bool at_end = (s == nl - 1);
        const bool inside = (s < nl - 1);
#if TGMS_JOINT_PREFETCH
        double w_next[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) w_next[a] = L.w(s, a);
        const double r_next = L.r(s);
#endif
        if (s + 1 < NS) {
            double B[3][3];
            {
                double pb[8];
#if TGMS_JOINT_PREFETCH
                rpowers(r_n, pb);
#else
                rpowers(L.r(s + 1), pb);
#endif
                coupling_p(pb, B);
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double b[3], x0, x1, x2;
#pragma unroll
                for (int d = 0; d < 3; ++d)
                    b[d] = Y[s][a][d] - (B[d][0] * Y[s + 1][a][0] + B[d][1] * Y[s + 1][a][1] + B[d][2] * Y[s + 1][a][2]);
                ldl3_solve(Fa.F[s], b[0], b[1], b[2], x0, x1, x2);
                Y[s][a][0] = at_end ? xm[a][0] : (inside ? x0 : Y[s][a][0]);
                Y[s][a][1] = at_end ? xm[a][1] : (inside ? x1 : Y[s][a][1]);
                Y[s][a][2] = at_end ? xm[a][2] : (inside ? x2 : Y[s][a][2]);
                fin += inside ? (x0 + x1) + x2 : 0.0;
            }
            pin33(Y[s]);
        } else {
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int d = 0; d < 3; ++d) Y[s][a][d] = at_end ? xm[a][d] : Y[s][a][d];
        }
        if constexpr (is_pair_lines<Out>::value) {
            if (s + 1 < NE) {
                double c[3][8];
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    axis_coeffs(L.w(s + 1, a), L.w(s + 2, a), L.r(s + 1), right, Y[s][a], Y[s + 1][a], !spd_pair,
                                c[a]);
                pair_emit_lines<M>(O, NE - 1 - (s + 1), right, c);
            }
        } else if (s + 1 < NE) {
#pragma unroll
            for (int a = 0; a < 3; ++a)
#if TGMS_JOINT_PREFETCH
                emit_axis_v<M, Out>(O, w_lo[a], w_hi[a], r_n, right, s + 1, a, Y[s][a], Y[s + 1][a], s + 1 < nR,
                                    !spd_pair);
#else
                emit_axis<M, Out>(O, L, right, s + 1, a, Y[s][a], Y[s + 1][a], s + 1 < nR, !spd_pair);
#endif
        }
#if TGMS_JOINT_PREFETCH
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            w_hi[a] = w_lo[a];
            w_lo[a] = w_next[a];
        }
        r_n = r_next;
#endif
    }
    SCHED_FENCE();
    if constexpr (is_pair_lines<Out>::value) {
        double c[3][8];
#pragma unroll
        for (int a = 0; a < 3; ++a) axis_coeffs(L.w(0, a), L.w(1, a), L.r(0), right, u0[a], Y[0][a], !spd_pair, c[a]);
        pair_emit_lines<M>(O, NE - 1, right, c);
        pair_flush_lines<M>(O);
    } else {
#pragma unroll
        for (int a = 0; a < 3; ++a)
#if TGMS_JOINT_PREFETCH
            emit_axis_v<M, Out>(O, w_lo[a], w_hi[a], r_n, right, 0, a, u0[a], Y[0][a], 0 < nR, !spd_pair);
#else
            emit_axis<M, Out>(O, L, right, 0, a, u0[a], Y[0][a], 0 < nR, !spd_pair);
#endif
    }
    const double fin_pair = fin + pair_swap(fin);
    if (!valid) return TGMS_ERR_INVALID_ARG;
    if (!spd_pair) return TGMS_ERR_SINGULAR;
    if (!finite(fin_pair)) return TGMS_ERR_NONFINITE;
    return TGMS_OK;
}

// Emit one segment (virtual knots 0, 1 with derivatives xs, xe [derivative][axis]).
template <int M, class Out>
__device__ __forceinline__ void emit_all_axes(const Out& O, const LaneView& L, bool right,
                                              const double (&xs)[3][3], const double (&xe)[3][3], bool has_r,
                                              bool zero = false) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double s3[3] = {xs[0][a], xs[1][a], xs[2][a]};
        const double e3[3] = {xe[0][a], xe[1][a], xe[2][a]};
        emit_axis<M, Out>(O, L, right, 0, a, s3, e3, has_r, zero);
    }
}

// Whole solve of one group (single-buffered kernels).
template <int M, bool HAS_ED, class Out, class V>
__device__ __forceinline__ int32_t pair_solve(const LaneView& L, bool right, V&& valid_src,
                                              const double* __restrict__ ed, const Out& O) {
    if constexpr (M <= 2) {
        const bool valid = get_valid(valid_src);
        double u0[3][3], uM[3][3];
        const double sg = right ? -1.0 : 1.0;
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const double s0 = (HAS_ED && valid) ? ed[d * 3 + a] : 0.0;
                const double s1 = (HAS_ED && valid) ? ed[9 + d * 3 + a] : 0.0;
                const double f = (d == 1) ? 1.0 : sg;
                u0[d][a] = (right ? f * s1 : s0) * PSI[d];  // scaled unknowns
                uM[d][a] = (right ? f * s0 : s1) * PSI[d];
            }
        bool spd = true;
        double fin = 0.0;
        if constexpr (M == 1) {
            emit_all_axes<M, Out>(O, L, right, u0, uM, false);
        } else {
            // one interior knot: virtual knot 1 on both lanes (physical 1 for both)
            double pp[8], pn[8], y[3][3], x[3][3];
            rpowers(L.r(0), pp);
            rpowers(L.r(1), pn);
            const Sym3 D = knot_diag_p(pp, pn);
            knot_rhs<HAS_ED>(L, 1, pp, pn, u0, y);
            if (HAS_ED) {  // final derivatives through C_1 (virtual segment 1)
                double C1[3][3];
                coupling_p(pn, C1);
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        y[d][a] -= C1[d][0] * uM[0][a] + C1[d][1] * uM[1][a] + C1[d][2] * uM[2][a];
            }
            const Ldl3 f = ldl3s(D, spd);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                ldl3_solve(f, y[0][a], y[1][a], y[2][a], x[0][a], x[1][a], x[2][a]);
                fin += (x[0][a] + x[1][a]) + x[2][a];
            }
            const bool spd2 = spd && (pair_swap(spd ? 1.0 : 0.0) != 0.0);
            emit_all_axes<M, Out>(O, L, right, u0, x, true, !spd2);
        }
        const bool spd_pair = spd && (pair_swap(spd ? 1.0 : 0.0) != 0.0);
        const double fin_pair = fin + pair_swap(fin);
        if (!valid) return TGMS_ERR_INVALID_ARG;
        if (!spd_pair) return TGMS_ERR_SINGULAR;
        if (!finite(fin_pair)) return TGMS_ERR_NONFINITE;
        return TGMS_OK;
    } else {
        if constexpr (M > TGMS_TWO_WAVE_MAX_M && TGMS_JOINT_AXES)
            return pair_solve_joint<M, HAS_ED, Out>(L, right, valid_src, ed, O);
        else
            return pair_solve_ax<M, HAS_ED, Out>(L, right, valid_src, ed, O);
    }
}

// ---------------------------------------------------------------------------
// Staging.

template <int M>
__device__ __forceinline__ void stage_row_w(In<M>& sm, int t, int q, double v) {
    sm.W[w_at<M>(q, t)] = v;
    if (!finite(v)) atomicOr(&sm.bad[t], 1);
}
template <int M>
__device__ __forceinline__ void stage_row_t(In<M>& sm, int t, int q, double v) {
    sm.R[r_at<M>(q, t)] = fast_rcp(v);
    if (!finite_pos(v)) atomicOr(&sm.bad[t], 1);
}

// A non-finite end derivative makes the trajectory invalid like a non-finite waypoint
// (TGMS_ERR_INVALID_ARG, exact zeros; the lane and band kernels check the same): the two
// lanes of the pair check 9 values each.
template <int M>
__device__ __forceinline__ void stage_check_ed(In<M>& sm, int t, bool right, const double* __restrict__ ed) {
    bool bad = false;
#pragma unroll
    for (int q = 0; q < 9; ++q) bad = bad || !finite(ed[2 * q + right]);
    if (bad) atomicOr(&sm.bad[t], 1);
}

// Invalid trajectories are replaced by an all-zero, unit-time one (whose solution
// is exactly zero), so the solver needs no per-coefficient masking.  Rare path.
template <int M>
__device__ __forceinline__ void sanitize(In<M>& sm, int lane) {
    if (lane < TPW && sm.bad[lane]) {
        for (int q = 0; q < (M + 1) * 3; ++q) sm.W[w_at<M>(q, lane)] = 0.0;
        for (int q = 0; q < M; ++q) sm.R[r_at<M>(q, lane)] = 1.0;
    }
}

// Stage a uniform group into the raw layout: 16-B loads (indices clamped into the
// arrays, so no lane branches), copied lane-linearly to LDS; 1/T computed in
// registers.  The times are issued first and staged first, so the factorisation
// (which needs only 1/T) runs while the waypoints are still in flight.  Only a wave
// that sees an invalid input builds per-trajectory flags (re-reading its rows from
// HBM) and sanitises the bad trajectories (all-zero waypoints, unit times).
template <int M, int NT = TPW>
struct RawLoader {
    static constexpr int NW = RawIn<M, NT>::NW;
    static constexpr int NW2 = (NT * NW / 2 + W64 - 1) / W64;  // double2 per lane, waypoints
    static constexpr int NT2 = (NT * M / 2 + W64 - 1) / W64;   // double2 per lane, times
    double2 wv[NW2], tv[NT2];
    double wl, tl;
    bool oddW, oddT, anyT;
    int nw, nt;
    const double* ed = nullptr;  // end derivatives [B][18] (nullptr: rest-to-rest)

    __device__ __forceinline__ void issue(const double* __restrict__ W, const double* __restrict__ T, int32_t B,
                                          int64_t b0, int nb, int lane) {
        const int64_t nW = (int64_t)B * NW, nT = (int64_t)B * M;
        const int64_t jW = b0 * NW / 2, jT = b0 * M / 2;  // first double2 of the group (b0 is even)
        const int64_t mW = nW / 2 - 1 - jW, mT = nT / 2 - 1 - jT;
        const int jmaxW = mW < (1 << 30) ? (int)mW : (1 << 30);  // last double2 inside the arrays
        const int jmaxT = mT < (1 << 30) ? (int)mT : (1 << 30);
        const double2* gW = reinterpret_cast<const double2*>(W) + jW;
        const double2* gT = reinterpret_cast<const double2*>(T) + jT;
#pragma unroll
        for (int i = 0; i < NT2; ++i) {
            const int j = lane + W64 * i;
            tv[i] = gT[j < jmaxT ? j : jmaxT];
        }
#pragma unroll
        for (int i = 0; i < NW2; ++i) {
            const int j = lane + W64 * i;
            wv[i] = gW[j < jmaxW ? j : jmaxW];
        }
        nw = nb * NW;
        nt = nb * M;
        // an array of odd length: its last double is outside every clamped pair
        oddW = (nW & 1) && (b0 + nb == B);
        oddT = (nT & 1) && (b0 + nb == B);
        wl = oddW ? W[nW - 1] : 0.0;
        tl = oddT ? T[nT - 1] : 1.0;
    }

    // Per-trajectory validity from HBM (rare path), sanitising the bad ones' times.
    __device__ __forceinline__ void flags(RawIn<M, NT>& sm, const double* __restrict__ W,
                                          const double* __restrict__ T, int64_t b0, int nb, int lane) {
        if (lane < NT) {
            int f = 0;
            if (lane < nb) {
                const double* w = W + (b0 + lane) * NW;
                const double* t = T + (b0 + lane) * M;
                for (int q = 0; q < NW; ++q) f |= !finite(w[q]);
                for (int q = 0; q < M; ++q) f |= !finite_pos(t[q]);
                if (ed)
                    for (int q = 0; q < 18; ++q) f |= !finite(ed[(b0 + lane) * 18 + q]);
            }
            sm.bad[lane] = f;
            if (f)
                for (int q = 0; q < M; ++q) sm.R[lane * M + q] = 1.0;
        }
    }

    __device__ __forceinline__ void stage_T(RawIn<M, NT>& sm, const double* __restrict__ W,
                                            const double* __restrict__ T, int64_t b0, int nb, int lane) {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < NT2; ++i) {
            const int e = 2 * (lane + W64 * i);
            if ((NT * M) % (2 * W64) == 0 || e < NT * M) {
                *reinterpret_cast<double2*>(sm.R + e) = make_double2(fast_rcp(tv[i].x), fast_rcp(tv[i].y));
                bad = bad || (e < nt && !finite_pos(tv[i].x)) || (e + 1 < nt && !finite_pos(tv[i].y));
            }
        }
        if (oddT) {
            if (lane == 0) sm.R[nt - 1] = fast_rcp(tl);
            bad = bad || !finite_pos(tl);
        }
        if (ed && (lane >> 1) < nb) {  // a trajectory's end derivatives: 9 values per lane of its pair
            const double* e = ed + (b0 + (lane >> 1)) * 18 + (lane & 1);
#pragma unroll
            for (int q = 0; q < 9; ++q) bad = bad || !finite(e[2 * q]);
        }
        anyT = __builtin_amdgcn_ballot_w64(bad) != 0;
        if (anyT) flags(sm, W, T, b0, nb, lane);
        wave_lds_sync();
    }

    // Returns (wave-uniform) whether any trajectory of the group is invalid.
    __device__ __forceinline__ bool stage_W(RawIn<M, NT>& sm, const double* __restrict__ W,
                                            const double* __restrict__ T, int64_t b0, int nb, int lane) {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < NW2; ++i) {
            const int e = 2 * (lane + W64 * i);
            if ((NT * NW) % (2 * W64) == 0 || e < NT * NW) {
                *reinterpret_cast<double2*>(sm.W + e) = wv[i];
                bad = bad || (e < nw && !finite(wv[i].x)) || (e + 1 < nw && !finite(wv[i].y));
            }
        }
        if (oddW) {
            if (lane == 0) sm.W[nw - 1] = wl;
            bad = bad || !finite(wl);
        }
        const bool anyW = __builtin_amdgcn_ballot_w64(bad) != 0;
        if (anyW && !anyT) flags(sm, W, T, b0, nb, lane);
        if (anyW || anyT) {
            if (lane < NT && sm.bad[lane])
                for (int q = 0; q < NW; ++q) sm.W[lane * NW + q] = 0.0;
        }
        wave_lds_sync();
        return anyW || anyT;
    }
};

template <int M>
__device__ __forceinline__ bool stage_raw(RawIn<M>& sm, const double* __restrict__ W, const double* __restrict__ T,
                                          const double* __restrict__ ED, int32_t B, int64_t b0, int nb, int lane) {
    RawLoader<M> ld;
    ld.ed = ED;
    ld.issue(W, T, B, b0, nb, lane);
    ld.stage_T(sm, W, T, b0, nb, lane);
    return ld.stage_W(sm, W, T, b0, nb, lane);
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(M)) void k_reduced_uniform(int32_t B, const double* __restrict__ W,
                                                                        const double* __restrict__ T,
                                                                        const double* __restrict__ ED,
                                                                        double* __restrict__ C,
                                                                        int32_t* __restrict__ status, int nt) {
    __shared__ RawStage<M> sm;
    STAMP_RT(6);
    STAMP(0);
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * TPW;
    const int nb = (int)((B - b0) < TPW ? (B - b0) : TPW);
    RawLoader<M> ld;
    ld.ed = HAS_ED ? ED : nullptr;
    ld.issue(W, T, B, b0, nb, lane);
    ld.stage_T(sm.in, W, T, b0, nb, lane);
    STAMP(1);
    // Every lane runs to the end (the output stage needs the whole wave); pairs
    // beyond nb compute on stale LDS and store nothing (their buffer range is empty).
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const bool live = slot < nb;
    const int64_t b = b0 + slot;
    // the waypoints are staged after the factorisation (which only needs 1/T)
    auto stage_w = [&]() {
        const bool any_bad = ld.stage_W(sm.in, W, T, b0, nb, lane);
        return !any_bad || sm.in.bad[slot] == 0;
    };
    const LaneView L = make_view_raw<M>(sm.in, slot, right);
    const OutBuf O = make_out_buf<M>(sm.O, C, b0, nb, lane, nt != 0);
    const int32_t st = pair_solve<M, HAS_ED, OutBuf>(L, right, stage_w, (HAS_ED && live) ? ED + b * 18 : ED, O);
    STAMP(5);
    STAMP_RT(7);
    if (live && st == TGMS_ERR_NONFINITE) zero_traj(C + b * (M * 24), M * 24, right, 2);
    if (live && !right && status) status[b] = st;
}

// ---------------------------------------------------------------------------
// Time-allocation refinement step: solve, then move every segment duration along
// the normalised gradient of  F(T) = sum_i J_i(T) + k_T sum_i T_i  in log space,
//   g_i = dJ_i/dT_i + k_T,   T_i <- T_i exp(clamp(-eta T_i g_i / F, -1/2, 1/2)),
// (the clamp bounds one step to a factor e^(+-1/2); trajectories whose solve failed
// keep their times).  oracle_refine_times restates the same step on the CPU.
//
// exp of the clamped step (|x| <= 1/2) as one degree-12 polynomial, Horner with FMAs: the
// library exp's range reduction, ldexp and overflow selects (~28 VALU per segment) are dead
// weight on this range.  Coefficients: Chebyshev interpolation at 60 digits
// (scripts/exp_poly.py), worst error 0.83 ulp over [-1/2, 1/2] with every FMA rounded.
// TGMS_EXP_LIBM=1 keeps the library exp (A/B builds).
#ifndef TGMS_EXP_LIBM
#define TGMS_EXP_LIBM 0
#endif
__device__ __forceinline__ double exp_step(double x) {
#if TGMS_EXP_LIBM
    return exp(x);
#else
    double p = 2.0970151215169475e-09;
    p = fma(p, x, 2.5182899238184787e-08);
    p = fma(p, x, 2.7557027169443954e-07);
    p = fma(p, x, 2.755691018636409e-06);
    p = fma(p, x, 2.480158773980975e-05);
    p = fma(p, x, 0.00019841270455051358);
    p = fma(p, x, 0.0013888888888569297);
    p = fma(p, x, 0.008333333332885695);
    p = fma(p, x, 0.041666666666667664);
    p = fma(p, x, 0.16666666666668065);
    p = fma(p, x, 0.5);
    p = fma(p, x, 0.9999999999999999);
    return fma(p, x, 1.0);
#endif
}
template <int M>
__device__ __forceinline__ void refine_update(const GradAcc<Chain<M>::NE>& G, bool right, int32_t st, bool live,
                                              double kT, double eta, const double* __restrict__ Tin,
                                              double* __restrict__ Tout, double* __restrict__ cost) {
    using CH = Chain<M>;
    constexpr int NE = CH::NE;
    const int nmine = right ? CH::nR : NE;
    double Tl[NE];
    double Fl = live ? G.J : 0.0;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int phys = right ? M - 1 - e : e;
        const bool mine = live && e < nmine;
        Tl[e] = mine ? Tin[phys] : 0.0;
        Fl += mine ? kT * Tl[e] : 0.0;
    }
    const double F = Fl + pair_swap(Fl);
    const bool ok = (st == TGMS_OK) && F > 0.0;
    const double iF = 1.0 / F;  // one division per lane, not one per segment (round 6)
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        if (live && e < nmine) {
            const int phys = right ? M - 1 - e : e;
            double dtau = -eta * Tl[e] * (G.dJ[e] + kT) * iF;
            dtau = fmin(fmax(dtau, -0.5), 0.5);
            Tout[phys] = ok ? Tl[e] * exp_step(dtau) : Tl[e];
        }
    }
    if (live && !right && cost) *cost = F;
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(M)) void k_refine_uniform(int32_t B, const double* __restrict__ W,
                                                                       const double* __restrict__ T,
                                                                       const double* __restrict__ ED, double kT,
                                                                       double eta, double* __restrict__ Tout,
                                                                       double* __restrict__ cost,
                                                                       int32_t* __restrict__ status) {
    __shared__ RawIn<M> sm;
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * TPW;
    const int nb = (int)((B - b0) < TPW ? (B - b0) : TPW);
    const bool any_bad = stage_raw<M>(sm, W, T, HAS_ED ? ED : nullptr, B, b0, nb, lane);
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const bool live = slot < nb;
    const int64_t b = b0 + slot;
    const bool valid = !any_bad || sm.bad[slot] == 0;
    const LaneView L = make_view_raw<M>(sm, slot, right);
    GradAcc<Chain<M>::NE> G;
    G.J = 0.0;
#pragma unroll
    for (int e = 0; e < Chain<M>::NE; ++e) G.dJ[e] = 0.0;
    const int32_t st =
        pair_solve<M, HAS_ED, GradAcc<Chain<M>::NE>>(L, right, valid, (HAS_ED && live) ? ED + b * 18 : ED, G);
    refine_update<M>(G, right, st, live, kT, eta, T + (live ? b : 0) * M, Tout + (live ? b : 0) * M,
                     cost ? cost + (live ? b : 0) : nullptr);
    if (live && !right && status) status[b] = st;
}

// One wavefront of a ragged group: trajectories perm[blk*TPW ...] (all with M segments).
template <int M, bool HAS_ED>
__device__ __forceinline__ void refine_ragged_block(Stage<M>& sm, int64_t blk, int32_t n,
                                                    const int32_t* __restrict__ perm,
                                                    const int32_t* __restrict__ seg_offsets,
                                                    const double* __restrict__ W, const double* __restrict__ T,
                                                    const double* __restrict__ ED, double kT, double eta,
                                                    double* __restrict__ Tout, double* __restrict__ cost,
                                                    int32_t* __restrict__ status) {
    constexpr int NW = (M + 1) * 3;
    const int lane = threadIdx.x;
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const int64_t i0 = blk * TPW;
    const int nb = (int)((n - i0) < TPW ? (n - i0) : TPW);
    const bool live = slot < nb;
    if (lane < TPW) sm.in.bad[lane] = 0;
    __syncthreads();
    int32_t b = 0;
    int64_t s0 = 0;
    if (live) {
        b = perm[i0 + slot];
        s0 = seg_offsets[b];
        const double* gW = W + (s0 + b) * 3;
        for (int q = right; q < NW; q += 2) stage_row_w(sm.in, slot, q, gW[q]);
        for (int q = right; q < M; q += 2) stage_row_t(sm.in, slot, q, T[s0 + q]);
        if (HAS_ED) stage_check_ed(sm.in, slot, right, ED + (int64_t)b * 18);
    }
    __syncthreads();
    sanitize(sm.in, lane);
    __syncthreads();
    const bool valid = sm.in.bad[slot] == 0;
    const LaneView L = make_view<M>(sm.in, slot, right);
    GradAcc<Chain<M>::NE> G;
    G.J = 0.0;
#pragma unroll
    for (int e = 0; e < Chain<M>::NE; ++e) G.dJ[e] = 0.0;
    const int32_t st = pair_solve<M, HAS_ED, GradAcc<Chain<M>::NE>>(
        L, right, valid, (HAS_ED && live) ? ED + (int64_t)b * 18 : ED, G);
    refine_update<M>(G, right, st, live, kT, eta, T + s0, Tout + s0, cost ? cost + b : nullptr);
    if (live && !right && status) status[b] = st;
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(M)) void k_refine_ragged(int32_t n, const int32_t* __restrict__ perm,
                                                                      const int32_t* __restrict__ seg_offsets,
                                                                      const double* __restrict__ W,
                                                                      const double* __restrict__ T,
                                                                      const double* __restrict__ ED, double kT,
                                                                      double eta, double* __restrict__ Tout,
                                                                      double* __restrict__ cost,
                                                                      int32_t* __restrict__ status) {
    __shared__ Stage<M> sm;
    refine_ragged_block<M, HAS_ED>(sm, blockIdx.x, n, perm, seg_offsets, W, T, ED, kT, eta, Tout, cost, status);
}

// Ragged batches: one wavefront = TPW trajectories of one segment count M (`perm`).
template <int M, bool HAS_ED>
__device__ __forceinline__ void reduced_ragged_block(Stage<M>& sm, int64_t blk, int32_t n,
                                                     const int32_t* __restrict__ perm,
                                                     const int32_t* __restrict__ seg_offsets,
                                                     const double* __restrict__ W, const double* __restrict__ T,
                                                     const double* __restrict__ ED, double* __restrict__ C,
                                                     int32_t* __restrict__ status, int32_t so_base = 0) {
    constexpr int NW = (M + 1) * 3;
    const int lane = threadIdx.x;
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const int64_t i0 = blk * TPW;
    const int nb = (int)((n - i0) < TPW ? (n - i0) : TPW);
    const bool live = slot < nb;
    if (lane < TPW) {
        sm.in.bad[lane] = 0;
        sm.in.base[lane] = 0;
    }
    __syncthreads();
    int32_t b = 0;
    if (live) {
        b = perm[i0 + slot];
        const int64_t s0 = (int64_t)seg_offsets[b] - so_base;  // (a slice of a larger batch's offsets)
        if (!right) sm.in.base[slot] = s0 * 24;
        const double* gW = W + (s0 + b) * 3;
        // the two lanes of a pair split the trajectory's rows
        for (int q = right; q < NW; q += 2) stage_row_w(sm.in, slot, q, gW[q]);
        for (int q = right; q < M; q += 2) stage_row_t(sm.in, slot, q, T[s0 + q]);
        if (HAS_ED) stage_check_ed(sm.in, slot, right, ED + (int64_t)b * 18);
    }
    __syncthreads();
    sanitize(sm.in, lane);
    __syncthreads();
    const bool valid = sm.in.bad[slot] == 0;
    const LaneView L = make_view<M>(sm.in, slot, right);
    const OutCtx O = make_out(sm.O, sm.in.base, C, nb, lane);
    const int32_t st = pair_solve<M, HAS_ED, OutCtx>(L, right, valid, (HAS_ED && live) ? ED + (int64_t)b * 18 : ED, O);
    if (live && st == TGMS_ERR_NONFINITE) zero_traj(C + sm.in.base[slot], M * 24, right, 2);
    if (live && !right && status) status[b] = st;
}

// The whole refinement loop of one wavefront's trajectories (config 5) in one pass:
// `iters` steps, the cost at the final times, the final solve into C.  Trajectories
// are independent across steps, so nothing synchronises beyond the wavefront: the times
// stay in the LDS stage between steps (and in the lanes that own them), and T is read
// once and written once (in place).  Step for step the same arithmetic as
// refine_ragged_block + refine_update + reduced_ragged_block.
template <int M, bool HAS_ED, bool OPQ = false>
__device__ __forceinline__ void refine_loop_block(Stage<M>& sm, int64_t blk, int32_t n,
                                                  const int32_t* __restrict__ perm,
                                                  const int32_t* __restrict__ seg_offsets,
                                                  const double* __restrict__ W, double* __restrict__ T,
                                                  const double* __restrict__ ED, double kT, double eta,
                                                  int32_t iters, double* __restrict__ cost, double* __restrict__ C,
                                                  int32_t* __restrict__ status, int32_t so_base) {
    using CH = Chain<M>;
    constexpr int NE = CH::NE;
    constexpr int NW = (M + 1) * 3;
    // OPQ (the one-wave class, whose kernel holds the persistent tile loop): an opaque copy
    // of the lane index, else every lane-derived LDS offset would be hoisted out of the
    // loop and held over it (~100 of them: 372-636 B of scratch at M = 14..16)
    int lane = threadIdx.x;
    if constexpr (OPQ) asm volatile("" : "+v"(lane));
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const int64_t i0 = blk * TPW;
    const int nb = (int)((n - i0) < TPW ? (n - i0) : TPW);
    const bool live = slot < nb;
    if (lane < TPW) {
        sm.in.bad[lane] = 0;
        sm.in.base[lane] = 0;
    }
    __syncthreads();
    int32_t b = 0;
    int64_t s0 = 0;
    if (live) {
        b = perm[i0 + slot];
        s0 = (int64_t)seg_offsets[b] - so_base;  // (a slice of a larger batch's offsets: rebased)
        if (!right) sm.in.base[slot] = s0 * 24;
        const double* gW = W + (s0 + b) * 3;
        for (int q = right; q < NW; q += 2) stage_row_w(sm.in, slot, q, gW[q]);
        for (int q = right; q < M; q += 2) stage_row_t(sm.in, slot, q, T[s0 + q]);
        if (HAS_ED) stage_check_ed(sm.in, slot, right, ED + (int64_t)b * 18);
    }
    // this lane updates the times of its half of the segments; between steps they live
    // in its registers (and as 1/T in the stage); an invalid trajectory keeps its times
    // (its stage row was sanitised to unit times; nothing is written back)
    const int nmine = right ? CH::nR : NE;
    double Tl[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) Tl[e] = (live && e < nmine) ? T[s0 + (right ? M - 1 - e : e)] : 0.0;
    __syncthreads();
    sanitize(sm.in, lane);
    __syncthreads();
    const bool valid = sm.in.bad[slot] == 0;
    const double* ed = (HAS_ED && live) ? ED + (int64_t)b * 18 : ED;
    int32_t st_last = TGMS_OK;
    for (int32_t it = 0; it <= iters; ++it) {  // it == iters: the cost at the final times
        const LaneView L = make_view<M>(sm.in, slot, right);
        if (C && it == iters) break;  // the last pass follows the loop
        GradAcc<NE> G;
        G.J = 0.0;
#pragma unroll
        for (int e = 0; e < NE; ++e) G.dJ[e] = 0.0;
        const int32_t st = pair_solve<M, HAS_ED, GradAcc<NE>>(L, right, valid, ed, G);
        st_last = st;
        double Fl = live ? G.J : 0.0;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            if (live && e < nmine) Fl += kT * Tl[e];
        }
        const double F = Fl + pair_swap(Fl);
        if (it == iters) {
            if (live && !right && cost) cost[b] = F;
            break;
        }
        const bool ok = (st == TGMS_OK) && F > 0.0;
        const double iF = 1.0 / F;  // one division per lane and step, not one per segment (round 6)
        __syncthreads();  // every lane has read the stage before the times change
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            if (live && valid && e < nmine) {
                const int phys = right ? M - 1 - e : e;
                const double tl = Tl[e];
                double dtau = -eta * tl * (G.dJ[e] + kT) * iF;
                dtau = fmin(fmax(dtau, -0.5), 0.5);
                const double tn = ok ? tl * exp_step(dtau) : tl;
                Tl[e] = tn;
                sm.in.R[r_at<M>(phys, slot)] = fast_rcp(tn);
            }
        }
        __syncthreads();
    }
    if (C) {
        const LaneView L = make_view<M>(sm.in, slot, right);
        // the last pass: the coefficients at the final times and the cost there from
        // one solve (a separate cost pass and emission pass before: 12 -> 11 solves
        // per trajectory at 10 steps)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            if (live && valid && e < nmine) T[s0 + (right ? M - 1 - e : e)] = Tl[e];
        }
        // kT sum T first: the times are dead during the solve
        double Ft = 0.0;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            if (live && e < nmine) Ft += kT * Tl[e];
        }
        const CostOut O{make_out(sm.O, sm.in.base, C, nb, lane), 0.0};
        const int32_t st = pair_solve<M, HAS_ED, CostOut>(L, right, valid, ed, O);
        const double Fl = live ? O.J + Ft : 0.0;
        const double F = Fl + pair_swap(Fl);
        if (live && !right && cost) cost[b] = F;
        if (live && st == TGMS_ERR_NONFINITE) zero_traj(C + sm.in.base[slot], M * 24, right, 2);
        if (live && !right && status) status[b] = st;
        return;
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        if (live && valid && e < nmine) T[s0 + (right ? M - 1 - e : e)] = Tl[e];
    }
    if (live && !right && status) status[b] = st_last;
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(M)) void k_reduced_ragged(int32_t n, const int32_t* __restrict__ perm,
                                                                       const int32_t* __restrict__ seg_offsets,
                                                                       const double* __restrict__ W,
                                                                       const double* __restrict__ T,
                                                                       const double* __restrict__ ED,
                                                                       double* __restrict__ C,
                                                                       int32_t* __restrict__ status) {
    __shared__ Stage<M> sm;
    reduced_ragged_block<M, HAS_ED>(sm, blockIdx.x, n, perm, seg_offsets, W, T, ED, C, status);
}

// Every M group of a ragged plan in ONE launch (one per occupancy class: M <= 11 at
// two waves per SIMD, M >= 12 at one): wavefront ranges [blk_end[g-1], blk_end[g])
// belong to group g, longest groups first.  The groups then share the machine at
// once instead of running one small grid after another.
static_assert(TPW == RAGGED_TPW, "host group tables assume TPW trajectories per wavefront");

template <int MLO, int MHI>
constexpr size_t max_stage_bytes() {
    size_t b = 0;
#define TGMS_STAGE_MAX(m) \
    if constexpr (m >= MLO && m <= MHI) b = b > sizeof(Stage<m>) ? b : sizeof(Stage<m>);
    TGMS_STAGE_MAX(1) TGMS_STAGE_MAX(2) TGMS_STAGE_MAX(3) TGMS_STAGE_MAX(4) TGMS_STAGE_MAX(5) TGMS_STAGE_MAX(6)
    TGMS_STAGE_MAX(7) TGMS_STAGE_MAX(8) TGMS_STAGE_MAX(9) TGMS_STAGE_MAX(10) TGMS_STAGE_MAX(11)
    TGMS_STAGE_MAX(12) TGMS_STAGE_MAX(13) TGMS_STAGE_MAX(14) TGMS_STAGE_MAX(15) TGMS_STAGE_MAX(16)
#undef TGMS_STAGE_MAX
    return b;
}

__device__ __forceinline__ int group_of(const GroupTable& tab, int64_t bid, int64_t& blk) {
    int g = 0;
    while (g + 1 < tab.ngroups && bid >= tab.blk_end[g]) ++g;  // uniform, <= 16 steps
    blk = bid - (g ? tab.blk_end[g - 1] : 0);
    return g;
}

template <int MLO, int MHI, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(MHI)) void k_reduced_multi(GroupTable tab,
                                                                        const int32_t* __restrict__ seg_offsets,
                                                                        const double* __restrict__ W,
                                                                        const double* __restrict__ T,
                                                                        const double* __restrict__ ED,
                                                                        double* __restrict__ C,
                                                                        int32_t* __restrict__ status) {
    __shared__ alignas(16) unsigned char raw[max_stage_bytes<MLO, MHI>()];
    int64_t blk;
    const int g = group_of(tab, blockIdx.x, blk);
    switch (tab.m[g]) {
#define TGMS_MULTI_CASE(mm)                                                                                \
    case mm:                                                                                              \
        if constexpr (mm >= MLO && mm <= MHI)                                                             \
            reduced_ragged_block<mm, HAS_ED>(*reinterpret_cast<Stage<mm>*>(raw), blk, tab.n[g], tab.perm[g], \
                                             seg_offsets, W, T, ED, C, status);                           \
        break;
        TGMS_MULTI_CASE(1) TGMS_MULTI_CASE(2) TGMS_MULTI_CASE(3) TGMS_MULTI_CASE(4) TGMS_MULTI_CASE(5)
        TGMS_MULTI_CASE(6) TGMS_MULTI_CASE(7) TGMS_MULTI_CASE(8) TGMS_MULTI_CASE(9) TGMS_MULTI_CASE(10)
        TGMS_MULTI_CASE(11) TGMS_MULTI_CASE(12) TGMS_MULTI_CASE(13) TGMS_MULTI_CASE(14) TGMS_MULTI_CASE(15)
        TGMS_MULTI_CASE(16)
#undef TGMS_MULTI_CASE
        default: break;
    }
}

template <int MLO, int MHI, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(MHI)) void k_refine_multi(GroupTable tab,
                                                                       const int32_t* __restrict__ seg_offsets,
                                                                       const double* __restrict__ W,
                                                                       const double* __restrict__ T,
                                                                       const double* __restrict__ ED, double kT,
                                                                       double eta, double* __restrict__ Tout,
                                                                       double* __restrict__ cost,
                                                                       int32_t* __restrict__ status) {
    __shared__ alignas(16) unsigned char raw[max_stage_bytes<MLO, MHI>()];
    int64_t blk;
    const int g = group_of(tab, blockIdx.x, blk);
    switch (tab.m[g]) {
#define TGMS_MULTI_CASE(mm)                                                                                 \
    case mm:                                                                                               \
        if constexpr (mm >= MLO && mm <= MHI)                                                              \
            refine_ragged_block<mm, HAS_ED>(*reinterpret_cast<Stage<mm>*>(raw), blk, tab.n[g], tab.perm[g], \
                                            seg_offsets, W, T, ED, kT, eta, Tout, cost, status);           \
        break;
        TGMS_MULTI_CASE(1) TGMS_MULTI_CASE(2) TGMS_MULTI_CASE(3) TGMS_MULTI_CASE(4) TGMS_MULTI_CASE(5)
        TGMS_MULTI_CASE(6) TGMS_MULTI_CASE(7) TGMS_MULTI_CASE(8) TGMS_MULTI_CASE(9) TGMS_MULTI_CASE(10)
        TGMS_MULTI_CASE(11) TGMS_MULTI_CASE(12) TGMS_MULTI_CASE(13) TGMS_MULTI_CASE(14) TGMS_MULTI_CASE(15)
        TGMS_MULTI_CASE(16)
#undef TGMS_MULTI_CASE
        default: break;
    }
}

// One wavefront tile of the refinement loop from the device plan: the class's group table
// is read from device memory (scalar loads); the tile's group gives M.
template <int MLO, int MHI, bool HAS_ED>
__device__ __forceinline__ void refine_loop_tile(unsigned char* raw, const GroupTable& tab, int64_t tile,
                                                 const int32_t* __restrict__ seg_offsets,
                                                 const double* __restrict__ W, double* __restrict__ T,
                                                 const double* __restrict__ ED, double kT, double eta, int32_t iters,
                                                 double* __restrict__ cost, double* __restrict__ C,
                                                 int32_t* __restrict__ status, int32_t so_base) {
    int64_t blk;
    const int g = group_of(tab, tile, blk);
    switch (tab.m[g]) {
#define TGMS_MULTI_CASE(mm)                                                                                    \
    case mm:                                                                                                  \
        if constexpr (mm >= MLO && mm <= MHI)                                                                 \
            refine_loop_block<mm, HAS_ED, TGMS_WAVES(MHI) == 1>(*reinterpret_cast<Stage<mm>*>(raw), blk,       \
                                                                 tab.n[g], tab.perm[g], seg_offsets, W, T, ED, kT, \
                                                                 eta, iters, cost, C, status, so_base);            \
        break;
        TGMS_MULTI_CASE(1) TGMS_MULTI_CASE(2) TGMS_MULTI_CASE(3) TGMS_MULTI_CASE(4) TGMS_MULTI_CASE(5)
        TGMS_MULTI_CASE(6) TGMS_MULTI_CASE(7) TGMS_MULTI_CASE(8) TGMS_MULTI_CASE(9) TGMS_MULTI_CASE(10)
        TGMS_MULTI_CASE(11) TGMS_MULTI_CASE(12) TGMS_MULTI_CASE(13) TGMS_MULTI_CASE(14) TGMS_MULTI_CASE(15)
        TGMS_MULTI_CASE(16)
#undef TGMS_MULTI_CASE
        default: break;
    }
}

// The refinement loop from the device plan, one launch per occupancy class, in one of two
// modes the plan chooses (k_plan_scatter):
//   * plan->waves[cls] == 0: one block per wavefront tile (longest groups first), blocks
//     past the class's last tile return; the hardware dispatches tiles into free slots;
//   * plan->waves[cls] > 0 (the one-wave class when it has more tiles than the GPU has
//     SIMDs, TGMS_C5_PERSIST): that many PERSISTENT wavefronts, each holding its SIMD and
//     taking tiles from plan->next[cls] (zeroed by the planner) until none is left.  A
//     one-wave tile needs a whole SIMD, which a SIMD shared with the two-wave class never
//     frees while two-wave tiles are pending: at full config-5 size (6,563 one-wave tiles)
//     the class was starved while the two-wave class ran and then ran alone as the tail;
//     sized from the plan's per-class work, the persistent class ends with the other one
//     (1,048,576 ragged on one device: 2.52-2.53 -> 2.35-2.37 ms pipelined, session r06v).
//     At one shard (822 tiles: one round) one block per tile is as fast (r06v, r06x).
// Which wave takes which tile does not change a tile's arithmetic: results are bit-identical.
template <int MLO, int MHI, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(MHI)) void k_refine_loop_dev(DevPlan* __restrict__ plan, int cls,
                                                                          const int32_t* __restrict__ seg_offsets,
                                                                          const double* __restrict__ W,
                                                                          double* __restrict__ T,
                                                                          const double* __restrict__ ED, double kT,
                                                                          double eta, int32_t iters,
                                                                          double* __restrict__ cost,
                                                                          double* __restrict__ C,
                                                                          int32_t* __restrict__ status) {
    __shared__ alignas(16) unsigned char raw[max_stage_bytes<MLO, MHI>()];
    const GroupTable& tab = plan->tab[cls];
    const int ng = tab.ngroups;
    if (ng <= 0) return;
    const int64_t ntiles = tab.blk_end[ng - 1];
    const int32_t so_base = plan->so_base;
    // (the persistent loop is compiled into the one-wave class only: at two waves per SIMD
    // its live ranges would not fit the 256 registers)
    const int nw = TGMS_WAVES(MHI) == 1 ? plan->waves[cls] : 0;
    if (nw <= 0) {
        if ((int64_t)blockIdx.x >= ntiles) return;
        refine_loop_tile<MLO, MHI, HAS_ED>(raw, tab, blockIdx.x, seg_offsets, W, T, ED, kT, eta, iters, cost, C,
                                           status, so_base);
        return;
    }
    if constexpr (TGMS_WAVES(MHI) == 1) {
        if ((int)blockIdx.x >= nw) return;
        for (;;) {
            int tile = 0;
            if (threadIdx.x == 0) tile = atomicAdd(&plan->next[cls], 1);  // a vector atomic, one lane
            tile = __builtin_amdgcn_readfirstlane(tile);
            if ((int64_t)tile >= ntiles) break;  // every wave leaves once the tiles run out
            refine_loop_tile<MLO, MHI, HAS_ED>(raw, tab, tile, seg_offsets, W, T, ED, kT, eta, iters, cost, C, status,
                                               so_base);
            __syncthreads();  // the next tile re-stages the LDS
        }
    }
}

// The ragged solve with the device-computed plan (round 6: the pieces of a multi-GPU ragged
// solve, and device 0's shard, are grouped on their device like the refinement loop's, so
// the host makes no pass over the offsets): k_reduced_multi's blocks with the class table
// read from device memory, grid dev_loop_grid(n), blocks past the last group return.
template <int MLO, int MHI, bool HAS_ED>
__global__ __launch_bounds__(64, TGMS_WAVES(MHI)) void k_reduced_multi_dev(const DevPlan* __restrict__ plan, int cls,
                                                                            const int32_t* __restrict__ seg_offsets,
                                                                            const double* __restrict__ W,
                                                                            const double* __restrict__ T,
                                                                            const double* __restrict__ ED,
                                                                            double* __restrict__ C,
                                                                            int32_t* __restrict__ status) {
    __shared__ alignas(16) unsigned char raw[max_stage_bytes<MLO, MHI>()];
    const GroupTable& tab = plan->tab[cls];
    const int ng = tab.ngroups;
    if (ng <= 0 || (int64_t)blockIdx.x >= tab.blk_end[ng - 1]) return;
    int64_t blk;
    const int g = group_of(tab, blockIdx.x, blk);
    const int32_t so_base = plan->so_base;
    switch (tab.m[g]) {
#define TGMS_MULTI_CASE(mm)                                                                                 \
    case mm:                                                                                               \
        if constexpr (mm >= MLO && mm <= MHI)                                                              \
            reduced_ragged_block<mm, HAS_ED>(*reinterpret_cast<Stage<mm>*>(raw), blk, tab.n[g], tab.perm[g], \
                                             seg_offsets, W, T, ED, C, status, so_base);                  \
        break;
        TGMS_MULTI_CASE(1) TGMS_MULTI_CASE(2) TGMS_MULTI_CASE(3) TGMS_MULTI_CASE(4) TGMS_MULTI_CASE(5)
        TGMS_MULTI_CASE(6) TGMS_MULTI_CASE(7) TGMS_MULTI_CASE(8) TGMS_MULTI_CASE(9) TGMS_MULTI_CASE(10)
        TGMS_MULTI_CASE(11) TGMS_MULTI_CASE(12) TGMS_MULTI_CASE(13) TGMS_MULTI_CASE(14) TGMS_MULTI_CASE(15)
        TGMS_MULTI_CASE(16)
#undef TGMS_MULTI_CASE
        default: break;
    }
}

// ---------------------------------------------------------------------------
// Grouping a ragged batch by M on the device (the refinement loop's plan, captured into
// its graph): a stable counting sort of the trajectory ids by M = so[b+1] - so[b], the
// same permutation the host planner builds (csrc/tgms_capi.hip upload_plan).  Blocks of
// PERM_BLOCK trajectories; k_perm_hist counts each block's trajectories per M (wave
// ballots), k_perm_scatter places them: the group's start + the counts of the blocks
// before + the counts of the waves before + the lanes before.  M is validated on the host.
constexpr int PERM_BLOCK = 1024;
constexpr int PERM_BINS = 17;  // M = 1..16 (bin 0 unused)
static_assert(PERM_BLOCK / W64 == PERM_BINS - 1, "k_perm_scatter: one wave per group");

__device__ __forceinline__ int perm_m(const int32_t* __restrict__ so, int64_t b, int32_t B) {
    return b < B ? (int)(so[b + 1] - so[b]) : 0;
}

__global__ __launch_bounds__(PERM_BLOCK) void k_perm_hist(int32_t B, const int32_t* __restrict__ so,
                                                          int32_t* __restrict__ hist) {
    __shared__ int32_t wc[PERM_BLOCK / W64][PERM_BINS];
    const int t = threadIdx.x, w = t / W64, l = t % W64;
    const int m = perm_m(so, (int64_t)blockIdx.x * PERM_BLOCK + t, B);
#pragma unroll
    for (int k = 1; k < PERM_BINS; ++k) {
        const unsigned long long mask = __ballot(m == k);
        if (l == 0) wc[w][k] = __popcll(mask);
    }
    __syncthreads();
    if (t > 0 && t < PERM_BINS) {
        int32_t s = 0;
        for (int v = 0; v < PERM_BLOCK / W64; ++v) s += wc[v][t];
        hist[(int64_t)blockIdx.x * PERM_BINS + t] = s;
    }
}

struct PermStarts {
    int32_t s[PERM_BINS];  // first index of group M in the permutation
};

template <class Starts>
__device__ __forceinline__ void perm_scatter_body(int32_t B, const int32_t* __restrict__ so,
                                                  const int32_t* __restrict__ hist, Starts&& start_of,
                                                  int32_t* __restrict__ perm) {
    __shared__ int32_t wc[PERM_BLOCK / W64][PERM_BINS];
    __shared__ int32_t base[PERM_BINS];
    const int t = threadIdx.x, w = t / W64, l = t % W64;
    const int64_t b = (int64_t)blockIdx.x * PERM_BLOCK + t;
    const int m = perm_m(so, b, B);
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 1; k < PERM_BINS; ++k) {
        const unsigned long long mask = __ballot(m == k);
        if (m == k) mine = mask;
        if (l == 0) wc[w][k] = __popcll(mask);
    }
    {  // the blocks before this one: wave w sums group w + 1 over them, 64 blocks per step
        const int g = w + 1;  // PERM_BLOCK / W64 == PERM_BINS - 1 waves, one per group
        int32_t s = 0;
        for (unsigned v = l; v < blockIdx.x; v += W64) s += hist[(int64_t)v * PERM_BINS + g];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        if (l == 0) base[g] = start_of(g) + s;
    }
    __syncthreads();
    if (m >= 1 && m < PERM_BINS) {  // (a device copy of the offsets that disagrees with the
        int32_t r = base[m];         // host's, which validated them, must not write out of range)
        for (int v = 0; v < w; ++v) r += wc[v][m];
        r += __popcll(mine & ((1ull << l) - 1ull));
        if (r >= 0 && r < B) perm[r] = (int32_t)b;
    }
}

__global__ __launch_bounds__(PERM_BLOCK) void k_perm_scatter(int32_t B, const int32_t* __restrict__ so,
                                                             const int32_t* __restrict__ hist, PermStarts st,
                                                             int32_t* __restrict__ perm) {
    perm_scatter_body(B, so, hist, [&](int g) { return st.s[g]; }, perm);
}

// The device-side plan (DevPlan, tgms_internal.h) and the scatter in ONE launch after
// k_perm_hist (round 6: a one-workgroup planning kernel between the two cost a launch, ~6 us
// of a 0.39 ms config-5 call).  Every block sums the per-block counts itself, one wave per
// group M: over the blocks before it (its scatter base) and over all blocks (the totals, so
// the starts); it checks the offsets against the host's B and S; block 0 also writes the
// plan the class loops read (so_base, starts and both classes' group tables in the order the
// host planner used, M descending within a class).  A bad plan scatters nothing and marks
// the trajectories whose own M is outside 1..16 TGMS_ERR_INVALID_ARG and the others
// TGMS_ERR_SKIPPED, all outputs exact zeros (each block its own trajectories and its share
// of the S x 24 coefficients).
__global__ __launch_bounds__(PERM_BLOCK) void k_plan_scatter(int32_t n, int64_t S, const int32_t* __restrict__ so,
                                                             int has_ed, int nsimd, const int32_t* __restrict__ hist,
                                                             int32_t* __restrict__ perm, DevPlan* __restrict__ plan,
                                                             int32_t* __restrict__ status, double* __restrict__ C,
                                                             double* __restrict__ cost) {
    __shared__ int32_t wc[PERM_BLOCK / W64][PERM_BINS];
    __shared__ int32_t before[PERM_BINS], cnt[PERM_BINS], base[PERM_BINS];
    __shared__ int32_t bad_s;
    const int t = threadIdx.x, w = t / W64, l = t % W64;
    const int nblk = (int)gridDim.x;
    const int64_t b = (int64_t)blockIdx.x * PERM_BLOCK + t;
    const int m = perm_m(so, b, n);
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 1; k < PERM_BINS; ++k) {
        const unsigned long long mask = __ballot(m == k);
        if (m == k) mine = mask;
        if (l == 0) wc[w][k] = __popcll(mask);
    }
    {  // PERM_BLOCK / W64 == PERM_BINS - 1 waves: wave w sums group w + 1 over the blocks
        const int g = w + 1;
        int32_t sb = 0, sa = 0;
        for (int v = l; v < nblk; v += W64) {
            const int32_t c = hist[(int64_t)v * PERM_BINS + g];
            sa += c;
            sb += (v < (int)blockIdx.x) ? c : 0;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            sa += __shfl_xor(sa, off);
            sb += __shfl_xor(sb, off);
        }
        if (l == 0) {
            before[g] = sb;
            cnt[g] = sa;
        }
    }
    __syncthreads();
    if (t == 0) {
        int64_t tot = 0;
        for (int k = 1; k < PERM_BINS; ++k) tot += cnt[k];
        const int32_t so0 = so[0];
        const bool bad = tot != n || (int64_t)so[n] - so0 != S;
        bad_s = bad ? 1 : 0;
        int32_t starts[PERM_BINS];
        int32_t st = 0;
        starts[0] = 0;
        for (int k = 1; k < PERM_BINS; ++k) {
            starts[k] = st;
            base[k] = st + before[k];
            st += bad ? 0 : cnt[k];
        }
        if (blockIdx.x == 0) {
            plan->so_base = so0;
            plan->bad = bad ? 1 : 0;
            for (int k = 0; k < PERM_BINS; ++k) plan->starts[k] = starts[k];
            const int max2 = has_ed ? TGMS_TWO_WAVE_MAX_M_ED : TGMS_TWO_WAVE_MAX_M;
            int ng[2] = {0, 0};
            int32_t be[2] = {0, 0};
            for (int k = PERM_BINS - 1; k >= 1; --k) {
                if (bad || !cnt[k]) continue;
                const int c = k > max2 ? 1 : 0;
                GroupTable& tb = plan->tab[c];
                const int g = ng[c]++;
                be[c] += (cnt[k] + RAGGED_TPW - 1) / RAGGED_TPW;
                tb.m[g] = k;
                tb.n[g] = cnt[k];
                tb.perm[g] = perm + starts[k];
                tb.blk_end[g] = be[c];
            }
            plan->tab[0].ngroups = ng[0];
            plan->tab[1].ngroups = ng[1];
            // the one-wave class's persistent waves (k_refine_loop_dev): its share of the
            // machine's SIMD time from the per-class work (tiles x (2 + M), the host
            // planner's cost), a one-wave tile taking TGMS_C5_W1 / 100 times the SIMD time
            // of a two-wave tile per unit (session r06r: 122 us per one-wave tile at M ~ 15
            // holding a SIMD, 87 us per two-wave tile at M ~ 7.5 sharing one), biased up by
            // TGMS_C5_BIAS % so the coarse class ends before the fine one, not after
            plan->next[0] = 0;
            plan->next[1] = 0;
            plan->waves[0] = 0;
            plan->waves[1] = 0;
            if (TGMS_C5_PERSIST && !bad) {
                int64_t w1 = 0, w2 = 0, t1 = 0;
                for (int k = 1; k < PERM_BINS; ++k) {
                    const int64_t tiles = (cnt[k] + RAGGED_TPW - 1) / RAGGED_TPW;
                    if (k > max2) {
                        w1 += tiles * (2 + k) * TGMS_C5_W1;
                        t1 += tiles;
                    } else {
                        w2 += tiles * (2 + k) * 100;
                    }
                }
                if (t1 > 0) {
                    int64_t p = ((int64_t)nsimd * w1 * TGMS_C5_BIAS + (w1 + w2) * 100 - 1) / ((w1 + w2) * 100);
                    p = p < 1 ? 1 : p;
                    p = p > nsimd ? nsimd : p;
                    // persistent only when the class has more tiles than the GPU has SIMDs
                    // (one block per tile then needs every one of them: grid <= nsimd)
                    plan->waves[1] = t1 > nsimd ? (int32_t)p : 0;
                }
            }
        }
    }
    __syncthreads();
    if (bad_s) {
        if (b < n) {
            const int64_t mb = (int64_t)so[b + 1] - so[b];
            if (status) status[b] = (mb < 1 || mb > TGMS_MAX_SEGMENTS) ? TGMS_ERR_INVALID_ARG : TGMS_ERR_SKIPPED;
            if (cost) cost[b] = 0.0;
        }
        if (C) {
            const int64_t total = S * 24, chunk = (total + nblk - 1) / nblk;
            const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = i0 + chunk < total ? i0 + chunk : total;
            for (int64_t i = i0 + t; i < i1; i += PERM_BLOCK) C[i] = 0.0;
        }
        return;
    }
    if (m >= 1 && m < PERM_BINS) {  // (a device copy of the offsets that disagrees with the
        int32_t r = base[m];         // host's must not write out of range)
        for (int v = 0; v < w; ++v) r += wc[v][m];
        r += __popcll(mine & ((1ull << l) - 1ull));
        if (r >= 0 && r < n) perm[r] = (int32_t)b;
    }
}

// ---------------------------------------------------------------------------
// Lane-per-trajectory solve of a uniform batch with an even number of segments
// (configs 2-4: M = 10 is the headline).  One LANE owns one trajectory, 64 per
// wavefront, one wavefront per SIMD: the 512-register budget holds the whole
// elimination state (every knot's G = D^-1 C and g = D^-1 z, 3 axes) at once, so
//   * the three axes are solved together — the shared powers, couplings and
//     right-hand-side factors are computed once per knot instead of once per axis,
//     and the three substitutions give the scheduler independent chains;
//   * there is no twisted interface: the chain runs knot 1 .. M-1 in one lane;
//   * every segment's 24 coefficients are final at the same moment, so the output
//     leaves as WHOLE 128-B lines.  In the [traj][seg][axis][8] layout the segment
//     pair (2k, 2k+1) is exactly three lines: (2k: x y), (2k: z | 2k+1: x),
//     (2k+1: y z).  Back substitution runs from the last segment down, so segment
//     2k+1 flushes its (y z) line and carries its x row until segment 2k completes
//     the other two.  Each flush stages one line per lane in LDS and stores it with
//     8 instructions of 8 whole lines each (half-line writes a pass apart, the
//     axis-sequential kernel's pattern, run at ~3.4 TB/s past the Infinity Cache;
//     whole lines at ~5.5, scripts/storebench.hip).
// Inputs arrive by LDS-DMA (global_load_lds_dwordx4, lane-linear in the HBM layout,
// no staging registers): the times first, so the factorisation (1/T only) runs while
// the waypoints are still in flight.  1/T stays in LDS (each lane's row) and is
// re-read per phase, which keeps the elimination state alone in registers.
// Same block LDL^T as the oracle's reduced formulation (oracle/minsnap_oracle.c),
// one-sided instead of twisted.

// The lane kernel anchors every knot's factors and elimination vectors (pin_ldl3,
// pin33): without the anchors it needs > 700 registers.

// LDS byte address of a __shared__ object.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// 16-B LDS-DMA (global_load_lds_dwordx4): lane l's 16 B from `src` land at LDS byte
// lds + 16 l.  Issued as asm so the compiler's wait bookkeeping ignores it (with the
// builtin it drains every copy, vmcnt(0), at the first LDS read of ANY object); the
// kernel counts completion itself.
__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}

constexpr int LTPW = 64;   // trajectories per wavefront (one per lane)
constexpr int LROW = 18;   // staged output line: 16 doubles padded to 144 B (conflict-free ds_*_b128)

// LDS-DMA copies of one wave's input block (lane-linear, 1 KiB per instruction).
template <int M>
struct LaneDma {
    static constexpr int NW = (M + 1) * 3;
    static constexpr int NTI = (LTPW * M * 8 + 1023) / 1024;   // instructions, times
    static constexpr int NWI = (LTPW * NW * 8 + 1023) / 1024;  // instructions, waypoints
};

struct LineOut {
    double* stage[2];              // LDS [LTPW][LROW], alternating per flush
    __amdgpu_buffer_rsrc_t rs[8];  // store q: trajectories 8q .. 8q+7 of the wave's block
    uint32_t voff;                 // lane's 16-B piece: trajectory (lane >> 3) of the group, piece (lane & 7)
    bool nt;                       // streaming stores (the batch's output exceeds the Infinity Cache)
    int lane;
};

template <int M>
__device__ __forceinline__ LineOut make_line_out(double* s0, double* s1, double* C, int64_t b0, int nb, int lane,
                                                 bool nt) {
    constexpr int TRAJ_B = M * 24 * 8;
    LineOut o;
    o.stage[0] = s0;
    o.stage[1] = s1;
    o.lane = lane;
    o.nt = nt;
    double* base = C + b0 * (M * 24);
    const int block = nb * TRAJ_B;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int lim = block - q * 8 * TRAJ_B;
        o.rs[q] = __builtin_amdgcn_make_buffer_rsrc(base + (int64_t)q * 8 * M * 24, (short)0, lim > 0 ? lim : 0,
                                                    0x00020000);
    }
    o.voff = (uint32_t)((lane >> 3) * TRAJ_B + (lane & 7) * 16);
    return o;
}

// Output lines are software-pipelined: a segment's lines are written to the stage
// (one 128-B line per lane per buffer, lo = first 64 B, hi = second) and stored one
// segment later, so the next segment's arithmetic covers the LDS write latency.
// Storing reads a buffer transposed — 8 consecutive lanes hold one line — and writes
// it with 8 instructions of 8 whole lines (the resources' range check drops a tail
// wave's missing trajectories).  LDS operations of a wave execute in order, so a
// buffer may be rewritten right after it was read.
__device__ __forceinline__ void stage_line(const LineOut& o, int buf, const double (&lo)[8], const double (&hi)[8]) {
#ifdef TGMS_ABL_NOSTAGE  // ablation build: the line's data stays live, no LDS traffic
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(lo[j]), "v"(hi[j]));
    return;
#endif
    double2* d = reinterpret_cast<double2*>(o.stage[buf] + o.lane * LROW);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = make_double2(lo[2 * j], lo[2 * j + 1]);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[4 + j] = make_double2(hi[2 * j], hi[2 * j + 1]);
}

struct StagedLine {
    double2 v[8];
};

__device__ __forceinline__ void read_line(const LineOut& o, int buf, StagedLine& L) {
#ifdef TGMS_ABL_NOSTAGE
#pragma unroll
    for (int q = 0; q < 8; ++q) L.v[q] = make_double2((double)buf, (double)q);
    return;
#endif
    const double* src = o.stage[buf] + (o.lane >> 3) * LROW + (o.lane & 7) * 2;
#pragma unroll
    for (int q = 0; q < 8; ++q) L.v[q] = *reinterpret_cast<const double2*>(src + q * 8 * LROW);
}

__device__ __forceinline__ void store_line(const LineOut& o, const StagedLine& L, int line_off) {
#ifdef TGMS_ABL_NOSTORE  // ablation build (scripts/gpu_kvar.sh): the stores' data stays live, nothing is written
#pragma unroll
    for (int q = 0; q < 8; ++q) asm volatile("" ::"v"(L.v[q].x), "v"(L.v[q].y));
    return;
#endif
    if (o.nt) {  // wave-uniform
#pragma unroll
        for (int q = 0; q < 8; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, L.v[q]), o.rs[q], o.voff, line_off,
                                                   TGMS_STORE_CPOL_NT);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, L.v[q]), o.rs[q], o.voff, line_off,
                                                   TGMS_STORE_CPOL);
    }
}

// The lines segment e leaves staged (M even, descending order): an odd segment its
// (y z) line in buffer 0, an even one (x y) in buffer 0 and (z | carry) in buffer 1.
__device__ __forceinline__ int seg_lines(int e) { return (e & 1) ? 1 : 2; }
__device__ __forceinline__ int seg_line_off(int e, int i) { return (e & 1) ? e * 192 + 64 : e * 192 + 128 * i; }

// Store the lines segment e staged (called one segment later, after wave_lds_sync).
__device__ __forceinline__ void put_segment_lines_read(const LineOut& o, int e, StagedLine& L0, StagedLine& L1) {
    read_line(o, 0, L0);
    if (seg_lines(e) == 2) read_line(o, 1, L1);
}
__device__ __forceinline__ void put_segment_lines_store(const LineOut& o, int e, const StagedLine& L0,
                                                        const StagedLine& L1) {
    store_line(o, L0, seg_line_off(e, 0));
    if (seg_lines(e) == 2) store_line(o, L1, seg_line_off(e, 1));
}

// ---------------------------------------------------------------------------
// Whole-line output of the joint lane-pair solve (uniform batches, even M >= 12): the even
// lane emits its segments nL, nL-1, .., 0 (nL = M/2 - 1), the odd lane nL+1, .., M-1, one
// segment per step each, all three axes at once.  A segment pair (2k, 2k+1) is three 128-B
// lines of [traj][seg][axis][8]: (2k: x y), (2k: z | 2k+1: x), (2k+1: y z).  The even lane
// meets a pair at its odd segment first: it stages (y z) and carries x; the odd lane meets it
// at its even segment: it stages (x y) and carries z; the next step completes the other two
// lines.  At every step both lanes of a pair stage the same number of lines (their segments
// have opposite parity), except at step 0 when nL is even: then the middle pair (nL, nL+1)
// is split between the lanes and the even lane completes (nL: z | nL+1: x) with the odd
// lane's x row (DPP swap).  Lines go through the lane kernel's transposed LDS stage: a lane
// stores rows (lane >> 3) + 8 q, all of one parity, so its line offsets are the even or the
// odd lane's, and eight buffer resources of four trajectories each drop a tail wave's
// missing trajectories (range check).  Half-line stores a pass apart run at ~3.4 TB/s past
// the Infinity Cache, whole lines at ~5.5 (scripts/storebench.hip).
struct PairLineOut {
    double* stage[2];              // LDS [W64][LROW]
    __amdgpu_buffer_rsrc_t rs[8];  // store q: trajectories 4q .. 4q+3 of the wave's block
    uint32_t voff;                 // (lane >> 4) * TRAJ_B + (lane & 7) * 16
    bool odd_rows;                 // the rows this lane stores were staged by odd (right) lanes
    bool nt;                       // streaming stores
    int lane;
    mutable double carry[8];
};

template <int M>
__device__ __forceinline__ PairLineOut make_pair_line_out(double* s0, double* s1, double* C, int64_t b0, int nb,
                                                          int lane, bool nt) {
    constexpr int TRAJ_B = M * 24 * 8;
    PairLineOut o;
    o.stage[0] = s0;
    o.stage[1] = s1;
    o.lane = lane;
    o.nt = nt;
    double* base = C + b0 * (M * 24);
    const int block = nb * TRAJ_B;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int lim = block - q * 4 * TRAJ_B;
        o.rs[q] = __builtin_amdgcn_make_buffer_rsrc(base + (int64_t)q * 4 * M * 24, (short)0, lim > 0 ? lim : 0,
                                                    0x00020000);
    }
    o.voff = (uint32_t)((lane >> 4) * TRAJ_B + (lane & 7) * 16);
    o.odd_rows = (lane >> 3) & 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.carry[k] = 0.0;
    return o;
}

// Step j's lines: count per lane (1 or 2) and byte offsets in the trajectory's block for
// the even and the odd lane (-1: none).  Constant-folded: j is a compile-time index.
template <int M>
__device__ __forceinline__ void pair_line_step(int j, int& nbuf, int (&offE)[2], int (&offO)[2]) {
    constexpr int nL = M / 2 - 1;
    const int eE = nL - j, eO = nL + 1 + j;
    if (j == 0 && nL % 2 == 0) {  // the middle pair split between the lanes
        nbuf = 2;
        offE[0] = eE * 192, offE[1] = eE * 192 + 128;
        offO[0] = eO * 192 + 64, offO[1] = -1;
    } else if (eE & 1) {
        nbuf = 1;
        offE[0] = eE * 192 + 64, offE[1] = -1;
        offO[0] = eO * 192, offO[1] = -1;
    } else {
        nbuf = 2;
        offE[0] = eE * 192, offE[1] = eE * 192 + 128;
        offO[0] = eO * 192 - 64, offO[1] = eO * 192 + 64;
    }
}

__device__ __forceinline__ void pair_store_line(const PairLineOut& o, const StagedLine& L, int offE, int offO) {
    const int off = o.odd_rows ? offO : offE;
    const uint32_t v = off >= 0 ? o.voff + (uint32_t)off : 0x80000000u;  // none: out of range, dropped
    if (o.nt) {  // wave-uniform
#pragma unroll
        for (int q = 0; q < 8; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, L.v[q]), o.rs[q], v, 0,
                                                   TGMS_STORE_CPOL_NT);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, L.v[q]), o.rs[q], v, 0, TGMS_STORE_CPOL);
    }
}

__device__ __forceinline__ void pair_read_line(const PairLineOut& o, int buf, StagedLine& L) {
    const double* src = o.stage[buf] + (o.lane >> 3) * LROW + (o.lane & 7) * 2;
#pragma unroll
    for (int q = 0; q < 8; ++q) L.v[q] = *reinterpret_cast<const double2*>(src + q * 8 * LROW);
}

__device__ __forceinline__ void pair_stage_line(const PairLineOut& o, int buf, const double (&lo)[8],
                                                const double (&hi)[8]) {
    double2* d = reinterpret_cast<double2*>(o.stage[buf] + o.lane * LROW);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = make_double2(lo[2 * k], lo[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[4 + k] = make_double2(hi[2 * k], hi[2 * k + 1]);
}

// Emission step j (c: this lane's segment, three axes): store the lines step j - 1 left
// staged (software-pipelined: the LDS writes of a step land while the next one computes),
// then stage this step's.
template <int M>
__device__ __forceinline__ void pair_emit_lines(const PairLineOut& o, int j, bool right, const double (&c)[3][8]) {
    static_assert(M % 2 == 0, "whole lines need even M");
    constexpr int nL = M / 2 - 1;
    StagedLine P0, P1;
    int pn = 0, pE[2] = {-1, -1}, pO[2] = {-1, -1};
    if (j > 0) {
        pair_line_step<M>(j - 1, pn, pE, pO);
        wave_lds_sync();  // the previous step's stage writes have landed
        pair_read_line(o, 0, P0);
        if (pn == 2) pair_read_line(o, 1, P1);
    }
    const int eE = nL - j;
    double lo[8], hi[8];
    if (j == 0 && nL % 2 == 0) {
        // even lane: (nL: x y) and (nL: z | nL+1: x), the odd lane's x row by DPP; odd lane:
        // (nL+1: y z)
        double xo[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) xo[k] = pair_swap(c[0][k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo[k] = right ? c[1][k] : c[0][k];
            hi[k] = right ? c[2][k] : c[1][k];
        }
        pair_stage_line(o, 0, lo, hi);
        pair_stage_line(o, 1, c[2], xo);  // (the odd lane's copy is never stored)
    } else if (eE & 1) {
        // even lane at an odd segment: (y z), carry x; odd lane at an even one: (x y), carry z
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo[k] = right ? c[0][k] : c[1][k];
            hi[k] = right ? c[1][k] : c[2][k];
            o.carry[k] = right ? c[2][k] : c[0][k];
        }
        pair_stage_line(o, 0, lo, hi);
    } else {
        // even lane at an even segment: (x y), (z | carry); odd lane at an odd one: (carry | x), (y z)
        double lo1[8], hi1[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo[k] = right ? o.carry[k] : c[0][k];
            hi[k] = right ? c[0][k] : c[1][k];
            lo1[k] = right ? c[1][k] : c[2][k];
            hi1[k] = right ? c[2][k] : o.carry[k];
        }
        pair_stage_line(o, 0, lo, hi);
        pair_stage_line(o, 1, lo1, hi1);
    }
    if (j > 0) {
        pair_store_line(o, P0, pE[0], pO[0]);
        if (pn == 2) pair_store_line(o, P1, pE[1], pO[1]);
    }
}

// After the last step (j = M/2 - 1): store what it staged.
template <int M>
__device__ __forceinline__ void pair_flush_lines(const PairLineOut& o) {
    int pn = 0, pE[2], pO[2];
    pair_line_step<M>(M / 2 - 1, pn, pE, pO);
    StagedLine P0, P1;
    wave_lds_sync();
    pair_read_line(o, 0, P0);
    if (pn == 2) pair_read_line(o, 1, P1);
    pair_store_line(o, P0, pE[0], pO[0]);
    if (pn == 2) pair_store_line(o, P1, pE[1], pO[1]);
}

template <int M>
struct alignas(16) RawLineStage {
    alignas(16) double O[2][W64 * LROW];  // two line buffers (the lane kernel's stage layout)
    RawIn<M> in;
};

// Uniform batches with even M >= TGMS_PAIR_LINES_MIN_M: the joint lane-pair solve (one
// wave per SIMD) with whole-line output; otherwise k_reduced_uniform.
template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, 1) void k_reduced_uniform_lines(int32_t B, const double* __restrict__ W,
                                                                 const double* __restrict__ T,
                                                                 const double* __restrict__ ED,
                                                                 double* __restrict__ C,
                                                                 int32_t* __restrict__ status, int nt) {
    __shared__ RawLineStage<M> sm;
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * TPW;
    const int nb = (int)((B - b0) < TPW ? (B - b0) : TPW);
    RawLoader<M> ld;
    ld.ed = HAS_ED ? ED : nullptr;
    ld.issue(W, T, B, b0, nb, lane);
    ld.stage_T(sm.in, W, T, b0, nb, lane);
    const int slot = lane >> 1;
    const bool right = lane & 1;
    const bool live = slot < nb;
    const int64_t b = b0 + slot;
    auto stage_w = [&]() {
        const bool any_bad = ld.stage_W(sm.in, W, T, b0, nb, lane);
        return !any_bad || sm.in.bad[slot] == 0;
    };
    const LaneView L = make_view_raw<M>(sm.in, slot, right);
    const PairLineOut O = make_pair_line_out<M>(sm.O[0], sm.O[1], C, b0, nb, lane, nt != 0);
    const int32_t st =
        pair_solve_joint<M, HAS_ED, PairLineOut>(L, right, stage_w, (HAS_ED && live) ? ED + b * 18 : ED, O);
    if (live && st == TGMS_ERR_NONFINITE) zero_traj(C + b * (M * 24), M * 24, right, 2);
    if (live && !right && status) status[b] = st;
}

// Monomial coefficients of segment e, all three axes, from the Hermite data at its
// knots (xs at knot e, xe at knot e+1, [derivative][axis]) in r = 1/T scaled
// variables (the same expressions as emit_axis).
__device__ __forceinline__ void seg_rows(const double (&ws)[3], const double (&we)[3], double r,
                                         const double (&xs)[3][3], const double (&xe)[3][3], double (&c)[3][8]) {
    const double r2 = r * r, r3 = r2 * r, r4 = r2 * r2;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double w0 = ws[a], w1 = we[a];
        const double v0 = xs[0][a], a0 = xs[1][a], j0 = xs[2][a];
        const double v1 = xe[0][a], a1 = xe[1][a], j1 = xe[2][a];
        const double D = (w1 - w0) * r3;
        const double V0 = v0 * r2, A0 = a0 * r, V1 = v1 * r2, A1 = a1 * r;
        const double P4 = 35.0 * D - 20.0 * V0 - 5.0 * A0 - (2.0 / 3.0) * j0 - 15.0 * V1 + 2.5 * A1 - (1.0 / 6.0) * j1;
        const double P5 = -84.0 * D + 45.0 * V0 + 10.0 * A0 + j0 + 39.0 * V1 - 7.0 * A1 + 0.5 * j1;
        const double P6 = 70.0 * D - 36.0 * V0 - 7.5 * A0 - (2.0 / 3.0) * j0 - 34.0 * V1 + 6.5 * A1 - 0.5 * j1;
        const double P7 = -20.0 * D + 10.0 * V0 + 2.0 * A0 + (1.0 / 6.0) * j0 + 10.0 * V1 - 2.0 * A1 + (1.0 / 6.0) * j1;
        c[a][0] = w0;
        c[a][1] = v0;
        c[a][2] = 0.5 * a0;
        c[a][3] = j0 * (1.0 / 6.0);
        c[a][4] = P4 * r;
        c[a][5] = P5 * r2;
        c[a][6] = P6 * r3;
        c[a][7] = P7 * r4;
    }
}

// Emit segment e (descending order, M even): store the lines the segment above left
// staged, then stage this segment's: an odd segment its (y z) line, keeping its x row
// in `carry`; the even segment below it (x y) and (z | carry).
__device__ __forceinline__ void emit_lane_segment(const LineOut& o, const double (&ws)[3], const double (&we)[3],
                                                  double r, int e, const double (&xs)[3][3],
                                                  const double (&xe)[3][3], double (&carry)[8], int e_prev) {
    double c[3][8];
#ifdef TGMS_ABL_NOEMIT  // ablation build: no coefficient arithmetic (the knot data stays live)
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int j = 0; j < 8; ++j) c[a][j] = (j < 3) ? xs[j][a] : ((j < 6) ? xe[j - 3][a] : ws[a] + r);
#else
    seg_rows(ws, we, r, xs, xe, c);
#endif
    StagedLine L0, L1;
    if (e_prev >= 0) {
        wave_lds_sync();  // the previous segment's stage writes have landed
        put_segment_lines_read(o, e_prev, L0, L1);
    }
    if (e & 1) {
        stage_line(o, 0, c[1], c[2]);
#pragma unroll
        for (int j = 0; j < 8; ++j) carry[j] = c[0][j];
    } else {
        stage_line(o, 0, c[0], c[1]);
        stage_line(o, 1, c[2], carry);
    }
    if (e_prev >= 0) put_segment_lines_store(o, e_prev, L0, L1);
}

template <int M, bool HAS_ED>
__global__ __launch_bounds__(64, 1) void k_lane_uniform(int32_t B, const double* __restrict__ W,
                                                         const double* __restrict__ T,
                                                         const double* __restrict__ ED, double* __restrict__ C,
                                                         int32_t* __restrict__ status, int nt) {
    static_assert(M >= 2 && M % 2 == 0, "segment pairs make whole lines only for even M");
    using DM = LaneDma<M>;
    constexpr int NK = M - 1;  // interior knots 1 .. M-1 (index k-1 below)
    constexpr int NW = DM::NW;
    __shared__ alignas(16) double sT[DM::NTI * 128];
    __shared__ alignas(16) double sW[DM::NWI * 128];
    __shared__ alignas(16) double sO[2][LTPW * LROW];
    STAMP_RT(6);
    STAMP(0);
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * LTPW;
    const int nb = (int)((B - b0) < LTPW ? (B - b0) : LTPW);
    const bool live = lane < nb;
    const int64_t b = b0 + lane;
    {
        // 16-B pieces of the wave's block, indices clamped into the arrays (a tail
        // wave copies junk for its missing trajectories; their results are dropped)
        const int64_t nT2 = (int64_t)B * M / 2, nW2 = (int64_t)B * NW / 2;
        const int64_t jT = b0 * M / 2, jW = b0 * NW / 2;  // b0 is a multiple of 64
        const double2* gT = reinterpret_cast<const double2*>(T);
        const double2* gW = reinterpret_cast<const double2*>(W);
        const uint32_t aT = lds_addr(sT), aW = lds_addr(sW);
#pragma unroll
        for (int i = 0; i < DM::NTI; ++i) {
            const int64_t j = jT + lane + W64 * i;
            glds16(gT + (j < nT2 ? j : nT2 - 1), aT + i * 1024);
        }
#pragma unroll
        for (int i = 0; i < DM::NWI; ++i) {
            const int64_t j = jW + lane + W64 * i;
            glds16(gW + (j < nW2 ? j : nW2 - 1), aW + i * 1024);
        }
    }
    // the times' copies retire before the waypoints' (in order)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DM::NWI) : "memory");
    double* __restrict__ Rl = sT + lane * M;  // this lane's row: T, then 1/T in place
    bool valid = true;
    {
        double t[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
            t[i] = Rl[i];
            valid = valid && finite_pos(t[i]);
        }
#pragma unroll
        for (int i = 0; i < M; ++i) Rl[i] = valid ? fast_rcp(t[i]) : 1.0;  // invalid: unit times
    }
    wave_lds_sync();
    STAMP(1);

    // ---- block LDL^T over the interior knots (needs 1/T only) ----
    // D_k = H_kk - C_{k-1}^T D_{k-1}^-1 C_{k-1};  G_{k-1} = D_{k-1}^-1 C_{k-1}
    Ldl3 F[NK];
    double G[NK > 1 ? NK - 1 : 1][3][3];
    bool spd = true;
    {
        double pp[8], rk = Rl[1];
        rpowers(Rl[0], pp);
#pragma unroll
        for (int k = 1; k <= NK; ++k) {
            SCHED_FENCE();
            double pn[8];
            rpowers(rk, pn);
            if (k < NK) rk = Rl[k + 1];  // LDS read one step ahead
            Sym3 D = knot_diag(pp, pn);
            if (k >= 2) {
                double Bc[3][3];
                coupling(pp, Bc);  // C_{k-1} = H_{k-1, k}
#pragma unroll
                for (int e = 0; e < 3; ++e)
                    ldl3_solve(F[k - 2], Bc[0][e], Bc[1][e], Bc[2][e], G[k - 2][0][e], G[k - 2][1][e], G[k - 2][2][e]);
                sym_sub_btw(D, Bc, G[k - 2]);
            }
            bool ok;
            F[k - 1] = ldl3s(D, ok);
            spd = spd && ok;
            pin_ldl3(F[k - 1]);
            if (k >= 2) pin33(G[k - 2]);
#pragma unroll
            for (int q = 0; q < 8; ++q) pp[q] = pn[q];
        }
    }
    STAMP(2);

    // ---- waypoints (in flight until now) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((((int64_t)B * NW) & 1) && b0 + nb == B) {  // the array's last double is in no 16-B piece
        if (lane == 0) sW[nb * NW - 1] = W[(int64_t)B * NW - 1];
        wave_lds_sync();
    }
    double* __restrict__ Wl = sW + lane * NW;
    STAMP(3);
    double u0[3][3], uM[3][3];  // end derivatives [derivative][axis]
    {
        const double* ed = ED + (live ? b : 0) * 18;
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                u0[d][a] = HAS_ED ? ed[d * 3 + a] : 0.0;
                uM[d][a] = HAS_ED ? ed[9 + d * 3 + a] : 0.0;
            }
    }

    // ---- forward substitution, 3 axes: z_k = y_k - G_{k-1}^T z_{k-1}, g_k = D_k^-1 z_k ----
    double g[NK][3][3];
    bool wfin = true;
    {
        // the waypoints of knots k-1, k, k+1 and 1/T of segment k, each read from LDS one
        // step before it is needed
        double pp[8], zp[3][3], wm[3], wc[3], wn[3], rk = Rl[1];
        rpowers(Rl[0], pp);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            wm[a] = Wl[a];
            wc[a] = Wl[3 + a];
            wn[a] = Wl[6 + a];
            wfin = wfin && finite(wm[a]) && finite(wc[a]);
        }
#pragma unroll
        for (int k = 1; k <= NK; ++k) {
            SCHED_FENCE();
            double pn[8];
            rpowers(rk, pn);
            double wnn[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) wnn[a] = (k < NK) ? Wl[(k + 2) * 3 + a] : 0.0;
            if (k < NK) rk = Rl[k + 1];
            const double fp[3] = {-KEP[0] * pp[6], -KEP[1] * pp[5], -KEP[2] * pp[4]};
            const double fn[3] = {-KSP[0] * pn[6], -KSP[1] * pn[5], -KSP[2] * pn[4]};
            double z[3][3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                wfin = wfin && finite(wn[a]);
                const double dp = wc[a] - wm[a];
                const double dn = wn[a] - wc[a];
#pragma unroll
                for (int d = 0; d < 3; ++d) z[d][a] = fp[d] * dp + fn[d] * dn;
                wm[a] = wc[a];
                wc[a] = wn[a];
                wn[a] = wnn[a];
            }
            if (HAS_ED && k == 1) {  // - C_0^T u0
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        const double c0 = KSE[e][d] * pp[5 - d - e];
#pragma unroll
                        for (int a = 0; a < 3; ++a) z[d][a] -= c0 * u0[e][a];
                    }
            }
            if (HAS_ED && k == NK) {  // - C_{M-1} uM
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        const double c1 = KSE[d][e] * pn[5 - d - e];
#pragma unroll
                        for (int a = 0; a < 3; ++a) z[d][a] -= c1 * uM[e][a];
                    }
            }
            if (k >= 2) {
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        z[d][a] -= G[k - 2][0][d] * zp[0][a] + G[k - 2][1][d] * zp[1][a] + G[k - 2][2][d] * zp[2][a];
            }
#pragma unroll
            for (int a = 0; a < 3; ++a)
                ldl3_solve(F[k - 1], z[0][a], z[1][a], z[2][a], g[k - 1][0][a], g[k - 1][1][a], g[k - 1][2][a]);
            pin33(g[k - 1]);
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) zp[d][a] = z[d][a];
#pragma unroll
            for (int q = 0; q < 8; ++q) pp[q] = pn[q];
        }
    }
    if (HAS_ED) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int a = 0; a < 3; ++a) wfin = wfin && finite(u0[d][a]) && finite(uM[d][a]);
    }
    // An invalid trajectory (non-finite input, T <= 0) or a failed factorisation comes
    // out as exact zeros: its elimination vectors and factors, end derivatives,
    // waypoint row and 1/T row (unit times) are zeroed (rare path).
    valid = valid && wfin;
    const bool keep = valid && spd;
    if (__builtin_amdgcn_ballot_w64(!keep) != 0) {
        if (!keep) {
#pragma unroll
            for (int q = 0; q < NW; ++q) Wl[q] = 0.0;
#pragma unroll
            for (int i = 0; i < M; ++i) Rl[i] = 1.0;
        }
#pragma unroll
        for (int k = 0; k < NK; ++k)
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    g[k][d][a] = keep ? g[k][d][a] : 0.0;
                    if (k < NK - 1) G[k][d][a] = keep ? G[k][d][a] : 0.0;
                }
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                u0[d][a] = keep ? u0[d][a] : 0.0;
                uM[d][a] = keep ? uM[d][a] : 0.0;
            }
        wave_lds_sync();
    }
    STAMP(4);

    // ---- back substitution x_k = g_k - G_k x_{k+1}, each segment emitted as soon as
    // both of its knots are final (last segment first); the next segment's waypoints
    // and 1/T are read one segment ahead ----
    const LineOut O = make_line_out<M>(sO[0], sO[1], C, b0, nb, lane, nt != 0);
    double carry[8];
    double fin = 0.0;
    double we[3], ws[3], rs = Rl[NK];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        we[a] = Wl[M * 3 + a];
        ws[a] = Wl[NK * 3 + a];
    }
#pragma unroll
    for (int k = NK; k >= 1; --k) {
        SCHED_FENCE();
        double wn[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) wn[a] = Wl[(k - 1) * 3 + a];
        const double rn = Rl[k - 1];
        if (k < NK) {
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    g[k - 1][d][a] -= G[k - 1][d][0] * g[k][0][a] + G[k - 1][d][1] * g[k][1][a] + G[k - 1][d][2] * g[k][2][a];
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) fin += (g[k - 1][d][0] + g[k - 1][d][1]) + g[k - 1][d][2];
        if (k == NK)
            emit_lane_segment(O, ws, we, rs, k, g[k - 1], uM, carry, -1);
        else
            emit_lane_segment(O, ws, we, rs, k, g[k - 1], g[k], carry, k + 1);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            we[a] = ws[a];
            ws[a] = wn[a];
        }
        rs = rn;
    }
    SCHED_FENCE();
    emit_lane_segment(O, ws, we, rs, 0, u0, g[0], carry, 1);
    {
        StagedLine L0, L1;
        wave_lds_sync();
        put_segment_lines_read(O, 0, L0, L1);
        put_segment_lines_store(O, 0, L0, L1);
    }
    STAMP(5);
    STAMP_RT(7);
    int32_t st = TGMS_OK;
    if (!valid)
        st = TGMS_ERR_INVALID_ARG;
    else if (!spd)
        st = TGMS_ERR_SINGULAR;
    else if (!finite(fin))
        st = TGMS_ERR_NONFINITE;
    if (live && st == TGMS_ERR_NONFINITE) zero_traj(C + b * (M * 24), M * 24, 0, 1);
    if (live && status) status[b] = st;
}

// Uniform batches with an even number of segments take the lane-per-trajectory kernel.
#ifndef TGMS_LANE_UNIFORM
#define TGMS_LANE_UNIFORM 1
#endif
// Largest M on the lane kernel: its whole elimination state lives in registers, which
// at M >= 12 spill to scratch (92-980 B per lane).  At M = 12 it still matches the
// lane-pair kernel (51.6 vs 52.4 us per 65,536, fresh batches); at 14 and 16 the pair is
// faster (60 vs 77 us, 69 vs 109 us; profiles/r04_lane_vs_pair_M12_16.jsonl), so M >= 14
// take the lane-pair kernel.
#ifndef TGMS_LANE_MAX_M
#define TGMS_LANE_MAX_M 10
#endif
template <int M>
constexpr bool use_lane_kernel() {
    return TGMS_LANE_UNIFORM && M >= 2 && M % 2 == 0 && M <= TGMS_LANE_MAX_M;
}
// Even M from here up (and above the lane kernel's range) take the joint lane-pair solve
// with whole-line output (k_reduced_uniform_lines).
#ifndef TGMS_PAIR_LINES_MIN_M
#define TGMS_PAIR_LINES_MIN_M 12
#endif
template <int M>
constexpr bool use_pair_lines() {
    return !use_lane_kernel<M>() && M % 2 == 0 && M >= TGMS_PAIR_LINES_MIN_M && M >= 4;
}

template <int M>
hipError_t uniform_M(int32_t B, const double* W, const double* T, const double* ED, double* C, int32_t* status,
                     hipStream_t stream) {
    const unsigned grid = (unsigned)((B + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    const int nt = (int64_t)B * M * 24 * 8 > kStreamingOutputBytes;
    if constexpr (use_lane_kernel<M>()) {
        const unsigned lgrid = (unsigned)((B + LTPW - 1) / LTPW);
        if (ED)
            TGMS_LAUNCH((k_lane_uniform<M, true>), dim3(lgrid), dim3(W64), 0, stream, B, W, T, ED, C, status, nt);
        else
            TGMS_LAUNCH((k_lane_uniform<M, false>), dim3(lgrid), dim3(W64), 0, stream, B, W, T, ED, C, status, nt);
        return hipSuccess;
    }
    if constexpr (use_pair_lines<M>()) {
        if (ED)
            TGMS_LAUNCH((k_reduced_uniform_lines<M, true>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status,
                        nt);
        else
            TGMS_LAUNCH((k_reduced_uniform_lines<M, false>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C,
                        status, nt);
        return hipSuccess;
    }
    if (ED)
        TGMS_LAUNCH((k_reduced_uniform<M, true>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status,
                           nt);
    else
        TGMS_LAUNCH((k_reduced_uniform<M, false>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, C, status,
                           nt);
    return hipSuccess;
}

template <int M>
hipError_t ragged_M(int32_t n, const int32_t* perm, const int32_t* so, const double* W, const double* T,
                    const double* ED, double* C, int32_t* status, hipStream_t stream) {
    const unsigned grid = (unsigned)((n + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    if (ED)
        TGMS_LAUNCH((k_reduced_ragged<M, true>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C,
                           status);
    else
        TGMS_LAUNCH((k_reduced_ragged<M, false>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, C,
                           status);
    return hipSuccess;
}

template <int M>
hipError_t refine_uniform_M(int32_t B, const double* W, const double* T, const double* ED, double kT, double eta,
                            double* Tout, double* cost, int32_t* status, hipStream_t stream) {
    const unsigned grid = (unsigned)((B + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    if (ED)
        TGMS_LAUNCH((k_refine_uniform<M, true>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, kT, eta, Tout,
                           cost, status);
    else
        TGMS_LAUNCH((k_refine_uniform<M, false>), dim3(grid), dim3(W64), 0, stream, B, W, T, ED, kT, eta,
                           Tout, cost, status);
    return hipSuccess;
}

template <int M>
hipError_t refine_ragged_M(int32_t n, const int32_t* perm, const int32_t* so, const double* W, const double* T,
                           const double* ED, double kT, double eta, double* Tout, double* cost, int32_t* status,
                           hipStream_t stream) {
    const unsigned grid = (unsigned)((n + TPW - 1) / TPW);
    if (grid == 0) return hipSuccess;
    if (ED)
        TGMS_LAUNCH((k_refine_ragged<M, true>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, kT,
                           eta, Tout, cost, status);
    else
        TGMS_LAUNCH((k_refine_ragged<M, false>), dim3(grid), dim3(W64), 0, stream, n, perm, so, W, T, ED, kT,
                           eta, Tout, cost, status);
    return hipSuccess;
}

template <int MLO, int MHI>
hipError_t multi_launch(const GroupTable& tab, bool refine, const int32_t* so, const double* W, const double* T,
                        const double* ED, double kT, double eta, double* Tout, double* cost, double* C,
                        int32_t* status, hipStream_t stream) {
    if (tab.ngroups <= 0) return hipSuccess;
    const unsigned grid = (unsigned)tab.blk_end[tab.ngroups - 1];
    if (grid == 0) return hipSuccess;
    if constexpr (MLO > MHI) return hipSuccess;  // an empty class
    else if (refine) {
        if (ED)
            TGMS_LAUNCH((k_refine_multi<MLO, MHI, true>), dim3(grid), dim3(W64), 0, stream, tab, so, W, T, ED,
                               kT, eta, Tout, cost, status);
        else
            TGMS_LAUNCH((k_refine_multi<MLO, MHI, false>), dim3(grid), dim3(W64), 0, stream, tab, so, W, T, ED,
                               kT, eta, Tout, cost, status);
    } else {
        if (ED)
            TGMS_LAUNCH((k_reduced_multi<MLO, MHI, true>), dim3(grid), dim3(W64), 0, stream, tab, so, W, T,
                               ED, C, status);
        else
            TGMS_LAUNCH((k_reduced_multi<MLO, MHI, false>), dim3(grid), dim3(W64), 0, stream, tab, so, W, T,
                               ED, C, status);
    }
    return hipSuccess;
}

}  // namespace

size_t perm_hist_bytes(int32_t B) {
    return (size_t)((B + PERM_BLOCK - 1) / PERM_BLOCK) * PERM_BINS * sizeof(int32_t);
}

hipError_t launch_group_perm(int32_t B, const int32_t* so, const int32_t* starts, int32_t* hist, int32_t* perm,
                             hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((B + PERM_BLOCK - 1) / PERM_BLOCK);
    PermStarts st{};
    for (int m = 1; m < PERM_BINS; ++m) st.s[m] = starts[m];
    TGMS_LAUNCH(k_perm_hist, dim3(grid), dim3(PERM_BLOCK), 0, stream, B, so, hist);
    TGMS_LAUNCH(k_perm_scatter, dim3(grid), dim3(PERM_BLOCK), 0, stream, B, so, hist, st, perm);
    return hipSuccess;
}

// SIMDs of the current device (4 per CU), cached per device
int device_simds() {
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return 1024;
        cache[dev] = 4 * cus;
    }
    return cache[dev];
}

hipError_t launch_group_plan_dev(int32_t n, int64_t S, const int32_t* so, int has_ed, int32_t* hist, int32_t* perm,
                                 DevPlan* plan, int32_t* status, double* C, double* cost, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + PERM_BLOCK - 1) / PERM_BLOCK);
    TGMS_LAUNCH(k_perm_hist, dim3(grid), dim3(PERM_BLOCK), 0, stream, n, so, hist);
    TGMS_LAUNCH(k_plan_scatter, dim3(grid), dim3(PERM_BLOCK), 0, stream, n, S, so, has_ed, device_simds(), hist, perm,
                plan, status, C, cost);
    return hipSuccess;
}

// (instantiated only for the classes a call can launch: end derivatives use the ED
// boundary, so e.g. <1, TWO_WAVE_MAX_M, true> never exists)
template <int MLO, int MHI, bool HAS_ED>
hipError_t loop_dev_launch(int cls, int32_t n, DevPlan* plan, const int32_t* so, const double* W, double* T,
                           const double* ED, double kT, double eta, int32_t iters, double* cost, double* C,
                           int32_t* status, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    // the one-wave class: as many blocks as SIMDs at most (persistent when it has more tiles
    // than that, k_plan_scatter); the two-wave class one block per tile
    unsigned grid = dev_loop_grid(n);
    if (TGMS_C5_PERSIST && cls == 1) grid = std::min<unsigned>(grid, (unsigned)device_simds());
    if constexpr (MLO <= MHI)  // (MLO > MHI: an empty class, every M at two waves)
        TGMS_LAUNCH((k_refine_loop_dev<MLO, MHI, HAS_ED>), dim3(grid), dim3(W64), 0, stream, plan, cls, so, W, T, ED,
                    kT, eta, iters, cost, C, status);
    return hipSuccess;
}

hipError_t launch_refine_loop_dev(int cls, int32_t n, DevPlan* plan, const int32_t* so, const double* W,
                                  double* T, const double* ED, double kT, double eta, int32_t iters, double* cost,
                                  double* C, int32_t* status, hipStream_t stream) {
    constexpr int A = TGMS_TWO_WAVE_MAX_M, E = TGMS_TWO_WAVE_MAX_M_ED;
    if (ED) {
        if (cls == 0) return loop_dev_launch<1, E, true>(0, n, plan, so, W, T, ED, kT, eta, iters, cost, C, status, stream);
        return loop_dev_launch<E + 1, 16, true>(1, n, plan, so, W, T, ED, kT, eta, iters, cost, C, status, stream);
    }
    if (cls == 0) return loop_dev_launch<1, A, false>(0, n, plan, so, W, T, ED, kT, eta, iters, cost, C, status, stream);
    return loop_dev_launch<A + 1, 16, false>(1, n, plan, so, W, T, ED, kT, eta, iters, cost, C, status, stream);
}

template <int MLO, int MHI, bool HAS_ED>
hipError_t solve_dev_launch(int cls, int32_t n, const DevPlan* plan, const int32_t* so, const double* W,
                            const double* T, const double* ED, double* C, int32_t* status, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if constexpr (MLO <= MHI)
        TGMS_LAUNCH((k_reduced_multi_dev<MLO, MHI, HAS_ED>), dim3(dev_loop_grid(n)), dim3(W64), 0, stream, plan, cls,
                    so, W, T, ED, C, status);
    return hipSuccess;
}

hipError_t launch_reduced_multi_dev(int cls, int32_t n, const DevPlan* plan, const int32_t* so, const double* W,
                                    const double* T, const double* ED, double* C, int32_t* status,
                                    hipStream_t stream) {
    constexpr int A = TGMS_TWO_WAVE_MAX_M, E = TGMS_TWO_WAVE_MAX_M_ED;
    if (ED) {
        if (cls == 0) return solve_dev_launch<1, E, true>(0, n, plan, so, W, T, ED, C, status, stream);
        return solve_dev_launch<E + 1, 16, true>(1, n, plan, so, W, T, ED, C, status, stream);
    }
    if (cls == 0) return solve_dev_launch<1, A, false>(0, n, plan, so, W, T, ED, C, status, stream);
    return solve_dev_launch<A + 1, 16, false>(1, n, plan, so, W, T, ED, C, status, stream);
}

hipError_t launch_ragged_multi(int cls, const GroupTable& tab, bool refine, const int32_t* so, const double* W,
                               const double* T, const double* ED, double kT, double eta, double* Tout, double* cost,
                               double* C, int32_t* status, hipStream_t stream) {
    constexpr int A = TGMS_TWO_WAVE_MAX_M, E = TGMS_TWO_WAVE_MAX_M_ED;
    if (ED) {
        if (cls == 0) return multi_launch<1, E>(tab, refine, so, W, T, ED, kT, eta, Tout, cost, C, status, stream);
        return multi_launch<E + 1, 16>(tab, refine, so, W, T, ED, kT, eta, Tout, cost, C, status, stream);
    }
    if (cls == 0) return multi_launch<1, A>(tab, refine, so, W, T, ED, kT, eta, Tout, cost, C, status, stream);
    return multi_launch<A + 1, 16>(tab, refine, so, W, T, ED, kT, eta, Tout, cost, C, status, stream);
}

#define TGMS_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

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

hipError_t launch_refine_uniform(int M, int32_t B, const double* W, const double* T, const double* ED, double kT,
                                 double eta, double* Tout, double* cost, int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return refine_uniform_M<m>(B, W, T, ED, kT, eta, Tout, cost, status, stream);
        TGMS_CASES(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_refine_ragged_group(int M, int32_t n, const int32_t* perm, const int32_t* so, const double* W,
                                      const double* T, const double* ED, double kT, double eta, double* Tout,
                                      double* cost, int32_t* status, hipStream_t stream) {
    switch (M) {
#define X(m) \
    case m: return refine_ragged_M<m>(n, perm, so, W, T, ED, kT, eta, Tout, cost, status, stream);
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

#ifdef TGMS_STAMPS
extern "C" int tgms_debug_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tgms::g_stamps), sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}
#endif
