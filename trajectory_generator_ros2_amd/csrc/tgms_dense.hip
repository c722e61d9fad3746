// tgms_dense.hip — TGMS_METHOD_DENSE_KKT: the survey's literal a1-a3 on gfx950.
//
// One WORKGROUP (NWV = 16 wavefronts) per trajectory; [[2Q, A^T],[A, 0]] (SURVEY.md
// §8(a) a1: snap Hessian Q, a2: endpoint/continuity rows A with right-hand side b) is
// assembled in LDS (N = 14M+2, N^2*8 B = 161,312 B at M = 10, so one trajectory per CU
// and all its parallelism is inside the workgroup).  LU with partial pivoting:
//   - rows never move; a position -> row permutation lives in registers (identical in
//     every wave), so a step has exactly one workgroup barrier;
//   - the rank-1 update of step k deals rows round-robin to the waves (lanes over
//     columns, rows with a zero multiplier skipped: the KKT stays sparse for a long
//     time); while updating, each wave also finds its best pivot candidate for column
//     k+1 and leaves it in a double-buffered LDS slot, so the pivot search of step k+1
//     is NWV LDS reads, not a column scan and shuffle reduction;
//   - the 3 right-hand sides live in wave 0's registers (lane = position), eliminated
//     on the fly; wave 0 back-substitutes with the stored inverse pivots.
// Measured (M = 10, B = 65536): 228 ms with one wave per trajectory -> ~122 ms; the
// per-step phase profile (scripts/dstamps.py) is LDS-latency bound, see DESIGN.md.
#include "tgms_device.h"
#include "tgms_internal.h"

namespace tgms {
namespace {


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

// broadcast lane src (wave-uniform) to the wave: two v_readlane, no LDS round trip
__device__ __forceinline__ double bcast(double v, int src) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, src);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), src);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

constexpr int NWV = 16;  // wavefronts per trajectory
#ifdef TGMS_DENSE_STAMPS  // diagnostic build: per-step phase timestamps of wave 0 in blocks < 64
constexpr int DST_BLOCKS = 64, DST_STEPS = 160;
__device__ unsigned long long g_dstamps[DST_BLOCKS * DST_STEPS * 4];
#define DSTAMP(k, i)                                                                          \
    do {                                                                                      \
        asm volatile("" ::: "memory");                                                        \
        if (bi < DST_BLOCKS && tid == 0)                                                      \
            g_dstamps[(bi * DST_STEPS + (k)) * 4 + (i)] = __builtin_amdgcn_s_memtime();       \
    } while (0)
#else
#define DSTAMP(k, i) \
    do {             \
    } while (0)
#endif
constexpr int DR = 1;  // rows per rank-1 update batch

template <int M, bool HAS_ED>
__global__ __launch_bounds__(W64 * NWV) void k_dense_kkt(int32_t n_traj, const int32_t* __restrict__ ids,
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
    double* A = smem;             // N x N row-major KKT

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar loop bounds
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
        double sum = 0.0;
        for (int q = 0; q < (M + 1) * 3; ++q) sum += w[q] * 0.0;
        if (HAS_ED)
            for (int q = 0; q < 18; ++q) sum += ed[q] * 0.0;
        valid = valid && (sum == 0.0);
    }

    DSTAMP(N + 1, 0);
    for (int e = tid; e < N * N; e += W64 * NWV) A[e] = 0.0;
    __syncthreads();
    // a1: 2Q blocks
    for (int e = tid; e < M * 16; e += W64 * NWV) {
        const int i = e >> 4, j = 4 + ((e >> 2) & 3), k = 4 + (e & 3);
        const int ex = j + k - 7;
        A[(8 * i + j) * N + 8 * i + k] = 2.0 * dfac(j, 4) * dfac(k, 4) * ipow(tt[i], ex) / (double)ex;
    }
    // a2: constraint rows (and their transposes), one thread per row
    for (int r = tid; r < m; r += W64 * NWV) {
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
    // right-hand sides in wave 0's registers: lane owns rows lane + 64*s
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

    // a3: LU with partial pivoting.  Rows never move: permv (registers; every wave holds
    // the same copy) maps elimination position -> physical row, so a step needs one
    // barrier: each wave repeats the pivot search on column k, then updates the rows it
    // owns (positions k+1+wave, k+1+wave+NWV, ...); wave 0 also the right-hand sides.
    static_assert(S <= 3, "N <= 192");
    int permv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) permv[s] = lane + W64 * s;
    auto perm_at = [&](int pos) -> int {  // wave-uniform position -> physical row
        // read every slot, select the scalar (a select on permv itself is folded into
        // an indexed access, i.e. scratch)
        const int l = pos & 63;
        int v = __builtin_amdgcn_readlane(permv[0], l);
        if constexpr (S > 1) v = pos >= W64 ? __builtin_amdgcn_readlane(permv[1], l) : v;
        if constexpr (S > 2) v = pos >= 2 * W64 ? __builtin_amdgcn_readlane(permv[S - 1], l) : v;
        return v;
    };
    // per-wave pivot candidates for column k+1, found while updating step k's rows
    // (double-buffered by step parity: a step's readers finish before the next writers)
    __shared__ double cand_v[2][NWV];
    __shared__ int cand_i[2][NWV];
    __shared__ double ipiv_s[N];  // 1 / pivot of each position, for the back substitution
    bool singular = false;
    for (int k = 0; k < N; ++k) {
        const int ks = k / W64, kl = k % W64;
        DSTAMP(k, 0);
        double best = -1.0;
        int bidx = N;
        if (k == 0) {  // first column: a full search (later columns: candidates of step k-1)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int i = lane + W64 * s;
                if (i < N) {
                    const double v = fabs(A[permv[s] * N]);
                    if (v > best) {
                        best = v;
                        bidx = i;
                    }
                }
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const double ov = __shfl_xor(best, off, W64);
                const int oi = __shfl_xor(bidx, off, W64);
                if (ov > best || (ov == best && oi < bidx)) {
                    best = ov;
                    bidx = oi;
                }
            }
        } else {  // max |.|, ties to the lowest position: the same order as the full search
            const double* cb = cand_v[(k - 1) & 1];
            const int* ci = cand_i[(k - 1) & 1];
            double ov[NWV];
            int oi[NWV];
#pragma unroll
            for (int q = 0; q < NWV; ++q) {  // all loads in flight, then branch-free selects
                ov[q] = cb[q];
                oi[q] = ci[q];
            }
#pragma unroll
            for (int q = 0; q < NWV; ++q) {
                const bool take = (ov[q] > best) | ((ov[q] == best) & (oi[q] < bidx));
                best = take ? ov[q] : best;
                bidx = take ? oi[q] : bidx;
            }
        }
        if (!__builtin_amdgcn_readfirstlane(best > 0.0)) {  // identical in every wave
            singular = true;
            break;
        }
        const int p = __builtin_amdgcn_readfirstlane(bidx);
        if (p != k) {
            const int ps = p / W64, pl = p % W64;
            const int rk = perm_at(k), rp = perm_at(p);
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int i = lane + W64 * s;
                permv[s] = i == k ? rp : (i == p ? rk : permv[s]);
            }
            if (wave == 0) {
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
        }
        DSTAMP(k, 1);
        const double* uk = A + perm_at(k) * N;
        const double ipiv = 1.0 / uk[k];
        if (tid == 0) ipiv_s[k] = ipiv;
        double u[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int j = k + 1 + lane + W64 * s;
            u[s] = (j < N) ? uk[j] : 0.0;
        }
        if (wave == 0) {
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
                    const double l = A[permv[s] * N + k] * ipiv;
#pragma unroll
                    for (int a = 0; a < 3; ++a) rhs[s][a] -= l * rk[a];
                }
            }
        }
        DSTAMP(k, 2);
        const double u1 = (k + 1 < N) ? uk[k + 1] : 0.0;  // = u[0] in lane 0
        double cbest = -1.0;
        int cidx = N;
        // rank-1 update, DR rows per batch so their LDS reads overlap; rows whose
        // multiplier is zero (most of them early on: the KKT is sparse) are skipped
        for (int pos0 = k + 1 + wave; pos0 < N; pos0 += NWV * DR) {
            int ph[DR];
            double l[DR], a1[DR];
#pragma unroll
            for (int r = 0; r < DR; ++r) {
                const int pos = pos0 + NWV * r;  // loads unconditional (clamped): one wait
                ph[r] = perm_at(pos < N ? pos : N - 1);
                const double akr = A[ph[r] * N + k];
                a1[r] = (k + 1 < N) ? A[ph[r] * N + k + 1] : 0.0;
                l[r] = pos < N ? akr * ipiv : 0.0;
            }
#pragma unroll
            for (int r = 0; r < DR; ++r) {  // this row's column k+1 after the update
                const int pos = pos0 + NWV * r;
                const double c = fabs(l[r] != 0.0 ? __builtin_fma(-l[r], u1, a1[r]) : a1[r]);
                const bool take = (pos < N) & (c > cbest);
                cbest = take ? c : cbest;
                cidx = take ? pos : cidx;
            }
            double v[DR][S];
#pragma unroll
            for (int r = 0; r < DR; ++r)
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int j = k + 1 + lane + W64 * s;
                    v[r][s] = (l[r] != 0.0 && j < N) ? A[ph[r] * N + j] : 0.0;
                }
#pragma unroll
            for (int r = 0; r < DR; ++r)
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int j = k + 1 + lane + W64 * s;
                    if (l[r] != 0.0 && j < N) A[ph[r] * N + j] = __builtin_fma(-l[r], u[s], v[r][s]);
                }
        }
        if (lane == 0) {
            cand_v[k & 1][wave] = cbest;
            cand_i[k & 1][wave] = cidx;
        }
        DSTAMP(k, 3);
        __syncthreads();
    }
    DSTAMP(N, 0);
    if (wave != 0) return;
    // back substitution (column oriented, wave 0); x overwrites rhs
    if (!singular) {
        for (int k = N - 1; k >= 0; --k) {
            const int ks = k / W64, kl = k % W64;
            const double ipiv = ipiv_s[k];
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
                    const double aik = A[permv[s] * N + k];
#pragma unroll
                    for (int a = 0; a < 3; ++a) rhs[s][a] -= aik * xk[a];
                }
            }
        }
    }
    DSTAMP(N, 1);
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

template <int M>
hipError_t dense_M(int32_t n_traj, const int32_t* ids, const int32_t* so, const double* W,
                   const double* T, const double* ED, double* C, int32_t* status,
                   hipStream_t stream) {
    constexpr int N = 14 * M + 2;
    const size_t lds = sizeof(double) * (size_t)(N * N);
    if (n_traj <= 0) return hipSuccess;
    hipError_t e;
    if (ED) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dense_kkt<M, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        TGMS_LAUNCH((k_dense_kkt<M, true>), dim3(n_traj), dim3(W64 * NWV), lds, stream, n_traj, ids, so, W, T, ED, C, status);
    } else {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dense_kkt<M, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        TGMS_LAUNCH((k_dense_kkt<M, false>), dim3(n_traj), dim3(W64 * NWV), lds, stream, n_traj, ids, so, W, T, ED, C, status);
    }
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

#ifdef TGMS_DENSE_STAMPS
extern "C" int tgms_debug_dense_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tgms::g_dstamps), sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}
#endif
