/*
 * minsnap_oracle.c — CPU fp64 restatement of the batched minimum-snap solve.
 *
 * TEST INFRASTRUCTURE ONLY (see minsnap_oracle.h): the checker for the HIP path
 * and the timed CPU baseline ("port") in bench.py.  Never linked into libtgms.
 *
 * Parity unpinned against the reference: jrached/trajectory_generator_ros2 has
 * no min-snap code at all (src/TrajectoryGenerator.cpp:1-789 holds
 * a ROS node, a parameter factory and an FSM; every primitive in
 * src/trajectories/ holds closed-form primitives only).  The oracle is pinned by exact
 * rational solves (oracle/exact.py -> tests/golden/) and closed forms instead.
 *
 * The formulation follows SURVEY.md §8(a):
 *   a1  snap-cost Hessian  Q_i[j][k] = (j!/(j-4)!)(k!/(k-4)!) T^(j+k-7)/(j+k-7), j,k in 4..7
 *   a2  endpoint + continuity rows built from r_k(t)_j = j!/(j-k)! t^(j-k)
 *   a3  KKT [[2Q, A^T],[A, 0]] [c; lambda] = [0; b], three right-hand sides,
 *       LU with partial pivoting
 *   a4  coefficients [seg][axis][8], ascending powers of local time
 *   a5  sampling at dt with the last sample pinned (Line.cpp:80-82 convention)
 */
#include "minsnap_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- helpers */

/* j!/(j-k)! : the k-th derivative factor of t^j (0 when k > j). */
static double dfac(int j, int k) {
    if (k > j) return 0.0;
    double r = 1.0;
    for (int q = 0; q < k; ++q) r *= (double)(j - q);
    return r;
}

/* r_k(t)_j = j!/(j-k)! t^(j-k) written into row[0..7]. */
static void deriv_row(int k, double t, double* row) {
    for (int j = 0; j < 8; ++j) {
        if (j < k) { row[j] = 0.0; continue; }
        double p = 1.0;
        for (int q = 0; q < j - k; ++q) p *= t;
        row[j] = dfac(j, k) * p;
    }
}

static int inputs_valid(int M, const double* W, const double* T, const double* ED) {
    if (M < 1 || M > ORACLE_MAX_SEGMENTS) return 0;
    for (int i = 0; i < M; ++i)
        if (!(T[i] > 0.0) || !isfinite(T[i])) return 0;
    for (int i = 0; i < 3 * (M + 1); ++i)
        if (!isfinite(W[i])) return 0;
    if (ED)
        for (int i = 0; i < 18; ++i)
            if (!isfinite(ED[i])) return 0;
    return 1;
}

/* end derivative k (1..3) at end e (0 start, 1 final), axis a */
static double end_deriv(const double* ED, int e, int k, int a) {
    return ED ? ED[e * 9 + (k - 1) * 3 + a] : 0.0;
}

/* Dense LU with partial pivoting, in place, n x n row-major A, nrhs columns in
 * row-major B ([n][nrhs]).  Solution overwrites B.  Returns 0 or ORACLE_SINGULAR. */
static int lu_solve(int n, double* A, int nrhs, double* B) {
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = fabs(A[i * n + k]);
            if (v > best) { best = v; p = i; }
        }
        if (!(best > 0.0)) return ORACLE_SINGULAR;
        if (p != k) {
            for (int j = 0; j < n; ++j) { double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
            for (int r = 0; r < nrhs; ++r) { double t = B[k * nrhs + r]; B[k * nrhs + r] = B[p * nrhs + r]; B[p * nrhs + r] = t; }
        }
        double piv = A[k * n + k];
        for (int i = k + 1; i < n; ++i) {
            double l = A[i * n + k];
            if (l == 0.0) continue;
            l /= piv;
            A[i * n + k] = l;
            for (int j = k + 1; j < n; ++j) A[i * n + j] -= l * A[k * n + j];
            for (int r = 0; r < nrhs; ++r) B[i * nrhs + r] -= l * B[k * nrhs + r];
        }
    }
    for (int k = n - 1; k >= 0; --k) {
        for (int r = 0; r < nrhs; ++r) {
            double s = B[k * nrhs + r];
            for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * B[j * nrhs + r];
            B[k * nrhs + r] = s / A[k * n + k];
        }
    }
    return ORACLE_OK;
}

/* Thread-local grow-only scratch: per-call malloc of a 160 KB KKT goes through
 * mmap/munmap and serialises OpenMP threads on page faults. */
static _Thread_local double* tls_buf = NULL;
static _Thread_local size_t tls_cap = 0;
static double* scratch(size_t n_doubles) {
    if (n_doubles > tls_cap) {
        free(tls_buf);
        tls_buf = (double*)malloc(sizeof(double) * n_doubles);
        tls_cap = tls_buf ? n_doubles : 0;
    }
    return tls_buf;
}

/* ------------------------------------------------- KKT formulations (a1–a3) */

/* Assemble [[2Q, A^T],[A, 0]] and [0; b].  cont = highest continuous derivative
 * at interior knots (3 or 4).  Returns N. */
static int assemble_kkt_cont(int M, int cont, const double* W, const double* T,
                             const double* ED, double* K, double* rhs) {
    const int n = 8 * M;
    const int m = 8 + (2 + cont) * (M - 1);
    const int N = n + m;
    memset(K, 0, sizeof(double) * (size_t)N * N);
    memset(rhs, 0, sizeof(double) * (size_t)N * 3);

    /* a1: block-diagonal snap Hessian, entries in rows/cols 4..7 of each segment */
    for (int i = 0; i < M; ++i) {
        for (int j = 4; j < 8; ++j)
            for (int k = 4; k < 8; ++k) {
                int e = j + k - 7;
                double tp = 1.0;
                for (int q = 0; q < e; ++q) tp *= T[i];
                double q = dfac(j, 4) * dfac(k, 4) * tp / (double)e;
                K[(8 * i + j) * N + (8 * i + k)] = 2.0 * q;
            }
    }

    /* a2: equality rows; row r of A is KKT row n+r, column n+r of A^T */
    double row[8];
    int r = 0;
#define PUT(seg, coefrow, scale)                                        \
    do {                                                                \
        for (int j_ = 0; j_ < 8; ++j_) {                                \
            double v_ = (scale) * (coefrow)[j_];                        \
            K[(n + r) * N + 8 * (seg) + j_] += v_;                      \
            K[(8 * (seg) + j_) * N + (n + r)] += v_;                    \
        }                                                               \
    } while (0)
    /* start endpoint: r_k(0) on segment 0 */
    for (int k = 0; k < 4; ++k, ++r) {
        deriv_row(k, 0.0, row);
        PUT(0, row, 1.0);
        for (int a = 0; a < 3; ++a) rhs[(n + r) * 3 + a] = (k == 0) ? W[a] : end_deriv(ED, 0, k, a);
    }
    /* final endpoint: r_k(T_{M-1}) on segment M-1 */
    for (int k = 0; k < 4; ++k, ++r) {
        deriv_row(k, T[M - 1], row);
        PUT(M - 1, row, 1.0);
        for (int a = 0; a < 3; ++a) rhs[(n + r) * 3 + a] = (k == 0) ? W[3 * M + a] : end_deriv(ED, 1, k, a);
    }
    /* interior knots i = 1..M-1 between segment i-1 and segment i */
    for (int i = 1; i < M; ++i) {
        deriv_row(0, T[i - 1], row);
        PUT(i - 1, row, 1.0);
        for (int a = 0; a < 3; ++a) rhs[(n + r) * 3 + a] = W[3 * i + a];
        ++r;
        deriv_row(0, 0.0, row);
        PUT(i, row, 1.0);
        for (int a = 0; a < 3; ++a) rhs[(n + r) * 3 + a] = W[3 * i + a];
        ++r;
        for (int k = 1; k <= cont; ++k, ++r) {
            deriv_row(k, T[i - 1], row);
            PUT(i - 1, row, 1.0);
            deriv_row(k, 0.0, row);
            PUT(i, row, -1.0);
        }
    }
#undef PUT
    return (r == m) ? N : -1;
}

int oracle_assemble_kkt(int M, const double* waypoints, const double* seg_times,
                        const double* end_derivs, double* K, double* rhs) {
    if (!inputs_valid(M, waypoints, seg_times, end_derivs)) return -1;
    return assemble_kkt_cont(M, 4, waypoints, seg_times, end_derivs, K, rhs);
}

static int solve_kkt(int M, int cont, const double* W, const double* T, const double* ED,
                     double* C) {
    const int N = 8 * M + 8 + (2 + cont) * (M - 1);
    double* K = scratch((size_t)N * N + (size_t)N * 3);
    if (!K) return ORACLE_INVALID;
    double* rhs = K + (size_t)N * N;
    assemble_kkt_cont(M, cont, W, T, ED, K, rhs);
    int st = lu_solve(N, K, 3, rhs);
    if (st == ORACLE_OK)
        for (int i = 0; i < M; ++i)
            for (int a = 0; a < 3; ++a)
                for (int j = 0; j < 8; ++j) C[(i * 3 + a) * 8 + j] = rhs[(8 * i + j) * 3 + a];
    return st;
}

/* ---------------------------------------- square C6 interpolation system */

/* The minimiser of the snap integral is a C6 septic spline (variational
 * argument), so the 8M x 8M system {endpoints, interpolation, continuity of
 * d1..d6} has the same unique solution as the KKT. */
static int solve_square_c6(int M, const double* W, const double* T, const double* ED,
                           double* C) {
    const int n = 8 * M;
    double* A = scratch((size_t)n * n + (size_t)n * 3);
    if (!A) return ORACLE_INVALID;
    double* B = A + (size_t)n * n;
    memset(A, 0, sizeof(double) * ((size_t)n * n + (size_t)n * 3));
    double row[8];
    int r = 0;
    for (int k = 0; k < 4; ++k, ++r) {
        deriv_row(k, 0.0, row);
        for (int j = 0; j < 8; ++j) A[r * n + j] = row[j];
        for (int a = 0; a < 3; ++a) B[r * 3 + a] = (k == 0) ? W[a] : end_deriv(ED, 0, k, a);
    }
    for (int k = 0; k < 4; ++k, ++r) {
        deriv_row(k, T[M - 1], row);
        for (int j = 0; j < 8; ++j) A[r * n + 8 * (M - 1) + j] = row[j];
        for (int a = 0; a < 3; ++a) B[r * 3 + a] = (k == 0) ? W[3 * M + a] : end_deriv(ED, 1, k, a);
    }
    for (int i = 1; i < M; ++i) {
        deriv_row(0, T[i - 1], row);
        for (int j = 0; j < 8; ++j) A[r * n + 8 * (i - 1) + j] = row[j];
        for (int a = 0; a < 3; ++a) B[r * 3 + a] = W[3 * i + a];
        ++r;
        deriv_row(0, 0.0, row);
        for (int j = 0; j < 8; ++j) A[r * n + 8 * i + j] = row[j];
        for (int a = 0; a < 3; ++a) B[r * 3 + a] = W[3 * i + a];
        ++r;
        for (int k = 1; k <= 6; ++k, ++r) {
            deriv_row(k, T[i - 1], row);
            for (int j = 0; j < 8; ++j) A[r * n + 8 * (i - 1) + j] = row[j];
            deriv_row(k, 0.0, row);
            for (int j = 0; j < 8; ++j) A[r * n + 8 * i + j] = -row[j];
        }
    }
    int st = lu_solve(n, A, 3, B);
    if (st == ORACLE_OK)
        for (int i = 0; i < M; ++i)
            for (int a = 0; a < 3; ++a)
                for (int j = 0; j < 8; ++j) C[(i * 3 + a) * 8 + j] = B[(8 * i + j) * 3 + a];
    return st;
}

/* ---------------------------------------- reduced free-derivative system */

/* Septic Hermite segment on s in [0,1] with scaled end data
 * h = [y0, y0', y0'', y0''', y1, y1', y1'', y1'''] (y' = dy/ds).
 * Snap cost integral_0^1 (q'''')^2 ds = h^T KH h with the integer matrix below
 * (derived once, exactly, in oracle/exact.py: hermite_cost_matrix()).
 * For duration T and unscaled data g (h_a = T^sigma_a g_a, sigma = 0,1,2,3,0,1,2,3):
 *   integral_0^T (p'''')^2 dt = sum_ab KH[a][b] T^(sigma_a + sigma_b - 7) g_a g_b. */
static const double KH[8][8] = {
    {100800, 50400, 10080, 840, -100800, 50400, -10080, 840},
    {50400, 25920, 5400, 480, -50400, 24480, -4680, 360},
    {10080, 5400, 1200, 120, -10080, 4680, -840, 60},
    {840, 480, 120, 16, -840, 360, -60, 4},
    {-100800, -50400, -10080, -840, 100800, -50400, 10080, -840},
    {50400, 24480, 4680, 360, -50400, 25920, -5400, 480},
    {-10080, -4680, -840, -60, 10080, -5400, 1200, -120},
    {840, 360, 60, 4, -840, 480, -120, 16}};
/* d_{4..7} = EH * h (rows 4..7 of the Hermite interpolation map). */
static const double EH[4][8] = {
    {-35, -20, -5, -2.0 / 3.0, 35, -15, 5.0 / 2.0, -1.0 / 6.0},
    {84, 45, 10, 1, -84, 39, -7, 1.0 / 2.0},
    {-70, -36, -15.0 / 2.0, -2.0 / 3.0, 70, -34, 13.0 / 2.0, -1.0 / 2.0},
    {20, 10, 2, 1.0 / 6.0, -20, 10, -2, 1.0 / 6.0}};
static const int SIG[8] = {0, 1, 2, 3, 0, 1, 2, 3};

/* Hermite data (p, v, a, j) at knot k, axis a, given the solved free derivatives */
static void knot_data(int M, int k, int a, const double* W, const double* ED,
                      const double* U /* [(M-1)][3 derivs][3 axes] */, double out[4]) {
    out[0] = W[3 * k + a];
    for (int d = 1; d <= 3; ++d) {
        if (k == 0) out[d] = end_deriv(ED, 0, d, a);
        else if (k == M) out[d] = end_deriv(ED, 1, d, a);
        else out[d] = U[((k - 1) * 3 + (d - 1)) * 3 + a];
    }
}

/* Coefficients of segment i from its end data (shared with the sampler tests). */
static void hermite_to_coeffs(double T, const double g0[4], const double g1[4], double c[8]) {
    double Tp[8];
    Tp[0] = 1.0;
    for (int q = 1; q < 8; ++q) Tp[q] = Tp[q - 1] * T;
    double h[8] = {g0[0], g0[1] * T, g0[2] * Tp[2], g0[3] * Tp[3],
                   g1[0], g1[1] * T, g1[2] * Tp[2], g1[3] * Tp[3]};
    c[0] = g0[0];
    c[1] = g0[1];
    c[2] = g0[2] * 0.5;
    c[3] = g0[3] / 6.0;
    for (int r = 0; r < 4; ++r) {
        /* translation invariance: EH[r][0] = -EH[r][4]; use the difference */
        double d = EH[r][4] * (h[4] - h[0]);
        for (int q = 1; q < 4; ++q) d += EH[r][q] * h[q] + EH[r][4 + q] * h[4 + q];
        c[4 + r] = d / Tp[4 + r];
    }
}

static int solve_reduced(int M, const double* W, const double* T, const double* ED,
                         double* C) {
    const int nf = 3 * (M - 1); /* free unknowns per axis: (v, a, j) at interior knots */
    double* U = NULL;
    if (nf > 0) {
        double* H = (double*)calloc((size_t)nf * nf, sizeof(double));
        double* R = (double*)calloc((size_t)nf * 3, sizeof(double));
        if (!H || !R) { free(H); free(R); return ORACLE_INVALID; }
        /* segment i couples knot i (slots 0..3) and knot i+1 (slots 4..7) */
        for (int i = 0; i < M; ++i) {
            double Ks[8][8];
            for (int x = 0; x < 8; ++x)
                for (int y = 0; y < 8; ++y) Ks[x][y] = KH[x][y] * pow(T[i], SIG[x] + SIG[y] - 7);
            for (int x = 0; x < 8; ++x) {
                int kx = (x < 4) ? i : i + 1, dx = x & 3;
                if (dx == 0 || kx == 0 || kx == M) continue; /* not a free unknown */
                int rx = 3 * (kx - 1) + (dx - 1);
                for (int y = 0; y < 8; ++y) {
                    int ky = (y < 4) ? i : i + 1, dy = y & 3;
                    if (y == 0) continue; /* folded into y == 4: KH[x][0] = -KH[x][4] */
                    if (dy != 0 && ky != 0 && ky != M) {
                        H[rx * nf + 3 * (ky - 1) + (dy - 1)] += Ks[x][y];
                    } else {
                        for (int a = 0; a < 3; ++a) {
                            /* positions enter only through the segment displacement
                             * (translation invariance), avoiding cancellation */
                            double g = (dy == 0) ? W[3 * (i + 1) + a] - W[3 * i + a]
                                                 : end_deriv(ED, ky == 0 ? 0 : 1, dy, a);
                            R[rx * 3 + a] -= Ks[x][y] * g;
                        }
                    }
                }
            }
        }
        /* dense Cholesky H = L L^T (H is SPD for T_i > 0) */
        for (int j = 0; j < nf; ++j) {
            double s = H[j * nf + j];
            for (int q = 0; q < j; ++q) s -= H[j * nf + q] * H[j * nf + q];
            if (!(s > 0.0)) { free(H); free(R); return ORACLE_SINGULAR; }
            double l = sqrt(s);
            H[j * nf + j] = l;
            for (int i2 = j + 1; i2 < nf; ++i2) {
                double t = H[i2 * nf + j];
                for (int q = 0; q < j; ++q) t -= H[i2 * nf + q] * H[j * nf + q];
                H[i2 * nf + j] = t / l;
            }
        }
        for (int a = 0; a < 3; ++a) {
            for (int i2 = 0; i2 < nf; ++i2) {
                double t = R[i2 * 3 + a];
                for (int q = 0; q < i2; ++q) t -= H[i2 * nf + q] * R[q * 3 + a];
                R[i2 * 3 + a] = t / H[i2 * nf + i2];
            }
            for (int i2 = nf - 1; i2 >= 0; --i2) {
                double t = R[i2 * 3 + a];
                for (int q = i2 + 1; q < nf; ++q) t -= H[q * nf + i2] * R[q * 3 + a];
                R[i2 * 3 + a] = t / H[i2 * nf + i2];
            }
        }
        free(H);
        U = R; /* [(M-1)][3][3] */
    }
    for (int i = 0; i < M; ++i)
        for (int a = 0; a < 3; ++a) {
            double g0[4], g1[4];
            knot_data(M, i, a, W, ED, U, g0);
            knot_data(M, i + 1, a, W, ED, U, g1);
            hermite_to_coeffs(T[i], g0, g1, &C[(i * 3 + a) * 8]);
        }
    free(U);
    return ORACLE_OK;
}

/* ------------------------------------------------------------------ driver */

/* Position of KKT_C4 row/column q in the segment-interleaved order
 *   [start rows (4) | c_0 (8) | knot-1 rows (6) | c_1 (8) | ... | c_{M-1} (8) | end rows (4)]
 * in which every nonzero lies within 9 of the diagonal. */
static int interleaved_pos(int M, int q) {
    const int n = 8 * M;
    if (q < n) return 4 + 14 * (q / 8) + q % 8;  /* coefficient j of segment i */
    const int r = q - n;
    if (r < 4) return r;                          /* start rows */
    if (r < 8) return 14 * M - 2 + (r - 4);       /* end rows */
    const int i = (r - 8) / 6, t = (r - 8) % 6;   /* knot after segment i */
    return 4 + 14 * i + 8 + t;
}

/* Dense GEPP of the permuted KKT: the same algorithm (lu_solve) the band kernel
 * performs, which skips only entries that are structurally zero in this order. */
static int solve_kkt_interleaved(int M, const double* W, const double* T, const double* ED, double* C) {
    const int N = 14 * M + 2;
    double* K = scratch((size_t)2 * N * N + (size_t)2 * N * 3);
    if (!K) return ORACLE_INVALID;
    double* rhs = K + (size_t)N * N;
    double* P = rhs + (size_t)N * 3;
    double* prhs = P + (size_t)N * N;
    assemble_kkt_cont(M, 4, W, T, ED, K, rhs);
    for (int q = 0; q < N; ++q) {
        const int pq = interleaved_pos(M, q);
        for (int s = 0; s < N; ++s) P[(size_t)pq * N + interleaved_pos(M, s)] = K[(size_t)q * N + s];
        for (int a = 0; a < 3; ++a) prhs[pq * 3 + a] = rhs[q * 3 + a];
    }
    int st = lu_solve(N, P, 3, prhs);
    if (st == ORACLE_OK)
        for (int i = 0; i < M; ++i)
            for (int a = 0; a < 3; ++a)
                for (int j = 0; j < 8; ++j) C[(i * 3 + a) * 8 + j] = prhs[interleaved_pos(M, 8 * i + j) * 3 + a];
    return st;
}

static int all_finite(const double* x, int n) {
    for (int i = 0; i < n; ++i)
        if (!isfinite(x[i])) return 0;
    return 1;
}

int oracle_solve(int formulation, int M, const double* W, const double* T, const double* ED,
                 double* C) {
    if (!W || !T || !C || !inputs_valid(M, W, T, ED)) return ORACLE_INVALID;
    int st;
    switch (formulation) {
        case ORACLE_KKT_C4: st = solve_kkt(M, 4, W, T, ED, C); break;
        case ORACLE_KKT_C3: st = solve_kkt(M, 3, W, T, ED, C); break;
        case ORACLE_SQUARE_C6: st = solve_square_c6(M, W, T, ED, C); break;
        case ORACLE_REDUCED: st = solve_reduced(M, W, T, ED, C); break;
        case ORACLE_KKT_BAND: st = solve_kkt_interleaved(M, W, T, ED, C); break;
        default: return ORACLE_INVALID;
    }
    if (st == ORACLE_OK && !all_finite(C, 24 * M)) st = ORACLE_NONFINITE;
    return st;
}

int oracle_solve_batch(int formulation, int32_t B, const int32_t* seg_offsets,
                       const double* waypoints, const double* seg_times,
                       const double* end_derivs, double* coeffs, int32_t* status,
                       int nthreads) {
    if (B < 0 || (B > 0 && (!seg_offsets || !waypoints || !seg_times || !coeffs)))
        return ORACLE_INVALID;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int worst = ORACLE_OK;
#pragma omp parallel for schedule(dynamic, 4) reduction(max : worst)
    for (int32_t b = 0; b < B; ++b) {
        int32_t s0 = seg_offsets[b], M = seg_offsets[b + 1] - s0;
        int st = oracle_solve(formulation, M, waypoints + 3 * ((int64_t)s0 + b), seg_times + s0,
                              end_derivs ? end_derivs + 18 * (int64_t)b : NULL,
                              coeffs + 24 * (int64_t)s0);
        if (status) status[b] = st;
        if (st > worst) worst = st;
    }
    return worst;
}

/* ----------------------------------------- time-allocation refinement */

/* Snap cost of one segment and its derivative in the duration, from the segment's
 * end data g = (w0, v0, a0, j0, w1, v1, a1, j1) per axis (KH above):
 *   J = sum_ab KH[a][b] T^(s_a+s_b-7) g_a g_b,
 *   dJ/dT = sum_ab KH[a][b] (s_a+s_b-7) T^(s_a+s_b-8) g_a g_b
 * (knot data held fixed: at the optimum only the explicit T dependence counts).
 * Evaluated in displacement form, as solve_reduced forms its right-hand side: with the
 * scaled data h_a = T^s_a g_a, J = T^-7 h^T KH h and dJ/dT = T^-8 h^T (KH o (s_a+s_b-7)) h;
 * KH (and its weighted copy, s = 0 at both positions) annihilates a common shift of the
 * two positions, so h_0 = 0 and h_4 = w1 - w0 — no absolute positions against KH's
 * +-100,800 entries.  The knot data are the solve's own: the start (v, a, j) are segment
 * i's c1, 2 c2, 6 c3; the end data are segment i+1's start (the shared knot) or the end
 * derivatives — no re-evaluation of the septic at T (whose terms cancel), no pow(). */
static void segment_cost(const double* c, const double* cn, const double* ED, const double* w0,
                         const double* w1, double T, double* J, double* dJ) {
    const double T2 = T * T, T3 = T2 * T, T4 = T2 * T2;
    const double T7 = T4 * T3, T8 = T4 * T4;
    double j = 0.0, dj = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double* ca = c + 8 * a;
        double e1[3];
        for (int d = 1; d <= 3; ++d)
            e1[d - 1] = cn ? (d == 1 ? cn[8 * a + 1] : d == 2 ? 2.0 * cn[8 * a + 2] : 6.0 * cn[8 * a + 3])
                           : end_deriv(ED, 1, d, a);
        const double h[8] = {0.0, ca[1] * T, 2.0 * ca[2] * T2, 6.0 * ca[3] * T3,
                             w1[a] - w0[a], e1[0] * T, e1[1] * T2, e1[2] * T3};
        for (int x = 0; x < 8; ++x) {
            double sj = 0.0, sd = 0.0;
            for (int y = 0; y < 8; ++y) {
                sj += KH[x][y] * h[y];
                sd += KH[x][y] * (double)(SIG[x] + SIG[y] - 7) * h[y];
            }
            j += h[x] * sj;
            dj += h[x] * sd;
        }
    }
    *J = j / T7;
    *dJ = dj / T8;
}

int oracle_refine_times(int formulation, int M, const double* W, double* T, const double* ED, double kT,
                        double eta, int iters, double* cost, double* C) {
    double buf[24 * ORACLE_MAX_SEGMENTS];
    double* c = C ? C : buf;
    if (!W || !T || !inputs_valid(M, W, T, ED)) return ORACLE_INVALID;
    for (int it = 0; it <= iters; ++it) {
        int st = oracle_solve(formulation, M, W, T, ED, c);
        if (st != ORACLE_OK) return st;
        double Jv[ORACLE_MAX_SEGMENTS], dJv[ORACLE_MAX_SEGMENTS], F = 0.0;
        for (int i = 0; i < M; ++i) {
            segment_cost(c + 24 * i, i + 1 < M ? c + 24 * (i + 1) : NULL, ED, W + 3 * i, W + 3 * (i + 1), T[i],
                         &Jv[i], &dJv[i]);
            F += Jv[i] + kT * T[i];
        }
        if (it == iters) { /* final times: report F, keep the final solve in C */
            if (cost) *cost = F;
            break;
        }
        if (!(F > 0.0)) continue;
        for (int i = 0; i < M; ++i) {
            double dtau = -eta * T[i] * (dJv[i] + kT) / F;
            dtau = dtau < -0.5 ? -0.5 : (dtau > 0.5 ? 0.5 : dtau);
            T[i] = T[i] * exp(dtau);
        }
    }
    return ORACLE_OK;
}

/* One step's ingredients at fixed times: the per-segment gradient dJ_i/dT_i and
 * F = sum_i J_i + kT sum_i T_i (what oracle_refine_times feeds its update), so a test
 * can pin a single GPU step, gradient included, without the iteration's amplification. */
int oracle_refine_grad(int formulation, int M, const double* W, const double* T, const double* ED, double kT,
                       double* dJ, double* cost) {
    double c[24 * ORACLE_MAX_SEGMENTS];
    if (!W || !T || !dJ || M < 1 || M > ORACLE_MAX_SEGMENTS || !inputs_valid(M, W, T, ED)) return ORACLE_INVALID;
    const int st = oracle_solve(formulation, M, W, T, ED, c);
    if (st != ORACLE_OK) return st;
    double F = 0.0;
    for (int i = 0; i < M; ++i) {
        double J;
        segment_cost(c + 24 * i, i + 1 < M ? c + 24 * (i + 1) : NULL, ED, W + 3 * i, W + 3 * (i + 1), T[i], &J,
                     &dJ[i]);
        F += J + kT * T[i];
    }
    if (cost) *cost = F;
    return ORACLE_OK;
}

int oracle_refine_batch(int formulation, int32_t B, const int32_t* seg_offsets, const double* waypoints,
                        double* seg_times, const double* end_derivs, double kT, double eta, int iters,
                        double* cost, double* coeffs, int32_t* status, int nthreads) {
    if (B < 0 || (B > 0 && (!seg_offsets || !waypoints || !seg_times))) return ORACLE_INVALID;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int worst = ORACLE_OK;
#pragma omp parallel for schedule(dynamic, 4) reduction(max : worst)
    for (int32_t b = 0; b < B; ++b) {
        int32_t s0 = seg_offsets[b], M = seg_offsets[b + 1] - s0;
        int st = oracle_refine_times(formulation, M, waypoints + 3 * ((int64_t)s0 + b), seg_times + s0,
                                     end_derivs ? end_derivs + 18 * (int64_t)b : NULL, kT, eta, iters,
                                     cost ? cost + b : NULL, coeffs ? coeffs + 24 * (int64_t)s0 : NULL);
        if (status) status[b] = st;
        if (st > worst) worst = st;
    }
    return worst;
}

/* --------------------------------------------------------------- sampling */

int64_t oracle_sample_count(double total_T, double dt) {
    if (!(dt > 0.0) || !(total_T >= 0.0)) return 0;
    double x = ceil(total_T / dt - 1e-9);
    int64_t n = (int64_t)x;
    if (n < 1) n = 1;
    return n + 1;
}

static void eval_poly(const double* c, double t, double out[4]) {
    /* p, p', p'', p''' by Horner on the derivative coefficients */
    for (int k = 0; k < 4; ++k) {
        double s = 0.0;
        for (int j = 7; j >= k; --j) s = s * t + dfac(j, k) * c[j];
        out[k] = s;
    }
}

static void yaw_of(int yaw_mode, double yaw_const, const double* v, const double* acc,
                   double* psi, double* dpsi) {
    double s2 = v[0] * v[0] + v[1] * v[1];
    if (yaw_mode == ORACLE_YAW_VELOCITY && s2 > 1e-6) {
        *psi = atan2(v[1], v[0]);
        *dpsi = (v[0] * acc[1] - v[1] * acc[0]) / s2;
    } else {
        *psi = yaw_const;
        *dpsi = 0.0;
    }
}

int64_t oracle_sample(int M, const double* coeffs, const double* T, const double* W,
                      const double* ED, double dt, int yaw_mode, double yaw_const,
                      double* out) {
    double tau[ORACLE_MAX_SEGMENTS + 1];
    if (M < 1 || M > ORACLE_MAX_SEGMENTS) return 0;
    tau[0] = 0.0;
    for (int i = 0; i < M; ++i) tau[i + 1] = tau[i] + T[i];
    int64_t n = oracle_sample_count(tau[M], dt);
    for (int64_t k = 0; k + 1 < n; ++k) {
        double t = (double)k * dt;
        int i = 0;
        while (i + 1 < M && tau[i + 1] <= t) ++i;
        double lt = t - tau[i];
        double* o = out + 14 * k;
        for (int a = 0; a < 3; ++a) {
            double d[4];
            eval_poly(coeffs + (i * 3 + a) * 8, lt, d);
            o[a] = d[0];
            o[3 + a] = d[1];
            o[6 + a] = d[2];
            o[9 + a] = d[3];
        }
        yaw_of(yaw_mode, yaw_const, o + 3, o + 6, o + 12, o + 13);
    }
    double* o = out + 14 * (n - 1);
    for (int a = 0; a < 3; ++a) {
        o[a] = W[3 * M + a];
        o[3 + a] = end_deriv(ED, 1, 1, a);
        o[6 + a] = end_deriv(ED, 1, 2, a);
        o[9 + a] = end_deriv(ED, 1, 3, a);
    }
    yaw_of(yaw_mode, yaw_const, o + 3, o + 6, o + 12, o + 13);
    return n;
}
