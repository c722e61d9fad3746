/*
 * minsnap_oracle.h — CPU fp64 restatement of the batched minimum-snap solve.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product library (libtgms.so) never links or calls it.
 *
 * Parity status: the reference (jrached/trajectory_generator_ros2) contains NO
 * minimum-snap solver, no tests and no fixtures, and its node
 * cannot be compiled here without stand-in headers (rclcpp, Eigen,
 * snapstack_msgs2 are absent).  Parity against the reference is therefore
 * UNPINNED for the coefficients.  This oracle is instead pinned by:
 *   (1) exact rational-arithmetic solves (oracle/exact.py, Python Fraction), which
 *       are the golden vectors in tests/golden/;
 *   (2) the closed-form single-segment rest-to-rest polynomial;
 *   (3) agreement of three independent formulations implemented below.
 *
 * Problem (SURVEY.md §8(a) rows a1–a4):
 *   M segments, segment i has duration T_i > 0, local time t in [0, T_i],
 *   p_i(t) = sum_{j=0..7} c_{i,j} t^j  (order 7, 8 coefficients, 3 axes).
 *   minimise  sum_axes sum_i  integral_0^{T_i} (p_i''''(t))^2 dt
 *   s.t. p_0^{(k)}(0) = (w_0, v_0, a_0, j_0)_k,  p_{M-1}^{(k)}(T_{M-1}) = (w_M, v_M, a_M, j_M)_k,
 *        interior knots: both adjacent segments pass through w_i and
 *        derivatives 1..4 are continuous (the survey's C4 KKT, N = 14M+2).
 *
 * Layouts (all fp64, row-major, trajectory-major "AoS"; these are the C-ABI
 * layouts of include/tgms.h):
 *   waypoints  [M+1][3]
 *   seg_times  [M]
 *   end_derivs [2][3][3]  = [start|final][v,a,j][x,y,z]; NULL = rest-to-rest
 *   coeffs     [M][3][8]  ascending powers in local time
 */
#ifndef MINSNAP_ORACLE_H
#define MINSNAP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_SEGMENTS 64

/* return codes (match tgms_status numerically) */
#define ORACLE_OK 0
#define ORACLE_INVALID 1
#define ORACLE_SINGULAR 2
#define ORACLE_NONFINITE 3

/* Formulation selectors for oracle_solve(). */
#define ORACLE_KKT_C4 0     /* survey a1-a3: [[2Q, A^T],[A, 0]], continuity of d1..d4, N = 14M+2 */
#define ORACLE_KKT_C3 1     /* same with continuity of d1..d3 only, N = 13M+3 */
#define ORACLE_SQUARE_C6 2  /* square 8M system: interpolation + continuity of d1..d6 */
#define ORACLE_REDUCED 3    /* reduced Hessian over free knot derivatives (v,a,j), dense Cholesky */
#define ORACLE_KKT_BAND 4   /* the KKT_C4 matrix in segment-interleaved order, dense GEPP (the
                               order in which it is banded; checker of TGMS_METHOD_BAND_KKT) */

/* Solve one trajectory. Returns ORACLE_* status. */
int oracle_solve(int formulation, int M, const double* waypoints, const double* seg_times,
                 const double* end_derivs, double* coeffs);

/* Batch over a CSR segment layout: trajectory b has seg_offsets[b+1]-seg_offsets[b]
 * segments; its waypoints start at row seg_offsets[b]+b of `waypoints` ([.][3]),
 * its times at seg_offsets[b], its coefficients at seg_offsets[b]*24.
 * end_derivs: NULL or [B][18].  status: nullable [B].  nthreads<=0: all cores. */
int oracle_solve_batch(int formulation, int32_t B, const int32_t* seg_offsets,
                       const double* waypoints, const double* seg_times,
                       const double* end_derivs, double* coeffs, int32_t* status,
                       int nthreads);

/* Dense KKT assembly exposed for tests (survey a1, a2): writes the N x N KKT matrix
 * (row-major) and the N x 3 right-hand side; returns N or -1. */
int oracle_assemble_kkt(int M, const double* waypoints, const double* seg_times,
                        const double* end_derivs, double* K, double* rhs);

/* Number of samples produced for one trajectory of total duration total_T at
 * period dt (see oracle_sample): ceil(total_T/dt - 1e-9) regular samples plus one
 * final sample pinned at total_T. */
int64_t oracle_sample_count(double total_T, double dt);

/* Time-allocation refinement (the GPU step of include/tgms.h, restated): `iters`
 * steps of  T_i <- T_i exp(clamp(-eta T_i (dJ_i/dT_i + kT) / F, -1/2, 1/2)),
 * F = sum_i J_i + kT sum_i T_i, each after a solve with `formulation`; T is
 * updated in place; cost (nullable) gets F at the final times and C (nullable)
 * the final solve. */
int oracle_refine_times(int formulation, int M, const double* waypoints, double* seg_times,
                        const double* end_derivs, double kT, double eta, int iters, double* cost,
                        double* coeffs);
/* The per-segment gradient dJ_i/dT_i (dJ[M]) and F at the given times (one solve, no
 * update): the ingredients of one refinement step. */
int oracle_refine_grad(int formulation, int M, const double* waypoints, const double* seg_times,
                       const double* end_derivs, double kT, double* dJ, double* cost);
int oracle_refine_batch(int formulation, int32_t B, const int32_t* seg_offsets, const double* waypoints,
                        double* seg_times, const double* end_derivs, double kT, double eta, int iters,
                        double* cost, double* coeffs, int32_t* status, int nthreads);

/* Yaw modes for sampling. */
#define ORACLE_YAW_CONSTANT 0
#define ORACLE_YAW_VELOCITY 1

/* Sample one trajectory at t_k = k*dt, k = 0..n-2, plus t = sum(T) as the last
 * sample, whose p/v/a/j are pinned exactly to (w_M, v_M, a_M, j_M).
 * out: [n][14] = p[3] v[3] a[3] j[3] psi dpsi.  Returns samples written. */
int64_t oracle_sample(int M, const double* coeffs, const double* seg_times,
                      const double* waypoints, const double* end_derivs, double dt,
                      int yaw_mode, double yaw_const, double* out);

#ifdef __cplusplus
}
#endif
#endif
