/*
 * tgms.h — C ABI of the MI355X-native batched minimum-snap solver (libtgms.so).
 *
 * This is the drop-in boundary of SURVEY.md §8(b).  The reference
 * (jrached/trajectory_generator_ros2) owns trajectories through
 *     std::unique_ptr<Trajectory> traj_           include/trajectory_generator_ros2/TrajectoryGenerator.hpp:83
 * built by the traj_type factory                  src/TrajectoryGenerator.cpp:175-388
 * and calls exactly three virtuals on it:
 *     generateTraj(goals, index_msgs, clock)      Trajectory.hpp:33-35, called at src/TrajectoryGenerator.cpp:71
 *     generateStopTraj(goals, msgs, idx, clock)   Trajectory.hpp:38-41, called at src/TrajectoryGenerator.cpp:516
 *     trajectoryInsideBounds(xmin..zmax)          Trajectory.hpp:44-46, called at src/TrajectoryGenerator.cpp:419
 * The reference has no solver behind those virtuals (every primitive is a
 * closed-form sampler).  A MinSnap primitive implements them on top
 * of the entry points below (trajectory_generator_ros2_amd/host/MinSnap.cpp):
 *     generateTraj            -> tgms_solve_batch (B = 1)  + tgms_sample_batch
 *     generateStopTraj        -> tgms_solve_batch with end_derivs (braking)  + tgms_sample_batch
 *     trajectoryInsideBounds  -> host check of waypoints and sampled extrema
 * and a swarm / sampling planner calls the same entry points with B up to 10^6.
 *
 * Conventions:
 *   - plain C, no exceptions cross the ABI; every call returns a tgms_status;
 *   - the caller owns every I/O buffer; the handle owns device workspace only;
 *   - a handle is bound to one HIP device and is single-thread-affine (the
 *     reference calls from its single rclcpp executor thread,
 *     src/trajectory_generator_node.cpp:30);
 *   - `*_device` entry points take device pointers and a hipStream_t passed as
 *     void* and are asynchronous; the others take host pointers and block.  Calls
 *     of one handle that use its device scratch (ragged plans, the refinement loop,
 *     the band-KKT method) may be issued on different streams: the handle orders
 *     them on the GPU with an event (each waits for the previous one's work);
 *     fp64 device arrays must be 16-byte aligned (TGMS_ERR_INVALID_ARG otherwise;
 *     hipMalloc allocations are, a slice at an odd element offset is not);
 *   - HIP-graph capture: uniform solves (tgms_solve_uniform_device, any method, and
 *     tgms_solve_batch_device / tgms_refine_*_device on a uniform batch) may be
 *     captured into a caller's graph.  Inside a capture the scratch event handshake
 *     is skipped.  A band-KKT capture needs the handle's slab sized by an earlier
 *     uncaptured band call of at least that M; from then on that slab belongs to
 *     graphs (uncaptured calls get a slab of their own and never free a graph's), so
 *     replays may run beside uncaptured calls, but graphs holding band launches of one
 *     handle must be replayed in stream order with each other.  Calls that upload a
 *     host-side launch plan or grow scratch at call time (ragged batches,
 *     tgms_refine_loop_device, the multi-GPU calls, a band capture with no slab large
 *     enough) return TGMS_ERR_UNSUPPORTED while their stream is capturing;
 *   - there is no CPU fallback: with no usable GPU, tgms_create fails with
 *     TGMS_ERR_NO_DEVICE.  A GPU-less node asks for the host backend explicitly
 *     (tgms_create_host: solve + sample on the CPU, config 1).
 *
 * Layouts (fp64, row-major, trajectory-major).  A batch is CSR over segments:
 * trajectory b has M_b = seg_offsets[b+1] - seg_offsets[b] segments (1..TGMS_MAX_SEGMENTS):
 *   seg_offsets  int32 [B+1], seg_offsets[0] = 0, strictly increasing (1 <= M_b <= max)
 *   waypoints    [sum_b (M_b+1)][3]   rows of b start at seg_offsets[b] + b
 *   seg_times    [sum_b M_b]          T_i > 0 and finite, starting at seg_offsets[b]
 *   end_derivs   NULL (rest-to-rest, as every reference primitive starts and ends
 *                at rest) or [B][2][3][3] = [start|final][v,a,j][x,y,z]
 *   coeffs       [sum_b M_b][3][8]    p(t) = sum_j c_j t^j on local t in [0, T_i]
 *   status       int32 [B], nullable: per-trajectory tgms_status
 */
#ifndef TGMS_H
#define TGMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TGMS_ABI_VERSION 2 /* 2: tgms_piece.ws_off gained the device plan regions (round 5) */
#define TGMS_MAX_SEGMENTS 16       /* reduced-Hessian kernel: M = 1..16 (config 5 range) */
#define TGMS_DENSE_MAX_SEGMENTS 10 /* dense KKT kernel: N = 14M+2 <= 142 (+3 right-hand sides) fits a 256-thread workgroup's registers */
#define TGMS_GOAL_STRIDE 14        /* doubles per sample: p[3] v[3] a[3] j[3] psi dpsi */

typedef enum tgms_status {
    TGMS_OK = 0,
    TGMS_ERR_INVALID_ARG = 1, /* bad sizes/pointers, M_b < 1 or > max, T <= 0, non-finite input */
    TGMS_ERR_SINGULAR = 2,    /* a pivot / Cholesky block broke down */
    TGMS_ERR_NONFINITE = 3,   /* solution contains inf/nan */
    TGMS_ERR_NO_DEVICE = 4,   /* no HIP device (no CPU fallback exists) */
    TGMS_ERR_DEVICE = 5,      /* a HIP runtime call failed (see tgms_last_error) */
    TGMS_ERR_UNSUPPORTED = 6, /* e.g. dense-KKT method with M_b > TGMS_DENSE_MAX_SEGMENTS */
    TGMS_ERR_SKIPPED = 7      /* per trajectory only: not solved because another trajectory of
                                 the same device shard piece had invalid offsets
                                 (tgms_refine_loop_multi_device; that one is INVALID_ARG) */
} tgms_status;

typedef enum tgms_method {
    TGMS_METHOD_REDUCED = 0,  /* default: Schur complement of the KKT onto the free knot
                                 derivatives, block-tridiagonal LDL^T, one lane per trajectory */
    TGMS_METHOD_DENSE_KKT = 1, /* the survey's literal a1-a3: KKT assembled in LDS, partial-
                                 pivoting LU, one workgroup per trajectory (M <= 10) */
    TGMS_METHOD_BAND_KKT = 2   /* the same KKT and LU with partial pivoting, in the
                                 segment-interleaved order where it is banded (kl = ku = 9);
                                 the structurally-zero entries are skipped, a 16-lane row of
                                 a wavefront per trajectory, M <= TGMS_MAX_SEGMENTS.  Its U rows live in a
                                 handle-owned scratch slab (calls of one handle on different
                                 streams are serialised on the GPU) */
} tgms_method;

typedef enum tgms_yaw_mode {
    TGMS_YAW_CONSTANT = 0, /* psi = yaw_const, dpsi = 0 */
    TGMS_YAW_VELOCITY = 1  /* psi = atan2(v_y, v_x) (Figure8.cpp:123 convention) when
                              |v_xy| > 1e-3, else yaw_const; dpsi = d/dt psi */
} tgms_yaw_mode;

typedef struct tgms_handle tgms_handle;

int tgms_abi_version(void);
const char* tgms_status_string(int status);

/* Create a handle on HIP device `device` (ordinal).  TGMS_ERR_NO_DEVICE if none. */
tgms_status tgms_create(tgms_handle** out, int device);
/* The explicit host backend (BASELINE config 1: a ROS 2 node with no GPU; the reference
 * generates on the executor thread's CPU, src/TrajectoryGenerator.cpp:54-57, :71).  A host
 * handle runs tgms_solve_batch (reduced method) and tgms_sample_batch on the calling thread
 * with the GPU path's conventions; every other entry point returns TGMS_ERR_UNSUPPORTED on
 * it.  Chosen by the caller only: tgms_create never falls back to it. */
tgms_status tgms_create_host(tgms_handle** out);
void tgms_destroy(tgms_handle* h);
/* Last error text of this handle ("" if none).  Valid until the next call. */
const char* tgms_last_error(const tgms_handle* h);
tgms_status tgms_set_method(tgms_handle* h, int method);

/* ---- solve (host pointers, blocking) ---- */
tgms_status tgms_solve_batch(tgms_handle* h, int32_t B, const int32_t* seg_offsets,
                             const double* waypoints, const double* seg_times,
                             const double* end_derivs, double* coeffs, int32_t* status);

/* ---- solve (device pointers, asynchronous on `stream`) ---- */
/* Uniform batch: every trajectory has M segments (configs 2-4). */
tgms_status tgms_solve_uniform_device(tgms_handle* h, int32_t B, int32_t M,
                                      const double* d_waypoints, const double* d_seg_times,
                                      const double* d_end_derivs, double* d_coeffs,
                                      int32_t* d_status, void* stream);
/* Ragged batch (config 5).  h_seg_offsets is a host copy used to plan the launch
 * (trajectories are grouped by M so every wavefront runs one M).  The refinement loops
 * group the batch on the device from d_seg_offsets, which must hold the same values as
 * h_seg_offsets: tgms_refine_loop_device reads h_seg_offsets once (validation, uniform
 * detection); tgms_refine_loop_multi_device reads only seg_offsets[0], [B] and the shard
 * and piece cuts (binary search), so per-trajectory M is checked on the devices alone.
 * Device offsets with an M outside 1..16 or another span run nothing in the shard piece
 * that holds them (failure granularity: one piece of one device's shard, <= 1/4 of the
 * shard): in d_status the trajectories whose own M is outside 1..16 read
 * TGMS_ERR_INVALID_ARG and the piece's other trajectories TGMS_ERR_SKIPPED, all with zero
 * coefficients and costs and the times kept; the call itself returns TGMS_OK, so a caller
 * checks d_status (a device-side finding cannot reach the return code without a
 * synchronisation the pipelined call avoids). */
tgms_status tgms_solve_batch_device(tgms_handle* h, int32_t B, const int32_t* h_seg_offsets,
                                    const int32_t* d_seg_offsets, const double* d_waypoints,
                                    const double* d_seg_times, const double* d_end_derivs,
                                    double* d_coeffs, int32_t* d_status, void* stream);

/* ---- time-allocation refinement ----
 * Minimises F(T) = sum_i J_i(T) + k_T * sum_i T_i per trajectory over its segment
 * durations, J_i the snap cost of segment i at the min-snap solution.  One step
 * solves, forms g_i = dJ_i/dT_i + k_T analytically (envelope theorem: knot
 * derivatives fixed), and moves in log space:
 *     T_i <- T_i * exp(clamp(-eta * T_i * g_i / F, -1/2, +1/2)).
 * Trajectories whose solve fails keep their times.  Reduced method only
 * (TGMS_ERR_UNSUPPORTED otherwise).  d_cost (nullable, [B]) receives F at the
 * step's input times; dT_out must not alias dT. */
tgms_status tgms_refine_uniform_device(tgms_handle* h, int32_t B, int32_t M, const double* d_waypoints,
                                       const double* d_seg_times, const double* d_end_derivs, double k_T,
                                       double eta, double* d_seg_times_out, double* d_cost, int32_t* d_status,
                                       void* stream);
tgms_status tgms_refine_batch_device(tgms_handle* h, int32_t B, const int32_t* h_seg_offsets,
                                     const int32_t* d_seg_offsets, const double* d_waypoints,
                                     const double* d_seg_times, const double* d_end_derivs, double k_T, double eta,
                                     double* d_seg_times_out, double* d_cost, int32_t* d_status, void* stream);
/* The whole config-5 pipeline on device, planned once: `iters` steps from
 * d_seg_times (updated in place), F at the final times into d_cost (nullable) and
 * the final solve into d_coeffs (nullable).  Uses the handle's workspace. */
tgms_status tgms_refine_loop_device(tgms_handle* h, int32_t B, const int32_t* h_seg_offsets,
                                    const int32_t* d_seg_offsets, const double* d_waypoints, double* d_seg_times,
                                    const double* d_end_derivs, double k_T, double eta, int32_t iters,
                                    double* d_coeffs, double* d_cost, int32_t* d_status, void* stream);
/* Host convenience (blocking): `iters` steps from seg_times (updated in place),
 * then F at the final times into cost (nullable) and, if coeffs is not NULL,
 * the final solve.  Returns the worst per-trajectory status. */
tgms_status tgms_refine_batch(tgms_handle* h, int32_t B, const int32_t* seg_offsets, const double* waypoints,
                              double* seg_times, const double* end_derivs, double k_T, double eta, int32_t iters,
                              double* coeffs, double* cost, int32_t* status);

/* ---- sampling at dt ----
 * Trajectory b yields tgms_sample_count(sum_i T_i, dt) samples: t_k = k*dt for
 * k = 0 .. n-2 and a final sample at sum_i T_i pinned exactly to the last
 * waypoint and final end derivatives (the Line.cpp:80-82 convention).  Each sample
 * is TGMS_GOAL_STRIDE doubles.  sample_offsets [B+1] comes from
 * tgms_sample_offsets(). */
int64_t tgms_sample_count(double total_T, double dt);
tgms_status tgms_sample_offsets(int32_t B, const int32_t* seg_offsets, const double* seg_times,
                                double dt, int64_t* sample_offsets);
tgms_status tgms_sample_batch(tgms_handle* h, int32_t B, const int32_t* seg_offsets,
                              const double* waypoints, const double* seg_times,
                              const double* end_derivs, const double* coeffs, double dt,
                              int yaw_mode, double yaw_const, const int64_t* sample_offsets,
                              double* out);
tgms_status tgms_sample_batch_device(tgms_handle* h, int32_t B, const int32_t* d_seg_offsets,
                                     const double* d_waypoints, const double* d_seg_times,
                                     const double* d_end_derivs, const double* d_coeffs,
                                     double dt, int yaw_mode, double yaw_const,
                                     const int64_t* d_sample_offsets, double* d_out,
                                     void* stream);

/* ---- multi-GPU ----
 * One process drives devices 0 .. device_count-1 through one handle that owns one RCCL
 * communicator per device (ncclCommInitAll, rccl.h:236; RCCL is loaded here, not at
 * library load).  The batch is split into contiguous shards of equal cost
 * (tgms_plan_shards), every shard into pieces; device 0 scatters each piece's inputs
 * to its device and gathers its coefficients / statuses back with grouped
 * ncclSend / ncclRecv (rccl.h:700, :722; per-piece counts, so ragged batches need no
 * padding) while the device solves the next piece.  Device 0 solves its own shard in
 * place.  The caller sees one device-0 batch, exactly as tgms_solve_batch_device
 * would produce it (identical coefficients: trajectories are independent).  The single-
 * device entry points applied to a multi handle run on device 0 only; the multi entry
 * points applied to a tgms_create handle run the single-device path.  Replaces nothing
 * in the reference, whose caller (TrajectoryGenerator.hpp:83, src/TrajectoryGenerator.cpp:71)
 * holds one Trajectory; this is the swarm / sampling planner's batch path (configs 4, 5). */
tgms_status tgms_create_multi(tgms_handle** out, int device_count);
int tgms_device_count(const tgms_handle* h); /* 1 for a tgms_create handle, 0 for a host handle */
/* Host-only shard planner: bounds [parts+1] of contiguous trajectory ranges with
 * ~equal cost (reduced / band: 2 + M_b, dense KKT: (14 M_b + 2)^3 per trajectory). */
tgms_status tgms_plan_shards(int32_t B, const int32_t* seg_offsets, int32_t parts, int method,
                             int32_t* bounds);
/* Host-only introspection of the multi-GPU schedule (no device, no RCCL needed): what a
 * tgms_solve_batch_multi_device / tgms_refine_loop_multi_device call over device_count
 * devices would do with this batch -- the shard bounds [device_count+1], every device's
 * piece-workspace size (ws_bytes [device_count], nullable), the pieces (trajectory /
 * segment ranges and the byte offsets of their arrays in the workspace) and every
 * point-to-point transfer in issue order: scatter groups 0..3 (piece k's inputs of every
 * device, device 0 -> dev), then gather groups 4..7 (piece k's results, dev -> device 0);
 * each transfer is one ncclSend on one side and one ncclRecv on the other.  flags:
 * TGMS_SCHED_* below.  Returns TGMS_ERR_INVALID_ARG (with *n_pieces / *n_xfers set to the
 * sizes needed) when piece_cap or xfer_cap is too small.  It does exactly the host work of
 * the call before its first transfer.  With TGMS_SCHED_REFINE: no pass over the offsets
 * (the cuts checked).  Without (a solve): for the reduced method the offsets' ends and a
 * uniform check that stops at the first 4,096-trajectory block holding two different M (a
 * ragged batch is then grouped and checked per trajectory on its devices, as a refinement
 * loop's; round 6); for the band / dense methods the full validation pass. */
#define TGMS_SCHED_REFINE 1
#define TGMS_SCHED_END_DERIVS 2
#define TGMS_SCHED_COEFFS 4
#define TGMS_SCHED_STATUS 8
#define TGMS_SCHED_COST 16
#define TGMS_SCHED_SELF_GATHER 32 /* device 0's shard through the pipeline too (TGMS_MULTI_SELF_GATHER=1) */
typedef struct tgms_piece {
    int32_t dev, piece, lo, hi; /* trajectories [lo, hi) */
    int64_t s0, s1;             /* segments [s0, s1) */
    int64_t ws_off[11];         /* byte offsets: seg_offsets (ragged: rebased for a band / dense solve,
                                   the raw slice for a refinement loop or a reduced solve),
                                   permutation, W, T, T2, ED, C, status, cost, and for a device-planned
                                   piece the device grouping's block counts and its device-side plan
                                   (uniform batches: empty regions) */
} tgms_piece;
typedef struct tgms_xfer {
    int32_t dev, piece, gather; /* gather 0: device 0 -> dev (scatter), 1: dev -> device 0 */
    int32_t array;              /* 0 W, 1 T, 2 end derivs, 3 coeffs, 4 status, 5 cost, 6 seg_offsets
                                   (the slice [lo, hi] of a device-planned piece) */
    int64_t batch_elem;         /* element offset in the device-0 batch array */
    int64_t ws_byte;            /* byte offset in dev's piece workspace */
    int64_t count;              /* elements */
    int32_t elem_bytes;         /* 8 (fp64) or 4 (int32) */
    int32_t group;              /* RCCL group (ncclGroupStart .. ncclGroupEnd) in issue order */
} tgms_xfer;
tgms_status tgms_multi_schedule(int32_t device_count, int32_t B, const int32_t* seg_offsets, int method,
                                int32_t flags, int32_t* bounds, int64_t* ws_bytes, tgms_piece* pieces,
                                int32_t piece_cap, int32_t* n_pieces, tgms_xfer* xfers, int32_t xfer_cap,
                                int32_t* n_xfers);
/* Host pointers, blocking: upload to device 0, the multi-GPU solve, one download. */
tgms_status tgms_solve_batch_multi(tgms_handle* h, int32_t B, const int32_t* seg_offsets,
                                   const double* waypoints, const double* seg_times,
                                   const double* end_derivs, double* coeffs, int32_t* status);
/* Device-0 pointers, asynchronous on `stream` (a device-0 stream).  Reduced method, ragged
 * batch (round 6): the host reads only the offsets' ends and the shard / piece cuts; every
 * device groups and checks its pieces' trajectories (as tgms_refine_loop_multi_device): a
 * trajectory with M outside 1..16 fails its piece -- TGMS_ERR_INVALID_ARG for it,
 * TGMS_ERR_SKIPPED for the piece's others, zero coefficients -- and the call returns
 * TGMS_OK, so check d_status.  Band / dense methods and uniform batches are validated on the
 * host as before (an error return names the first offending trajectory). */
tgms_status tgms_solve_batch_multi_device(tgms_handle* h, int32_t B, const int32_t* h_seg_offsets,
                                          const int32_t* d_seg_offsets, const double* d_waypoints,
                                          const double* d_seg_times, const double* d_end_derivs,
                                          double* d_coeffs, int32_t* d_status, void* stream);
/* tgms_refine_loop_device over the devices (config 5): times (in place), costs,
 * coefficients and statuses gathered back to device 0.  Every batch (uniform ones too) runs
 * the device-grouped loop; the host does no pass over the offsets (see
 * tgms_solve_batch_device above: a piece with bad offsets fails on its device). */
tgms_status tgms_refine_loop_multi_device(tgms_handle* h, int32_t B, const int32_t* h_seg_offsets,
                                          const int32_t* d_seg_offsets, const double* d_waypoints,
                                          double* d_seg_times, const double* d_end_derivs, double k_T,
                                          double eta, int32_t iters, double* d_coeffs, double* d_cost,
                                          int32_t* d_status, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TGMS_H */
