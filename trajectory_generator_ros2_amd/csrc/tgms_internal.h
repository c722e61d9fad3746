// tgms_internal.h — declarations shared by the kernels TU and the C-ABI TU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tgms {

// Largest M solved at two wavefronts per SIMD (the axis-sequential state of larger M
// needs more than 256 registers); ragged batches launch one kernel per class.  13: the
// fused refinement loop keeps 4 VGPRs in scratch at M = 12..13 and still beats running
// them at one wave (config 5: 0.489-0.494 against 0.494-0.506 ms with 11, round 4).
#ifndef TGMS_TWO_WAVE_MAX_M
#define TGMS_TWO_WAVE_MAX_M 13
#endif
// ... and with end derivatives (their extra state spills the fused refinement loop by
// 79 VGPRs at M = 12..13 within 256 registers; M <= 11 fits with none)
#ifndef TGMS_TWO_WAVE_MAX_M_ED
#define TGMS_TWO_WAVE_MAX_M_ED 11
#endif
constexpr int two_wave_max_m(bool has_ed) { return has_ed ? TGMS_TWO_WAVE_MAX_M_ED : TGMS_TWO_WAVE_MAX_M; }

// Reduced-Hessian solve, uniform M (configs 2-4).  Grid: ceil(B/64) waves.
hipError_t launch_reduced_uniform(int M, int32_t B, const double* W, const double* T,
                                  const double* ED, double* C, int32_t* status,
                                  hipStream_t stream);

// Reduced-Hessian solve for one group of a ragged CSR batch: the n trajectories
// perm[0..n) all have M segments (the host groups a ragged batch by M so every
// wavefront runs a single M).
hipError_t launch_reduced_ragged_group(int M, int32_t n, const int32_t* perm,
                                       const int32_t* seg_offsets, const double* W,
                                       const double* T, const double* ED, double* C,
                                       int32_t* status, hipStream_t stream);

// Dense-KKT solve (survey a1-a3 literally): one wavefront per trajectory, KKT in LDS.
// Uniform M only (1..TGMS_DENSE_MAX_SEGMENTS); ragged batches loop over M groups.
hipError_t launch_dense_kkt(int M, int32_t n_traj, const int32_t* traj_ids /*nullable*/,
                            const int32_t* seg_offsets /*nullable if uniform*/, const double* W,
                            const double* T, const double* ED, double* C, int32_t* status,
                            hipStream_t stream);

// Band-KKT solve (the same KKT and partial-pivoting LU, segment-interleaved order, the
// structurally-zero entries skipped): sixteen trajectories per wavefront, persistent grid
// of `grid` wavefronts, each with private U slabs in `scratch` (band_scratch_bytes).
// grid = CUs x BAND_WAVES_PER_CU (the scratch is sized for it: two wavefronts per SIMD,
// the kernel's register budget); the launch uses the resident part of it.
#ifndef TGMS_BAND_WAVES_PER_CU
#define TGMS_BAND_WAVES_PER_CU 8
#endif
constexpr int BAND_WAVES_PER_CU = TGMS_BAND_WAVES_PER_CU;
size_t band_scratch_bytes(int M, int32_t grid);
hipError_t launch_band_kkt(int M, int32_t n_traj, const int32_t* traj_ids /*nullable*/,
                           const int32_t* seg_offsets /*nullable if uniform*/, const double* W,
                           const double* T, const double* ED, double* C, int32_t* status, double* scratch,
                           int32_t grid, hipStream_t stream);

// Time-allocation refinement step (solve + snap-cost gradient + log-space step on T):
// uniform batches, and one M group of a ragged batch.  Tout may not alias T.
hipError_t launch_refine_uniform(int M, int32_t B, const double* W, const double* T, const double* ED, double kT,
                                 double eta, double* Tout, double* cost, int32_t* status, hipStream_t stream);
hipError_t launch_refine_ragged_group(int M, int32_t n, const int32_t* perm, const int32_t* seg_offsets,
                                      const double* W, const double* T, const double* ED, double kT, double eta,
                                      double* Tout, double* cost, int32_t* status, hipStream_t stream);

// Several M groups of a ragged batch in one launch.  Group g owns wavefronts
// [blk_end[g-1], blk_end[g]) and its n[g] trajectories perm[g][0..n) have m[g] segments.
// cls 0 takes M in 1..two_wave_max_m(ED) (two waves per SIMD), cls 1 the larger M (one wave
// per SIMD).
constexpr int RAGGED_TPW = 32;  // trajectories per wavefront of the reduced kernels
struct GroupTable {
    int32_t ngroups;
    int32_t m[16];
    int32_t n[16];
    int32_t blk_end[16];
    const int32_t* perm[16];
};
hipError_t launch_ragged_multi(int cls, const GroupTable& tab, bool refine, const int32_t* seg_offsets,
                               const double* W, const double* T, const double* ED, double kT, double eta,
                               double* Tout, double* cost, double* C, int32_t* status, hipStream_t stream);

// The M-grouping permutation of a ragged batch computed on the device (stable counting
// sort of the ids by so[b+1] - so[b]; M validated on the host): starts[m] (m = 1..16) is
// where group m begins, hist a workspace of perm_hist_bytes(B).
size_t perm_hist_bytes(int32_t B);
hipError_t launch_group_perm(int32_t B, const int32_t* seg_offsets, const int32_t* starts, int32_t* hist,
                             int32_t* perm, hipStream_t stream);

// The launch plan of a ragged refinement loop computed entirely on the device (round 5):
// the per-M totals summed from k_perm_hist's block counts, the starts of the M groups in
// the permutation and both occupancy classes' group tables.  The host plans nothing per
// trajectory, and a captured graph stays valid for any offsets of the same B and S: each
// replay regroups.  `so` may be a slice of a larger batch's offsets (so[0] != 0: the
// kernels subtract so_base = so[0]); offsets whose M leave 1..16 or whose span is not S
// mark the plan bad and nothing runs: statuses TGMS_ERR_INVALID_ARG, the S segments'
// coefficients (C, nullable) and the n costs (cost, nullable) exact zeros, times kept.
// This is the only per-trajectory check of tgms_refine_loop_multi_device's offsets.
struct DevPlan {
    GroupTable tab[2];
    int32_t starts[17];  // starts[m]: first index of group m in the permutation (m = 1..16)
    int32_t so_base;     // so[0]
    int32_t bad;
    // waves[1] > 0: the refinement loop's one-wave class runs as that many PERSISTENT
    // wavefronts (round 6, k_refine_loop_dev), each taking the class's tiles from the counter
    // next[1] (longest groups first) until none is left; 0: one block per tile (always for
    // the two-wave class, and for a one-wave class with no more tiles than SIMDs)
    int32_t waves[2];
    int32_t next[2];
};
// Grid of one class's loop launch: every wavefront a group table can hold, whatever the
// offsets (the blocks beyond the class's last group return at once).
inline unsigned dev_loop_grid(int32_t n) { return (unsigned)((n + RAGGED_TPW - 1) / RAGGED_TPW + 16); }
hipError_t launch_group_plan_dev(int32_t n, int64_t S, const int32_t* so, int has_ed, int32_t* hist, int32_t* perm,
                                 DevPlan* plan, int32_t* status, double* C, double* cost, hipStream_t stream);
hipError_t launch_refine_loop_dev(int cls, int32_t n, DevPlan* plan, const int32_t* so, const double* W,
                                  double* T, const double* ED, double kT, double eta, int32_t iters, double* cost,
                                  double* C, int32_t* status, hipStream_t stream);
// The ragged solve of one occupancy class from a device plan (k_reduced_multi's blocks).
hipError_t launch_reduced_multi_dev(int cls, int32_t n, const DevPlan* plan, const int32_t* so, const double* W,
                                    const double* T, const double* ED, double* C, int32_t* status,
                                    hipStream_t stream);

// Sampler: one workgroup per trajectory (grid-stride), 14 doubles per sample.
hipError_t launch_sample(int32_t B, const int32_t* seg_offsets, const double* W, const double* T,
                         const double* ED, const double* C, double dt, int yaw_mode,
                         double yaw_const, const int64_t* sample_offsets, double* out,
                         hipStream_t stream);

}  // namespace tgms
