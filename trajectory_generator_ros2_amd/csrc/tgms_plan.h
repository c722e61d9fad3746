// tgms_plan.h — host-only planning of the multi-GPU pipeline.
//
// Pure C++ (no HIP, no RCCL): the shard cuts, the pieces of every shard, the byte layout
// of every device's piece workspace and the complete list of point-to-point transfers
// (scatter of the inputs from device 0, gather of the results back to device 0) are
// computed here, and tgms_capi.hip's multi_enqueue only turns that list into grouped
// ncclSend / ncclRecv calls (rccl.h:700/722) and kernel launches.  The same code is
// exported through tgms_multi_schedule (include/tgms.h), so the schedule is checked on
// the CPU at 2..8 devices (tests/test_multi_schedule.py) without a GPU or RCCL.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace tgms {

// Cost of one trajectory with M segments for `method` (the shard planner's unit).
// Reduced / band: 2 + M (a fixed part per trajectory plus one per segment; the same
// rule as shard.trajectory_cost); dense KKT: (14 M + 2)^3.
double traj_cost(int method, int32_t M);

// Contiguous cost-balanced shards: bounds[parts + 1].  The rule of
// shard.ragged_bounds (trajectory_generator_ros2_amd/shard.py), step for step in the
// same fp64 arithmetic.  `so` may be NULL when uniform_m > 0, and may be a slice of a
// larger batch's offsets (so[0] != 0).  Reduced / band cost 2 + M, whose running sum is
// the integer 2 (b + 1) + so[b + 1] - so[0]: cut by binary search, O(parts log B), no pass
// over the batch.
void plan_shards(int32_t B, const int32_t* so, int parts, int method, int32_t* bounds, int uniform_m = 0);

constexpr int MULTI_PIECES = 4;  // pieces per shard: the gather of piece p overlaps the solve of p + 1

// Arrays a transfer moves (batch array on device 0 <-> a piece's region of a workspace)
enum XferArray : int32_t { XA_W = 0, XA_T = 1, XA_ED = 2, XA_C = 3, XA_ST = 4, XA_COST = 5, XA_SO = 6 };

// Device-side plan of a ragged refinement-loop piece (tgms::DevPlan, tgms_internal.h; its
// size is checked against this bound where both are visible) and the per-block counts of
// the device grouping (perm_hist_bytes: 17 int32 per 1,024 trajectories).
constexpr size_t DEV_PLAN_BYTES = 1024;
inline size_t dev_hist_bytes(int32_t n) { return (size_t)((n + 1023) / 1024) * 17 * sizeof(int32_t); }

struct Xfer {
    int32_t dev;         // the piece's device (the peer of device 0)
    int32_t piece;       // piece index k within the device's shard
    int32_t gather;      // 0: scatter (device 0 -> dev), 1: gather (dev -> device 0)
    int32_t array;       // XferArray
    int64_t batch_elem;  // element offset in the device-0 batch array
    int64_t ws_byte;     // byte offset in dev's piece workspace
    int64_t count;       // elements
    int32_t elem_bytes;  // 8 (fp64) or 4 (int32)
    int32_t group;       // RCCL group: scatter groups 0..K-1 (one per piece index), gathers K..2K-1
};

struct PiecePlan {
    int32_t lo = 0, hi = 0;  // trajectories [lo, hi) of the batch
    int64_t s0 = 0, s1 = 0;  // segments [s0, s1)
    // byte offsets inside the device's workspace.  A ragged solve: the plan block (rebased
    // offsets, the grouping permutation, uploaded from the host) first, then the piece's
    // arrays.  A ragged refinement loop: the raw offsets slice (scattered from device 0 with
    // the inputs), the permutation, the device grouping's block counts and its plan, all
    // filled on the device.  A uniform batch: none of these (size 0).
    size_t oSo = 0, oPerm = 0, oW = 0, oT = 0, oT2 = 0, oED = 0, oC = 0, oSt = 0, oCost = 0, oHist = 0, oPlan = 0;
    int32_t n() const { return hi - lo; }
    int64_t S() const { return s1 - s0; }
};

struct MultiFlags {
    bool refine = false;       // tgms_refine_loop_multi_device (times in/out, a second time buffer)
    bool has_ed = false;       // end derivatives scattered
    bool has_c = false;        // coefficients gathered
    bool has_st = false;       // statuses gathered
    bool has_cost = false;     // costs gathered (refine)
    bool self_gather = false;  // device 0's own shard through the pipeline as well
};

struct MultiPlan {
    int n = 0;
    std::vector<int32_t> bounds;              // [n + 1]
    std::vector<std::vector<PiecePlan>> pieces;  // per device (empty: solved in place or no work)
    std::vector<size_t> plan_bytes;           // per device: the plan block (uploaded from pinned staging; ragged solves only)
    std::vector<size_t> ws_bytes;             // per device: the whole piece workspace
    std::vector<Xfer> xfers;                  // in issue order, grouped by Xfer::group
    int32_t n_groups = 0;                     // 2 * MULTI_PIECES
};

// The whole schedule of one multi-GPU call over devices 0..n-1.
// The schedule's shard and piece cuts are consistent with offsets nobody scanned: every
// shard and piece spans between 1 and TGMS_MAX_SEGMENTS segments per trajectory (the
// workspaces are sized from these spans).  O(devices x pieces).
bool cuts_valid(const MultiPlan& P, const int32_t* so);
void plan_multi(int n, int32_t B, const int32_t* so, int method, int uniform_m, const MultiFlags& f, MultiPlan* out);

}  // namespace tgms
