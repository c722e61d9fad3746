// MinSnap.hpp — minimum-snap trajectory primitive behind the reference's Trajectory
// interface (SURVEY.md §8(a) a6, §8(b) "Adapter").
//
// It is one more trajectory next to Circle / Line / Figure8 ... (reference
// include/trajectory_generator_ros2/trajectories/*.hpp), built by the traj_type
// factory branch "MinSnap" (factory.hpp, mirrors src/TrajectoryGenerator.cpp:175-388).
// Every solve and every sample runs on the GPU through the C ABI (include/tgms.h),
// unless the node's YAML asks for the host backend (`minsnap_backend: host`, config 1: a
// node with no GPU); there is no silent CPU fallback.
//
//   generateTraj            tgms_solve_batch (B = 1, rest-to-rest) + tgms_sample_batch at dt,
//                           appended to goals (Line.cpp:33-89 append convention)
//   generateStopTraj        one braking segment from goals[pub_index]'s p/v/a/j to rest
//                           (end_derivs), replaces goals / index_msgs, pub_index = 0
//                           (Line.cpp:145-147 replace convention)
//   trajectoryInsideBounds  every waypoint AND every sampled position inside the room
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "Trajectory.hpp"
#include "tgms.h"

namespace trajectory_generator {

struct MinSnapParams {
    std::vector<double> waypoints;  // flat [x0 y0 z0 x1 y1 z1 ...], >= 2 points
    std::vector<double> seg_times;  // one per segment, > 0
    int yaw_mode = TGMS_YAW_CONSTANT;
    double yaw = 0.0;               // psi for TGMS_YAW_CONSTANT (and at rest)
    double stop_accel = 1.0;        // braking deceleration for generateStopTraj [m/s^2]
    int device = 0;                 // HIP device ordinal
    bool host_backend = false;      // `minsnap_backend: host`: the explicit CPU backend (config 1,
                                    // a node with no GPU; tgms_create_host), never a fallback
};

class MinSnap : public Trajectory {
public:
    MinSnap(const MinSnapParams& params, double dt);
    ~MinSnap() override;
    MinSnap(const MinSnap&) = delete;
    MinSnap& operator=(const MinSnap&) = delete;

    void generateTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                      const ClockPtr& clock) override;
    void generateStopTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                          int& pub_index, const ClockPtr& clock) override;
    bool trajectoryInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin,
                                double zmax) override;

    // Solved coefficients [M][3][8] of the main trajectory (solves on first use).
    const std::vector<double>& coefficients();
    int segments() const { return (int)p_.seg_times.size(); }

private:
    tgms_handle* handle();
    // Solve one trajectory and sample it at dt_; false + message on failure.
    bool solve_and_sample(const std::vector<double>& W, const std::vector<double>& T, const double* end_derivs,
                          std::vector<double>& coeffs, std::vector<double>& samples, std::string& err);
    bool ensure_main();

    MinSnapParams p_;
    tgms_handle* h_ = nullptr;
    bool solved_ = false;
    std::vector<double> coeffs_;   // [M][3][8]
    std::vector<double> samples_;  // [n][TGMS_GOAL_STRIDE]
};

}  // namespace trajectory_generator
