// factory.hpp — the traj_type == "MinSnap" branch of the reference's parameter
// reader (src/TrajectoryGenerator.cpp:175-388), written against any node type with
// rclcpp::Node's `bool get_parameter(const std::string&, T&)`, so the same code runs
// inside the ROS node and against ParamMap in the standalone build.
//
// Parameters (same validation style as :184-195: "must be > 0" -> return false):
//   waypoints    double[]  flat x,y,z triples, >= 2 points, finite
//   seg_times    double[]  optional, one per segment, all > 0; when absent or empty
//                          T_i = max(|w_{i+1} - w_i| / v_goals[0], min_seg_time)
//   v_goals      double[]  all > 0 (as for Circle/Line); used only for the time allocation
//   min_seg_time double    optional, > 0, default 0.5 s
//   yaw_mode     string    optional, "constant" (default) or "velocity" (Figure8.cpp:123)
//   yaw          double    optional, psi in constant mode, default 0
//   stop_accel   double    optional, > 0, braking deceleration, default 1.0 m/s^2
#pragma once

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "MinSnap.hpp"

namespace trajectory_generator {

template <class Node>
bool readMinSnapParameters(Node& node, double dt, std::unique_ptr<Trajectory>& traj) {
    MinSnapParams p;
    if (!node.get_parameter("waypoints", p.waypoints)) return false;
    if (p.waypoints.size() < 6 || p.waypoints.size() % 3 != 0) {
        log_error("waypoints must hold at least 2 x,y,z triples");
        return false;
    }
    const size_t M = p.waypoints.size() / 3 - 1;
    if (M > (size_t)TGMS_MAX_SEGMENTS) {
        log_error("MinSnap supports at most %d segments", TGMS_MAX_SEGMENTS);
        return false;
    }
    for (double w : p.waypoints)
        if (!std::isfinite(w)) {
            log_error("All waypoints must be finite");
            return false;
        }
    node.get_parameter("seg_times", p.seg_times);
    if (p.seg_times.empty()) {
        std::vector<double> v_goals;
        if (!node.get_parameter("v_goals", v_goals) || v_goals.empty()) return false;
        for (double vel : v_goals)
            if (vel <= 0) {
                log_error("All velocities must be > 0");
                return false;
            }
        double tmin = 0.5;
        node.get_parameter("min_seg_time", tmin);
        if (!(tmin > 0)) {
            log_error("min_seg_time must be > 0");
            return false;
        }
        for (size_t i = 0; i < M; ++i) {
            const double* a = &p.waypoints[3 * i];
            const double* b = a + 3;
            const double d = std::sqrt((b[0] - a[0]) * (b[0] - a[0]) + (b[1] - a[1]) * (b[1] - a[1]) +
                                       (b[2] - a[2]) * (b[2] - a[2]));
            p.seg_times.push_back(std::max(d / v_goals[0], tmin));
        }
    }
    if (p.seg_times.size() != M) {
        log_error("seg_times must have one entry per segment (%zu)", M);
        return false;
    }
    for (double t : p.seg_times)
        if (!(t > 0) || !std::isfinite(t)) {
            log_error("All segment times must be > 0");
            return false;
        }
    std::string yaw_mode = "constant";
    node.get_parameter("yaw_mode", yaw_mode);
    if (yaw_mode == "constant")
        p.yaw_mode = TGMS_YAW_CONSTANT;
    else if (yaw_mode == "velocity")
        p.yaw_mode = TGMS_YAW_VELOCITY;
    else {
        log_error("yaw_mode must be \"constant\" or \"velocity\"");
        return false;
    }
    node.get_parameter("yaw", p.yaw);
    node.get_parameter("stop_accel", p.stop_accel);
    if (!(p.stop_accel > 0)) {
        log_error("accel must be > 0");
        return false;
    }
    double device = 0;
    node.get_parameter("device", device);
    p.device = (int)device;
    traj = std::make_unique<MinSnap>(p, dt);
    return true;
}

// Parameter store with rclcpp::Node's get_parameter shape (standalone build / tests).
class ParamMap {
public:
    void set(const std::string& k, double v) { d_[k] = v; }
    void set(const std::string& k, const std::vector<double>& v) { a_[k] = v; }
    void set(const std::string& k, const std::string& v) { s_[k] = v; }
    bool get_parameter(const std::string& k, double& v) const { return get(d_, k, v); }
    bool get_parameter(const std::string& k, std::vector<double>& v) const { return get(a_, k, v); }
    bool get_parameter(const std::string& k, std::string& v) const { return get(s_, k, v); }

private:
    template <class Map, class T>
    static bool get(const Map& m, const std::string& k, T& v) {
        auto it = m.find(k);
        if (it == m.end()) return false;
        v = it->second;
        return true;
    }
    std::map<std::string, double> d_;
    std::map<std::string, std::vector<double>> a_;
    std::map<std::string, std::string> s_;
};

// The parts of TrajectoryGenerator::readParameters (src/TrajectoryGenerator.cpp:150-425)
// that frame the factory: alt, pub_freq -> dt = 1/freq (:171-172), traj_type dispatch,
// room bounds (:407-413) and the trajectoryInsideBounds check (:417-421).
struct GeneratorSettings {
    double alt = 0.0, dt = 0.0;
    double xmin = 0, xmax = 0, ymin = 0, ymax = 0, zmin = 0, zmax = 0;
    std::string traj_type;
};

bool readParameters(const ParamMap& node, GeneratorSettings& s, std::unique_ptr<Trajectory>& traj);

}  // namespace trajectory_generator
