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

// Waypoints of the reference's polyline primitives, so a
// MinSnap trajectory can fly a smooth version of them.  Local (x, y) points, rotated
// by `orientation` about (cx, cy) as those primitives do, at altitude z:
//   "M"      M.cpp:20-26       (-w/2,-l/2) (-w/2,l/2) (0,-l/2) (w/2,l/2) (w/2,-l/2)
//   "I"      I.cpp:28-35       (-w/2,l/2) (w/2,l/2) (0,l/2) (0,-l/2) (-w/2,-l/2) (w/2,-l/2)
//   "T"      T.cpp:28-33       (-w/2,l/2) (w/2,l/2) (0,l/2) (0,-l/2)
//   "Square" Square.cpp:26-43  corners (-h,h) (h,h) (h,-h) (-h,-h) with h = l/2, closed
// `laps` traversals alternate direction like the reference's back-and-forth loop
// (M.cpp:50-62); a closed Square simply repeats.  Returns the number of points
// (0 for an unknown shape or more than cap).
inline int shapeWaypoints(const std::string& shape, double cx, double cy, double orientation, double length,
                          double width, double z, int laps, double* out, int cap) {
    std::vector<std::pair<double, double>> pts;
    const double l = length, w = width;
    if (shape == "M")
        pts = {{-w / 2, -l / 2}, {-w / 2, l / 2}, {0.0, -l / 2}, {w / 2, l / 2}, {w / 2, -l / 2}};
    else if (shape == "I")
        pts = {{-w / 2, l / 2}, {w / 2, l / 2}, {0.0, l / 2}, {0.0, -l / 2}, {-w / 2, -l / 2}, {w / 2, -l / 2}};
    else if (shape == "T")
        pts = {{-w / 2, l / 2}, {w / 2, l / 2}, {0.0, l / 2}, {0.0, -l / 2}};
    else if (shape == "Square")
        pts = {{-l / 2, l / 2}, {l / 2, l / 2}, {l / 2, -l / 2}, {-l / 2, -l / 2}, {-l / 2, l / 2}};
    else
        return 0;
    if (laps < 1) return 0;
    const bool closed = shape == "Square";
    std::vector<std::pair<double, double>> path = pts;
    for (int lap = 1; lap < laps; ++lap) {
        if (closed) {
            path.insert(path.end(), pts.begin() + 1, pts.end());
        } else {  // reverse direction each lap, sharing the turning point
            const bool rev = lap & 1;
            for (size_t i = 1; i < pts.size(); ++i) path.push_back(rev ? pts[pts.size() - 1 - i] : pts[i]);
        }
    }
    if ((int)path.size() > cap) return 0;
    const double c = std::cos(orientation), s = std::sin(orientation);
    for (size_t i = 0; i < path.size(); ++i) {
        const double x = path[i].first, y = path[i].second;
        out[3 * i] = c * x - s * y + cx;
        out[3 * i + 1] = s * x + c * y + cy;
        out[3 * i + 2] = z;
    }
    return (int)path.size();
}

template <class Node>
bool readMinSnapParameters(Node& node, double dt, std::unique_ptr<Trajectory>& traj) {
    MinSnapParams p;
    std::string source = "list";
    node.get_parameter("waypoint_source", source);
    if (source != "list") {
        // shape parameters named as in config/default.yaml (M_length, I_width, side_length, ...)
        double cx = 0, cy = 0, orientation = 0, alt = 0, length = 0, width = 0, laps = 1;
        if (!node.get_parameter("alt", alt)) return false;
        node.get_parameter("center_x", cx);
        node.get_parameter("center_y", cy);
        node.get_parameter("orientation", orientation);
        node.get_parameter("laps", laps);
        if (source == "Square") {
            if (!node.get_parameter("side_length", length)) return false;
            width = length;
        } else {
            if (!node.get_parameter(source + "_length", length)) return false;
            if (!node.get_parameter(source + "_width", width)) return false;
        }
        if (!(length > 0) || !(width > 0)) {
            log_error("%s dimensions must be > 0", source.c_str());
            return false;
        }
        double buf[3 * (TGMS_MAX_SEGMENTS + 1)];
        const int n = shapeWaypoints(source, cx, cy, orientation, length, width, alt, (int)laps, buf,
                                     TGMS_MAX_SEGMENTS + 1);
        if (n < 2) {
            log_error("waypoint_source %s with %d laps is not available (at most %d segments)", source.c_str(),
                      (int)laps, TGMS_MAX_SEGMENTS);
            return false;
        }
        p.waypoints.assign(buf, buf + 3 * n);
    } else if (!node.get_parameter("waypoints", p.waypoints)) {
        return false;
    }
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
    std::string backend = "hip";  // "host": the explicit CPU backend for a node with no GPU (config 1)
    node.get_parameter("minsnap_backend", backend);
    if (backend != "hip" && backend != "host") {
        log_error("minsnap_backend must be \"hip\" or \"host\"");
        return false;
    }
    p.host_backend = backend == "host";
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
