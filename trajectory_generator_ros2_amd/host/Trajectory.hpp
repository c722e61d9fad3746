// Trajectory.hpp — host-side mirror of the reference's trajectory plugin interface.
//
// Reference: include/trajectory_generator_ros2/trajectories/Trajectory.hpp:24-61.
// Same class name, same three pure virtuals, same argument meaning and ownership:
//   generateTraj            appends to `goals`, fills index_msgs[goal index] = text
//   generateStopTraj        replaces goals / index_msgs, sets pub_index = 0
//   trajectoryInsideBounds  validates the parameters against the room bounds
// Only the ROS types are replaced, because rclcpp / snapstack_msgs2 are not present
// in this image:
//   snapstack_msgs2::msg::Goal  -> trajectory_generator::Goal   (Goal.hpp, same fields)
//   rclcpp::Clock::SharedPtr    -> trajectory_generator::ClockPtr (steady clock)
//   RCLCPP_INFO / RCLCPP_ERROR  -> log_info / log_error (stderr; rclcpp logger under TGMS_ROS2)
// With TGMS_ROS2 defined the real ROS types are used instead;
// that configuration needs a ROS 2 workspace and is not built here.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#ifdef TGMS_ROS2
#include <rclcpp/rclcpp.hpp>

#include "snapstack_msgs2/msg/goal.hpp"
#include "trajectory_generator_ros2/trajectories/Trajectory.hpp"
namespace trajectory_generator {
using GoalMsg = snapstack_msgs2::msg::Goal;
using ClockPtr = rclcpp::Clock::SharedPtr;
inline double clock_seconds(const ClockPtr& c) { return c->now().seconds(); }
}  // namespace trajectory_generator
#else
#include <chrono>

#include "Goal.hpp"

namespace trajectory_generator {

using GoalMsg = Goal;

// Stand-in for rclcpp::Clock: only now() is used by trajectories (Line.cpp:33).
struct Clock {
    double now() const {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};
using ClockPtr = std::shared_ptr<Clock>;
inline double clock_seconds(const ClockPtr& c) { return c ? c->now() : Clock().now(); }

struct Vector3d {
    double v[3];
    double x() const { return v[0]; }
    double y() const { return v[1]; }
    double z() const { return v[2]; }
};

class Trajectory {
public:
    explicit Trajectory(double dt) : dt_(dt) {}
    virtual ~Trajectory() {}

    // Generate the trajectory to be followed; may exit the program (Trajectory.hpp:31-35)
    virtual void generateTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                              const ClockPtr& clock) = 0;

    // Generate a stopping (braking) trajectory (Trajectory.hpp:37-41)
    virtual void generateStopTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                                  int& pub_index, const ClockPtr& clock) = 0;

    // Return if the trajectory params conflict with the room bounds (Trajectory.hpp:43-46)
    virtual bool trajectoryInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin,
                                        double zmax) = 0;

protected:
    // Trajectory.hpp:50-57
    static bool isPointInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin, double zmax,
                                    const Vector3d& point) {
        if (point.x() < xmin || point.x() > xmax) return false;
        if (point.y() < ymin || point.y() > ymax) return false;
        if (point.z() < zmin || point.z() > zmax) return false;
        return true;
    }

    static constexpr double GRAVITY = 9.81;  // m/s^2
    double dt_;                               // goal publication period [s]
};

}  // namespace trajectory_generator
#endif

namespace trajectory_generator {

// RCLCPP_INFO / RCLCPP_ERROR with the reference's printf-style formatting: through the
// node's rclcpp logger when built into the node (TGMS_ROS2), else to stderr.  Info
// lines are always emitted, as the reference logs "Time to calculate the traj" on every
// generation (Line.cpp:87-88); TGMS_NODE_QUIET silences them outside ROS (test runs).
inline void log_msg(bool error, const char* fmt, va_list ap) {
#ifdef TGMS_ROS2
    char buf[512];
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    if (error)
        RCLCPP_ERROR(rclcpp::get_logger("trajectory_generator"), "%s", buf);
    else
        RCLCPP_INFO(rclcpp::get_logger("trajectory_generator"), "%s", buf);
#else
    std::fprintf(stderr, "[%s] [trajectory_generator]: ", error ? "ERROR" : "INFO");
    std::vfprintf(stderr, fmt, ap);
    std::fputc('\n', stderr);
#endif
}
inline void log_info(const char* fmt, ...) {
#ifndef TGMS_ROS2
    if (std::getenv("TGMS_NODE_QUIET")) return;
#endif
    va_list ap;
    va_start(ap, fmt);
    log_msg(false, fmt, ap);
    va_end(ap);
}
inline void log_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    log_msg(true, fmt, ap);
    va_end(ap);
}

}  // namespace trajectory_generator
