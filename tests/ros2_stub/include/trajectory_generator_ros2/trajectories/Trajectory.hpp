// Signature restatement of the reference base class
// (include/trajectory_generator_ros2/trajectories/Trajectory.hpp:24-61): namespace,
// constructor, the three pure virtuals with their exact parameter types, the protected
// helper and members.  Written for the TGMS_ROS2 type check only.
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

#include <Eigen/Core>
#include <rclcpp/rclcpp.hpp>

#include "snapstack_msgs2/msg/goal.hpp"

namespace trajectory_generator {

class Trajectory {
public:
    explicit Trajectory(double dt) : dt_(dt) {}
    virtual ~Trajectory() {}

    virtual void generateTraj(std::vector<snapstack_msgs2::msg::Goal>& goals,
                              std::unordered_map<int, std::string>& index_msgs,
                              const rclcpp::Clock::SharedPtr& clock) = 0;
    virtual void generateStopTraj(std::vector<snapstack_msgs2::msg::Goal>& goals,
                                  std::unordered_map<int, std::string>& index_msgs, int& pub_index,
                                  const rclcpp::Clock::SharedPtr& clock) = 0;
    virtual bool trajectoryInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin,
                                        double zmax) = 0;

protected:
    static bool isPointInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin, double zmax,
                                    Eigen::Vector3d point);
    static constexpr double GRAVITY = 9.81;
    double dt_;
};

}  // namespace trajectory_generator
