// Signature stub of snapstack_msgs2::msg::Goal: the fields the reference writes
// (src/TrajectoryGenerator.cpp:621-634, src/trajectories/Circle.cpp:105-127).
#pragma once
#include <cstdint>
#include <string>

namespace builtin_interfaces::msg {
struct Time {
    int32_t sec = 0;
    uint32_t nanosec = 0;
};
}  // namespace builtin_interfaces::msg

namespace std_msgs::msg {
struct Header {
    builtin_interfaces::msg::Time stamp;
    std::string frame_id;
};
}  // namespace std_msgs::msg

namespace geometry_msgs::msg {
struct Vector3 {
    double x = 0.0, y = 0.0, z = 0.0;
};
}  // namespace geometry_msgs::msg

namespace snapstack_msgs2::msg {
struct Goal {
    std_msgs::msg::Header header;
    geometry_msgs::msg::Vector3 p, v, a, j, s;
    double psi = 0.0;
    double dpsi = 0.0;
    bool power = false;
    uint8_t mode_xy = 0, mode_z = 0;
};
}  // namespace snapstack_msgs2::msg
