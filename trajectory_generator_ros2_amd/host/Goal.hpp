// Goal.hpp — the fields of snapstack_msgs2::msg::Goal that the reference trajectories
// write (Line.cpp createLineGoal, Circle.cpp:96-130): header.frame_id, p, v, a, j,
// psi, dpsi, power.  snapstack_msgs2 is an un-vendored ROS message package
// (SURVEY.md §8(c)); this struct stands in for it in the standalone build only.
#pragma once

#include <string>

namespace trajectory_generator {

struct Vector3 {
    double x = 0.0, y = 0.0, z = 0.0;
};

struct Header {
    std::string frame_id;
};

struct Goal {
    Header header;
    Vector3 p, v, a, j;
    double psi = 0.0;
    double dpsi = 0.0;
    bool power = false;
};

}  // namespace trajectory_generator
