// The reference node's use of its trajectory, made on a MinSnap built by the factory
// branch INTEGRATION.md §1 adds -- type-checked with -DTGMS_ROS2 against the stubs.
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "factory.hpp"

namespace trajectory_generator {

class TrajectoryGeneratorLike : public rclcpp::Node {
public:
    bool readParameters() {  // src/TrajectoryGenerator.cpp:99-425, MinSnap branch
        double freq = 100.0;
        if (!this->get_parameter("pub_freq", freq)) return false;
        dt_ = 1.0 / freq;
        std::string traj_type;
        if (!this->get_parameter("traj_type", traj_type)) return false;
        if (traj_type == "MinSnap") {
            if (!readMinSnapParameters(*this, dt_, traj_)) return false;
        }
        // :419
        return traj_->trajectoryInsideBounds(-5.0, 5.0, -5.0, 5.0, 0.0, 5.0);
    }
    void start() {  // :71
        traj_->generateTraj(traj_goals_full_, index_msgs_full_, this->get_clock());
    }
    void pressedEnd() {  // :516
        traj_->generateStopTraj(traj_goals_, index_msgs_, pub_index_, this->get_clock());
    }

private:
    double dt_ = 0.01;
    std::unique_ptr<Trajectory> traj_;  // TrajectoryGenerator.hpp:83
    std::vector<snapstack_msgs2::msg::Goal> traj_goals_full_, traj_goals_;
    std::unordered_map<int, std::string> index_msgs_full_, index_msgs_;
    int pub_index_ = 0;
};

}  // namespace trajectory_generator
