// factory.cpp — readParameters() mirror around the MinSnap branch (factory.hpp).
// Reference: src/TrajectoryGenerator.cpp:150-425.  Only traj_type "MinSnap" is built
// here; the reference's closed-form primitives (Circle, Line, ...) are outside the
// accelerated path and are reported as unsupported.
#include "factory.hpp"

namespace trajectory_generator {

template bool readMinSnapParameters<const ParamMap>(const ParamMap&, double, std::unique_ptr<Trajectory>&);

bool readParameters(const ParamMap& node, GeneratorSettings& s, std::unique_ptr<Trajectory>& traj) {
    if (!node.get_parameter("alt", s.alt)) return false;
    double freq;
    if (!node.get_parameter("pub_freq", freq)) return false;
    if (!(freq > 0)) {
        log_error("pub_freq must be > 0");
        return false;
    }
    s.dt = 1.0 / freq;
    if (!node.get_parameter("traj_type", s.traj_type)) return false;
    if (s.traj_type == "MinSnap") {
        if (!readMinSnapParameters(node, s.dt, traj)) return false;
    } else {
        log_error("traj_type %s is not provided by this build (only MinSnap)", s.traj_type.c_str());
        return false;
    }
    if (!node.get_parameter("x_min", s.xmin)) return false;
    if (!node.get_parameter("x_max", s.xmax)) return false;
    if (!node.get_parameter("y_min", s.ymin)) return false;
    if (!node.get_parameter("y_max", s.ymax)) return false;
    if (!node.get_parameter("z_min", s.zmin)) return false;
    if (!node.get_parameter("z_max", s.zmax)) return false;
    if (!traj->trajectoryInsideBounds(s.xmin, s.xmax, s.ymin, s.ymax, s.zmin, s.zmax)) {
        log_error("The trajectory parameters conflict with the room bounds.");
        return false;
    }
    return true;
}

}  // namespace trajectory_generator
