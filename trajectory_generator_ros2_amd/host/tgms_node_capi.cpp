// tgms_node_capi.cpp — include/tgms_node.h over the C++ MinSnap trajectory.
#include <algorithm>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "MinSnap.hpp"
#include "factory.hpp"
#include "tgms_node.h"

using namespace trajectory_generator;

struct tgms_node {
    ParamMap params;
    GeneratorSettings settings;
    std::unique_ptr<Trajectory> traj;
    std::vector<GoalMsg> goals;
    std::unordered_map<int, std::string> index_msgs;
    int pub_index = 0;
    ClockPtr clock = std::make_shared<Clock>();
};

extern "C" {

tgms_node* tgms_node_new(void) { return new tgms_node(); }
void tgms_node_free(tgms_node* n) { delete n; }

void tgms_node_set_double(tgms_node* n, const char* name, double v) { n->params.set(name, v); }
void tgms_node_set_array(tgms_node* n, const char* name, const double* v, int32_t count) {
    n->params.set(name, std::vector<double>(v, v + std::max(count, 0)));
}
void tgms_node_set_string(tgms_node* n, const char* name, const char* v) { n->params.set(name, std::string(v)); }

int tgms_node_read_parameters(tgms_node* n) {
    n->traj.reset();
    if (!readParameters(n->params, n->settings, n->traj)) {
        log_error("Could not read parameters.");
        n->traj.reset();
        return 0;
    }
    return 1;
}

int64_t tgms_node_generate_traj(tgms_node* n) {
    if (!n->traj) return -1;
    n->traj->generateTraj(n->goals, n->index_msgs, n->clock);
    return (int64_t)n->goals.size();
}

int64_t tgms_node_generate_stop_traj(tgms_node* n, int32_t pub_index) {
    if (!n->traj) return -1;
    n->pub_index = pub_index;
    n->traj->generateStopTraj(n->goals, n->index_msgs, n->pub_index, n->clock);
    return (int64_t)n->goals.size();
}

int32_t tgms_node_pub_index(const tgms_node* n) { return n->pub_index; }
int64_t tgms_node_goal_count(const tgms_node* n) { return (int64_t)n->goals.size(); }

int tgms_node_goals(const tgms_node* n, int64_t first, int64_t count, double* out) {
    if (first < 0 || count < 0 || first + count > (int64_t)n->goals.size()) return 0;
    for (int64_t k = 0; k < count; ++k) {
        const GoalMsg& g = n->goals[first + k];
        double* o = out + k * TGMS_NODE_GOAL_FIELDS;
        const double f[TGMS_NODE_GOAL_FIELDS] = {g.p.x, g.p.y, g.p.z, g.v.x, g.v.y, g.v.z, g.a.x, g.a.y,
                                                g.a.z, g.j.x, g.j.y, g.j.z, g.psi, g.dpsi, g.power ? 1.0 : 0.0};
        std::copy(f, f + TGMS_NODE_GOAL_FIELDS, o);
    }
    return 1;
}

const char* tgms_node_frame_id(const tgms_node* n, int64_t i) {
    if (i < 0 || i >= (int64_t)n->goals.size()) return nullptr;
    return n->goals[i].header.frame_id.c_str();
}

int32_t tgms_node_index_keys(const tgms_node* n, int32_t* keys, int32_t cap) {
    std::vector<int32_t> k;
    for (const auto& kv : n->index_msgs) k.push_back(kv.first);
    std::sort(k.begin(), k.end());
    for (int32_t i = 0; i < (int32_t)k.size() && i < cap; ++i) keys[i] = k[i];
    return (int32_t)k.size();
}

const char* tgms_node_index_msg(const tgms_node* n, int32_t key) {
    auto it = n->index_msgs.find(key);
    return it == n->index_msgs.end() ? nullptr : it->second.c_str();
}

int tgms_node_inside_bounds(tgms_node* n, double xmin, double xmax, double ymin, double ymax, double zmin,
                            double zmax) {
    if (!n->traj) return 0;
    return n->traj->trajectoryInsideBounds(xmin, xmax, ymin, ymax, zmin, zmax) ? 1 : 0;
}

int32_t tgms_node_coefficients(tgms_node* n, double* out, int32_t cap_doubles) {
    MinSnap* ms = dynamic_cast<MinSnap*>(n->traj.get());
    if (!ms) return 0;
    const std::vector<double>& c = ms->coefficients();
    std::copy(c.begin(), c.begin() + std::min<size_t>(c.size(), (size_t)std::max(cap_doubles, 0)), out);
    return ms->segments();
}

double tgms_node_dt(const tgms_node* n) { return n->settings.dt; }

int32_t tgms_node_shape_waypoints(const char* shape, double cx, double cy, double orientation, double length,
                                  double width, double z, int32_t laps, double* out, int32_t cap) {
    return shapeWaypoints(shape, cx, cy, orientation, length, width, z, laps, out, cap);
}

}  // extern "C"
