// MinSnap.cpp — see MinSnap.hpp.  Conventions follow the reference primitives:
//   goal.header.frame_id = "world", goal.power = true      (Line.cpp:91-115, Circle.cpp:106/127)
//   generation errors: log + exit(1)                         (Line.cpp:77-78, Circle.cpp:86-87)
//   last goal pinned to the end point                        (Line.cpp:80-82; done by the sampler)
//   "Time to calculate the traj" / "Goal vector size" logs   (Line.cpp:87-88)
#include "MinSnap.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

namespace trajectory_generator {

namespace {

GoalMsg to_goal(const double* s) {
    GoalMsg g;
    g.header.frame_id = "world";
    g.p.x = s[0];
    g.p.y = s[1];
    g.p.z = s[2];
    g.v.x = s[3];
    g.v.y = s[4];
    g.v.z = s[5];
    g.a.x = s[6];
    g.a.y = s[7];
    g.a.z = s[8];
    g.j.x = s[9];
    g.j.y = s[10];
    g.j.z = s[11];
    g.psi = s[12];
    g.dpsi = s[13];
    g.power = true;
    return g;
}

bool inside(double xmin, double xmax, double ymin, double ymax, double zmin, double zmax, const double* q) {
    return !(q[0] < xmin || q[0] > xmax || q[1] < ymin || q[1] > ymax || q[2] < zmin || q[2] > zmax);
}

std::string fmt_double(double v) { return std::to_string(v); }

}  // namespace

MinSnap::MinSnap(const MinSnapParams& params, double dt) : Trajectory(dt), p_(params) {}

MinSnap::~MinSnap() {
    if (h_) tgms_destroy(h_);
}

tgms_handle* MinSnap::handle() {
    if (!h_) {
        const tgms_status s = p_.host_backend ? tgms_create_host(&h_) : tgms_create(&h_, p_.device);
        if (s != TGMS_OK) {
            h_ = nullptr;
            if (p_.host_backend)
                log_error("MinSnap: cannot create the host solver: %s", tgms_status_string(s));
            else
                log_error("MinSnap: cannot create the GPU solver on device %d: %s", p_.device,
                          tgms_status_string(s));
        }
    }
    return h_;
}

bool MinSnap::solve_and_sample(const std::vector<double>& W, const std::vector<double>& T, const double* end_derivs,
                               std::vector<double>& coeffs, std::vector<double>& samples, std::string& err) {
    tgms_handle* h = handle();
    if (!h) {
        err = p_.host_backend ? "no host solver" : "no GPU solver";
        return false;
    }
    const int32_t M = (int32_t)T.size();
    const int32_t so[2] = {0, M};
    int32_t st = TGMS_OK;
    coeffs.assign((size_t)M * 24, 0.0);
    tgms_status s = tgms_solve_batch(h, 1, so, W.data(), T.data(), end_derivs, coeffs.data(), &st);
    if (s != TGMS_OK || st != TGMS_OK) {
        err = std::string("solve failed: ") + tgms_status_string(s != TGMS_OK ? s : st) + " " + tgms_last_error(h);
        return false;
    }
    int64_t offs[2];
    s = tgms_sample_offsets(1, so, T.data(), dt_, offs);
    if (s != TGMS_OK) {
        err = std::string("sample_offsets failed: ") + tgms_status_string(s);
        return false;
    }
    samples.assign((size_t)offs[1] * TGMS_GOAL_STRIDE, 0.0);
    s = tgms_sample_batch(h, 1, so, W.data(), T.data(), end_derivs, coeffs.data(), dt_, p_.yaw_mode, p_.yaw, offs,
                          samples.data());
    if (s != TGMS_OK) {
        err = std::string("sampling failed: ") + tgms_status_string(s) + " " + tgms_last_error(h);
        return false;
    }
    return true;
}

bool MinSnap::ensure_main() {
    if (solved_) return true;
    std::string err;
    if (!solve_and_sample(p_.waypoints, p_.seg_times, nullptr, coeffs_, samples_, err)) {
        log_error("MinSnap traj: %s", err.c_str());
        return false;
    }
    solved_ = true;
    return true;
}

const std::vector<double>& MinSnap::coefficients() {
    if (!ensure_main()) std::exit(1);
    return coeffs_;
}

void MinSnap::generateTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                           const ClockPtr& clock) {
    const double tstart = clock_seconds(clock);
    if (!ensure_main()) {
        log_error("Error: could not generate the MinSnap trajectory");
        std::exit(1);
    }
    const int M = segments();
    double total = 0.0;
    for (double t : p_.seg_times) total += t;
    const size_t first = goals.size();
    const size_t n = samples_.size() / TGMS_GOAL_STRIDE;
    goals.reserve(first + n);
    for (size_t k = 0; k < n; ++k) goals.push_back(to_goal(&samples_[k * TGMS_GOAL_STRIDE]));

    index_msgs[(int)first] = "MinSnap traj: following " + std::to_string(M) + " segments through " +
                             std::to_string(M + 1) + " waypoints in " + fmt_double(total) + " s";
    // the first goal at or after each interior waypoint's arrival time
    double tau = 0.0;
    for (int i = 1; i < M; ++i) {
        tau += p_.seg_times[i - 1];
        const size_t k = (size_t)std::ceil(tau / dt_ - 1e-9);
        if (k > 0 && k + 1 < n)
            index_msgs[(int)(first + k)] = "MinSnap traj: reached waypoint " + std::to_string(i);
    }
    index_msgs[(int)goals.size() - 1] = "MinSnap traj: stopped";

    log_info("Time to calculate the traj (s): %f", clock_seconds(clock) - tstart);
    log_info("Goal vector size = %lu", (unsigned long)goals.size());
}

void MinSnap::generateStopTraj(std::vector<GoalMsg>& goals, std::unordered_map<int, std::string>& index_msgs,
                               int& pub_index, const ClockPtr& clock) {
    const double tstart = clock_seconds(clock);
    if (goals.empty()) {
        log_error("MinSnap traj: no current goal to brake from");
        std::exit(1);
    }
    const int idx = std::min(std::max(pub_index, 0), (int)goals.size() - 1);
    const GoalMsg& g = goals[idx];
    const double p0[3] = {g.p.x, g.p.y, g.p.z};
    const double v0[3] = {g.v.x, g.v.y, g.v.z};
    const double speed = std::sqrt(v0[0] * v0[0] + v0[1] * v0[1] + v0[2] * v0[2]);
    // one septic segment from the current p/v/a/j to rest; duration from the braking
    // deceleration, end point where a constant deceleration would stop
    const double T = std::max(2.0 * speed / p_.stop_accel, 4.0 * dt_);
    std::vector<double> W = {p0[0], p0[1], p0[2], p0[0] + 0.5 * v0[0] * T, p0[1] + 0.5 * v0[1] * T,
                             p0[2] + 0.5 * v0[2] * T};
    std::vector<double> Ts = {T};
    double ed[18] = {g.v.x, g.v.y, g.v.z, g.a.x, g.a.y, g.a.z, g.j.x, g.j.y, g.j.z};  // final: rest

    MinSnapParams keep = p_;
    p_.yaw = g.psi;  // hold the current heading (constant mode, and velocity mode at rest)
    std::vector<double> c, s;
    std::string err;
    const bool ok = solve_and_sample(W, Ts, ed, c, s, err);
    p_ = keep;
    if (!ok) {
        log_error("MinSnap traj: braking trajectory failed: %s", err.c_str());
        std::exit(1);
    }
    std::vector<GoalMsg> goals_tmp;
    std::unordered_map<int, std::string> index_msgs_tmp;
    const size_t n = s.size() / TGMS_GOAL_STRIDE;
    goals_tmp.reserve(n);
    for (size_t k = 0; k < n; ++k) goals_tmp.push_back(to_goal(&s[k * TGMS_GOAL_STRIDE]));
    index_msgs_tmp[0] = "MinSnap traj: pressed END, braking to rest in " + fmt_double(T) + " s";
    index_msgs_tmp[(int)goals_tmp.size() - 1] = "MinSnap traj: stopped";

    goals = std::move(goals_tmp);
    index_msgs = std::move(index_msgs_tmp);
    pub_index = 0;

    log_info("Time to calculate the braking traj (s): %f", clock_seconds(clock) - tstart);
    log_info("Goal vector size = %lu", (unsigned long)goals.size());
}

bool MinSnap::trajectoryInsideBounds(double xmin, double xmax, double ymin, double ymax, double zmin,
                                     double zmax) {
    const size_t npts = p_.waypoints.size() / 3;
    for (size_t i = 0; i < npts; ++i) {
        if (!inside(xmin, xmax, ymin, ymax, zmin, zmax, &p_.waypoints[3 * i])) {
            log_error("MinSnap waypoint %zu (%f, %f, %f) is outside the room bounds", i, p_.waypoints[3 * i],
                      p_.waypoints[3 * i + 1], p_.waypoints[3 * i + 2]);
            return false;
        }
    }
    // a min-snap spline can overshoot between waypoints: check every sampled position
    if (!ensure_main()) return false;
    const size_t n = samples_.size() / TGMS_GOAL_STRIDE;
    for (size_t k = 0; k < n; ++k) {
        const double* q = &samples_[k * TGMS_GOAL_STRIDE];
        if (!inside(xmin, xmax, ymin, ymax, zmin, zmax, q)) {
            log_error("MinSnap trajectory leaves the room bounds at t = %f s (%f, %f, %f)", (double)k * dt_, q[0],
                      q[1], q[2]);
            return false;
        }
    }
    return true;
}

}  // namespace trajectory_generator
