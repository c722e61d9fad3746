"""GPU: the C++ MinSnap adapter driven like TrajectoryGenerator drives a primitive
(readParameters -> generateTraj -> modeCB END -> generateStopTraj), checked against
the oracle.  Reference conventions: frame_id "world" and power = true
(Line.cpp:91-115), last goal pinned to the end point (Line.cpp:80-82), generateTraj
appends (Line.cpp:33-89), generateStopTraj replaces and sets pub_index = 0
(Line.cpp:145-147)."""
import numpy as np
import pytest

from test_node_host import WAYPOINTS, base_params

pytestmark = pytest.mark.gpu

TOL = 1e-9


def _node(**kw):
    from trajectory_generator_ros2_amd.node import MinSnapNode
    n = MinSnapNode(base_params(**kw))
    assert n.read_parameters()
    return n


def test_generate_traj_matches_oracle(oracle):
    n = _node()
    W = np.array(WAYPOINTS).reshape(-1, 3)
    T = np.array([2.0, 2.0, 2.5])
    C = n.coefficients()
    R, st = oracle.solve(W, T)
    assert st == 0
    err = np.abs(C - R).max(axis=(0, 2)) / np.abs(R).max(axis=(0, 2))
    assert err.max() <= TOL, err
    cnt = n.generate_traj()
    G = n.goals()
    ref = oracle.sample(R, T, W, None, 0.01, oracle.YAW_CONSTANT, 0.3)
    assert cnt == G.shape[0] == ref.shape[0] == oracle.sample_count(6.5, 0.01)
    scale = max(1.0, np.abs(ref[:, :12]).max())
    assert np.abs(G[:, :14] - ref[:, :14]).max() <= TOL * scale
    assert (G[:, 14] == 1.0).all()                               # power = true
    assert n.frame_id(0) == "world" and n.frame_id(cnt - 1) == "world"
    np.testing.assert_array_equal(G[-1, :3], W[-1])              # pinned end point
    np.testing.assert_array_equal(G[-1, 3:12], np.zeros(9))     # at rest
    msgs = n.index_msgs()
    assert 0 in msgs and msgs[cnt - 1] == "MinSnap traj: stopped"
    assert msgs[200].endswith("waypoint 1") and msgs[400].endswith("waypoint 2")


def test_generate_traj_appends(oracle):
    n = _node()
    a = n.generate_traj()
    b = n.generate_traj()
    assert b == 2 * a
    G = n.goals()
    np.testing.assert_array_equal(G[:a], G[a:])
    assert n.index_msgs()[a].startswith("MinSnap traj: following")


def test_velocity_yaw_matches_oracle(oracle):
    n = _node(yaw_mode="velocity")
    n.generate_traj()
    G = n.goals()
    W = np.array(WAYPOINTS).reshape(-1, 3)
    T = np.array([2.0, 2.0, 2.5])
    ref = oracle.sample(oracle.solve(W, T)[0], T, W, None, 0.01, oracle.YAW_VELOCITY, 0.3)
    moving = np.hypot(ref[:, 3], ref[:, 4]) > 1e-2
    d = np.angle(np.exp(1j * (G[moving, 12] - ref[moving, 12])))
    assert np.abs(d).max() <= 1e-9


def test_auto_time_allocation(oracle):
    n = _node(seg_times=None, v_goals=[1.0], min_seg_time=0.5)
    n.generate_traj()
    W = np.array(WAYPOINTS).reshape(-1, 3)
    T = np.maximum(np.linalg.norm(np.diff(W, axis=0), axis=1) / 1.0, 0.5)
    R, _ = oracle.solve(W, T)
    C = n.coefficients()
    assert (np.abs(C - R).max(axis=(0, 2)) / np.abs(R).max(axis=(0, 2))).max() <= TOL
    assert n.goals().shape[0] == oracle.sample_count(float(T.sum()), 0.01)


def test_stop_traj_brakes_from_current_goal(oracle):
    n = _node()
    n.generate_traj()
    G = n.goals()
    k = 250
    g = G[k]
    cnt = n.generate_stop_traj(k)
    assert n.pub_index == 0
    S = n.goals()
    assert S.shape[0] == cnt
    v = g[3:6]
    T = max(2.0 * np.linalg.norm(v) / 1.0, 4 * 0.01)
    W = np.stack([g[0:3], g[0:3] + 0.5 * v * T])
    ED = np.zeros((2, 3, 3))
    ED[0] = g[3:12].reshape(3, 3)
    R, st = oracle.solve(W, np.array([T]), ED)
    assert st == 0
    ref = oracle.sample(R, np.array([T]), W, ED, 0.01, oracle.YAW_CONSTANT, g[12])
    assert S.shape[0] == ref.shape[0]
    assert np.abs(S[:, :14] - ref[:, :14]).max() <= TOL * max(1.0, np.abs(ref[:, :12]).max())
    np.testing.assert_allclose(S[0, :12], g[:12], rtol=0, atol=1e-12)  # continues from p/v/a/j
    np.testing.assert_array_equal(S[-1, 3:12], np.zeros(9))            # ends at rest
    assert (S[:, 12] == g[12]).all()                                   # holds the heading
    msgs = n.index_msgs()
    assert set(msgs) == {0, cnt - 1} and msgs[cnt - 1] == "MinSnap traj: stopped"


def test_inside_bounds_checks_sampled_overshoot(oracle):
    n = _node()
    G = None
    n.generate_traj()
    G = n.goals()
    lo, hi = G[:, :3].min(axis=0), G[:, :3].max(axis=0)
    W = np.array(WAYPOINTS).reshape(-1, 3)
    assert n.inside_bounds(lo[0], hi[0], lo[1], hi[1], lo[2], hi[2])
    # every waypoint inside, but the spline overshoots the waypoints' bounding box
    wl, wh = W.min(axis=0), W.max(axis=0)
    assert (lo < wl - 1e-6).any() or (hi > wh + 1e-6).any()
    assert not n.inside_bounds(wl[0], wh[0], wl[1], wh[1], wl[2], wh[2])
    m = _node()
    assert not m.inside_bounds(-5, 5, -5, 5, 1.2, 5)  # first waypoint z = 1.0 below z_min


def test_read_parameters_rejects_overshoot():
    """readParameters fails when the sampled trajectory leaves the room, even though
    every waypoint is inside (src/TrajectoryGenerator.cpp:417-421)."""
    from trajectory_generator_ros2_amd.node import MinSnapNode
    W = np.array(WAYPOINTS).reshape(-1, 3)
    wl, wh = W.min(axis=0), W.max(axis=0)
    n = MinSnapNode(base_params(x_min=wl[0], x_max=wh[0], y_min=wl[1], y_max=wh[1], z_min=wl[2], z_max=wh[2]))
    assert not n.read_parameters()


def test_smooth_M_from_reference_shape(oracle):
    """waypoint_source "M": the reference's M corners flown as one min-snap spline
    (SURVEY.md §8(f) rank 4), matching the oracle through the same waypoints."""
    from trajectory_generator_ros2_amd.node import MinSnapNode, shape_waypoints
    p = base_params(waypoint_source="M", M_length=3.0, M_width=4.0, center_x=0.0, center_y=0.0,
                    orientation=0.2, laps=2.0, yaw_mode="velocity")
    p.pop("seg_times")
    p.pop("waypoints")
    p["v_goals"] = [1.0]
    n = MinSnapNode(p)
    assert n.read_parameters()
    W = shape_waypoints("M", 0.0, 0.0, 0.2, 3.0, 4.0, 1.8, 2)
    T = np.maximum(np.linalg.norm(np.diff(W, axis=0), axis=1), 0.5)
    R, st = oracle.solve(W, T)
    assert st == 0 and W.shape[0] == 9
    C = n.coefficients()
    assert (np.abs(C - R).max(axis=(0, 2)) / np.abs(R).max(axis=(0, 2))).max() <= TOL
    n.generate_traj()
    G = n.goals()
    np.testing.assert_array_equal(G[-1, :3], W[-1])
    assert np.allclose(G[:, 2], 1.8, atol=1e-12)   # planar shape stays at alt
