"""Type check of the TGMS_ROS2 adapter configuration.

INTEGRATION.md §1 tells a maintainer to copy host/{MinSnap.hpp,MinSnap.cpp,factory.hpp,
Trajectory.hpp} into the reference package and build them with TGMS_ROS2, which swaps
in rclcpp::Clock::SharedPtr, snapstack_msgs2::msg::Goal, the reference Trajectory base
and RCLCPP_* logging.  No ROS 2 workspace exists here, so this compiles those sources
with `g++ -fsyntax-only -DTGMS_ROS2` against minimal committed signature stubs
(tests/ros2_stub/).  A signature/type check only: it catches drift from the
reference's virtual signatures (Trajectory.hpp:33-46: `override` fails on any
mismatch) and from the node's three call sites (src/TrajectoryGenerator.cpp:71, :419,
:516); it runs and links nothing."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "trajectory_generator_ros2_amd", "host")
STUB = os.path.join(ROOT, "tests", "ros2_stub")


def _gxx(src, extra=()):
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-DTGMS_ROS2",
           "-I" + os.path.join(STUB, "include"), "-I" + os.path.join(ROOT, "include"), "-I" + HOST, *extra, src]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("src", [os.path.join(HOST, "MinSnap.cpp"), os.path.join(STUB, "check_node_calls.cpp")],
                         ids=["MinSnap.cpp", "node_call_sites"])
def test_tgms_ros2_configuration_type_checks(src):
    r = _gxx(src)
    assert r.returncode == 0, r.stderr


def test_signature_drift_is_caught(tmp_path):
    """The check has teeth: a MinSnap whose generateTraj took the mirror's steady clock
    instead of rclcpp::Clock::SharedPtr would no longer override the reference virtual."""
    bad = tmp_path / "bad.cpp"
    bad.write_text('#include "Trajectory.hpp"\n'
                   "#include <chrono>\n"
                   "namespace trajectory_generator {\n"
                   "struct Bad : Trajectory {\n"
                   "  Bad() : Trajectory(0.01) {}\n"
                   "  void generateTraj(std::vector<GoalMsg>&, std::unordered_map<int, std::string>&,\n"
                   "                    const std::shared_ptr<std::chrono::steady_clock>&) override {}\n"
                   "};\n}\n")
    r = _gxx(str(bad))
    assert r.returncode != 0 and "override" in r.stderr
