"""CPU: the ROS drop-in's parameters and scan gating (dm/ros_node.py) — the
decisions of the stage it replaces (slam_toolbox's shouldProcessScan front
gate and Karto's HasMovedEnough over throttle_scans, minimum_time_interval,
minimum_travel_distance / _heading; server/thymio_project/config/
slam_config.yaml:23,28,37-38; restated, parity unpinned) on fake message
streams, the parameter file, and the launch file's wiring."""
import ast
import math
import os

import pytest

from dm.ros_node import ScanGate, SlamParams, quaternion_from_yaw, stamp_seconds, yaw_from_quaternion

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_YAML = "/root/reference/server/thymio_project/config/slam_config.yaml"


def test_defaults_are_the_reference_config():
    p = SlamParams()
    assert (p.throttle_scans, p.map_update_interval, p.resolution, p.max_laser_range) == (1, 5.0, 0.05, 12.0)
    assert (p.minimum_time_interval, p.minimum_travel_distance, p.minimum_travel_heading) == (0.5, 0.1, 0.1)
    assert (p.map_frame, p.base_frame, p.scan_topic) == ("map", "base_link", "/scan")
    gp = p.grid_params()
    assert gp.resolution == 0.05 and gp.range_max == 12.0 and gp.width == 4096


@pytest.mark.skipif(not os.path.exists(REF_YAML), reason="reference checkout not present")
def test_reads_the_reference_parameter_file():
    p = SlamParams.from_yaml(REF_YAML)
    assert p == SlamParams()  # every value the stage uses equals the defaults above


def test_parameter_file_overrides(tmp_path):
    f = tmp_path / "p.yaml"
    f.write_text("slam_toolbox:\n  ros__parameters:\n    resolution: 0.1\n    max_laser_range: 8.0\n"
                 "    throttle_scans: 3\n    minimum_time_interval: 0.2\n    do_loop_closing: true\n"
                 "    dm_width: 1000\n")
    p = SlamParams.from_yaml(str(f))
    assert (p.resolution, p.max_laser_range, p.throttle_scans, p.minimum_time_interval, p.dm_width) == \
        (0.1, 8.0, 3, 0.2, 1000)
    gp = p.grid_params()
    assert gp.resolution == 0.1 and gp.range_max == 8.0 and gp.origin_x == -50.0


def test_gate_time_distance_heading():
    """slam_toolbox's front gate, then Karto's HasMovedEnough (ScanGate's
    docstring); the slam_config.yaml thresholds 0.5 s / 0.1 m / 0.1 rad."""
    g = ScanGate()
    assert g.accept(0.0, (0, 0, 0))            # the first scan always
    assert not g.accept(0.3, (1.0, 0, 0))      # moved, but too soon (< 0.5 s)
    assert not g.accept(0.6, (0.05, 0, 0))     # in time, moved 5 cm < sqrt(0.8) * 0.1 m
    assert not g.accept(0.7, (0.1, 0, 0))      # enough, but the 4th scan: warm-up (counter < 5)
    assert g.accept(0.8, (0.1, 0, 0))          # 5th scan, 0.1 m, 0.8 s
    assert not g.accept(1.5, (0.1, 0, 1.0))    # turned 1 rad in place: no translation, rejected
    assert not g.accept(2.0, (0.1 + 0.0894, 0, 1.0))  # 0.0894^2 < 0.8 * 0.01
    assert g.accept(2.1, (0.1 + 0.0895, 0, 1.0))      # 0.0895^2 >= 0.8 * 0.01 (within 10 %)


def test_karto_layer_heading_and_wrap():
    """Karto's HasMovedEnough on its own (it only decides when its thresholds
    differ from the front gate's): time, or heading (normalised), or
    distance (less KT_TOLERANCE)."""
    g = ScanGate()
    g.last = (0.0, 0.0, 0.0, 0.1)
    assert g._moved_enough(0.5, 0.0, 0.0, 0.1)                          # 0.5 s passed
    assert not g._moved_enough(0.4, 0.05, 0.0, 0.15)                    # 5 cm, 0.05 rad
    assert g._moved_enough(0.4, 0.0, 0.0, 0.2)                          # turned 0.1 rad
    assert g._moved_enough(0.4, 0.0, 0.0, 0.1 + 2 * math.pi - 0.15)     # wraps: 0.15 rad
    assert not g._moved_enough(0.4, 0.0, 0.0, 0.1 + 2 * math.pi - 0.05)  # wraps: 0.05 rad
    assert g._moved_enough(0.4, 0.1, 0.0, 0.1)                          # 0.1 m


def test_gate_throttle():
    g = ScanGate(throttle_scans=3, minimum_time_interval=0.0, minimum_travel_distance=0.0,
                 minimum_travel_heading=0.0)
    got = [g.accept(float(k), (k, 0, 0)) for k in range(10)]
    # first scan, then every third scan of the counter once past the warm-up
    # (counter 3 < 5 is dropped; 6 and 9 pass -> calls 5 and 8)
    assert got == [True, False, False, False, False, True, False, False, True, False]


def test_gate_stream_rate():
    """A 10 Hz LD06 stream of a robot at 0.2 m/s: a scan every 0.5 s passes."""
    g = ScanGate()
    acc = [k for k in range(100) if g.accept(0.1 * k, (0.02 * k, 0.0, 0.0))]
    assert acc[:4] == [0, 5, 10, 15] and len(acc) == 20


def test_stamps_and_quaternions():
    class T:
        sec, nanosec = 12, 500_000_000
    assert stamp_seconds(T()) == 12.5 and stamp_seconds(3.25) == 3.25
    for yaw in (-3.0, -0.5, 0.0, 1.2, 3.1):
        assert abs(yaw_from_quaternion(quaternion_from_yaw(yaw)) - yaw) < 1e-12


def test_launch_file_remaps_slam_toolbox_map_and_starts_dm_mapper():
    path = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd", "launch",
                        "dm_pc_server.launch.py")
    tree = ast.parse(open(path).read())
    calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call)]
    names = [getattr(c.func, "id", getattr(c.func, "attr", None)) for c in calls]
    remaps = [c for c in calls if getattr(c.func, "id", None) == "SetRemap"]
    assert any(kw.arg == "src" and kw.value.value == "/map" for c in remaps for kw in c.keywords)
    nodes = [c for c in calls if getattr(c.func, "id", None) == "Node"]
    execs = {kw.value.value for c in nodes for kw in c.keywords if kw.arg == "executable"}
    assert {"dm_mapper", "main", "rviz2"} <= execs  # the reference's thymio_driver and rviz2 stay
    assert "IncludeLaunchDescription" in names and "generate_launch_description" in \
        [f.name for f in tree.body if isinstance(f, ast.FunctionDef)]


def test_launch_file_exposes_the_sharded_map():
    """dm_devices (one map in row bands over several GPUs, dm_create_sharded)
    is a launch argument passed to the mapper node like dm_device."""
    path = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd", "launch",
                        "dm_pc_server.launch.py")
    tree = ast.parse(open(path).read())
    calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call)]
    declared = {c.args[0].value for c in calls if getattr(c.func, "id", None) == "DeclareLaunchArgument"}
    assert {"dm_width", "dm_height", "dm_device", "dm_devices", "dm_explore"} <= declared
    passed = {k.value for c in calls if getattr(c.func, "id", None) == "Node"
              for kw in c.keywords if kw.arg == "parameters"
              for d in kw.value.elts if isinstance(d, ast.Dict) for k in d.keys}
    assert "dm_devices" in passed
