"""CPU: ROS-side helpers of the drop-in node (no GPU needed)."""
import math

import numpy as np

from dm.ros_node import Quaternion, yaw_from_quaternion


def reference_euler_to_quaternion(roll, pitch, yaw):
    # formula of server/thymio_project/thymio_project/main.py:31-36
    qx = np.sin(roll / 2) * np.cos(pitch / 2) * np.cos(yaw / 2) - np.cos(roll / 2) * np.sin(pitch / 2) * np.sin(yaw / 2)
    qy = np.cos(roll / 2) * np.sin(pitch / 2) * np.cos(yaw / 2) + np.sin(roll / 2) * np.cos(pitch / 2) * np.sin(yaw / 2)
    qz = np.cos(roll / 2) * np.cos(pitch / 2) * np.sin(yaw / 2) - np.sin(roll / 2) * np.sin(pitch / 2) * np.cos(yaw / 2)
    qw = np.cos(roll / 2) * np.cos(pitch / 2) * np.cos(yaw / 2) + np.sin(roll / 2) * np.sin(pitch / 2) * np.sin(yaw / 2)
    return [qx, qy, qz, qw]


def test_yaw_roundtrip_with_reference_tf_quaternions():
    for yaw in np.linspace(-math.pi + 1e-6, math.pi - 1e-6, 101):
        q = reference_euler_to_quaternion(0.0, 0.0, yaw)
        got = yaw_from_quaternion(Quaternion(*q))
        assert abs(math.remainder(got - yaw, 2 * math.pi)) < 1e-12


# -- the node's host logic on an oracle-backed stand-in (tests/oracle_mapper.py)
import cases  # noqa: E402
from dm import synth  # noqa: E402
from dm.ros_node import Header, LaserScan, MappingNode  # noqa: E402
from oracle_mapper import OracleMapper  # noqa: E402


class _Executor:
    """What rclpy's executor does for MappingNode (main()): scans at 10 Hz,
    the map_update_interval timer, the frontier poll timer, on a fake clock."""

    def __init__(self, node, interval):
        self.node, self.interval, self.t, self.next_tick = node, interval, 0.0, interval

    def run(self, until, scan_at=None):
        while self.t < until - 1e-9:
            self.t = round(self.t + 0.1, 10)
            if scan_at is not None:
                self.node.scan_cb(scan_at(self.t))
            if self.t >= self.next_tick - 1e-9:
                self.node.timer_cb()
                self.next_tick += self.interval
            self.node.poll_frontiers()


def _node(p_world, pose, latency=0, **kw):
    p, batches, amin, inc = p_world
    mapper = OracleMapper(p, pass_latency=latency)
    clock = [0.0]
    node = MappingNode(dm_width=int(p.width), dm_height=int(p.height), resolution=float(p.resolution),
                       pose_provider=lambda m: pose(m), clock=lambda: clock[0], mapper=mapper, **kw)
    return node, mapper, clock


def test_stationary_robot_republishes_every_interval(oracle_lib):
    """slam_toolbox publishes /map every map_update_interval (slam_config.yaml:25)
    from its own loop: a robot that stopped (every scan after the first
    gated out by minimum_travel_*, :37-38) still gets a map every 5 s, stamped
    with the tick's time; frontiers follow each map."""
    world = cases.world_case(11, 300, 300, 0.05, 1, 450, 1)
    p, batches, amin, inc = world
    poses, ranges = batches[0]
    node, mapper, clock = _node(world, lambda m: tuple(poses[0]))
    ex = _Executor(node, 5.0)

    def scan(t):
        clock[0] = t
        return LaserScan(header=Header(stamp=t, frame_id="base_laser"), angle_min=amin,
                         angle_increment=inc, ranges=ranges[0])

    ex.run(20.0, scan)
    assert node.scans_seen == 200 and node.scans_integrated == 1  # stationary: gated out
    stamps = [m.header.stamp for m in node.map_pub.messages]
    assert stamps == [5.0, 10.0, 15.0, 20.0]
    assert all(m.info.map_load_time == m.header.stamp for m in node.map_pub.messages)
    om = oracle_lib.OracleMap(p)
    om.integrate(poses, ranges, amin, inc)
    np.testing.assert_array_equal(np.frombuffer(node.map_pub.messages[-1].data, np.int8).reshape(300, 300),
                                  om.state)
    assert len(node.frontier_pub.messages) == 4
    exp = om.frontiers(want_mask=False, want_labels=False)[2]
    assert [c.label for c in node.frontier_pub.messages[-1]] == exp["label"].tolist()


def test_no_map_before_the_first_scan():
    world = cases.world_case(12, 128, 128, 0.05, 1, 90, 1)
    node, mapper, clock = _node(world, lambda m: None)
    ex = _Executor(node, 1.0)
    ex.run(3.0)
    assert node.map_pub.messages == [] and mapper.begins == 0


def test_frontier_pass_never_blocks_the_callbacks(oracle_lib):
    """The timer starts the GPU pass (frontiers_begin) and returns; the
    clusters go out from a later callback once frontiers_ready() says the
    pass is done (here: 3 polls find it running), with the goal stamped like its map."""
    world = cases.world_case(13, 300, 300, 0.05, 1, 450, 3)
    p, batches, amin, inc = world
    k = [0]
    node, mapper, clock = _node(world, lambda m: tuple(batches[min(k[0], 2)][0][0]), latency=3,
                                gate=False, dm_explore=True, dm_goal_min_size=1)
    for j in range(3):
        k[0] = j
        node.scan_cb(LaserScan(angle_min=amin, angle_increment=inc, ranges=batches[j][1][0]))
    clock[0] = 5.0
    node.timer_cb()
    assert len(node.map_pub.messages) == 1 and node.frontier_pub.messages == []
    assert not any(node.poll_frontiers() for _ in range(3))  # still running on the "GPU"
    assert node.frontier_pub.messages == []
    assert node.poll_frontiers()  # done now
    assert len(node.frontier_pub.messages) == 1
    om = oracle_lib.OracleMap(p)
    for poses, ranges in batches:
        om.integrate(poses, ranges, amin, inc)
    exp = om.frontiers(want_mask=False, want_labels=False)[2]
    assert [c.label for c in node.frontier_pub.messages[0]] == exp["label"].tolist()
    assert len(node.goal_pub.messages) == 1 and node.goal_pub.messages[0].header.stamp == 5.0
    # a pass still pending at the next tick is collected first (one in flight)
    clock[0] = 10.0
    node.timer_cb()
    clock[0] = 15.0
    node.timer_cb()
    assert len(node.frontier_pub.messages) == 2 and mapper.begins == 3
