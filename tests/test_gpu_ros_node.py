"""GPU: the ROS 2 drop-in (dm/ros_node.py) driven with duck-typed LaserScan
messages, as the LD06 driver publishes them: it integrates exactly the scans
slam_toolbox's gating accepts (slam_config.yaml:23,28,37-38), publishes the
/map the oracle builds from those scans, the frontier clusters, a frontier
goal on /goal_pose, and the /map-image pixels get_map_image would serve
(server/thymio_project/thymio_project/main.py:241-279)."""
import io

import numpy as np
import pytest

import cases
import np_oracle
from dm import synth
from dm.ros_node import Header, LaserScan, MappingNode, ScanGate, yaw_from_quaternion

pytestmark = pytest.mark.gpu


def _stream(seed, n, N=450):
    p, batches, amin, inc = cases.world_case(seed, 400, 400, 0.05, 1, N, n)
    return p, batches, amin, inc


def test_mapping_node_publishes_oracle_map(oracle_lib):
    p, batches, amin, inc = _stream(5, 15)
    om = oracle_lib.OracleMap(p)
    t = [0.0]
    poses_by_scan = {}

    def pose_provider(msg):
        return poses_by_scan[id(msg)]

    node = MappingNode(dm_width=400, dm_height=400, resolution=0.05, map_update_interval=5.0,
                       pose_provider=pose_provider, clock=lambda: t[0], gate=False)
    try:
        for k, (poses, ranges) in enumerate(batches):
            msg = LaserScan(angle_min=float(synth.LD06_ANGLE_MIN), angle_increment=inc, ranges=ranges[0])
            poses_by_scan[id(msg)] = tuple(poses[0])
            t[0] = 0.7 * k
            node.scan_cb(msg)
            om.integrate(poses, ranges, amin, inc)
        assert node.map_pub.messages == []  # /map comes from the timer, not from scans
        node.timer_cb()  # the map_update_interval tick
        assert node.poll_frontiers(wait=True)  # the GPU frontier pass the tick started
        assert len(node.map_pub.messages) == 1
        grid = node.map_pub.messages[-1]
        assert grid.header.stamp == t[0] and grid.info.map_load_time == t[0]
        assert (grid.info.width, grid.info.height) == (400, 400)
        assert grid.info.resolution == 0.05 and grid.header.frame_id == "map"
        assert grid.data.typecode == "b" and len(grid.data) == 400 * 400
        data = np.frombuffer(grid.data, dtype=np.int8).reshape(grid.info.height, grid.info.width)
        np.testing.assert_array_equal(data, om.state)
        _, _, clusters = om.frontiers()
        fr = node.frontier_pub.messages[-1]
        assert [c.label for c in fr] == clusters["label"].tolist()
        assert [c.x for c in fr] == clusters["cx_m"].tolist()
        from PIL import Image
        img = np.array(Image.open(io.BytesIO(node.map_image_png())))
        np.testing.assert_array_equal(img, np_oracle.map_image(om.state))
    finally:
        node.destroy_node()


def test_gated_stream_integrates_exactly_the_accepted_scans(oracle_lib):
    """A 10 Hz stream (stamps 0.1 s apart) of a robot random-walking 0.1 m /
    <= 0.1 rad per scan: the node integrates only what ScanGate accepts, and
    its map equals the oracle's over exactly those scans."""
    p, batches, amin, inc = _stream(6, 40)
    om = oracle_lib.OracleMap(p)
    ref_gate = ScanGate()
    poses_by_scan = {}
    node = MappingNode(dm_width=400, dm_height=400, map_update_interval=1.0,
                       pose_provider=lambda m: poses_by_scan[id(m)], clock=lambda: 0.0)
    try:
        accepted = 0
        for k, (poses, ranges) in enumerate(batches):
            msg = LaserScan(header=Header(stamp=0.1 * k, frame_id="base_laser"), angle_increment=inc,
                            ranges=ranges[0])
            poses_by_scan[id(msg)] = tuple(poses[0])
            node.scan_cb(msg)
            if ref_gate.accept(0.1 * k, poses[0]):
                om.integrate(poses, ranges, amin, inc)
                accepted += 1
        assert node.scans_seen == 40 and node.scans_integrated == accepted
        assert 0 < accepted < 40
        np.testing.assert_array_equal(node.mapper.state(), om.state)
        np.testing.assert_array_equal(node.mapper.logodds().view(np.uint32), om.L.view(np.uint32))
    finally:
        node.destroy_node()


def test_exploration_goal_topic(oracle_lib):
    """With dm_explore, every map update also publishes the frontier goal the
    host policy (dm.goals.select_goal) picks from the oracle's clusters for
    the robot's latest pose, as a PoseStamped facing the goal."""
    from dm.goals import select_goal

    p, batches, amin, inc = _stream(7, 12)
    om = oracle_lib.OracleMap(p)
    poses_by_scan = {}
    node = MappingNode(dm_width=400, dm_height=400, pose_provider=lambda m: poses_by_scan[id(m)],
                       clock=lambda: 0.0, gate=False, dm_explore=True, dm_goal_min_size=4)
    try:
        for k, (poses, ranges) in enumerate(batches):
            msg = LaserScan(angle_increment=inc, ranges=ranges[0])
            poses_by_scan[id(msg)] = tuple(poses[0])
            node.scan_cb(msg)
            om.integrate(poses, ranges, amin, inc)
        node.publish_map(stamp=1.0)
        while not node.poll_frontiers():  # frontiers_ready() polls the GPU pass, never blocks
            pass
        clusters = om.frontiers(want_mask=False, want_labels=False)[2]
        x, y, _ = batches[-1][0][0]
        exp = select_goal(clusters, (x, y), min_size=4, min_distance=0.3)
        assert exp is not None
        goal = node.goal_pub.messages[-1]
        assert goal.header.frame_id == "map"
        assert (goal.pose.position.x, goal.pose.position.y) == exp[1]
        yaw = yaw_from_quaternion(goal.pose.orientation)
        assert abs(yaw - np.arctan2(exp[1][1] - y, exp[1][0] - x)) < 1e-9
    finally:
        node.destroy_node()


def test_scan_without_pose_is_dropped():
    node = MappingNode(dm_width=128, dm_height=128, pose_provider=lambda m: None)
    try:
        node.scan_cb(LaserScan(angle_increment=0.1, ranges=np.full(10, 1.0, np.float32)))
        assert node.scans_integrated == 0 and node.latest_scan is not None
    finally:
        node.destroy_node()
