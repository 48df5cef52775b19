"""GPU: the ROS 2 drop-in (dm/ros_node.py) driven with duck-typed LaserScan
messages, as the LD06 driver publishes them, produces the /map the oracle
produces, and the /map-image pixels get_map_image would serve
(server/thymio_project/thymio_project/main.py:241-279)."""
import io

import numpy as np
import pytest

import cases
import np_oracle
from dm import synth
from dm.ros_node import LaserScan, MappingNode

pytestmark = pytest.mark.gpu


def test_mapping_node_publishes_oracle_map(oracle_lib):
    p, batches, amin, inc = cases.world_case(5, 400, 400, 0.05, 1, 450, 15)
    om = oracle_lib.OracleMap(p)
    t = [0.0]
    poses_by_scan = {}

    def pose_provider(msg):
        return poses_by_scan[id(msg)]

    node = MappingNode(width=400, height=400, resolution=0.05, map_update_interval=5.0,
                       pose_provider=pose_provider, clock=lambda: t[0])
    try:
        for k, (poses, ranges) in enumerate(batches):
            msg = LaserScan(angle_min=float(synth.LD06_ANGLE_MIN), angle_increment=inc,
                            ranges=ranges[0])
            poses_by_scan[id(msg)] = tuple(poses[0])
            t[0] = 0.7 * k
            node.scan_cb(msg)
            om.integrate(poses, ranges, amin, inc)
        node.publish_map(stamp=t[0])
        assert len(node.map_pub.messages) >= 2  # interval-driven + explicit
        grid = node.map_pub.messages[-1]
        assert (grid.info.width, grid.info.height) == (400, 400)
        assert grid.info.resolution == 0.05 and grid.header.frame_id == "map"
        data = np.array(grid.data, dtype=np.int8).reshape(grid.info.height, grid.info.width)
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


def test_scan_without_pose_is_dropped():
    node = MappingNode(width=128, height=128, pose_provider=lambda m: None)
    try:
        node.scan_cb(LaserScan(angle_increment=0.1, ranges=np.full(10, 1.0, np.float32)))
        assert node.scans_integrated == 0 and node.latest_scan is not None
    finally:
        node.destroy_node()
