"""ROS 2 drop-in for the mapping stage.

The reference gets its ``/map`` from slam_toolbox (server/thymio_project/
launch/pc_server.launch.py:12-19) and consumes it in ``ThymioBrain.map_cb``
(server/thymio_project/thymio_project/main.py:46,80-81) and ``get_map_image``
(main.py:241-279).  ``MappingNode`` keeps those topics, message types and
callback signatures:

* subscribes ``/scan`` (``sensor_msgs/LaserScan``; ``scan_cb(self, msg)`` as
  main.py:77-78) and looks up the laser pose ``map -> base_laser`` through a
  pose provider (tf2 in ROS; any callable in tests);
* integrates each scan with libdm on the GPU (``dm_integrate``);
* every ``map_update_interval`` seconds (slam_config.yaml:25) publishes
  ``/map`` as ``nav_msgs/OccupancyGrid`` (frame ``map``, resolution and
  origin from the grid, int8 -1/0/100 row-major) and the frontier clusters on
  ``/frontiers`` (``geometry_msgs/PoseArray`` of centroids when ROS is
  present, plain records otherwise).

Without rclpy (this container and the GPU box) the same class runs on
duck-typed messages: tests drive ``scan_cb`` directly and read what was
"published" from the publisher stubs.
"""
from __future__ import annotations

import io
import math
import time
from dataclasses import dataclass, field

import numpy as np

from .grid import OccupancyMapper, default_params

try:  # pragma: no cover - ROS is absent in CI and on the GPU box
    import rclpy  # noqa: F401
    from nav_msgs.msg import OccupancyGrid as _RosOccupancyGrid
    HAVE_ROS = True
except Exception:  # ModuleNotFoundError or a broken ROS env
    HAVE_ROS = False


# -- duck-typed message stand-ins (same field names as the ROS messages) -------
@dataclass
class Header:
    stamp: float = 0.0
    frame_id: str = "map"


@dataclass
class Point:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class Quaternion:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0
    w: float = 1.0


@dataclass
class Pose:
    position: Point = field(default_factory=Point)
    orientation: Quaternion = field(default_factory=Quaternion)


@dataclass
class MapMetaData:
    map_load_time: float = 0.0
    resolution: float = 0.05
    width: int = 0
    height: int = 0
    origin: Pose = field(default_factory=Pose)


@dataclass
class OccupancyGrid:
    header: Header = field(default_factory=Header)
    info: MapMetaData = field(default_factory=MapMetaData)
    data: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int8))


@dataclass
class LaserScan:
    header: Header = field(default_factory=lambda: Header(frame_id="base_laser"))
    angle_min: float = 0.0
    angle_max: float = 6.2831855
    angle_increment: float = 0.0
    time_increment: float = 0.0
    scan_time: float = 0.1
    range_min: float = 0.02
    range_max: float = 25.0
    ranges: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))
    intensities: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))


@dataclass
class FrontierCluster:
    label: int
    size: int
    x: float
    y: float


class ListPublisher:
    """Publisher stub: keeps what was published."""

    def __init__(self, topic: str):
        self.topic = topic
        self.messages: list = []

    def publish(self, msg):
        self.messages.append(msg)


def yaw_from_quaternion(q) -> float:
    """Planar yaw of a quaternion (inverse of main.py:31-36 for roll=pitch=0)."""
    return math.atan2(2.0 * (q.w * q.z + q.x * q.y), 1.0 - 2.0 * (q.y * q.y + q.z * q.z))


class MappingNode:
    """GPU mapping stage: /scan (+TF) -> /map + /frontiers."""

    def __init__(self, width: int = 4096, height: int = 4096, resolution: float = 0.05,
                 origin=None, map_update_interval: float = 5.0, pose_provider=None,
                 map_publisher=None, frontier_publisher=None, device: int = 0,
                 clock=time.monotonic, **param_overrides):
        kw = dict(resolution=resolution)
        if origin is not None:
            kw["origin_x"], kw["origin_y"] = origin
        kw.update(param_overrides)
        self.params = default_params(width, height, **kw)
        self.mapper = OccupancyMapper(self.params, device=device)
        self.map_update_interval = float(map_update_interval)
        self.pose_provider = pose_provider
        self.map_pub = map_publisher or ListPublisher("/map")
        self.frontier_pub = frontier_publisher or ListPublisher("/frontiers")
        self.clock = clock
        self._last_publish = -math.inf
        self.latest_scan = None
        self.scans_integrated = 0
        self.updates = 0

    # main.py:77-78 keeps the signature scan_cb(self, msg)
    def scan_cb(self, msg):
        self.latest_scan = msg
        pose = self.pose_provider(msg) if self.pose_provider is not None else None
        if pose is None:
            return  # no transform yet: slam_toolbox drops such scans too
        u, _ = self.mapper.integrate_scan(msg, pose)
        self.updates += u
        self.scans_integrated += 1
        now = self.clock()
        if now - self._last_publish >= self.map_update_interval:
            self.publish_map(stamp=now)

    def occupancy_grid(self, stamp: float = 0.0):
        st = self.mapper.state()
        p = self.params
        if HAVE_ROS:  # pragma: no cover
            msg = _RosOccupancyGrid()
            msg.header.frame_id = "map"
            msg.info.resolution = float(p.resolution)
            msg.info.width = int(p.width)
            msg.info.height = int(p.height)
            msg.info.origin.position.x = float(p.origin_x)
            msg.info.origin.position.y = float(p.origin_y)
            msg.info.origin.orientation.w = 1.0
            msg.data = st.reshape(-1).tolist()
            return msg
        return OccupancyGrid(
            header=Header(stamp=stamp, frame_id="map"),
            info=MapMetaData(map_load_time=stamp, resolution=float(p.resolution), width=int(p.width),
                             height=int(p.height),
                             origin=Pose(position=Point(float(p.origin_x), float(p.origin_y), 0.0))),
            data=st.reshape(-1))

    def frontier_clusters(self) -> list:
        fr = self.mapper.frontiers()
        return [FrontierCluster(int(c["label"]), int(c["size"]), float(c["cx_m"]), float(c["cy_m"]))
                for c in fr.clusters]

    def publish_map(self, stamp: float = 0.0):
        self._last_publish = stamp
        self.map_pub.publish(self.occupancy_grid(stamp))
        self.frontier_pub.publish(self.frontier_clusters())

    def map_image_png(self) -> bytes:
        """What get_map_image serves (main.py:256-273), rendered on the GPU
        (dm_map_image) and PNG-encoded with PIL."""
        from PIL import Image

        img = Image.fromarray(self.mapper.map_image(), mode="L")
        buf = io.BytesIO()
        img.save(buf, "PNG")
        return buf.getvalue()

    def destroy_node(self):
        self.mapper.close()


def main(args=None):  # pragma: no cover - needs ROS 2
    """ros2 run entry point: wires MappingNode into rclpy (tf2 pose lookup)."""
    if not HAVE_ROS:
        raise SystemExit("rclpy is not available; MappingNode can still be used as a library")
    import rclpy
    from rclpy.node import Node
    from sensor_msgs.msg import LaserScan as RosLaserScan
    from nav_msgs.msg import OccupancyGrid as RosGrid
    from geometry_msgs.msg import PoseArray, Pose as RosPose
    import tf2_ros

    rclpy.init(args=args)
    node = Node("dm_mapper")
    tf_buffer = tf2_ros.Buffer()
    tf2_ros.TransformListener(tf_buffer, node)

    def lookup(msg):
        try:
            t = tf_buffer.lookup_transform("map", msg.header.frame_id, msg.header.stamp)
        except Exception:
            return None
        tr = t.transform
        return (tr.translation.x, tr.translation.y, yaw_from_quaternion(tr.rotation))

    map_pub = node.create_publisher(RosGrid, "/map", 10)
    fr_pub = node.create_publisher(PoseArray, "/frontiers", 10)

    class _FrontierAdapter:
        def publish(self, clusters):
            pa = PoseArray()
            pa.header.frame_id = "map"
            for c in clusters:
                ps = RosPose()
                ps.position.x, ps.position.y = c.x, c.y
                pa.poses.append(ps)
            fr_pub.publish(pa)

    mn = MappingNode(pose_provider=lookup, map_publisher=map_pub, frontier_publisher=_FrontierAdapter(),
                     clock=lambda: node.get_clock().now().nanoseconds * 1e-9)
    node.create_subscription(RosLaserScan, "/scan", mn.scan_cb, 10)
    try:
        rclpy.spin(node)
    finally:
        mn.destroy_node()
        node.destroy_node()
        rclpy.shutdown()


if __name__ == "__main__":  # pragma: no cover
    main()
