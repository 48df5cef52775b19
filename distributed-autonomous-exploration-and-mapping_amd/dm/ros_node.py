"""ROS 2 drop-in for the mapping stage.

The reference gets its ``/map`` from slam_toolbox (server/thymio_project/
launch/pc_server.launch.py:12-19, parameters server/thymio_project/config/
slam_config.yaml) and consumes it in ``ThymioBrain.map_cb``
(server/thymio_project/thymio_project/main.py:46,80-81) and ``get_map_image``
(main.py:241-279).  ``MappingNode`` keeps those topics, message types and
callback signatures:

* subscribes ``/scan`` (``sensor_msgs/LaserScan``; ``scan_cb(self, msg)`` as
  main.py:77-78 — every scan is cached as ``latest_scan``) and looks up the
  laser pose ``map -> base_laser`` through a pose provider (tf2 in ROS; any
  callable in tests);
* gates scans the way the stage it replaces does (``ScanGate``: slam_toolbox's
  ``shouldProcessScan`` front gate, then Karto's ``HasMovedEnough``;
  slam_config.yaml:23,28,37-38) and integrates the accepted ones with libdm on
  the GPU (``dm_integrate``);
* on a timer of ``map_update_interval`` seconds (slam_config.yaml:25) —
  like slam_toolbox's map-publishing loop, whether or not scans were accepted
  in between, so a robot that stopped moving still republishes and a late
  subscriber gets a map — publishes ``/map`` as ``nav_msgs/OccupancyGrid``
  (frame ``map_frame``, ``header.stamp`` and ``info.map_load_time`` = the
  tick's time, resolution and origin from the grid, int8 -1/0/100 row-major,
  ``data`` handed over as an ``array('b')`` built from the device copy's bytes
  — no per-cell Python objects) and starts a frontier pass on the GPU
  (``dm_frontiers_begin``).  The pass is collected without blocking the
  callback thread (``dm_frontiers_poll`` from the scan / timer callbacks) and
  then published: the clusters on ``/frontiers`` (``geometry_msgs/PoseArray``
  of centroids) and, with exploration enabled, the chosen frontier goal on
  ``/goal_pose`` (``geometry_msgs/PoseStamped``, the topic Nav2's navigator
  and RViz's "2D Goal Pose" use) — the map-based replacement of the reactive
  IR/LiDAR policy (main.py:123-188) that the report lists as future work
  (report.pdf p.5 §VI-2);
* with ``dm_devices`` naming several GPUs, the map is one sharded handle
  (``dm_create_sharded``: row bands over those devices, the exchange inside
  libdm) behind the same calls.

All parameters come from the slam_toolbox parameter file the reference
launches (``SlamParams.from_yaml``), plus the fixed grid size this build needs
(slam_toolbox grows its map from the scans' bounding box; a device-resident
grid is allocated once).  Without rclpy (this container and the GPU box) the
same class runs on duck-typed messages: tests drive ``scan_cb`` directly and
read what was "published" from the publisher stubs.
"""
from __future__ import annotations

import array
import io
import math
import time
from dataclasses import dataclass, field, fields

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
class PoseStamped:
    header: Header = field(default_factory=Header)
    pose: Pose = field(default_factory=Pose)


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
    data: array.array = field(default_factory=lambda: array.array("b"))


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


def quaternion_from_yaw(yaw: float) -> Quaternion:
    """main.py:31-36's euler_to_quaternion(0, 0, yaw)."""
    return Quaternion(0.0, 0.0, math.sin(yaw / 2.0), math.cos(yaw / 2.0))


def stamp_seconds(stamp) -> float:
    """builtin_interfaces/Time (sec, nanosec) or plain seconds."""
    if hasattr(stamp, "sec"):
        return float(stamp.sec) + 1e-9 * float(stamp.nanosec)
    return float(stamp)


@dataclass
class SlamParams:
    """The slam_toolbox parameters the mapping stage uses, with the values of
    server/thymio_project/config/slam_config.yaml as defaults (line numbers
    there), plus this build's fixed grid size and exploration switches."""

    map_frame: str = "map"                # :17
    base_frame: str = "base_link"         # :18
    scan_topic: str = "/scan"             # :19
    throttle_scans: int = 1               # :23
    map_update_interval: float = 5.0      # :25
    resolution: float = 0.05              # :26
    max_laser_range: float = 12.0         # :27
    minimum_time_interval: float = 0.5    # :28
    minimum_travel_distance: float = 0.1  # :37
    minimum_travel_heading: float = 0.1   # :38
    # this build (not slam_toolbox parameters)
    dm_width: int = 4096                  # cells; a 204.8 m square at 5 cm
    dm_height: int = 4096
    dm_origin_x: float = float("nan")     # NaN: map centred on the world origin
    dm_origin_y: float = float("nan")
    dm_device: int = 0
    dm_devices: str = ""                  # e.g. "0,1,2,3": one map sharded in row bands over these GPUs
    dm_explore: bool = False              # publish /goal_pose after each map update
    dm_goal_min_size: int = 8
    dm_goal_distance_weight: float = 1.0
    dm_goal_min_distance: float = 0.3

    @classmethod
    def from_dict(cls, d: dict) -> "SlamParams":
        """Known keys of a ros__parameters mapping; others are ignored
        (slam_toolbox's matcher / loop-closure settings are not this stage's)."""
        p = cls()
        for f in fields(cls):
            if f.name in d:
                setattr(p, f.name, type(getattr(p, f.name))(d[f.name]))
        return p

    @classmethod
    def from_yaml(cls, path: str, node_name: str = "slam_toolbox") -> "SlamParams":
        import yaml

        with open(path) as fh:
            doc = yaml.safe_load(fh) or {}
        section = doc.get(node_name, doc.get("/**", {}))
        return cls.from_dict(section.get("ros__parameters", {}))

    def grid_params(self):
        kw = dict(resolution=float(self.resolution), range_max=float(self.max_laser_range))
        if not math.isnan(self.dm_origin_x):
            kw["origin_x"] = float(self.dm_origin_x)
        if not math.isnan(self.dm_origin_y):
            kw["origin_y"] = float(self.dm_origin_y)
        return default_params(int(self.dm_width), int(self.dm_height), **kw)


class ScanGate:
    """Which scans the mapping stage integrates, as slam_toolbox decides it.
    slam_toolbox is not vendored and its version is not pinned (README.md:28
    names the apt package ros-jazzy-slam-toolbox), so this restates its
    published sources (SlamToolbox::shouldProcessScan in
    slam_toolbox_common.cpp, then the Karto mapper's Mapper::HasMovedEnough in
    lib/karto_sdk/src/Mapper.cpp); parity with them is unpinned (SURVEY.md
    §8(c)).  Two layers, in this order:

    1. slam_toolbox's front gate (``shouldProcessScan``; its scan counter counts
       every scan offered, the first included):
       * the first scan is always processed;
       * ``throttle_scans``: dropped unless counter % throttle_scans == 0;
       * ``minimum_time_interval``: dropped if closer in time than this to the
         last scan that passed this gate;
       * dropped if it moved less than ``0.8 * minimum_travel_distance²``
         (squared, "within 10 % for correction error") from that scan's
         pose, or while the counter is below 5 (warm-up).  A robot turning
         in place is therefore never integrated, whatever it turned.
    2. Karto's ``HasMovedEnough`` against the last *processed* scan: processed
       if ``minimum_time_interval`` has passed, or the laser turned by
       ``minimum_travel_heading`` (normalised angle), or moved
       ``minimum_travel_distance`` (squared, less Karto's KT_TOLERANCE 1e-9).
       After layer 1 the time test already holds, so this layer only matters
       when the thresholds are configured differently for the two.

    The values of the reference's slam_config.yaml (lines 23, 28, 37, 38) are
    ``SlamParams``' defaults."""

    KT_TOLERANCE = 1e-9

    def __init__(self, throttle_scans=1, minimum_time_interval=0.5, minimum_travel_distance=0.1,
                 minimum_travel_heading=0.1):
        self.throttle = max(1, int(throttle_scans))
        self.min_dt = float(minimum_time_interval)
        self.min_d2 = float(minimum_travel_distance) ** 2
        self.min_heading = float(minimum_travel_heading)
        self.counter = 0
        self.front = None  # (stamp, x, y) of the last scan past slam_toolbox's gate
        self.last = None   # (stamp, x, y, yaw) of the last processed scan (Karto)

    @classmethod
    def from_params(cls, p: SlamParams) -> "ScanGate":
        return cls(p.throttle_scans, p.minimum_time_interval, p.minimum_travel_distance,
                   p.minimum_travel_heading)

    def _front(self, stamp: float, x: float, y: float) -> bool:
        self.counter += 1
        if self.front is None:
            self.front = (stamp, x, y)
            return True
        if self.counter % self.throttle != 0:
            return False
        t0, x0, y0 = self.front
        if stamp - t0 < self.min_dt:
            return False
        if (x - x0) ** 2 + (y - y0) ** 2 < 0.8 * self.min_d2 or self.counter < 5:
            return False
        self.front = (stamp, x, y)
        return True

    def _moved_enough(self, stamp: float, x: float, y: float, yaw: float) -> bool:
        if self.last is None:
            return True
        t0, x0, y0, yaw0 = self.last
        if stamp - t0 >= self.min_dt:
            return True
        if abs(math.remainder(yaw - yaw0, 2.0 * math.pi)) >= self.min_heading:
            return True
        return (x - x0) ** 2 + (y - y0) ** 2 >= self.min_d2 - self.KT_TOLERANCE

    def accept(self, stamp: float, pose) -> bool:
        x, y, yaw = (float(v) for v in pose)
        if not self._front(stamp, x, y):
            return False
        if not self._moved_enough(stamp, x, y, yaw):
            return False
        self.last = (stamp, x, y, yaw)
        return True


def parse_devices(spec) -> list[int]:
    """dm_devices: "0,1,2,3" (or a list) -> [0, 1, 2, 3]; "" -> []."""
    if isinstance(spec, (list, tuple)):
        return [int(d) for d in spec]
    return [int(d) for d in str(spec).replace(" ", "").split(",") if d != ""]


class MappingNode:
    """GPU mapping stage: /scan (+TF) -> /map + /frontiers (+ /goal_pose).

    Callbacks (all non-blocking on the GPU except the /map readback itself):
    ``scan_cb`` per LaserScan, ``timer_cb`` every ``map_update_interval``
    seconds, ``poll_frontiers`` whenever convenient (the rclpy wiring in
    ``main`` runs it on a short timer)."""

    def __init__(self, params: SlamParams | None = None, pose_provider=None, map_publisher=None,
                 frontier_publisher=None, goal_publisher=None, clock=time.monotonic, gate: bool = True,
                 mapper=None, **overrides):
        """`overrides` set SlamParams fields (tests: dm_width=..., ...).
        `mapper`: an object with OccupancyMapper's interface to use instead of
        creating one (tests inject CPU stand-ins)."""
        p = params or SlamParams()
        for k, v in overrides.items():
            if not hasattr(p, k):
                raise TypeError(f"unknown parameter {k!r}")
            setattr(p, k, v)
        self.slam = p
        self.params = p.grid_params()
        if mapper is None:
            devices = parse_devices(p.dm_devices)
            if len(devices) > 1:
                mapper = OccupancyMapper(self.params, devices=devices)
            else:
                mapper = OccupancyMapper(self.params, device=devices[0] if devices else int(p.dm_device))
        self.mapper = mapper
        self.map_update_interval = float(p.map_update_interval)
        self.gate = ScanGate.from_params(p) if gate else None
        self.pose_provider = pose_provider
        self.map_pub = map_publisher or ListPublisher("/map")
        self.frontier_pub = frontier_publisher or ListPublisher("/frontiers")
        self.goal_pub = goal_publisher or ListPublisher("/goal_pose")
        self.clock = clock
        self._last_publish = -math.inf
        self._pass_stamp = None  # stamp of the frontier pass in flight (None: none)
        self.latest_scan = None
        self.latest_pose = None
        self.scans_seen = 0
        self.scans_integrated = 0
        self.updates = 0
        self.last_frontiers = None

    # main.py:77-78 keeps the signature scan_cb(self, msg)
    def scan_cb(self, msg):
        self.latest_scan = msg
        self.scans_seen += 1
        self.poll_frontiers()
        pose = self.pose_provider(msg) if self.pose_provider is not None else None
        if pose is None:
            return  # no transform yet: slam_toolbox drops such scans too
        self.latest_pose = tuple(float(v) for v in pose)
        stamp = stamp_seconds(msg.header.stamp)
        if self.gate is not None and not self.gate.accept(stamp, pose):
            return
        u, _ = self.mapper.integrate_scan(msg, pose)
        self.updates += u
        self.scans_integrated += 1

    def timer_cb(self):
        """The map_update_interval timer: publish /map and start a frontier
        pass, independent of scan gating.  Before the first integrated scan
        there is no map (slam_toolbox has no grid before its first processed
        scan either)."""
        self.poll_frontiers()
        if self.scans_integrated == 0:
            return
        self.publish_map(stamp=self.clock())

    def occupancy_grid(self, stamp: float = 0.0):
        st = self.mapper.state()
        p = self.params
        data = array.array("b")
        data.frombytes(st.tobytes())  # one copy of the device readback, no per-cell objects
        if HAVE_ROS:  # pragma: no cover
            msg = _RosOccupancyGrid()
            msg.header.frame_id = self.slam.map_frame
            msg.header.stamp = time_msg(stamp)
            msg.info.map_load_time = time_msg(stamp)
            msg.info.resolution = float(p.resolution)
            msg.info.width = int(p.width)
            msg.info.height = int(p.height)
            msg.info.origin.position.x = float(p.origin_x)
            msg.info.origin.position.y = float(p.origin_y)
            msg.info.origin.orientation.w = 1.0
            msg.data = data
            return msg
        return OccupancyGrid(
            header=Header(stamp=stamp, frame_id=self.slam.map_frame),
            info=MapMetaData(map_load_time=stamp, resolution=float(p.resolution), width=int(p.width),
                             height=int(p.height),
                             origin=Pose(position=Point(float(p.origin_x), float(p.origin_y), 0.0))),
            data=data)

    def frontier_clusters(self) -> list:
        """Synchronous frontier extraction of the map as it is now."""
        fr = self.mapper.frontiers()
        self.last_frontiers = fr.clusters
        return self._cluster_msgs(fr.clusters)

    @staticmethod
    def _cluster_msgs(clusters) -> list:
        return [FrontierCluster(int(c["label"]), int(c["size"]), float(c["cx_m"]), float(c["cy_m"]))
                for c in clusters]

    def choose_goal(self, stamp: float | None = None):
        """The frontier goal for the robot at its latest pose, chosen on the
        device over the last published frontier clusters (dm_assign_goals;
        policy: dm.goals): PoseStamped in the map frame facing the goal, or
        None."""
        if self.last_frontiers is None or self.latest_pose is None:
            return None
        x, y, _ = self.latest_pose
        s = self.slam
        g = self.mapper.assign_goals([(x, y)], min_size=s.dm_goal_min_size,
                                     distance_weight=s.dm_goal_distance_weight,
                                     min_distance=s.dm_goal_min_distance)[0]
        if g is None:
            return None
        gx, gy = g[1]
        msg = PoseStamped(header=Header(stamp=self._last_publish if stamp is None else stamp,
                                        frame_id=s.map_frame))
        msg.pose.position = Point(gx, gy, 0.0)
        msg.pose.orientation = quaternion_from_yaw(math.atan2(gy - y, gx - x))
        return msg

    def publish_map(self, stamp: float = 0.0):
        """Publish /map now and start the frontier pass of this map (its
        clusters are published by poll_frontiers once the GPU is done)."""
        self._last_publish = stamp
        self.map_pub.publish(self.occupancy_grid(stamp))
        if self._pass_stamp is not None:
            self.poll_frontiers(wait=True)  # the previous tick's pass (long done by now)
        self.mapper.frontiers_begin()
        self._pass_stamp = stamp

    def poll_frontiers(self, wait: bool = False) -> bool:
        """Publish the frontier pass in flight if the GPU has finished it
        (never blocks unless `wait`).  Returns True if it published."""
        if self._pass_stamp is None:
            return False
        if not wait and not self.mapper.frontiers_ready():
            return False
        stamp, self._pass_stamp = self._pass_stamp, None
        fr = self.mapper.frontiers_end()
        clusters = fr.clusters if fr is not None else self.mapper.frontiers().clusters  # overflowed: rerun
        self.last_frontiers = clusters
        self.frontier_pub.publish(self._cluster_msgs(clusters))
        if self.slam.dm_explore:
            goal = self.choose_goal(stamp)
            if goal is not None:
                self.goal_pub.publish(goal)
        return True

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


def time_msg(t: float):  # pragma: no cover - needs ROS 2
    """Seconds -> builtin_interfaces/Time."""
    from builtin_interfaces.msg import Time

    sec = int(math.floor(t))
    return Time(sec=sec, nanosec=int(round((t - sec) * 1e9)) % 1_000_000_000)


def main(args=None):  # pragma: no cover - needs ROS 2
    """ros2 run entry point: wires MappingNode into rclpy (tf2 pose lookup).
    Parameters are declared with SlamParams' defaults, so the node takes the
    reference's slam_config.yaml (launch/dm_pc_server.launch.py passes it)."""
    if not HAVE_ROS:
        raise SystemExit("rclpy is not available; MappingNode can still be used as a library")
    import rclpy
    from rclpy.node import Node
    from sensor_msgs.msg import LaserScan as RosLaserScan
    from nav_msgs.msg import OccupancyGrid as RosGrid
    from geometry_msgs.msg import PoseArray, Pose as RosPose, PoseStamped as RosPoseStamped
    import tf2_ros

    rclpy.init(args=args)
    node = Node("dm_mapper")
    defaults = SlamParams()
    values = {}
    for f in fields(SlamParams):
        node.declare_parameter(f.name, getattr(defaults, f.name))
        values[f.name] = node.get_parameter(f.name).value
    sp = SlamParams.from_dict(values)
    tf_buffer = tf2_ros.Buffer()
    tf2_ros.TransformListener(tf_buffer, node)

    def lookup(msg):
        try:
            t = tf_buffer.lookup_transform(sp.map_frame, msg.header.frame_id, msg.header.stamp)
        except Exception:
            return None
        tr = t.transform
        return (tr.translation.x, tr.translation.y, yaw_from_quaternion(tr.rotation))

    map_pub = node.create_publisher(RosGrid, "/map", 10)
    fr_pub = node.create_publisher(PoseArray, "/frontiers", 10)
    goal_pub = node.create_publisher(RosPoseStamped, "/goal_pose", 10)

    class _FrontierAdapter:
        def publish(self, clusters):
            pa = PoseArray()
            pa.header.frame_id = sp.map_frame
            pa.header.stamp = node.get_clock().now().to_msg()
            for c in clusters:
                ps = RosPose()
                ps.position.x, ps.position.y = c.x, c.y
                pa.poses.append(ps)
            fr_pub.publish(pa)

    class _GoalAdapter:
        def publish(self, g):
            m = RosPoseStamped()
            m.header.frame_id = g.header.frame_id
            m.header.stamp = node.get_clock().now().to_msg()
            m.pose.position.x, m.pose.position.y = g.pose.position.x, g.pose.position.y
            q = g.pose.orientation
            m.pose.orientation.z, m.pose.orientation.w = q.z, q.w
            goal_pub.publish(m)

    mn = MappingNode(sp, pose_provider=lookup, map_publisher=map_pub, frontier_publisher=_FrontierAdapter(),
                     goal_publisher=_GoalAdapter(), clock=lambda: node.get_clock().now().nanoseconds * 1e-9)
    node.create_subscription(RosLaserScan, sp.scan_topic, mn.scan_cb, 10)
    # slam_toolbox publishes the map on its own period, not per scan
    node.create_timer(sp.map_update_interval, mn.timer_cb)
    node.create_timer(0.01, mn.poll_frontiers)  # frontiers go out as soon as the GPU pass is done
    try:
        rclpy.spin(node)
    finally:
        mn.destroy_node()
        node.destroy_node()
        rclpy.shutdown()


if __name__ == "__main__":  # pragma: no cover
    main()
