"""TEST INFRASTRUCTURE: an oracle-backed stand-in with OccupancyMapper's
interface (dm/grid.py), so the ROS drop-in's host logic (dm/ros_node.py:
timer, gating, asynchronous frontier collection) can be tested on CPU.  The
product never uses it; GPU tests drive the same node with libdm."""
import numpy as np

import oracle
from dm.goals import assign_goals
from dm.grid import Frontiers


class OracleMapper:
    def __init__(self, params, pass_latency=0):
        """pass_latency: how many frontiers_ready() polls a frontier pass
        stays 'in flight' (a GPU pass that has not finished yet)."""
        self.om = oracle.OracleMap(params)
        self.params = params
        self.pass_latency = pass_latency
        self._pending = []  # [clusters, polls left]
        self._last = None
        self.begins = 0
        self.closed = False

    def integrate(self, poses, ranges, amin, inc):
        return self.om.integrate(poses, ranges, amin, inc)

    def integrate_scan(self, scan, pose):
        ranges = np.asarray(scan.ranges, dtype=np.float32)[None, :]
        return self.integrate(np.asarray(pose, np.float64)[None, :], ranges,
                              np.float32(scan.angle_min), np.float32(scan.angle_increment))

    def state(self):
        return self.om.state.copy()

    def logodds(self):
        return self.om.L.copy()

    def frontiers(self, want_mask=False, want_labels=False):
        mask, labels, clusters = self.om.frontiers(want_mask=want_mask, want_labels=want_labels)
        self._last = clusters
        return Frontiers(clusters=clusters, mask=mask, labels=labels)

    def frontiers_begin(self):
        if len(self._pending) >= 2:
            raise RuntimeError("two passes in flight")
        self.begins += 1
        self._pending.append([self.om.frontiers(want_mask=False, want_labels=False)[2], self.pass_latency])

    def frontiers_ready(self):
        if not self._pending:
            raise RuntimeError("no pass in flight")
        head = self._pending[0]
        if head[1] > 0:
            head[1] -= 1
            return False
        return True

    def frontiers_end(self):
        clusters, _ = self._pending.pop(0)
        self._last = clusters
        return Frontiers(clusters=clusters)

    def assign_goals(self, robots_xy, min_size=8, distance_weight=1.0, min_distance=0.0):
        return assign_goals(self._last, robots_xy, min_size, distance_weight, min_distance)

    def map_image(self):
        return self.om.map_image()

    def close(self):
        self.closed = True
