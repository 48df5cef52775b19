"""Frontier goal selection.

The reference explores reactively (IR/LiDAR subsumption in
server/thymio_project/thymio_project/main.py:123-188) and lists map-based
planning as future work (report.pdf p.5 §VI-2), so there is no reference
behaviour to match.  This is the classic frontier-exploration policy
(Yamauchi 1997): pick the cluster with the best size-over-distance utility,
ignoring clusters below ``min_size`` cells.  Deterministic: ties go to the
smaller label.  The cluster list comes from dm_frontiers; the device version is
dm_assign_goals (csrc/dm_goals.hip).
"""
from __future__ import annotations

import numpy as np


def _utility(clusters: np.ndarray, robot_xy, min_size: int, distance_weight: float,
             min_distance: float) -> np.ndarray:
    """util = size / (1 + w * dist), dist = sqrt(dx*dx + dy*dy) (IEEE double,
    each operation rounded: the device computes the same bits,
    csrc/dm_goals.hip); -inf where the cluster is not eligible."""
    dx = clusters["cx_m"] - float(robot_xy[0])
    dy = clusters["cy_m"] - float(robot_xy[1])
    dist = np.sqrt(dx * dx + dy * dy)
    ok = (clusters["size"] >= min_size) & (dist >= min_distance)
    util = clusters["size"].astype(np.float64) / (1.0 + float(distance_weight) * dist)
    return np.where(ok, util, -np.inf)


def select_goal(clusters: np.ndarray, robot_xy, min_size: int = 8, distance_weight: float = 1.0,
                min_distance: float = 0.0):
    """Return (index, (x, y)) of the chosen frontier cluster, or None.

    utility = size / (1 + distance_weight * distance), distance from the robot
    to the cluster centroid in metres; clusters closer than ``min_distance``
    (e.g. the one the robot is standing in) are skipped."""
    r = assign_goals(clusters, [robot_xy], min_size, distance_weight, min_distance)
    return r[0] if r else None


def assign_goals(clusters: np.ndarray, robots_xy, min_size: int = 8, distance_weight: float = 1.0,
                 min_distance: float = 0.0):
    """Greedy multi-robot assignment: robots in order each take the best
    eligible cluster not yet taken (ties to the smaller label, i.e. the
    smaller index of the label-sorted list).  Returns a list of
    (cluster index, (x, y)) or None per robot.  The device path is
    OccupancyMapper.assign_goals (dm_assign_goals); this is its host
    restatement, used by the tests."""
    if not float(distance_weight) >= 0.0:
        raise ValueError("distance_weight must be >= 0 (dm_assign_goals rejects it too)")
    robots = list(robots_xy)
    if clusters is None or len(clusters) == 0:
        return [None] * len(robots)
    taken = np.zeros(len(clusters), bool)
    out = []
    for xy in robots:
        util = _utility(clusters, xy, min_size, distance_weight, min_distance)
        util[taken] = -np.inf
        m = util.max()
        if not np.isfinite(m):
            out.append(None)
            continue
        best = np.flatnonzero(util == m)
        i = int(best[np.argmin(clusters["label"][best])])  # ties: the smaller label
        taken[i] = True
        out.append((i, (float(clusters["cx_m"][i]), float(clusters["cy_m"][i]))))
    return out
