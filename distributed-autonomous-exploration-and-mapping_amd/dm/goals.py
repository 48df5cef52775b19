"""Frontier goal selection.

The reference explores reactively (IR/LiDAR subsumption in
server/thymio_project/thymio_project/main.py:123-188) and lists map-based
planning as future work (report.pdf p.5 §VI-2), so there is no reference
behaviour to match.  This is the classic frontier-exploration policy
(Yamauchi 1997): pick the cluster with the best size-over-distance utility,
ignoring clusters below ``min_size`` cells.  Deterministic: ties go to the
smaller label.  Host-side; the cluster list comes from dm_frontiers.
"""
from __future__ import annotations

import numpy as np


def select_goal(clusters: np.ndarray, robot_xy, min_size: int = 8, distance_weight: float = 1.0,
                min_distance: float = 0.0):
    """Return (index, (x, y)) of the chosen frontier cluster, or None.

    utility = size / (1 + distance_weight * distance), distance from the robot
    to the cluster centroid in metres; clusters closer than ``min_distance``
    (e.g. the one the robot is standing in) are skipped."""
    if clusters is None or len(clusters) == 0:
        return None
    size = clusters["size"].astype(np.float64)
    dx = clusters["cx_m"] - float(robot_xy[0])
    dy = clusters["cy_m"] - float(robot_xy[1])
    dist = np.hypot(dx, dy)
    ok = (clusters["size"] >= min_size) & (dist >= min_distance)
    if not ok.any():
        return None
    util = np.where(ok, size / (1.0 + distance_weight * dist), -np.inf)
    best = np.flatnonzero(util == util.max())
    i = int(best[np.argmin(clusters["label"][best])])
    return i, (float(clusters["cx_m"][i]), float(clusters["cy_m"][i]))


def assign_goals(clusters: np.ndarray, robots_xy, min_size: int = 8, distance_weight: float = 1.0):
    """Greedy multi-robot assignment: robots in order each take the best
    cluster not yet taken.  Returns a list of (cluster index, (x, y)) or None
    per robot."""
    taken = np.zeros(len(clusters), bool) if clusters is not None else np.zeros(0, bool)
    out = []
    for xy in robots_xy:
        if clusters is None or len(clusters) == 0 or taken.all():
            out.append(None)
            continue
        free = clusters[~taken]
        idx = np.flatnonzero(~taken)
        g = select_goal(free, xy, min_size, distance_weight)
        if g is None:
            out.append(None)
            continue
        j = int(idx[g[0]])
        taken[j] = True
        out.append((j, g[1]))
    return out
