"""dm — MI355X-native occupancy mapping + exploration frontiers.

Drop-in for the mapping hot path of rafaelgmv/Distributed-Autonomous-
Exploration-and-Mapping (BASELINE.json north_star): LD06 ``LaserScan`` ->
log-odds ray-cast integration into a ``nav_msgs/OccupancyGrid`` -> frontier
mask, 8-connected CCL labels, cluster centroids and sizes.  The compute runs
in hand-written HIP kernels for gfx950 behind the C-ABI in include/dm.h
(libdm.so, loaded with ctypes); this package is the host side.
"""
from ._ffi import (CLUSTER_DTYPE, DM_TILE, DmCluster, DmError, DmParams, exported_symbols,
                   load_library)
from .grid import Frontiers, OccupancyMapper, atomic_peak, default_params, params_from_dict

__all__ = [
    "CLUSTER_DTYPE",
    "DM_TILE",
    "DmCluster",
    "DmError",
    "DmParams",
    "Frontiers",
    "OccupancyMapper",
    "atomic_peak",
    "default_params",
    "exported_symbols",
    "load_library",
    "params_from_dict",
]
