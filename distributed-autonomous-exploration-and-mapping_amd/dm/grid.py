"""Python host side of the hot path: a locked handle over libdm.so.

``OccupancyMapper`` is what a ROS 2 node calls (dm/ros_node.py): it takes the
same data a ``sensor_msgs/LaserScan`` carries (ranges, angle_min,
angle_increment) plus the laser pose, and yields what ``nav_msgs/OccupancyGrid``
carries (int8 row-major -1/0/100, origin bottom-left), i.e. the data
``ThymioBrain.map_cb`` caches and ``get_map_image`` renders
(server/thymio_project/thymio_project/main.py:80-81, 241-279).

Threading: the reference writes ``latest_map`` on the
rclpy spin thread and reads it on the Flask thread (main.py:80-81 vs
:244-256); a libdm handle is not thread-safe, so every call here holds a
per-handle lock and every array returned is a fresh copy.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _ffi
from ._ffi import CLUSTER_DTYPE, DmError, DmParams, check, load_library


def default_params(width: int, height: int, **overrides) -> DmParams:
    """dm_default_params + keyword overrides (resolution 0.05 and max range
    12.0 from slam_config.yaml:26-27)."""
    lib = load_library()
    p = DmParams()
    check(lib.dm_default_params(ctypes.byref(p), int(width), int(height)))
    res_given = "resolution" in overrides
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise DmError(_ffi.DM_ERR_INVALID_ARG, f"unknown parameter {k!r}")
        setattr(p, k, v)
    if res_given and "origin_x" not in overrides:
        p.origin_x = -0.5 * p.width * p.resolution
    if res_given and "origin_y" not in overrides:
        p.origin_y = -0.5 * p.height * p.resolution
    return p


def params_from_dict(d: dict) -> DmParams:
    p = DmParams()
    for k, v in d.items():
        setattr(p, k, v)
    return p


def atomic_peak(device: int = 0) -> dict:
    """Measured uncontended atomic throughput of the device (dm_atomic_peak):
    LDS ds_add_u32 and global no-return atomicAdd u32, operations per second."""
    lib = load_library()
    out = (ctypes.c_double * 2)()
    n = ctypes.c_int32(0)
    check(lib.dm_atomic_peak(int(device), out, 2, ctypes.byref(n)))
    return {"lds_add_u32_per_s": float(out[0]), "global_add_u32_per_s": float(out[1])}


@dataclass
class Frontiers:
    """Result of one frontier extraction."""

    clusters: np.ndarray            # structured CLUSTER_DTYPE, sorted by label
    mask: np.ndarray | None = None  # uint8 [rows, W]
    labels: np.ndarray | None = None  # int64 [rows, W], -1 off-frontier

    def __len__(self) -> int:
        return int(self.clusters.shape[0])


def _vp(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OccupancyMapper:
    """One device-resident map (or one row band of a sharded map)."""

    def __init__(self, params: DmParams, device: int = 0, devices=None):
        """`devices`: a list of HIP devices to shard the map over in row bands
        (dm_create_sharded; a device may repeat); the handle then takes the
        same calls, with results identical to one handle."""
        self._lib = load_library()
        self._lock = threading.RLock()
        self._h = ctypes.c_void_p()
        if devices is not None:
            devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
            check(self._lib.dm_create_sharded(ctypes.byref(self._h), ctypes.byref(params), len(devices), devs))
            device = int(devices[0])
        else:
            check(self._lib.dm_create(ctypes.byref(self._h), ctypes.byref(params), int(device)))
        self.devices = list(devices) if devices is not None else [int(device)]
        out = DmParams()
        check(self._lib.dm_get_params(self._h, ctypes.byref(out)))
        self.params = out
        self.device = device
        self.width = int(out.width)
        self.rows = int(out.band_rows)
        self.row0 = int(out.band_row0)
        self._cap = 1 << 12  # cluster records per frontiers() buffer (grown on demand)
        self.last_incomplete = None  # dm_last_error() of the last pass that returned no result

    # -- lifetime ---------------------------------------------------------
    def close(self):
        with self._lock:
            if self._h:
                self._lib.dm_destroy(self._h)
                self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _handle(self):
        if not self._h:
            raise DmError(_ffi.DM_ERR_STATE, "mapper is closed")
        return self._h

    # -- integration ------------------------------------------------------
    def integrate(self, poses, ranges, angle_min, angle_increment):
        """Integrate S scans: poses [S,3] (x, y, yaw), ranges [S,N] float32.
        Returns (updates U, touched cells T)."""
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        ranges = np.ascontiguousarray(ranges, dtype=np.float32)
        if ranges.ndim != 2:
            ranges = ranges.reshape(poses.shape[0], -1)
        S, N = ranges.shape
        U = ctypes.c_uint64(0)
        T = ctypes.c_uint64(0)
        with self._lock:
            check(self._lib.dm_integrate(self._handle(), S, _vp(poses), N, _vp(ranges),
                                         float(angle_min), float(angle_increment),
                                         ctypes.byref(U), ctypes.byref(T)))
        return int(U.value), int(T.value)

    def integrate_scan(self, scan, pose):
        """One LaserScan-like message (attributes ranges, angle_min,
        angle_increment) at laser pose (x, y, yaw) in the map frame."""
        ranges = np.asarray(scan.ranges, dtype=np.float32)[None, :]
        return self.integrate(np.asarray(pose, np.float64)[None, :], ranges,
                              np.float32(scan.angle_min), np.float32(scan.angle_increment))

    def integrate_async(self, poses, ranges_ptr: int, S: int, N: int, angle_min, angle_increment):
        """dm_integrate_async: poses [S,3] (read now), ranges a host pointer to
        float32 [S,N] — pinned memory for a truly asynchronous upload — that
        must stay valid until the second integrate_async call after this one
        (or synchronize()).  Returns at once; U/T via last_counts()."""
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        if poses.shape[0] != S:
            raise DmError(_ffi.DM_ERR_SHAPE, f"poses has {poses.shape[0]} rows, S = {S}")
        with self._lock:
            check(self._lib.dm_integrate_async(self._handle(), int(S), _vp(poses), int(N),
                                               ctypes.c_void_p(ranges_ptr), float(angle_min),
                                               float(angle_increment)))

    def integrate_device(self, d_pose4_ptr: int, S: int, d_ranges_ptr: int, N: int,
                         angle_min, angle_increment):
        """Asynchronous integrate from device pointers (pose4 = x, y, cos yaw,
        sin yaw as float64 [S,4]; ranges float32 [S,N])."""
        with self._lock:
            check(self._lib.dm_integrate_device(self._handle(), int(S), ctypes.c_void_p(d_pose4_ptr),
                                                int(N), ctypes.c_void_p(d_ranges_ptr),
                                                float(angle_min), float(angle_increment)))

    def last_counts(self):
        U = ctypes.c_uint64(0)
        T = ctypes.c_uint64(0)
        with self._lock:
            check(self._lib.dm_last_counts(self._handle(), ctypes.byref(U), ctypes.byref(T)))
        return int(U.value), int(T.value)

    STAT_NAMES = ("updates", "touched", "touched_heavy", "pieces", "active_tiles", "work_items",
                  "heavy_tiles", "frontier_tiles", "frontier_slots", "frontier_clusters", "sparse_items")

    def last_stats(self) -> dict:
        """Diagnostics of the most recent integrate call (dm_last_stats)."""
        k = len(self.STAT_NAMES)
        out = (ctypes.c_uint64 * k)()
        n = ctypes.c_int32(0)
        with self._lock:
            check(self._lib.dm_last_stats(self._handle(), out, k, ctypes.byref(n)))
        return {k: int(out[i]) for i, k in enumerate(self.STAT_NAMES)}

    def ld06_to_scans(self, points, offsets, n_beams: int, laser_scan_dir: bool = True,
                      want_intensities: bool = False):
        """LD06 PointData -> LaserScan ranges on the GPU, as the driver's
        ToLaserscanMessagePublish (dm_ld06_to_scans).  points: structured
        array of LD06_POINT_DTYPE; offsets: int64 [S+1].  Returns ranges
        float32 [S, N] (and intensities)."""
        pts = np.ascontiguousarray(points, dtype=np.dtype(_ffi.LD06_POINT_DTYPE))
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        S = off.shape[0] - 1
        ranges = np.empty((S, n_beams), np.float32)
        inten = np.empty((S, n_beams), np.float32) if want_intensities else None
        with self._lock:
            check(self._lib.dm_ld06_to_scans(self._handle(), S, _vp(pts), _vp(off), int(n_beams),
                                             1 if laser_scan_dir else 0, _vp(ranges), _vp(inten)))
        return (ranges, inten) if want_intensities else ranges

    # -- map access -------------------------------------------------------
    def state(self) -> np.ndarray:
        out = np.empty((self.rows, self.width), np.int8)
        with self._lock:
            check(self._lib.dm_get_state(self._handle(), _vp(out)))
        return out

    def logodds(self) -> np.ndarray:
        out = np.empty((self.rows, self.width), np.float32)
        with self._lock:
            check(self._lib.dm_get_logodds(self._handle(), _vp(out)))
        return out

    def set_logodds(self, L):
        L = np.ascontiguousarray(L, dtype=np.float32).reshape(self.rows, self.width)
        with self._lock:
            check(self._lib.dm_set_logodds(self._handle(), _vp(L)))

    def set_state(self, st):
        st = np.ascontiguousarray(st, dtype=np.int8).reshape(self.rows, self.width)
        with self._lock:
            check(self._lib.dm_set_state(self._handle(), _vp(st)))

    def reset(self):
        with self._lock:
            check(self._lib.dm_reset(self._handle()))

    def map_image(self) -> np.ndarray:
        """get_map_image's grayscale pixels (main.py:256-266), rendered on
        the GPU: uint8 [rows, W], already flipped."""
        out = np.empty((self.rows, self.width), np.uint8)
        with self._lock:
            check(self._lib.dm_map_image(self._handle(), _vp(out)))
        return out

    def assign_goals(self, robots_xy, min_size: int = 8, distance_weight: float = 1.0,
                     min_distance: float = 0.0):
        """Frontier goals on the device (dm_assign_goals) over the clusters of
        the last collected frontier result: per robot, in order, (index into
        that result's cluster list, (x, y)) or None.  Same policy as
        dm.goals.assign_goals (the host restatement the tests compare with)."""
        xy = np.ascontiguousarray(np.asarray(robots_xy, np.float64).reshape(-1, 2))
        R = xy.shape[0]
        idx = np.empty(R, np.int64)
        out = np.empty((R, 2), np.float64)
        with self._lock:
            check(self._lib.dm_assign_goals(self._handle(), _vp(xy), R, int(min_size), float(distance_weight),
                                            float(min_distance), _vp(idx), _vp(out)))
        return [(int(i), (float(p[0]), float(p[1]))) if i >= 0 else None for i, p in zip(idx, out)]

    # -- frontiers --------------------------------------------------------
    def frontiers(self, want_mask=False, want_labels=False, cap=None) -> Frontiers:
        """Frontier mask / labels (optional dense copies) and the cluster
        list sorted by label.  The cluster buffer is reused across calls and
        grown when the library reports more clusters than it holds."""
        mask = np.empty((self.rows, self.width), np.uint8) if want_mask else None
        labels = np.empty((self.rows, self.width), np.int64) if want_labels else None
        n = ctypes.c_int64(0)
        with self._lock:
            if cap is not None and self._cap < cap:
                self._cap = max(1, int(cap))
            while True:
                # a fresh array per call: the library writes the records straight
                # into it and the caller owns the result (no second copy)
                buf = np.empty(self._cap, dtype=np.dtype(CLUSTER_DTYPE))
                rc = self._lib.dm_frontiers(self._handle(), _vp(mask), _vp(labels), _vp(buf),
                                            buf.shape[0], ctypes.byref(n))
                if rc == _ffi.DM_ERR_CAPACITY and n.value > buf.shape[0]:
                    self._cap = int(n.value) * 2
                    continue
                check(rc)
                break
            clusters = buf[: int(n.value)]
        return Frontiers(clusters=clusters, mask=mask, labels=labels)

    def frontiers_begin(self):
        """Enqueue a clusters-only frontier pass and return at once
        (dm_frontiers_begin); collect it with frontiers_end()."""
        with self._lock:
            check(self._lib.dm_frontiers_begin(self._handle()))

    def frontiers_ready(self) -> bool:
        """True when the oldest frontiers_begin() pass has completed, so
        frontiers_end() returns without waiting (dm_frontiers_poll; never
        blocks)."""
        r = ctypes.c_int32(0)
        with self._lock:
            check(self._lib.dm_frontiers_poll(self._handle(), ctypes.byref(r)))
        return bool(r.value)

    def frontiers_end(self) -> Frontiers | None:
        """Clusters of the pass started by frontiers_begin(), as frontiers()
        would have returned them on the map at that time; None if the pass
        overflowed the library's slot arrays (grown now: call frontiers())."""
        n = ctypes.c_int64(0)
        with self._lock:
            while True:
                buf = np.empty(self._cap, dtype=np.dtype(CLUSTER_DTYPE))
                rc = self._lib.dm_frontiers_end(self._handle(), _vp(buf), buf.shape[0], ctypes.byref(n))
                if rc == _ffi.DM_ERR_CAPACITY and n.value > buf.shape[0]:
                    self._cap = int(n.value) * 2  # the pass stays pending: read it again
                    continue
                if rc == _ffi.DM_ERR_INCOMPLETE:
                    self.last_incomplete = _ffi.last_error()
                    return None
                check(rc)
                return Frontiers(clusters=buf[: int(n.value)])

    def set_overlap(self, on: bool = True):
        """dm_set_overlap: run the integrate front-end beside an in-flight
        frontier pass (results unchanged)."""
        with self._lock:
            check(self._lib.dm_set_overlap(self._handle(), 1 if on else 0))

    # -- sharding support -------------------------------------------------
    def set_halo(self, before=None, after=None):
        b = None if before is None else np.ascontiguousarray(before, np.int8)
        a = None if after is None else np.ascontiguousarray(after, np.int8)
        with self._lock:
            check(self._lib.dm_set_halo(self._handle(), _vp(b), _vp(a)))

    def set_halo_device(self, before_ptr: int | None, after_ptr: int | None):
        with self._lock:
            check(self._lib.dm_set_halo_device(self._handle(),
                                               None if before_ptr is None else ctypes.c_void_p(before_ptr),
                                               None if after_ptr is None else ctypes.c_void_p(after_ptr)))

    def edge_rows(self):
        first = np.empty(self.width, np.int8)
        last = np.empty(self.width, np.int8)
        with self._lock:
            check(self._lib.dm_get_edge_rows(self._handle(), _vp(first), _vp(last)))
        return first, last

    def edge_rows_device(self, first_ptr: int, last_ptr: int):
        with self._lock:
            check(self._lib.dm_get_edge_rows_device(self._handle(), ctypes.c_void_p(first_ptr),
                                                    ctypes.c_void_p(last_ptr)))

    def edge_labels(self):
        first = np.empty(self.width, np.int64)
        last = np.empty(self.width, np.int64)
        with self._lock:
            check(self._lib.dm_get_edge_labels(self._handle(), _vp(first), _vp(last)))
        return first, last

    # -- cross-band exchange (device-resident; dm/sharded.py) --------------
    def export_bytes(self, rec_cap: int) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.dm_export_bytes(self._handle(), int(rec_cap), ctypes.byref(n)))
        return int(n.value)

    def frontiers_export_device(self, d_export_ptr: int, rec_cap: int):
        """Band frontiers + export record into a device buffer of
        export_bytes(rec_cap) bytes; asynchronous, complete on
        exchange_stream() (the pass stream with overlap on)."""
        with self._lock:
            check(self._lib.dm_frontiers_export_device(self._handle(), ctypes.c_void_p(d_export_ptr),
                                                       int(rec_cap)))

    def exchange_stream(self) -> int:
        """hipStream_t (as an int) on which exports are complete and merges
        run (dm_exchange_stream): order the records' all-gather on it."""
        s = ctypes.c_void_p(0)
        with self._lock:
            check(self._lib.dm_exchange_stream(self._handle(), ctypes.byref(s)))
        return int(s.value or 0)

    def merge_bands(self, d_gathered_ptr: int, nranks: int, rec_cap: int, min_size: int):
        """Merge all-gathered export records on the device.  Returns
        (clusters, None) or (None, largest band K) when a band's record was
        incomplete (DM_ERR_INCOMPLETE: rerun with more capacity)."""
        n = ctypes.c_int64(0)
        with self._lock:
            while True:
                buf = self._mbuf if getattr(self, "_mbuf", None) is not None else \
                    np.empty(1 << 14, dtype=np.dtype(CLUSTER_DTYPE))
                rc = self._lib.dm_merge_bands(self._handle(), ctypes.c_void_p(d_gathered_ptr), int(nranks),
                                              int(rec_cap), int(min_size), _vp(buf), buf.shape[0],
                                              ctypes.byref(n))
                self._mbuf = buf
                if rc == _ffi.DM_ERR_INCOMPLETE:
                    self.last_incomplete = _ffi.last_error()
                    return None, int(n.value)
                if rc == _ffi.DM_ERR_CAPACITY and n.value > buf.shape[0]:
                    self._mbuf = np.empty(int(n.value) * 2, dtype=np.dtype(CLUSTER_DTYPE))
                    continue
                check(rc)
                return buf[: int(n.value)].copy(), None

    def merge_max_band_k(self) -> int:
        """Largest band cluster count of the last collected merge."""
        k = ctypes.c_int64(0)
        with self._lock:
            check(self._lib.dm_merge_max_band_k(self._handle(), ctypes.byref(k)))
        return int(k.value)

    def merge_bands_begin(self, d_gathered_ptr: int, nranks: int, rec_cap: int, min_size: int):
        """Enqueue the device merge of gathered export records and return
        (dm_merge_bands_begin); collect it with merge_bands_end()."""
        with self._lock:
            check(self._lib.dm_merge_bands_begin(self._handle(), ctypes.c_void_p(d_gathered_ptr), int(nranks),
                                                 int(rec_cap), int(min_size)))

    def merge_bands_end(self):
        """merge_bands()'s result for the pass started by merge_bands_begin()."""
        n = ctypes.c_int64(0)
        with self._lock:
            while True:
                buf = self._mbuf if getattr(self, "_mbuf", None) is not None else \
                    np.empty(1 << 14, dtype=np.dtype(CLUSTER_DTYPE))
                rc = self._lib.dm_merge_bands_end(self._handle(), _vp(buf), buf.shape[0], ctypes.byref(n))
                self._mbuf = buf
                if rc == _ffi.DM_ERR_INCOMPLETE:
                    self.last_incomplete = _ffi.last_error()
                    return None, int(n.value)
                if rc == _ffi.DM_ERR_CAPACITY and n.value > buf.shape[0]:
                    self._mbuf = np.empty(int(n.value) * 2, dtype=np.dtype(CLUSTER_DTYPE))
                    continue  # the pass stays pending: read it again
                check(rc)
                return buf[: int(n.value)].copy(), None

    # -- checkpoint / streams / profiling ----------------------------------
    def save(self, path: str):
        with self._lock:
            check(self._lib.dm_save(self._handle(), str(path).encode()))

    def load(self, path: str):
        with self._lock:
            check(self._lib.dm_load(self._handle(), str(path).encode()))

    def set_stream(self, stream_ptr: int | None):
        with self._lock:
            check(self._lib.dm_set_stream(self._handle(),
                                          None if not stream_ptr else ctypes.c_void_p(stream_ptr)))

    def synchronize(self):
        with self._lock:
            check(self._lib.dm_synchronize(self._handle()))

    def profile(self, enable: bool = True):
        with self._lock:
            check(self._lib.dm_profile_enable(self._handle(), 1 if enable else 0))

    def profile_read(self) -> dict:
        cap = 64
        arr = (_ffi.DmKernelStat * cap)()
        n = ctypes.c_int32(0)
        with self._lock:
            check(self._lib.dm_profile_read(self._handle(), arr, cap, ctypes.byref(n)))
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].total_ms))
                for i in range(min(n.value, cap))}

    def profile_reset(self):
        with self._lock:
            check(self._lib.dm_profile_reset(self._handle()))
