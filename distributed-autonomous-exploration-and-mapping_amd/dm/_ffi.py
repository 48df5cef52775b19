"""ctypes binding of libdm.so (the C-ABI declared in include/dm.h).

This is the "thin C-ABI shared library (ctypes)" that BASELINE.json's
north_star puts between the ROS 2 Python nodes and the HIP kernels.  The
library is built in-tree (``csrc/Makefile`` -> ``dm/libdm.so``); there is no
fallback: if it is missing, every entry point raises ``DmError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DM_LIB", os.path.join(_HERE, "libdm.so"))

DM_OK = 0
DM_ERR_INVALID_ARG = -1
DM_ERR_SHAPE = -2
DM_ERR_HIP = -3
DM_ERR_OOM = -4
DM_ERR_CAPACITY = -5
DM_ERR_IO = -6
DM_ERR_STATE = -7
DM_ERR_INCOMPLETE = -8
DM_ERR_PIPELINE = -9
DM_ERR_COLLECTIVE = -10
DM_TILE = 64

_ERR_NAMES = {
    DM_ERR_INVALID_ARG: "DM_ERR_INVALID_ARG",
    DM_ERR_SHAPE: "DM_ERR_SHAPE",
    DM_ERR_HIP: "DM_ERR_HIP",
    DM_ERR_OOM: "DM_ERR_OOM",
    DM_ERR_CAPACITY: "DM_ERR_CAPACITY",
    DM_ERR_IO: "DM_ERR_IO",
    DM_ERR_STATE: "DM_ERR_STATE",
    DM_ERR_INCOMPLETE: "DM_ERR_INCOMPLETE",
    DM_ERR_PIPELINE: "DM_ERR_PIPELINE",
    DM_ERR_COLLECTIVE: "DM_ERR_COLLECTIVE",
}


class DmError(RuntimeError):
    """Raised for every negative return code of libdm (include/dm.h)."""

    def __init__(self, code: int, message: str):
        self.code = code
        super().__init__(f"{_ERR_NAMES.get(code, code)}: {message}")


class DmParams(ctypes.Structure):
    """Mirror of ``dm_params`` (include/dm.h)."""

    _fields_ = [
        ("width", ctypes.c_int64),
        ("height", ctypes.c_int64),
        ("resolution", ctypes.c_double),
        ("origin_x", ctypes.c_double),
        ("origin_y", ctypes.c_double),
        ("range_min", ctypes.c_float),
        ("range_max", ctypes.c_float),
        ("l_occ", ctypes.c_float),
        ("l_free", ctypes.c_float),
        ("l_min", ctypes.c_float),
        ("l_max", ctypes.c_float),
        ("occ_thresh", ctypes.c_float),
        ("free_thresh", ctypes.c_float),
        ("min_frontier_size", ctypes.c_int64),
        ("band_row0", ctypes.c_int64),
        ("band_rows", ctypes.c_int64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class DmCluster(ctypes.Structure):
    """Mirror of ``dm_cluster`` (include/dm.h)."""

    _fields_ = [
        ("label", ctypes.c_int64),
        ("size", ctypes.c_int64),
        ("sum_x", ctypes.c_int64),
        ("sum_y", ctypes.c_int64),
        ("cx_m", ctypes.c_double),
        ("cy_m", ctypes.c_double),
    ]


class DmLd06Point(ctypes.Structure):
    """Mirror of ``dm_ld06_point`` (include/dm.h)."""

    _fields_ = [
        ("angle_deg", ctypes.c_float),
        ("distance_mm", ctypes.c_uint16),
        ("intensity", ctypes.c_uint8),
        ("pad", ctypes.c_uint8),
    ]


LD06_POINT_DTYPE = [("angle_deg", "<f4"), ("distance_mm", "<u2"), ("intensity", "u1"), ("pad", "u1")]


class DmKernelStat(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 32),
        ("launches", ctypes.c_uint64),
        ("total_ms", ctypes.c_double),
    ]


CLUSTER_DTYPE = [
    ("label", "<i8"),
    ("size", "<i8"),
    ("sum_x", "<i8"),
    ("sum_y", "<i8"),
    ("cx_m", "<f8"),
    ("cy_m", "<f8"),
]

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> argtypes (every function returns int)
SIGNATURES = {
    "dm_default_params": [ctypes.POINTER(DmParams), _i64, _i64],
    "dm_create": [ctypes.POINTER(_vp), ctypes.POINTER(DmParams), ctypes.c_int],
    "dm_create_sharded": [ctypes.POINTER(_vp), ctypes.POINTER(DmParams), _i32, ctypes.POINTER(_i32)],
    "dm_sharded_band_rows": [_i64, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_i64)],
    "dm_sharded_info": [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64)],
    "dm_destroy": [_vp],
    "dm_reset": [_vp],
    "dm_get_params": [_vp, ctypes.POINTER(DmParams)],
    "dm_integrate": [_vp, _i32, _vp, _i32, _vp, _f32, _f32, _vp, _vp],
    "dm_integrate_device": [_vp, _i32, _vp, _i32, _vp, _f32, _f32],
    "dm_integrate_async": [_vp, _i32, _vp, _i32, _vp, _f32, _f32],
    "dm_last_counts": [_vp, _vp, _vp],
    "dm_last_stats": [_vp, _vp, _i32, ctypes.POINTER(_i32)],
    "dm_get_state": [_vp, _vp],
    "dm_get_logodds": [_vp, _vp],
    "dm_set_logodds": [_vp, _vp],
    "dm_set_state": [_vp, _vp],
    "dm_frontiers": [_vp, _vp, _vp, _vp, _i64, ctypes.POINTER(_i64)],
    "dm_set_halo": [_vp, _vp, _vp],
    "dm_set_halo_device": [_vp, _vp, _vp],
    "dm_get_edge_rows": [_vp, _vp, _vp],
    "dm_get_edge_rows_device": [_vp, _vp, _vp],
    "dm_get_edge_labels": [_vp, _vp, _vp],
    "dm_save": [_vp, ctypes.c_char_p],
    "dm_load": [_vp, ctypes.c_char_p],
    "dm_set_stream": [_vp, _vp],
    "dm_exchange_stream": [_vp, ctypes.POINTER(ctypes.c_void_p)],
    "dm_synchronize": [_vp],
    "dm_profile_enable": [_vp, ctypes.c_int],
    "dm_profile_read": [_vp, ctypes.POINTER(DmKernelStat), _i32, ctypes.POINTER(_i32)],
    "dm_profile_reset": [_vp],
    "dm_map_image": [_vp, _vp],
    "dm_ld06_to_scans": [_vp, _i32, _vp, _vp, _i32, ctypes.c_int, _vp, _vp],
    "dm_ld06_to_scans_device": [_vp, _i32, _vp, _vp, _i32, ctypes.c_int, _vp, _vp],
    "dm_export_bytes": [_vp, _i64, ctypes.POINTER(_i64)],
    "dm_frontiers_export_device": [_vp, _vp, _i64],
    "dm_merge_bands": [_vp, _vp, _i32, _i64, _i64, _vp, _i64, ctypes.POINTER(_i64)],
    "dm_merge_bands_begin": [_vp, _vp, _i32, _i64, _i64],
    "dm_merge_bands_end": [_vp, _vp, _i64, ctypes.POINTER(_i64)],
    "dm_merge_max_band_k": [_vp, ctypes.POINTER(_i64)],
    "dm_frontiers_begin": [_vp],
    "dm_max_passes_in_flight": [],
    "dm_frontiers_end": [_vp, _vp, _i64, ctypes.POINTER(_i64)],
    "dm_frontiers_poll": [_vp, ctypes.POINTER(_i32)],
    "dm_set_overlap": [_vp, _i32],
    "dm_atomic_peak": [ctypes.c_int, _vp, _i32, ctypes.POINTER(_i32)],
    "dm_assign_goals": [_vp, _vp, _i32, ctypes.c_int64, ctypes.c_double, ctypes.c_double, _vp, _vp],
}
# functions returning const char*
STRING_FUNCS = ("dm_last_error", "dm_version")

_lib = None
_lib_lock = threading.Lock()


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libdm.so (once).  Raises DmError if it is missing: there is no
    CPU fallback for the product path."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise DmError(
                DM_ERR_STATE,
                f"libdm.so not found at {p}; build it with "
                "`make -C distributed-autonomous-exploration-and-mapping_amd/csrc` "
                "(or __graft_entry__.build())",
            )
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        for name in STRING_FUNCS:
            fn = getattr(lib, name)
            fn.argtypes = []
            fn.restype = ctypes.c_char_p
        _lib = lib
        return lib


def last_error() -> str:
    v = load_library().dm_last_error()
    return v.decode() if isinstance(v, bytes) else str(v)


def check(rc: int) -> int:
    if rc < 0:
        msg = load_library().dm_last_error()
        raise DmError(rc, msg.decode() if msg else "")
    return rc


def exported_symbols() -> list[str]:
    return list(SIGNATURES) + list(STRING_FUNCS)
