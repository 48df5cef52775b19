"""Generate tests/golden/map_image_golden.npz from the REFERENCE's own
get_map_image (server/thymio_project/thymio_project/main.py:241-279).

Run in the build container (where /root/reference exists):
    python tests/golden/make_map_image_golden.py
The reference module imports rclpy / tf2_ros / ROS message packages /
thymiodirect, which are absent; they are replaced by inert sys.modules stubs
(only so the module body can execute: get_map_image uses none of them).
Flask and PIL are real.  The reference never travels to the GPU box: only
the .npz (inputs + the PNG pixels the reference produced) is committed.
"""
from __future__ import annotations

import importlib.util
import io
import os
import sys
import types

import numpy as np

REF = "/root/reference/server/thymio_project/thymio_project/main.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "map_image_golden.npz")


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def load_reference():
    class _Any:
        def __init__(self, *a, **k):
            pass

    _stub("rclpy", init=lambda *a, **k: None, spin=lambda *a, **k: None,
          shutdown=lambda *a, **k: None)
    _stub("rclpy.node", Node=_Any)
    _stub("rclpy.duration", Duration=_Any)
    _stub("sensor_msgs")
    _stub("sensor_msgs.msg", LaserScan=_Any)
    _stub("nav_msgs")
    _stub("nav_msgs.msg", OccupancyGrid=_Any, Odometry=_Any)
    _stub("geometry_msgs")
    _stub("geometry_msgs.msg", TransformStamped=_Any)
    _stub("tf2_ros", TransformBroadcaster=_Any)
    _stub("thymiodirect", Thymio=_Any)
    spec = importlib.util.spec_from_file_location("ref_main", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Info:
    def __init__(self, w, h):
        self.width = w
        self.height = h


class _Grid:
    """Duck-typed nav_msgs/OccupancyGrid (the fields get_map_image reads)."""

    def __init__(self, data: np.ndarray):
        h, w = data.shape
        self.info = _Info(w, h)
        self.data = [int(v) for v in data.reshape(-1)]


def main():
    from PIL import Image

    ref = load_reference()

    class _Node:
        latest_map = None
        last_png = None
        last_png_time = 0

    ref.robot_node = _Node()
    client = ref.app.test_client()
    rng = np.random.Generator(np.random.PCG64(7))
    cases = [np.array([[-1, 0, 100, 0], [0, 0, -1, 100], [100, -1, 0, 0]], np.int8)]
    for (h, w) in [(1, 1), (5, 7), (64, 64), (33, 70)]:
        cases.append(rng.choice(np.array([-1, 0, 100], np.int8), size=(h, w)))
    # values outside {-1, 0, 100} (a probability-valued OccupancyGrid) -> 127
    cases.append(rng.integers(-1, 101, size=(9, 11)).astype(np.int8))
    arrays = {}
    for i, grid in enumerate(cases):
        ref.robot_node.latest_map = _Grid(grid)
        resp = client.get("/map-image")
        assert resp.status_code == 200, resp.status_code
        img = np.array(Image.open(io.BytesIO(resp.data)))
        arrays[f"state_{i}"] = grid
        arrays[f"image_{i}"] = img.astype(np.uint8)
    # "Map not ready yet" path
    ref.robot_node.latest_map = None
    resp = client.get("/map-image")
    arrays["not_ready_status"] = np.array(resp.status_code)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT} ({len(cases)} grids)")


if __name__ == "__main__":
    main()
