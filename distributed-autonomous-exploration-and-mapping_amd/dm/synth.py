"""Seeded synthetic worlds, trajectories and LD06-format scans.

Only workload generation (tests and bench.py); not on the hot path.  Scans
follow the LD06 driver's LaserScan encoding (ToLaserscanMessagePublish,
ldlidar_stl_ros2_node @0x7f853):

* ``angle_min = 0.0f``, ``angle_max = 6.2831855f``,
  ``angle_increment = (angle_max - angle_min) / (float)(N - 1)``;
* range = (float)distance_mm / 1000.0f on a 1 mm grid;
* no return -> NaN; LD06 ``range_max = 25.0f``, so targets beyond 25 m give NaN;
* 2 % random dropout -> NaN.

World: axis-aligned rectangles covering ``density`` of the area (2 % by
default) plus four boundary walls.  Trajectories: random walk of 0.1 m /
<= 0.1 rad steps (the slam_toolbox gating, slam_config.yaml:37-38).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

LD06_ANGLE_MIN = np.float32(0.0)
LD06_ANGLE_MAX = np.float32(6.2831855)
LD06_RANGE_MAX = 25.0
LD06_RANGE_MIN = np.float32(0.02)


def ld06_angle_increment(n_beams: int) -> np.float32:
    """angle_increment exactly as the driver computes it (float32)."""
    return np.float32((LD06_ANGLE_MAX - LD06_ANGLE_MIN) / np.float32(n_beams - 1))


@dataclass
class World:
    rects: np.ndarray  # [K, 4] xmin, ymin, xmax, ymax (metres)
    xmin: float
    ymin: float
    xmax: float
    ymax: float
    cell: float = 8.0  # spatial-hash bucket (m)

    def __post_init__(self):
        self._build_hash()

    def _build_hash(self):
        c = self.cell
        self._nx = max(1, int(math.ceil((self.xmax - self.xmin) / c)))
        self._ny = max(1, int(math.ceil((self.ymax - self.ymin) / c)))
        buckets: dict[int, list[int]] = {}
        for k, (x0, y0, x1, y1) in enumerate(self.rects):
            bx0 = int(np.clip((x0 - self.xmin) // c, 0, self._nx - 1))
            bx1 = int(np.clip((x1 - self.xmin) // c, 0, self._nx - 1))
            by0 = int(np.clip((y0 - self.ymin) // c, 0, self._ny - 1))
            by1 = int(np.clip((y1 - self.ymin) // c, 0, self._ny - 1))
            for by in range(by0, by1 + 1):
                for bx in range(bx0, bx1 + 1):
                    buckets.setdefault(by * self._nx + bx, []).append(k)
        self._buckets = {k: np.array(v, np.int64) for k, v in buckets.items()}

    def near(self, x: float, y: float, radius: float) -> np.ndarray:
        c = self.cell
        bx0 = int(np.clip((x - radius - self.xmin) // c, 0, self._nx - 1))
        bx1 = int(np.clip((x + radius - self.xmin) // c, 0, self._nx - 1))
        by0 = int(np.clip((y - radius - self.ymin) // c, 0, self._ny - 1))
        by1 = int(np.clip((y + radius - self.ymin) // c, 0, self._ny - 1))
        parts = [self._buckets[b] for by in range(by0, by1 + 1)
                 for b in range(by * self._nx + bx0, by * self._nx + bx1 + 1) if b in self._buckets]
        if not parts:
            return np.zeros(0, np.int64)
        return np.unique(np.concatenate(parts))

    def occupied(self, x: float, y: float, margin: float = 0.0) -> bool:
        if not (self.xmin + 0.5 <= x <= self.xmax - 0.5 and self.ymin + 0.5 <= y <= self.ymax - 0.5):
            return True
        idx = self.near(x, y, margin + 0.01)
        if idx.size == 0:
            return False
        r = self.rects[idx]
        return bool(np.any((x >= r[:, 0] - margin) & (x <= r[:, 2] + margin)
                           & (y >= r[:, 1] - margin) & (y <= r[:, 3] + margin)))


def make_world(seed: int, xmin: float, ymin: float, xmax: float, ymax: float,
               density: float = 0.02, size_lo: float = 0.2, size_hi: float = 1.5,
               walls: bool = True) -> World:
    rng = np.random.Generator(np.random.PCG64(seed))
    area = (xmax - xmin) * (ymax - ymin)
    mean_area = ((size_lo + size_hi) / 2.0) ** 2
    k = int(round(density * area / mean_area))
    w = rng.uniform(size_lo, size_hi, k)
    h = rng.uniform(size_lo, size_hi, k)
    cx = rng.uniform(xmin, xmax, k)
    cy = rng.uniform(ymin, ymax, k)
    rects = np.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], axis=1)
    if walls:
        t = 0.1
        wall = np.array([
            [xmin + 0.2, ymin + 0.2, xmax - 0.2, ymin + 0.2 + t],
            [xmin + 0.2, ymax - 0.2 - t, xmax - 0.2, ymax - 0.2],
            [xmin + 0.2, ymin + 0.2, xmin + 0.2 + t, ymax - 0.2],
            [xmax - 0.2 - t, ymin + 0.2, xmax - 0.2, ymax - 0.2],
        ])
        rects = np.concatenate([rects, wall], axis=0)
    return World(rects=rects, xmin=xmin, ymin=ymin, xmax=xmax, ymax=ymax)


def ray_distances(world: World, x: float, y: float, theta: np.ndarray,
                  max_dist: float = LD06_RANGE_MAX) -> np.ndarray:
    """Exact float64 distance along each ray to the nearest rectangle (inf if
    none within max_dist)."""
    idx = world.near(x, y, max_dist)
    out = np.full(theta.shape, np.inf)
    if idx.size == 0:
        return out
    r = world.rects[idx]
    # keep rectangles whose nearest point is within max_dist
    px = np.clip(x, r[:, 0], r[:, 2])
    py = np.clip(y, r[:, 1], r[:, 3])
    r = r[(px - x) ** 2 + (py - y) ** 2 <= max_dist * max_dist]
    if r.shape[0] == 0:
        return out
    dx = np.cos(theta)[:, None]
    dy = np.sin(theta)[:, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        inv_x = 1.0 / dx
        inv_y = 1.0 / dy
        tx1 = (r[None, :, 0] - x) * inv_x
        tx2 = (r[None, :, 2] - x) * inv_x
        ty1 = (r[None, :, 1] - y) * inv_y
        ty2 = (r[None, :, 3] - y) * inv_y
        tmin = np.maximum(np.minimum(tx1, tx2), np.minimum(ty1, ty2))
        tmax = np.minimum(np.maximum(tx1, tx2), np.maximum(ty1, ty2))
    ok = (tmax >= np.maximum(tmin, 0.0)) & np.isfinite(tmin)
    t = np.where(ok, np.maximum(tmin, 0.0), np.inf)
    return t.min(axis=1)


def ld06_scan(world: World, x: float, y: float, yaw: float, n_beams: int,
              rng: np.random.Generator, dropout: float = 0.02) -> np.ndarray:
    """One LaserScan.ranges array (float32[N]) in the LD06 encoding."""
    inc = ld06_angle_increment(n_beams)
    phi = np.float64(LD06_ANGLE_MIN) + np.arange(n_beams, dtype=np.float64) * np.float64(inc)
    d = ray_distances(world, x, y, yaw + phi)
    mm = np.round(d * 1000.0)
    rng_out = np.where(np.isfinite(d) & (d <= LD06_RANGE_MAX),
                       (mm.astype(np.float32) / np.float32(1000.0)), np.float32(np.nan))
    rng_out = rng_out.astype(np.float32)
    drop = rng.random(n_beams) < dropout
    rng_out[drop] = np.float32(np.nan)
    # the LD06 publishes distance 0 with intensity 0 as NaN; a 0 mm return
    # with intensity is a 0.0 range (below range_min, skipped downstream)
    return rng_out


class ScanStream:
    """n_robots random-walking robots; each next_batch() advances every robot
    one step and returns their poses (S,3) and scans (S,N)."""

    def __init__(self, world: World, n_robots: int, n_beams: int, seed: int,
                 step: float = 0.1, turn: float = 0.1, region=None):
        self.world = world
        self.n_beams = n_beams
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.step = step
        self.turn = turn
        x0, y0, x1, y1 = region if region is not None else (world.xmin, world.ymin,
                                                             world.xmax, world.ymax)
        poses = []
        while len(poses) < n_robots:
            x = self.rng.uniform(x0 + 1.0, x1 - 1.0)
            y = self.rng.uniform(y0 + 1.0, y1 - 1.0)
            if world.occupied(x, y, margin=0.3):
                continue
            poses.append([x, y, self.rng.uniform(-math.pi, math.pi)])
        self.poses = np.array(poses, np.float64)

    def advance(self):
        for r in range(self.poses.shape[0]):
            x, y, yaw = self.poses[r]
            yaw = yaw + self.rng.uniform(-self.turn, self.turn)
            nx, ny = x + self.step * math.cos(yaw), y + self.step * math.sin(yaw)
            if self.world.occupied(nx, ny, margin=0.2):
                yaw += math.pi / 2
                nx, ny = x, y
            yaw = math.atan2(math.sin(yaw), math.cos(yaw))
            self.poses[r] = (nx, ny, yaw)

    def scans(self) -> np.ndarray:
        return np.stack([ld06_scan(self.world, p[0], p[1], p[2], self.n_beams, self.rng)
                         for p in self.poses]).astype(np.float32)

    def next_batch(self):
        self.advance()
        return self.poses.copy(), self.scans()


def config_world(cfg: str, seed: int = 0):
    """Worlds and map parameters for BASELINE.json configs.
    Returns (world, width, height, resolution, origin_x, origin_y)."""
    table = {
        "C1": (400, 0.05),
        "C2": (4096, 0.05),
        "C3": (16384, 0.05),
        "C4": (32768, 0.05),
        "C5": (65536, 0.01),
    }
    n, res = table[cfg]
    half = n * res / 2.0
    world = make_world(seed, -half, -half, half, half)
    return world, n, n, res, -half, -half


def explored_state(world: World, W: int, H: int, res: float, ox: float, oy: float, seed: int = 0,
                   row0: int = 0, rows: int | None = None, unknown_frac: float = 0.08,
                   r_lo: float = 0.5, r_hi: float = 6.0) -> np.ndarray:
    """Rows [row0, row0 + rows) of a mostly explored map (OccupancyGrid.data
    encoding, int8 [rows, W]): free space; every obstacle of `world` as an
    occupied outline around an unobserved (unknown) interior, as a scanner
    sees it; unexplored pockets (shadows behind obstacles, rooms not yet
    entered) as unknown discs of radius r_lo..r_hi metres covering about
    `unknown_frac` of the area.  Nearly every 64x64 tile holds free cells and
    the pocket rims are frontiers: the frontier pass's worst case (every tile
    read), as get_map_image (main.py:251-263) sees a map late in a run.
    Seeded and independent of the row window, so bands of one map agree."""
    rows = H - row0 if rows is None else rows
    st = np.zeros((rows, W), np.int8)

    def cells(x0, y0, x1, y1):
        return (int(math.floor((x0 - ox) / res)), int(math.floor((y0 - oy) / res)),
                int(math.floor((x1 - ox) / res)), int(math.floor((y1 - oy) / res)))

    for x0, y0, x1, y1 in world.rects:
        cx0, cy0, cx1, cy1 = cells(x0, y0, x1, y1)
        cx0, cx1 = max(cx0, 0), min(cx1, W - 1)
        ya, yb = max(cy0, row0), min(cy1, row0 + rows - 1)
        if cx0 > cx1 or ya > yb:
            continue
        st[ya - row0:yb - row0 + 1, cx0:cx1 + 1] = 100
        ia, ib = max(cy0 + 1, row0), min(cy1 - 1, row0 + rows - 1)
        if cx1 - cx0 >= 2 and ia <= ib:
            st[ia - row0:ib - row0 + 1, cx0 + 1:cx1] = -1
    rng = np.random.Generator(np.random.PCG64(seed))
    area = W * H * res * res
    mean_r2 = (r_hi ** 3 - r_lo ** 3) / (3.0 * (r_hi - r_lo))
    n = int(round(unknown_frac * area / (math.pi * mean_r2)))
    cxs = rng.uniform(0, W, n)
    cys = rng.uniform(0, H, n)
    rads = rng.uniform(r_lo, r_hi, n) / res
    for cx, cy, rr in zip(cxs, cys, rads):
        ya, yb = max(int(cy - rr), row0), min(int(cy + rr) + 1, row0 + rows - 1)
        xa, xb = max(int(cx - rr), 0), min(int(cx + rr) + 1, W - 1)
        if ya > yb or xa > xb:
            continue
        yy = np.arange(ya, yb + 1)[:, None] + 0.5 - cy
        xx = np.arange(xa, xb + 1)[None, :] + 0.5 - cx
        sub = st[ya - row0:yb - row0 + 1, xa:xb + 1]
        sub[(yy * yy + xx * xx <= rr * rr) & (sub == 0)] = -1
    return st


def pose4(poses: np.ndarray) -> np.ndarray:
    """(x, y, yaw) -> (x, y, cos yaw, sin yaw) with the C library's cos/sin
    (math.cos), the device-resident pose format of dm_integrate_device."""
    poses = np.asarray(poses, np.float64).reshape(-1, 3)
    out = np.empty((poses.shape[0], 4), np.float64)
    for i, (x, y, yaw) in enumerate(poses):
        out[i] = (x, y, math.cos(yaw), math.sin(yaw))
    return out


def ld06_points(world: World, x: float, y: float, yaw: float, rng: np.random.Generator,
                n_points: int = 450, dropout: float = 0.02) -> np.ndarray:
    """One revolution of raw LD06 PointData (angle in degrees, distance in mm,
    intensity), as LiPkg hands them to ToLaserscanMessagePublish: ~4500 Hz /
    10 Hz = 450 points with slightly jittered angles, no return = (0 mm, 0)."""
    from ._ffi import LD06_POINT_DTYPE

    ang = (np.arange(n_points) + rng.uniform(-0.3, 0.3, n_points)) * (360.0 / n_points)
    ang = np.mod(ang, 360.0).astype(np.float32)
    d = ray_distances(world, x, y, yaw + np.deg2rad(ang.astype(np.float64)))
    pts = np.zeros(n_points, dtype=np.dtype(LD06_POINT_DTYPE))
    pts["angle_deg"] = ang
    ok = np.isfinite(d) & (d * 1000.0 < 65535) & (rng.random(n_points) >= dropout)
    pts["distance_mm"] = np.where(ok, np.round(d * 1000.0), 0).astype(np.uint16)
    pts["intensity"] = np.where(ok, rng.integers(100, 255, n_points), 0).astype(np.uint8)
    return pts


def c3_pool(seed: int, G: int, robots: int, beams: int, n: int, world_size: int = 1, rank: int = 0,
            res: float = 0.05):
    """The bench line's C3 batches (bench.py): rank
    `rank` of `world_size` owns a G-row band of a G x G*world_size map; each
    band has `robots` robots random-walking anywhere in it, in one world over
    the whole map; a rank integrates its own robots' scans plus the
    neighbouring bands' scans whose max-range disk reaches its band.
    Returns (world, (origin_x, origin_y), pool): pool is n (poses [S,3],
    ranges [S,beams]) batches.  Tests replay exactly what bench.py times."""
    from .sharded import band_rows

    H_total = G * world_size
    half_w = G * res / 2.0
    oy_global = -H_total * res / 2.0
    world = make_world(seed * 1000, -half_w, oy_global, half_w, -oy_global)
    b_row0, b_rows = band_rows(H_total, world_size, rank) if world_size > 1 else (0, H_total)

    def band_stream(q):
        y0 = oy_global + q * G * res
        return ScanStream(world, robots, beams, seed * 1000 + 500 + q,
                          region=(-half_w + 1.0, y0 + 1.0, half_w - 1.0, y0 + G * res - 1.0))

    reach = 12.0 + 2 * res
    ylo = oy_global + b_row0 * res - reach
    yhi = oy_global + (b_row0 + b_rows) * res + reach
    streams = {q: band_stream(q) for q in (rank - 1, rank, rank + 1) if 0 <= q < world_size}
    pool = []
    for _ in range(n):
        poses, ranges = [], []
        for q, st in streams.items():
            p_, r_ = st.next_batch()
            keep = np.ones(len(p_), bool) if q == rank else (p_[:, 1] >= ylo) & (p_[:, 1] <= yhi)
            poses.append(p_[keep])
            ranges.append(r_[keep])
        pool.append((np.concatenate(poses), np.concatenate(ranges)))
    return world, (-half_w, oy_global), pool
