"""Seeded parity cases shared by the CPU oracle tests and the GPU parity tests."""
from __future__ import annotations

import numpy as np

from dm._ffi import DmParams
from dm import synth


def make_params(width, height, resolution=0.05, origin=None, **kw) -> DmParams:
    """Same defaults as dm_default_params (include/dm.h), without the library."""
    p = DmParams()
    p.width, p.height, p.resolution = width, height, resolution
    ox, oy = origin if origin is not None else (-0.5 * width * resolution, -0.5 * height * resolution)
    p.origin_x, p.origin_y = ox, oy
    p.range_min, p.range_max = np.float32(0.02), 12.0
    p.l_occ, p.l_free, p.l_min, p.l_max = 0.85, -0.4, -2.0, 3.5
    p.occ_thresh = p.free_thresh = 0.0
    p.min_frontier_size = 1
    p.band_row0 = 0
    p.band_rows = 0
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def world_case(seed, width, height, resolution, n_robots, n_beams, n_batches, region_frac=0.9):
    """A synthetic world covering the map, robots random-walking inside it.
    Returns (params, list of (poses[S,3], ranges[S,N])), angle_min, angle_inc."""
    p = make_params(width, height, resolution)
    half_w, half_h = width * resolution / 2, height * resolution / 2
    world = synth.make_world(seed, -half_w, -half_h, half_w, half_h)
    f = region_frac
    stream = synth.ScanStream(world, n_robots, n_beams, seed + 1,
                              region=(-half_w * f, -half_h * f, half_w * f, half_h * f))
    batches = [stream.next_batch() for _ in range(n_batches)]
    return p, batches, float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(n_beams))


def random_scans(seed, p, S, N, spread=1.0, nan_frac=0.05, far_frac=0.1):
    """Unstructured scans: poses anywhere around the map (also outside it),
    ranges uniform in [0, 1.3*range_max] with NaNs, zeros and infinities."""
    rng = np.random.Generator(np.random.PCG64(seed))
    wx, wy = p.width * p.resolution, p.height * p.resolution
    x = p.origin_x + rng.uniform(-0.2 * spread, 1 + 0.2 * spread, S) * wx
    y = p.origin_y + rng.uniform(-0.2 * spread, 1 + 0.2 * spread, S) * wy
    yaw = rng.uniform(-np.pi, np.pi, S)
    poses = np.stack([x, y, yaw], 1)
    r = rng.uniform(0.0, 1.3 * p.range_max, (S, N)).astype(np.float32)
    r = (np.round(r * 1000) / 1000).astype(np.float32)
    m = rng.random((S, N))
    r[m < nan_frac] = np.nan
    r[(m >= nan_frac) & (m < nan_frac + 0.01)] = 0.0
    r[(m >= nan_frac + 0.01) & (m < nan_frac + 0.02)] = np.inf
    r[(m >= 1 - far_frac)] = np.float32(p.range_max + 1.0)
    inc = float(np.float32(2 * np.pi / max(N - 1, 1)))
    return poses, r, 0.0, inc


def random_state(seed, R, W, p_free=0.5, p_occ=0.1):
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.random((R, W))
    st = np.full((R, W), -1, np.int8)
    st[u < p_free] = 0
    st[(u >= p_free) & (u < p_free + p_occ)] = 100
    return st


def blob_state(seed, R, W, n_blobs=20):
    """Unknown background with free discs (explored areas) and occupied specks:
    long, winding frontier components that cross many 64x64 tiles."""
    rng = np.random.Generator(np.random.PCG64(seed))
    st = np.full((R, W), -1, np.int8)
    yy, xx = np.mgrid[0:R, 0:W]
    for _ in range(n_blobs):
        cy, cx = rng.uniform(0, R), rng.uniform(0, W)
        rad = rng.uniform(3, max(4, min(R, W) / 4))
        st[(yy - cy) ** 2 + (xx - cx) ** 2 <= rad * rad] = 0
    occ = rng.random((R, W)) < 0.03
    st[occ & (st == 0)] = 100
    return st
