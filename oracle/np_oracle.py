"""TEST INFRASTRUCTURE ONLY — second, independent restatement of the SPEC in
NumPy/scipy and pure-Python loops (small cases only).  It exists to pin the C
oracle (dm_oracle.c): two restatements written differently must agree bit for
bit on seeded inputs (tests/test_oracle.py).  Written in the reference's
numpy idiom (server/thymio_project/thymio_project/main.py:151-156, 256-263).

Trig: ``math.cos``/``math.sin`` call the C library like dm_oracle.c does
(NumPy's vectorised cos may differ by an ulp, SURVEY.md §7 "Hard parts").
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage


def endpoints(p, poses, ranges, angle_min, angle_increment):
    """SPEC a4.  Returns list of (sx, sy, ex, ey, hit) per valid beam and a
    parallel list of flat beam indices."""
    poses = np.asarray(poses, np.float64).reshape(-1, 3)
    ranges = np.asarray(ranges, np.float32).reshape(poses.shape[0], -1)
    S, N = ranges.shape
    f32 = np.float32
    amin = float(f32(angle_min))
    inc = float(f32(angle_increment))
    phis = [amin + float(i) * inc for i in range(N)]
    cph = [math.cos(v) for v in phis]
    sph = [math.sin(v) for v in phis]
    rmin = f32(p.range_min)
    rmax = f32(p.range_max)
    out = []
    for s in range(S):
        x, y, yaw = (float(v) for v in poses[s])
        if not (math.isfinite(x) and math.isfinite(y) and math.isfinite(yaw)):
            continue
        cy, sy = math.cos(yaw), math.sin(yaw)
        for i in range(N):
            r = ranges[s, i]
            if not (r >= rmin):
                continue
            hit = bool(r <= rmax)
            rr = float(r) if hit else float(rmax)
            dcx = cy * cph[i] - sy * sph[i]
            dcy = sy * cph[i] + cy * sph[i]
            ex = x + rr * dcx
            ey = y + rr * dcy
            res = float(p.resolution)
            v = [math.floor((x - p.origin_x) / res), math.floor((y - p.origin_y) / res),
                 math.floor((ex - p.origin_x) / res), math.floor((ey - p.origin_y) / res)]
            if any(abs(c) >= 2 ** 30 for c in v):
                continue
            out.append((s * N + i, v[0], v[1], v[2], v[3], hit))
    return out


def line(sx, sy, ex, ey):
    """SPEC a5: closed-form Bresenham cells k = 0..n."""
    dx, dy = ex - sx, ey - sy
    adx, ady = abs(dx), abs(dy)
    ix = (dx > 0) - (dx < 0)
    iy = (dy > 0) - (dy < 0)
    n = max(adx, ady)
    cells = []
    for k in range(n + 1):
        if n == 0:
            cells.append((sx, sy))
        elif adx >= ady:
            cells.append((sx + k * ix, sy + iy * ((2 * k * ady + adx) // (2 * adx))))
        else:
            cells.append((sx + ix * ((2 * k * adx + ady) // (2 * ady)), sy + k * iy))
    return cells


def band_rows(p):
    return int(p.band_rows) if p.band_rows > 0 else int(p.height - p.band_row0)


def integrate(p, L, state, poses, ranges, angle_min, angle_increment):
    """SPEC a5-a7 on band arrays L (float32) / state (int8), in place."""
    W, H, r0, R = int(p.width), int(p.height), int(p.band_row0), band_rows(p)
    h = np.zeros((R, W), np.uint32)
    m = np.zeros((R, W), np.uint32)
    U = 0
    for _, sx, sy, ex, ey, hit in endpoints(p, poses, ranges, angle_min, angle_increment):
        cells = line(sx, sy, ex, ey)
        n = len(cells) - 1
        for k, (cx, cy) in enumerate(cells):
            if not (0 <= cx < W and 0 <= cy < H and r0 <= cy < r0 + R):
                continue
            if k == n and hit:
                h[cy - r0, cx] += 1
            else:
                m[cy - r0, cx] += 1
            U += 1
    touched = (h > 0) | (m > 0)
    f32 = np.float32
    t = h[touched].astype(f32) * f32(p.l_occ)
    u = m[touched].astype(f32) * f32(p.l_free)
    l = L[touched]
    l = (l + t).astype(f32)
    l = (l + u).astype(f32)
    l = np.minimum(np.maximum(l, f32(p.l_min)), f32(p.l_max))
    L[touched] = l
    state[touched] = state_of(p, l)
    return U, int(touched.sum())


def state_of(p, L):
    L = np.asarray(L, np.float32)
    s = np.full(L.shape, -1, np.int8)
    s[L >= np.float32(p.occ_thresh)] = 100
    s[(L <= np.float32(p.free_thresh)) & ~(L >= np.float32(p.occ_thresh))] = 0
    s[L == 0] = -1
    return s


def frontiers(p, state, halo_before=None, halo_after=None):
    """SPEC a8-a10 via numpy shifts + scipy.ndimage.label (8-connectivity)."""
    R, W = state.shape
    pad = np.zeros((R + 2, W + 2), np.int8)  # out-of-grid neighbours: not unknown
    pad[1:-1, 1:-1] = state
    if halo_before is not None:
        pad[0, 1:-1] = halo_before
    if halo_after is not None:
        pad[-1, 1:-1] = halo_after
    unk = np.zeros((R, W), bool)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy == 0 and dx == 0:
                continue
            unk |= pad[1 + dy:1 + dy + R, 1 + dx:1 + dx + W] == -1
    F = (state == 0) & unk
    lab, n = ndimage.label(F, structure=np.ones((3, 3), int))
    r0 = int(p.band_row0)
    labels = np.full((R, W), -1, np.int64)
    clusters = []
    if n:
        idx = np.arange(R * W, dtype=np.int64).reshape(R, W) + r0 * W
        ys, xs = np.nonzero(F)
        comp = lab[ys, xs] - 1
        minidx = np.full(n, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(minidx, comp, idx[ys, xs])
        labels[ys, xs] = minidx[comp]
        size = np.bincount(comp, minlength=n).astype(np.int64)
        sx = np.zeros(n, np.int64)
        sy = np.zeros(n, np.int64)
        np.add.at(sx, comp, xs.astype(np.int64))
        np.add.at(sy, comp, ys.astype(np.int64) + r0)
        order = np.argsort(minidx)
        for c in order:
            if size[c] < p.min_frontier_size:
                continue
            mx = float(sx[c]) / float(size[c])
            my = float(sy[c]) / float(size[c])
            clusters.append((int(minidx[c]), int(size[c]), int(sx[c]), int(sy[c]),
                             p.origin_x + (mx + 0.5) * p.resolution,
                             p.origin_y + (my + 0.5) * p.resolution))
    return F.astype(np.uint8), labels, clusters


def map_image(state):
    """get_map_image's mapping (main.py:258-266)."""
    img = np.full(state.shape, 127, np.uint8)
    img[state == 0] = 255
    img[state == 100] = 0
    return np.flipud(img)


def ld06_to_scan(points, n_beams, laser_scan_dir=True):
    """The LD06 driver's PointData -> LaserScan, float32
    arithmetic step by step in NumPy, points in order."""
    f32 = np.float32
    inc = (f32(6.2831855) - f32(0.0)) / f32(n_beams - 1)
    ranges = np.full(n_beams, np.nan, np.float32)
    inten = np.full(n_beams, np.nan, np.float32)
    for pt in points:
        d, it = int(pt["distance_mm"]), int(pt["intensity"])
        r = f32(d) / f32(1000.0)
        iv = f32(it)
        if d == 0 and it == 0:
            r, iv = f32(np.nan), f32(np.nan)
        ang = f32(float(np.float64(pt["angle_deg"])) * 3141.59 / 180000.0)
        q = (ang - f32(0.0)) / inc
        c = np.ceil(q)
        if not (c >= 0 and c < n_beams):
            continue
        idx = int(c)
        if laser_scan_dir:
            idx = n_beams - idx - 1
        if np.isnan(ranges[idx]) or ranges[idx] > r:
            ranges[idx] = r
        inten[idx] = iv
    return ranges, inten
