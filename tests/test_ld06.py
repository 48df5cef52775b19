"""LD06 PointData -> LaserScan.

CPU: the C restatement (oracle/dm_oracle.c) agrees with a step-by-step NumPy
restatement of the driver's ToLaserscanMessagePublish.  GPU: libdm's device
conversion (dm_ld06_to_scans) agrees with both, bit for bit (NaN in the same
beams)."""
import numpy as np
import pytest

import np_oracle
from dm._ffi import LD06_POINT_DTYPE


def random_points(seed, n, collide=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    pts = np.zeros(n, dtype=np.dtype(LD06_POINT_DTYPE))
    if collide:  # few distinct angles: many points share a beam
        pts["angle_deg"] = rng.choice(np.float32([0.0, 0.4, 90.0, 179.99, 359.9, 360.0]), n)
    else:
        pts["angle_deg"] = rng.uniform(0.0, 360.0, n).astype(np.float32)
    pts["distance_mm"] = rng.integers(0, 12000, n).astype(np.uint16)
    pts["intensity"] = rng.integers(0, 255, n).astype(np.uint8)
    z = rng.random(n) < 0.1
    pts["distance_mm"][z] = 0
    pts["intensity"][z & (rng.random(n) < 0.7)] = 0
    return pts


CASES = [(1, 450, 450, False), (2, 900, 450, True), (3, 4500, 4096, False), (4, 300, 12, True),
         (5, 60, 2, False)]


@pytest.mark.parametrize("seed,n,N,collide", CASES)
@pytest.mark.parametrize("direction", [True, False])
def test_oracle_matches_numpy(oracle_lib, seed, n, N, collide, direction):
    pts = random_points(seed, n, collide)
    r, i = oracle_lib.ld06_to_scans(pts, [0, n], N, direction)
    r2, i2 = np_oracle.ld06_to_scan(pts, N, direction)
    np.testing.assert_array_equal(r[0].view(np.uint32) * ~np.isnan(r[0]), r2.view(np.uint32) * ~np.isnan(r2))
    np.testing.assert_array_equal(np.isnan(r[0]), np.isnan(r2))
    np.testing.assert_array_equal(np.isnan(i[0]), np.isnan(i2))
    np.testing.assert_array_equal(np.nan_to_num(i[0]), np.nan_to_num(i2))


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [True, False])
def test_gpu_matches_oracle(oracle_lib, direction):
    import dm

    segs = [random_points(10 + k, n, collide=(k % 2 == 1)) for k, n in enumerate([450, 900, 0, 4500, 37])]
    pts = np.concatenate(segs)
    off = np.cumsum([0] + [len(s) for s in segs]).astype(np.int64)
    with dm.OccupancyMapper(dm.default_params(64, 64)) as m:
        for N in (450, 4096, 12):
            r, i = m.ld06_to_scans(pts, off, N, direction, want_intensities=True)
            er, ei = oracle_lib.ld06_to_scans(pts, off, N, direction)
            np.testing.assert_array_equal(np.isnan(r), np.isnan(er))
            np.testing.assert_array_equal(np.nan_to_num(r).view(np.uint32), np.nan_to_num(er).view(np.uint32))
            np.testing.assert_array_equal(np.isnan(i), np.isnan(ei))
            np.testing.assert_array_equal(np.nan_to_num(i), np.nan_to_num(ei))


@pytest.mark.gpu
def test_gpu_ld06_stream_into_map(oracle_lib):
    """Raw LD06 revolutions -> GPU scans -> GPU map equals the oracle chain."""
    import cases
    import dm
    from dm import synth

    p = cases.make_params(400, 400)
    world = synth.make_world(3, -10, -10, 10, 10)
    rng = np.random.Generator(np.random.PCG64(4))
    revs = [synth.ld06_points(world, 0.5 * k - 2, 0.3, 0.1 * k, rng) for k in range(8)]
    pts = np.concatenate(revs)
    off = np.cumsum([0] + [len(r) for r in revs]).astype(np.int64)
    N = 450
    poses = np.array([[0.5 * k - 2, 0.3, 0.1 * k] for k in range(8)])
    inc = float(synth.ld06_angle_increment(N))
    om = oracle_lib.OracleMap(p)
    er, _ = oracle_lib.ld06_to_scans(pts, off, N, True)
    with dm.OccupancyMapper(p) as m:
        r = m.ld06_to_scans(pts, off, N, True)
        np.testing.assert_array_equal(np.isnan(r), np.isnan(er))
        assert m.integrate(poses, r, 0.0, inc) == om.integrate(poses, er, 0.0, inc)
        np.testing.assert_array_equal(m.state(), om.state)


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [True, False])
def test_gpu_ld06_edge_angles_and_sizes(oracle_lib, direction):
    """Angles at and past the scan's ends (a hair below 0, 0, 359.999, 360,
    past 360, +-1e30, +-inf, NaN: out-of-range ones are dropped, as the
    driver's idx >= N / idx < 0 test does), the largest distance, zero
    distance with and without intensity, empty first and last revolutions,
    and the smallest and largest beam counts the boundary accepts."""
    import dm

    ang = np.float32([-0.001, 0.0, 0.0, 359.999, 360.0, 360.001, 1e30, -1e30, np.inf, -np.inf, np.nan, 180.0, 180.0])
    pts = np.zeros(ang.size, dtype=np.dtype(LD06_POINT_DTYPE))
    pts["angle_deg"] = ang
    pts["distance_mm"] = [5, 65535, 0, 12000, 1, 7, 9, 9, 9, 9, 9, 0, 3]
    pts["intensity"] = [1, 2, 0, 4, 5, 6, 7, 7, 7, 7, 7, 9, 0]
    segs = [pts[:0], pts, random_points(20, 500, collide=True), pts[::-1].copy(), pts[:0]]
    allp = np.concatenate(segs)
    off = np.cumsum([0] + [len(s) for s in segs]).astype(np.int64)
    with dm.OccupancyMapper(dm.default_params(64, 64)) as m:
        for N in (2, 3, 360, 8192):
            r, i = m.ld06_to_scans(allp, off, N, direction, want_intensities=True)
            er, ei = oracle_lib.ld06_to_scans(allp, off, N, direction)
            np.testing.assert_array_equal(np.isnan(r), np.isnan(er))
            np.testing.assert_array_equal(np.nan_to_num(r).view(np.uint32), np.nan_to_num(er).view(np.uint32))
            np.testing.assert_array_equal(np.isnan(i), np.isnan(ei))
            np.testing.assert_array_equal(np.nan_to_num(i), np.nan_to_num(ei))
            assert np.isnan(r[0]).all() and np.isnan(r[-1]).all()  # the empty revolutions
