"""GPU: the direct integrate front-end (k_scan_plan -> k_direct_accum,
csrc/dm_integrate.hip; dm_set_integrate_mode) against the CPU oracle, bit for
bit, and against the binned front-end on the same calls.

The direct form finds each beam's pieces per scan tile from the beams whose
angle reaches the tile (a superset) and their exact k-ranges; the CPU
emulation checks that it finds exactly the binned pieces
(test_emulated_kernels.py).  Here: the device kernels on cases that exercise
every branch — exclusive tiles, tiles reached by several scans (one unit
list), heavy sensor tiles split over workgroups and merged in a slab (packed
and wide), region-A spills, bands, ragged maps, scanner layouts other than
the LD06's, host inputs with overlap (per-set staging), mode switches."""
import numpy as np
import pytest

import cases
import dm
from test_gpu_parity import assert_frontiers_equal, assert_map_equal
from test_gpu_pipeline import _device_batches, _oracle_steps

pytestmark = pytest.mark.gpu


def _run(m, om, batches, amin, inc, expect_direct=True):
    for poses, ranges in batches:
        assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert m.last_integrate_direct() == expect_direct
    assert_map_equal(m, om)
    assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


@pytest.mark.parametrize("W,H,S,N,res,seed,r0,rows", [
    (400, 400, 8, 360, 0.05, 2, 0, 0),
    (130, 70, 5, 500, 0.05, 3, 0, 0),       # W % 4 != 0, ragged tiles
    (257, 513, 16, 1024, 0.05, 4, 0, 0),
    (1000, 300, 32, 4096, 0.02, 5, 0, 0),   # long rays (600 cells)
    (300, 700, 8, 600, 0.05, 7, 320, 192),  # a band
    (700, 500, 3, 3000, 0.01, 8, 128, 0),   # 1 cm, a band from row 128
])
def test_direct_random_scans(oracle_lib, W, H, S, N, res, seed, r0, rows):
    p = cases.make_params(W, H, resolution=res, band_row0=r0, band_rows=rows)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_integrate_mode("direct")
        batches = []
        for k in range(3):
            poses, ranges, amin, inc = cases.random_scans(seed * 10 + k, p, S, N, spread=1.0)
            batches.append((poses, ranges))
        _run(m, om, batches, amin, inc)


@pytest.mark.parametrize("S", [3, 17, 40])
def test_direct_colocated_sensors(oracle_lib, S):
    """Sensors at a few spots: every tile near them is reached by several
    scans (one unit list), the sensor tiles are heavy (chunks + slab); S=17
    and 40 at one spot put more than 65535 candidates on a tile (wide slab),
    and 40 heavy units overflow region A into region B."""
    p = cases.make_params(500, 400)
    rng = np.random.Generator(np.random.PCG64(77 + S))
    centres = np.array([[0.013, -0.021, 0.3], [4.41, 2.07, 1.1], [-6.3, -3.9, 2.0]])
    N = 4096
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        batches = []
        for k in range(3):
            idx = np.arange(S) % 3 if S < 17 else np.zeros(S, int)
            poses = centres[idx].copy()
            poses[:, 2] += rng.uniform(-0.5, 0.5, S)
            poses[:, :2] += rng.uniform(-0.04, 0.04, (S, 2))  # sensors near tile corners too
            ranges = (np.round(rng.uniform(0.05, 8.0, (S, N)) * 1000) / 1000).astype(np.float32)
            batches.append((poses, ranges))
        m.set_integrate_mode("direct")
        _run(m, om, batches, amin, inc)
        assert m.last_stats()["heavy_tiles"] >= 1


def test_direct_sensor_on_tile_corners(oracle_lib):
    """Sensors exactly on tile corners / edges (a sensor in up to four widened
    tile boxes: four heavy units of one scan)."""
    p = cases.make_params(512, 512)  # origin -12.8: tile corners every 3.2 m
    N = 2048
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    rng = np.random.Generator(np.random.PCG64(5))
    xs = [-9.6, -6.4, -3.2, 0.0, 3.2, 6.4, 9.6, -9.6 + 0.001, 3.2 - 0.001, 0.05]
    poses = np.array([[x, y, rng.uniform(-3, 3)] for x, y in zip(xs, xs[::-1])])
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_integrate_mode("direct")
        batches = [(poses, (np.round(rng.uniform(0.02, 13.0, (len(xs), N)) * 1000) / 1000).astype(np.float32))
                   for _ in range(2)]
        _run(m, om, batches, amin, inc)


@pytest.mark.parametrize("amin,span,N", [(-2.356194490192345, 4.71238898038469, 1081), (1.0, 6.283185307179586, 1440),
                                          (-3.0, 9.0, 1200)])
def test_direct_scanner_layouts(oracle_lib, amin, span, N):
    p = cases.make_params(384, 320, resolution=0.03)
    amin32 = float(np.float32(amin))
    inc32 = float(np.float32(span / (N - 1)))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_integrate_mode("direct")
        batches = []
        for k in range(3):
            poses, ranges, _, _ = cases.random_scans(900 + k, p, 6, N, spread=0.5)
            batches.append((poses, ranges))
        _run(m, om, batches, amin32, inc32)


def test_direct_and_binned_agree_and_switch(oracle_lib):
    """auto picks direct for dense scans that fill the chip unchunked
    (32 x 4096 beams), binned for sparse ones; switching modes between calls
    leaves every per-tile array at rest."""
    p, batches, amin, inc = cases.world_case(61, 1024, 1024, 0.05, 32, 4096, 3, region_frac=0.6)
    _, sparse, amin_s, inc_s = cases.world_case(62, 1024, 1024, 0.05, 8, 360, 2, region_frac=0.6)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k, (poses, ranges) in enumerate(batches):
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            assert m.last_integrate_direct()  # auto: 4096 beams, 32 scans
            poses_s, ranges_s = sparse[k % 2]
            assert m.integrate(poses_s, ranges_s, amin_s, inc_s) == om.integrate(poses_s, ranges_s, amin_s, inc_s)
            assert not m.last_integrate_direct()  # auto: 360 beams
        m.set_integrate_mode("binned")
        poses, ranges = batches[0]
        assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert not m.last_integrate_direct()
        m.set_integrate_mode("direct")
        poses_s, ranges_s = sparse[0]
        assert m.integrate(poses_s, ranges_s, amin_s, inc_s) == om.integrate(poses_s, ranges_s, amin_s, inc_s)
        assert m.last_integrate_direct()
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


def test_direct_pipelined_device_and_host_inputs(oracle_lib):
    """Overlap on (front-end stream + gate): pipelined passes over direct
    calls from device inputs, then from host inputs through the per-set
    device staging (the accumulation reads the inputs on the map stream)."""
    p, batches, amin, inc = cases.world_case(63, 2048, 2048, 0.05, 16, 4096, 6, region_frac=0.6)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    dev = _device_batches(batches)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        m.set_integrate_mode("direct")  # 16 x 4096 beams: auto would chunk them (binned)
        got = []
        for k, (pose4, rng) in enumerate(dev):
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), rng.shape[1], amin, inc)
            if k >= 2:
                got.append(m.frontiers_end())
            m.frontiers_begin()
        got += [m.frontiers_end(), m.frontiers_end()]
        assert m.last_integrate_direct()
        for fr, exp in zip(got, expect):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, exp)
        assert_map_equal(m, om)
        # host inputs, several calls in flight before any synchronising call
        m.reset()
        om2 = oracle_lib.OracleMap(p)
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om2.integrate(poses, ranges, amin, inc)
        assert_map_equal(m, om2)


def test_direct_async_host_inputs_overlap(oracle_lib):
    """dm_integrate_async with overlap: each call's inputs are copied into its
    workspace set's device buffers after that set's last accumulation; three
    calls are queued before the first synchronising call."""
    import torch

    p, batches, amin, inc = cases.world_case(64, 1536, 1536, 0.05, 12, 4096, 5, region_frac=0.6)
    om = oracle_lib.OracleMap(p)
    pinned = [torch.from_numpy(np.ascontiguousarray(r, np.float32)).pin_memory() for _, r in batches]
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        m.set_integrate_mode("direct")
        for k, (poses, ranges) in enumerate(batches):
            m.integrate_async(poses, pinned[k].data_ptr(), poses.shape[0], ranges.shape[1], amin, inc)
            om.integrate(poses, ranges, amin, inc)
        m.synchronize()
        assert m.last_integrate_direct()
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())
