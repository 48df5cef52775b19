"""GPU parity: libdm (HIP, gfx950) vs the CPU oracle, bit-exact.

L is compared bit for bit (the north-star tolerance is 1e-5 absolute; the
SPEC's fixed float32 op order without FMA makes it exact), state / mask /
labels / cluster integers exactly, centroids exactly (same double formula).
Run on the GPU box: python -m pytest tests -m gpu
"""
import os

import numpy as np
import pytest

import cases
import dm
from golden_io import load_case

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
LOGODDS_ATOL = 1e-5  # north_star; the comparison below is exact, which implies it


def assert_map_equal(m, om):
    L = m.logodds()
    np.testing.assert_allclose(L, om.L, rtol=0, atol=LOGODDS_ATOL)
    np.testing.assert_array_equal(L.view(np.uint32), om.L.view(np.uint32))
    np.testing.assert_array_equal(m.state(), om.state)


def assert_frontiers_equal(fr, mask, labels, clusters):
    if fr.mask is not None:
        np.testing.assert_array_equal(fr.mask, mask)
    if fr.labels is not None:
        np.testing.assert_array_equal(fr.labels, labels)
    np.testing.assert_array_equal(fr.clusters, clusters)


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLD, "oracle_golden.npz"))


@pytest.mark.parametrize("name", ["tiny64", "c1_room", "ragged", "offgrid"])
def test_golden_fixture(golden, name):
    c = load_case(golden, name)
    with dm.OccupancyMapper(c["params"]) as m:
        for k, (poses, ranges) in enumerate(c["batches"]):
            assert m.integrate(poses, ranges, c["amin"], c["inc"]) == tuple(c["counts"][k])
        L = m.logodds()
        np.testing.assert_array_equal(L.view(np.uint32), c["L"].view(np.uint32))
        np.testing.assert_array_equal(m.state(), c["state"])
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, c["mask"], c["labels"], c["clusters"])


@pytest.mark.parametrize("W,H,S,N,res,seed", [
    (64, 64, 1, 1, 0.05, 1),
    (400, 400, 8, 360, 0.05, 2),
    (130, 70, 5, 500, 0.05, 3),     # W % 4 != 0: scalar apply path, ragged tiles
    (257, 513, 16, 1024, 0.05, 4),  # ragged tiles in both axes
    (1000, 300, 32, 4096, 0.02, 5), # 12 m = 600 cells: long rays, many tiles per ray
    (96, 96, 12, 256, 0.1, 6),      # sensors far outside the map
])
def test_random_scans_vs_oracle(oracle_lib, W, H, S, N, res, seed):
    p = cases.make_params(W, H, resolution=res)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k in range(3):
            poses, ranges, amin, inc = cases.random_scans(seed * 100 + k, p, S, N,
                                                          spread=4.0 if seed == 6 else 1.0)
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert_map_equal(m, om)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())


def test_world_stream_c2_scale(oracle_lib):
    """C2 geometry (4096^2 @ 5 cm), single robot, scan-by-scan replay."""
    p, batches, amin, inc = cases.world_case(21, 4096, 4096, 0.05, 1, 450, 30, region_frac=0.05)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            fr = m.frontiers()
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())
        assert len(fr) > 0


def test_c3_full_size_batch(oracle_lib):
    """BASELINE C3 at full size: 16384^2 @ 5 cm, one 64-scan x 4096-beam batch
    from 64 robots; the oracle does this in seconds."""
    p, batches, amin, inc = cases.world_case(31, 16384, 16384, 0.05, 64, 4096, 1)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        poses, ranges = batches[0]
        got = m.integrate(poses, ranges, amin, inc)
        exp = om.integrate(poses, ranges, amin, inc)
        assert got == exp and got[0] > 10_000_000
        assert_map_equal(m, om)
        fr = m.frontiers()
        _, _, clusters = om.frontiers(want_mask=False, want_labels=False)
        np.testing.assert_array_equal(fr.clusters, clusters)


FRONTIER_STATE_CASES = [("random", 64, 64, 1), ("random", 200, 333, 2), ("blob", 700, 650, 3),
                        ("blob", 1, 300, 4), ("blob", 300, 1, 5), ("checker", 128, 192, 6),
                        ("stripes", 256, 256, 7), ("random", 1024, 1024, 8),
                        ("sparse", 400, 330, 9), ("sparse", 2048, 2048, 10)]


@pytest.mark.parametrize("kind,R,W,seed", FRONTIER_STATE_CASES)
def test_frontiers_on_states(oracle_lib, kind, R, W, seed):
    if kind == "random":
        st = cases.random_state(seed, R, W)
    elif kind == "blob":
        st = cases.blob_state(seed, R, W, n_blobs=40)
    elif kind == "checker":
        yy, xx = np.mgrid[0:R, 0:W]
        st = np.where((yy + xx) % 2 == 0, 0, -1).astype(np.int8)
    elif kind == "sparse":  # isolated free cells in unknown space: one cluster each
        rng = np.random.Generator(np.random.PCG64(seed))
        st = np.full((R, W), -1, np.int8)
        st[::3, ::3] = np.where(rng.random(st[::3, ::3].shape) < 0.9, 0, -1)
    else:  # long diagonal frontier stripes crossing many tiles
        yy, xx = np.mgrid[0:R, 0:W]
        st = np.where(((xx + yy) // 3) % 4 == 0, -1, 0).astype(np.int8)
    p = cases.make_params(W, R)
    om = oracle_lib.OracleMap(p)
    om.state[...] = st
    with dm.OccupancyMapper(p) as m:
        m.set_state(st)
        np.testing.assert_array_equal(m.state(), st)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())
        assert m.last_stats()["frontier_clusters"] == len(fr.clusters)


def test_frontier_band_with_halo(oracle_lib):
    W, H = 300, 640
    full = cases.blob_state(8, H, W, n_blobs=30)
    for r0, rows in [(0, 192), (192, 256), (448, 192), (128, 100), (64, 37)]:
        p = cases.make_params(W, H, band_row0=r0, band_rows=rows)
        om = oracle_lib.OracleMap(p)
        om.state[...] = full[r0:r0 + rows]
        hb = full[r0 - 1] if r0 > 0 else None
        ha = full[r0 + rows] if r0 + rows < H else None
        with dm.OccupancyMapper(p) as m:
            m.set_state(full[r0:r0 + rows])
            m.set_halo(hb, ha)
            fr = m.frontiers(want_mask=True, want_labels=True)
            mask, labels, clusters = om.frontiers(hb, ha)
            assert_frontiers_equal(fr, mask, labels, clusters)
            first, last = m.edge_labels()
            np.testing.assert_array_equal(first, labels[0])
            np.testing.assert_array_equal(last, labels[-1])


def test_edge_cases(oracle_lib):
    p = cases.make_params(200, 120)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        # empty batch, then empty map: no frontiers
        assert m.integrate(np.zeros((0, 3)), np.zeros((0, 5), np.float32), 0.0, 0.1) == (0, 0)
        assert len(m.frontiers()) == 0
        # all-NaN / too-short ranges: skipped
        poses = np.array([[0.0, 0.0, 0.3]])
        for bad in (np.nan, 0.0, 0.019):
            assert m.integrate(poses, np.full((1, 50), bad, np.float32), 0.0, 0.1) == (0, 0)
        # single beam, non-finite pose skipped
        poses = np.array([[0.1, 0.2, 0.0], [np.nan, 0.0, 0.0], [0.0, 0.0, np.inf]])
        r = np.full((3, 1), 3.0, np.float32)
        assert m.integrate(poses, r, 0.0, 0.0) == om.integrate(poses, r, 0.0, 0.0)
        # exactly range_max (hit) and just beyond (truncated, no hit)
        r = np.array([[12.0, np.nextafter(np.float32(12.0), np.float32(20.0)), np.inf]], np.float32)
        poses = np.array([[-1.0, 0.5, 0.2]])
        assert m.integrate(poses, r, 0.1, 2.0) == om.integrate(poses, r, 0.1, 2.0)
        assert_map_equal(m, om)
        # saturation: many hits on the same cells clamp at l_max / l_min
        poses = np.tile(np.array([[0.0, 0.0, 0.0]]), (64, 1))
        r = np.full((64, 64), 1.0, np.float32)
        for _ in range(3):
            assert m.integrate(poses, r, 0.0, 0.01) == om.integrate(poses, r, 0.0, 0.01)
        assert_map_equal(m, om)
        assert m.logodds().max() == np.float32(3.5) and m.logodds().min() == np.float32(-2.0)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


def test_deterministic_and_order_independent(oracle_lib):
    p = cases.make_params(512, 512)
    poses, ranges, amin, inc = cases.random_scans(77, p, 32, 1024)
    perm = np.random.Generator(np.random.PCG64(1)).permutation(32)
    outs = []
    for order in (np.arange(32), np.arange(32), perm):
        with dm.OccupancyMapper(p) as m:
            m.integrate(poses[order], ranges[order], amin, inc)
            outs.append((m.logodds(), m.state(), m.frontiers(want_labels=True)))
    for L, st, fr in outs[1:]:
        np.testing.assert_array_equal(L.view(np.uint32), outs[0][0].view(np.uint32))
        np.testing.assert_array_equal(st, outs[0][1])
        np.testing.assert_array_equal(fr.labels, outs[0][2].labels)
        np.testing.assert_array_equal(fr.clusters, outs[0][2].clusters)


def test_device_entry_point_matches_host(oracle_lib):
    import torch

    p = cases.make_params(640, 480)
    poses, ranges, amin, inc = cases.random_scans(5, p, 16, 720)
    from dm import synth
    pose4 = torch.from_numpy(synth.pose4(poses)).cuda()
    rng_d = torch.from_numpy(ranges).cuda()
    om = oracle_lib.OracleMap(p)
    exp = om.integrate(poses, ranges, amin, inc)
    with dm.OccupancyMapper(p) as m:
        torch.cuda.synchronize()
        m.integrate_device(pose4.data_ptr(), 16, rng_d.data_ptr(), 720, amin, inc)
        assert m.last_counts() == exp
        assert_map_equal(m, om)


def test_checkpoint_roundtrip(tmp_path, oracle_lib):
    p = cases.make_params(300, 200)
    poses, ranges, amin, inc = cases.random_scans(9, p, 8, 300)
    with dm.OccupancyMapper(p) as a:
        a.integrate(poses, ranges, amin, inc)
        a.save(str(tmp_path / "m.dmap"))
        poses2, ranges2, _, _ = cases.random_scans(10, p, 8, 300)
        a.integrate(poses2, ranges2, amin, inc)
        with dm.OccupancyMapper(p) as b:
            b.load(str(tmp_path / "m.dmap"))
            b.integrate(poses2, ranges2, amin, inc)
            np.testing.assert_array_equal(a.logodds().view(np.uint32), b.logodds().view(np.uint32))
            np.testing.assert_array_equal(a.frontiers().clusters, b.frontiers().clusters)
    with dm.OccupancyMapper(cases.make_params(100, 100)) as c:
        with pytest.raises(dm.DmError):
            c.load(str(tmp_path / "m.dmap"))


def test_map_image_matches_reference_golden():
    d = np.load(os.path.join(GOLD, "map_image_golden.npz"))
    n = len([k for k in d.files if k.startswith("state_")])
    for i in range(n):
        st = d[f"state_{i}"]
        with dm.OccupancyMapper(cases.make_params(st.shape[1], st.shape[0])) as m:
            m.set_state(np.where(np.isin(st, (-1, 0, 100)), st, -1).astype(np.int8))
            img = m.map_image()
        exp = d[f"image_{i}"]
        ok = np.isin(st, (-1, 0, 100))  # set_state stores only the three states
        np.testing.assert_array_equal(img[np.flipud(ok)], exp[np.flipud(ok)])


def test_profiling_counters():
    p = cases.make_params(256, 256)
    poses, ranges, amin, inc = cases.random_scans(3, p, 4, 256)
    with dm.OccupancyMapper(p) as m:
        m.profile(True)
        m.integrate(poses, ranges, amin, inc)
        m.frontiers()
        st = m.profile_read()
    assert st["tile_accum"][0] == 1 and st["tile_accum"][1] > 0
    assert "frontier_tile" in st


def _window_world(seed, p, n_robots, n_beams, x0, y0, x1, y1, n_batches):
    from dm import synth
    world = synth.make_world(seed, x0 - 15, y0 - 15, x1 + 15, y1 + 15)
    stream = synth.ScanStream(world, n_robots, n_beams, seed + 1, region=(x0, y0, x1, y1))
    return [stream.next_batch() for _ in range(n_batches)]


def test_c5_geometry_band_near_top(oracle_lib):
    """C5 geometry (65536^2 @ 1 cm, rays of 1200 cells): a 2048-row band near
    the top of the map, so global linear indices exceed 2^31 (int64 labels)."""
    from dm import synth
    W = H = 65536
    res = 0.01
    r0, rows = 62464, 2048
    p = cases.make_params(W, H, resolution=res, band_row0=r0, band_rows=rows)
    y0 = p.origin_y + (r0 + 300) * res
    y1 = p.origin_y + (r0 + rows - 300) * res
    batches = _window_world(51, p, 6, 4096, -3.0, y0, 3.0, y1, 2)
    amin, inc = 0.0, float(synth.ld06_angle_increment(4096))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert_map_equal(m, om)
        fr = m.frontiers(want_mask=True, want_labels=True)
        mask, labels, clusters = om.frontiers()
        assert_frontiers_equal(fr, mask, labels, clusters)
        assert len(clusters) and clusters["label"].max() > 2 ** 31  # beyond int32


@pytest.mark.parametrize("N", [12, 48, 192, 768, 4096])
def test_c5_beam_density_sweep(oracle_lib, N):
    """C5 scan-density sweep (12 .. 4096 beams per scan) on a 1 cm band."""
    from dm import synth
    W, H, res = 65536, 65536, 0.01
    r0, rows = 30720, 2560
    p = cases.make_params(W, H, resolution=res, band_row0=r0, band_rows=rows)
    y0 = p.origin_y + (r0 + 100) * res
    y1 = p.origin_y + (r0 + rows - 100) * res
    batches = _window_world(60 + N, p, 8, N, -10.0, y0, 10.0, y1, 2)
    amin, inc = 0.0, float(synth.ld06_angle_increment(N))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(), None, None, om.frontiers(want_mask=False,
                                                                         want_labels=False)[2])


@pytest.mark.parametrize("S", [15, 17])
def test_colocated_scans_heavy_slab_widths(oracle_lib, S):
    """S scans of 4096 beams from one pose in one call: the sensor's tile gets
    S*4096 pieces, so its cells' counts approach (S=15: 61440, packed 16-bit
    slab) or exceed (S=17: 69632, wide slab) 65535 (csrc/dm_integrate.hip,
    k_plan's per-tile slab width)."""
    p = cases.make_params(300, 300)
    rng = np.random.Generator(np.random.PCG64(7 + S))
    poses = np.tile(np.array([[0.013, -0.021, 0.3]]), (S, 1))
    poses[:, 2] += rng.uniform(-0.01, 0.01, S)
    N = 4096
    ranges = (np.round(rng.uniform(0.05, 8.0, (S, N)) * 1000) / 1000).astype(np.float32)
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k in range(2):
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        st = m.last_stats()
        assert st["heavy_tiles"] >= 1
        assert_map_equal(m, om)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())


@pytest.mark.parametrize("S,N", [(1, 360), (1, 512), (1, 513), (2, 256), (1, 1100), (3, 400)])
def test_heavy_apply_skip_boundary(oracle_lib, S, N):
    """Co-located scans around the bound below which no tile can be heavy
    (a tile gets <= 1 piece per beam, <= 2 when beams are chunked: no tile can
    exceed kMedium = 1024 pieces).  Above the bound the sensor tile may be
    heavy and must be applied."""
    p = cases.make_params(700, 600, resolution=0.02)
    rng = np.random.Generator(np.random.PCG64(100 + N + S))
    poses = np.tile(np.array([[0.011, 0.017, 0.2]]), (S, 1))
    ranges = (np.round(rng.uniform(0.05, 6.0, (S, N)) * 1000) / 1000).astype(np.float32)
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k in range(2):
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        if S * N > 1024:
            assert m.last_stats()["heavy_tiles"] >= 1
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


@pytest.mark.parametrize("S", [6, 17])
def test_heavy_apply_ticket(oracle_lib, S):
    """Heavy tiles applied by their last k_tile_accum item (the ticket in
    heavy_done): bit-exact against the oracle over several calls (the
    tickets are reset by the finisher for the next call), with three sensors
    sharing the batch (several heavy tiles per call; S=17 puts > 65535
    pieces on one tile: wide slab)."""
    p = cases.make_params(500, 400)
    rng = np.random.Generator(np.random.PCG64(31 + S))
    centres = np.array([[0.013, -0.021, 0.3], [4.41, 2.07, 1.1], [-6.3, -3.9, 2.0]])
    N = 4096
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k in range(3):
            poses = centres[np.arange(S) % 3 if S < 17 else np.zeros(S, int)].copy()
            poses[:, 2] += rng.uniform(-0.01, 0.01, S)
            ranges = (np.round(rng.uniform(0.05, 8.0, (S, N)) * 1000) / 1000).astype(np.float32)
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            assert m.last_stats()["heavy_tiles"] >= (1 if S >= 17 else 3)
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


def test_heavy_ticket_under_uneven_load(oracle_lib):
    """The fused heavy apply's ticket hand-off (csrc/dm_integrate.hip,
    k_tile_accum) while another stream keeps CUs busy with long GEMMs, so
    the heavy items of one tile run on different XCDs at very different
    times: 12 calls, each bit-exact against the oracle (17 co-located scans:
    wide slabs; one sensor tile split into 272 items)."""
    import torch

    p = cases.make_params(600, 500)
    rng = np.random.Generator(np.random.PCG64(2024))
    N = 4096
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    om = oracle_lib.OracleMap(p)
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    with dm.OccupancyMapper(p) as m:
        for k in range(12):
            with torch.cuda.stream(side):
                for _ in range(3 + k % 4):
                    a = torch.tanh(a @ a * 1e-3)
            S = 17 if k % 2 == 0 else 9
            poses = np.tile(np.array([[0.013 + 0.3 * k, -0.021, 0.3]]), (S, 1))
            poses[:, 2] += rng.uniform(-0.01, 0.01, S)
            ranges = (np.round(rng.uniform(0.05, 8.0, (S, N)) * 1000) / 1000).astype(np.float32)
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            assert m.last_stats()["heavy_tiles"] >= 1
            np.testing.assert_array_equal(m.logodds().view(np.uint32), om.L.view(np.uint32))
        torch.cuda.synchronize()
        assert_map_equal(m, om)


@pytest.mark.parametrize("sparse", ["0", "8", "15", "256"])
def test_sparse_items_threshold(oracle_lib, monkeypatch, sparse):
    """Light tiles with at most DM_SPARSE_PIECES pieces are sparse items
    (two per workgroup, byte-packed counts; walk first, then load only the
    touched cells; listed from the top of the light list).  0: none; the
    library caps the threshold at 15 pieces (one byte of counts per cell), so
    256 behaves as 15.  1 cm map with few beams per
    scan (C5's sparse end) and ragged edge tiles; fmask records forced on so
    k_fmask_items covers the sparse range too."""
    monkeypatch.setenv("DM_SPARSE_PIECES", sparse)
    monkeypatch.setenv("DM_FMASK", "on")
    for W, H, S, N, res, seed in [(1000, 900, 16, 12, 0.01, 41), (130, 70, 5, 64, 0.05, 42),
                                  (2050, 1030, 32, 48, 0.01, 43)]:
        p = cases.make_params(W, H, resolution=res)
        om = oracle_lib.OracleMap(p)
        with dm.OccupancyMapper(p) as m:
            for k in range(4):
                poses, ranges, amin, inc = cases.random_scans(seed * 100 + k, p, S, N)
                assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            assert_map_equal(m, om)
            fr = m.frontiers(want_mask=True, want_labels=True)
            assert_frontiers_equal(fr, *om.frontiers())


def test_geometry_edge_cases(oracle_lib):
    """Ray geometry at its degenerate points, bit-exact against the oracle:
    beams along the axes and the diagonals (yaw multiples of pi/4: Bresenham's
    ties), sensors on cell corners with ranges that end exactly on cell
    boundaries, negative / -inf / subnormal ranges (skipped as too short),
    sensors far outside the map whose rays cross it or miss it, and sensors
    on the map's last row / column."""
    res = np.float32(0.05)
    p = cases.make_params(160, 96, resolution=float(res), origin=(-4.0, -2.4))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        def both(poses, ranges, amin, inc):
            poses = np.asarray(poses, np.float64)
            ranges = np.asarray(ranges, np.float32)
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)

        # eight beams at yaw + k * pi/4 from cell corners, lengths on cell boundaries
        corners = [[0.0, 0.0, 0.0], [0.05, -0.05, 0.0], [1.0, 1.0, np.pi / 2], [-2.0, 0.5, np.pi]]
        lens = np.float32([0.05, 0.1, 0.25, 1.0, 1.5, 2.0, 0.5, 3.0])
        both(corners, np.tile(lens, (4, 1)), 0.0, float(np.float32(np.pi / 4)))
        # the same from cell centres, and just off the corners
        both([[0.025, 0.025, 0.0], [1e-9, -1e-9, 0.0]], np.tile(lens, (2, 1)), 0.0, float(np.float32(np.pi / 4)))
        # negative, -inf, subnormal and zero ranges among valid ones
        bad = np.float32([-1.0, -np.inf, 1e-40, 0.0, 2.0, -0.0, 0.0199, 0.02])
        both([[0.3, 0.2, 0.1]], bad[None, :], 0.0, 0.7)
        # sensors far outside the map: rays crossing it, ending inside it, missing it
        far = [[-9.0, 0.0, 0.0], [0.0, -7.5, np.pi / 2], [9.5, 3.0, np.pi], [-9.0, -9.0, np.pi / 4]]
        rr = np.float32([[12.0, 6.0, 11.9, 3.0]] * 4)
        both(far, rr, -0.05, 0.05)
        # sensors on the last row / column and on the map's corner cells
        W, H = 160 * res, 96 * res
        edge = [[-4.0 + W - 0.01, 0.0, 0.3], [0.0, -2.4 + H - 0.01, -1.2], [-3.99, -2.39, 0.8],
                [-4.0 + W - 0.01, -2.4 + H - 0.01, 3.5]]
        both(edge, np.full((4, 90), 2.5, np.float32), -np.pi, float(np.float32(2 * np.pi / 90)))
        assert_map_equal(m, om)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())


def spiral_state(n, gap=2):
    """A one-cell-wide free spiral in unknown space, `gap` cells between its
    turns: every free cell is a frontier cell and the whole spiral is ONE
    8-connected component that winds through every tile many times, the
    longest tile-to-tile union chains a map of this size can hold."""
    st = np.full((n, n), -1, np.int8)
    lo, hi = 0, n - 1
    y = x = 0
    while lo <= hi:
        st[lo, lo:hi + 1] = 0                      # top row, left to right
        st[lo:hi + 1, hi] = 0                      # right column, down
        if hi - lo <= gap:
            break
        st[hi, lo + gap - 1:hi + 1] = 0            # bottom row, right to left
        st[lo + gap:hi + 1, lo + gap - 1] = 0      # left column, up (stops short of the top row)
        lo += gap
        hi -= gap
        st[lo, lo - 1:lo + 1] = 0                  # step into the next turn
    return st


@pytest.mark.parametrize("n", [300, 1536])
def test_frontiers_on_spiral(oracle_lib, n):
    import time

    st = spiral_state(n)
    p = cases.make_params(n, n)
    om = oracle_lib.OracleMap(p)
    om.state[...] = st
    expect = om.frontiers()
    with dm.OccupancyMapper(p) as m:
        m.set_state(st)
        m.frontiers()  # first pass: lists, grids, hints
        t0 = time.perf_counter()
        fr = m.frontiers(want_mask=True, want_labels=True)
        dt = time.perf_counter() - t0
        assert_frontiers_equal(fr, *expect)
    assert len(expect[2]) >= 1
    assert dt < 0.5, f"spiral frontier pass took {dt:.3f} s"
