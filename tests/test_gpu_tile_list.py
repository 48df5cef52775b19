"""GPU: the persistent frontier tile list (dm_internal.h `ftiles`): every
tile that has held a free cell since the last rebuild, appended by the
integrate apply when a tile's free count first rises above 0 (listed flag in
`tile_free`), rebuilt in tile order by k_list_tiles after bulk writes
(dm_set_state, dm_set_logodds, dm_reset, dm_load) and periodically (after 1,
2, 4, 8 passes, then every 16).  A pass's `frontier_tiles` statistic is its
snapshot of the list length: at least the tiles holding a free cell, at most
the tiles that held one since the last bulk write; tiles that lost every free
cell stay listed until the next rebuild without changing any result, and a
rebuild drops them (flag cleared, so a tile that regains a free cell is
appended again)."""
import numpy as np
import pytest

import cases
import dm
from test_gpu_parity import assert_frontiers_equal, assert_map_equal

pytestmark = pytest.mark.gpu


def _tiles_with_free(st):
    H, W = st.shape
    TY, TX = -(-H // 64), -(-W // 64)
    pad = np.full((TY * 64, TX * 64), 1, np.int8)
    pad[:H, :W] = st
    return (pad.reshape(TY, 64, TX, 64) == 0).any(axis=(1, 3))


def test_list_grows_with_every_tile_that_held_a_free_cell(oracle_lib):
    p, batches, amin, inc = cases.world_case(71, 1100, 900, 0.05, 12, 1500, 6, region_frac=0.8)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        ever = np.zeros_like(_tiles_with_free(om.state))
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            ever |= _tiles_with_free(om.state)
            fr = m.frontiers()
            np.testing.assert_array_equal(fr.clusters, om.frontiers(want_mask=False, want_labels=False)[2])
            n = m.last_stats()["frontier_tiles"]
            assert int(_tiles_with_free(om.state).sum()) <= n <= int(ever.sum())
        assert_map_equal(m, om)


def test_bulk_writes_rebuild_the_list(oracle_lib):
    """set_state lists exactly the tiles with free cells; tiles whose free
    cells all turn occupied stay listed; a map set back to unknown lists
    nothing; reset likewise."""
    p = cases.make_params(700, 520)
    rng = np.random.Generator(np.random.PCG64(5))
    st = np.full((520, 700), -1, np.int8)
    st[100:300, 50:400] = 0
    st[120:140, 60:200] = 100
    st[rng.random(st.shape) < 0.01] = 0
    om = oracle_lib.OracleMap(p)
    om.L[...] = np.where(st == 100, np.float32(p.l_occ), np.where(st == 0, np.float32(p.l_free), np.float32(0)))
    om.state[...] = st
    with dm.OccupancyMapper(p) as m:
        m.set_state(st)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())
        assert m.last_stats()["frontier_tiles"] == int(_tiles_with_free(st).sum())
        # every free cell of one tile row band turns occupied through the
        # integrate path is hard to arrange; a bulk write re-lists instead
        st2 = st.copy()
        st2[100:300, 50:400][st2[100:300, 50:400] == 0] = 100
        m.set_state(st2)
        om.L[...] = np.where(st2 == 100, np.float32(p.l_occ),
                             np.where(st2 == 0, np.float32(p.l_free), np.float32(0)))
        om.state[...] = st2
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *om.frontiers())
        assert m.last_stats()["frontier_tiles"] == int(_tiles_with_free(st2).sum())
        m.set_logodds(np.zeros((520, 700), np.float32))
        fr = m.frontiers()
        assert len(fr.clusters) == 0 and m.last_stats()["frontier_tiles"] == 0
        m.set_state(st)
        m.reset()
        fr = m.frontiers()
        assert len(fr.clusters) == 0 and m.last_stats()["frontier_tiles"] == 0


def test_listed_tiles_that_lose_their_free_cells(oracle_lib):
    """Scans from one spot: early batches free a region, later batches with
    the same rays hitting close by turn part of it occupied; the tiles stay
    on the list (no result changes) and the pipelined passes match."""
    p = cases.make_params(640, 640)
    N = 2048
    amin, inc = 0.0, float(np.float32(2 * np.pi / (N - 1)))
    rng = np.random.Generator(np.random.PCG64(9))
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        got, exp = [], []
        for k in range(8):
            poses = np.array([[0.3, -0.2, 0.1 * k], [3.1, 2.2, -0.4 * k]])
            far = 9.0 if k < 3 else 1.2  # later batches: short ranges, hits inside the freed region
            ranges = (np.round(rng.uniform(0.5, far, (2, N)) * 1000) / 1000).astype(np.float32)
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            if k >= 2:
                got.append(m.frontiers_end())
            m.frontiers_begin()
            exp.append(om.frontiers(want_mask=False, want_labels=False)[2])
        got += [m.frontiers_end(), m.frontiers_end()]
        for fr, e in zip(got, exp):
            np.testing.assert_array_equal(fr.clusters, e)
        assert_map_equal(m, om)


def test_periodic_rebuilds_keep_results(oracle_lib):
    """40 pipelined passes (two periodic rebuilds, with passes in flight),
    rays that free cells early and occupy some of them later: every pass
    equals the oracle's frontiers of its own batch."""
    p, batches, amin, inc = cases.world_case(73, 900, 800, 0.05, 6, 720, 40, region_frac=0.8)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        got, exp = [], []
        for k, (poses, ranges) in enumerate(batches):
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            if k >= 2:
                got.append(m.frontiers_end())
            m.frontiers_begin()
            exp.append(om.frontiers(want_mask=False, want_labels=False)[2])
        got += [m.frontiers_end(), m.frontiers_end()]
        for fr, e in zip(got, exp):
            np.testing.assert_array_equal(fr.clusters, e)
        assert_map_equal(m, om)
