"""GPU: both ways of uniting frontier components across tile edges give the
oracle's frontiers: in the tile kernels through the stamped
hand-off words (dense passes, forced with DM_FRONTIER_KERNEL=wg) and in
k_frontier_edges after publish-only tile kernels (sparse passes, forced with
DM_FRONTIER_KERNEL=wave, where run-rich tiles still go to the 256-thread
kernel beside the wave kernel).  Passes of both kinds alternate on one handle
(the two encodings live in separate halves of the hand-off array), on a
single map, pipelined, and on a sharded handle whose band edges are halos."""
import numpy as np
import pytest

import cases
import dm
from test_gpu_parity import assert_frontiers_equal, assert_map_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", ["wave", "wg"])
@pytest.mark.parametrize("W,H,seed,res", [(900, 700, 71, 0.05), (1500, 1100, 72, 0.02)])
def test_edge_modes_match_oracle(oracle_lib, monkeypatch, kernel, W, H, seed, res):
    monkeypatch.setenv("DM_FRONTIER_KERNEL", kernel)
    p, batches, amin, inc = cases.world_case(seed, W, H, res, 6, 1024, 4, region_frac=0.8)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for k, (poses, ranges) in enumerate(batches):
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
            fr = m.frontiers(want_mask=k % 2 == 0, want_labels=k % 2 == 0)
            assert_frontiers_equal(fr, *om.frontiers(want_mask=k % 2 == 0, want_labels=k % 2 == 0))
        assert_map_equal(m, om)


def test_edge_modes_alternate_on_one_handle(oracle_lib):
    """Pipelined passes under the automatic choice, which picks the edge
    kernel or the in-kernel unions per pass from the last collected pass
    (a growing map can change kind between passes): every pass equals the
    oracle's, whichever kind it and its predecessors were."""
    p, batches, amin, inc = cases.world_case(73, 1024, 1024, 0.05, 12, 2048, 8, region_frac=0.5)
    om = oracle_lib.OracleMap(p)
    expect = []
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        got = []
        for k, (poses, ranges) in enumerate(batches):
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            expect.append(om.frontiers(want_mask=False, want_labels=False)[2])
            if k >= 2:
                got.append(m.frontiers_end())
            m.frontiers_begin()
        got += [m.frontiers_end(), m.frontiers_end()]
        for k, fr in enumerate(got):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, expect[k])
        assert_map_equal(m, om)


@pytest.mark.parametrize("kernel", ["wave", "wg"])
def test_edge_modes_on_band_handles(oracle_lib, monkeypatch, kernel):
    monkeypatch.setenv("DM_FRONTIER_KERNEL", kernel)
    p, batches, amin, inc = cases.world_case(74, 640, 900, 0.05, 6, 720, 3, region_frac=0.9)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p, devices=[0, 0, 0]) as sh:
        for poses, ranges in batches:
            assert sh.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        assert_frontiers_equal(sh.frontiers(want_mask=True, want_labels=True), *om.frontiers())


def test_sparse_item_stat(oracle_lib):
    """dm_last_stats out[10]: the call's sparse work items (light tiles with at
    most 15 pieces) -- a 12-beam scan set on a 1 cm map is almost all sparse
    tiles, a dense fan has few; never more than the active tiles (a tile is
    one item of one kind) and counted in the work items too.  The map itself
    stays bit-exact."""
    p, batches, amin, inc = cases.world_case(75, 1200, 1000, 0.01, 8, 12, 2, region_frac=0.8)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        for poses, ranges in batches:
            assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
        st = m.last_stats()
        assert 0 < st["sparse_items"] <= st["active_tiles"] <= st["work_items"]
        assert st["sparse_items"] >= st["active_tiles"] // 2
        assert_map_equal(m, om)
    p, batches, amin, inc = cases.world_case(76, 800, 800, 0.05, 4, 4096, 1, region_frac=0.5)
    with dm.OccupancyMapper(p) as m:
        m.integrate(*batches[0], amin, inc)
        st = m.last_stats()
        assert st["sparse_items"] < st["active_tiles"] <= st["work_items"]
