"""GPU: the frontier pass reading the per-tile free / unknown bit records
(fmask, DM_FMASK=on: maintained by k_fmask_items after every map update and by k_recount after bulk state writes, with the per-tile edge
words fedge the pass reads for a tile's neighbours) instead of the state bytes, against the
CPU oracle: integrate sequences on aligned, ragged and unaligned (W % 4 != 0:
the cell-by-cell path) maps, the state families of the frontier parity tests,
band halos (the halo rows come from the state bytes at band edges), and the
automatic switch (DM_FMASK=auto: on once a pass lists >= 8192 tiles, with a
rebuild of records that went stale while it was off)."""
import numpy as np
import pytest

import cases
import dm
import test_gpu_parity as par
from test_gpu_parity import assert_frontiers_equal, assert_map_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def fmask_on(monkeypatch):
    monkeypatch.setenv("DM_FMASK", "on")


@pytest.mark.parametrize("W,H,S,N,nb,seed", [(1024, 1024, 8, 1024, 4, 61), (1000, 700, 6, 720, 4, 62),
                                             (1001, 703, 5, 900, 4, 63), (700, 1300, 3, 200, 6, 64)])
def test_integrate_then_frontiers(oracle_lib, fmask_on, W, H, S, N, nb, seed):
    """The fmask writer (k_fmask_items, with sparse items that rewrite only
    some rows) and the edge words (fedge) the pass reads for a tile's
    neighbours."""
    p, batches, amin, inc = cases.world_case(seed, W, H, 0.05, S, N, nb, region_frac=0.7)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        for poses, ranges in batches:
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            m.frontiers_begin()
            fr = m.frontiers_end()
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, om.frontiers(want_mask=False, want_labels=False)[2])
        assert_map_equal(m, om)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())


@pytest.mark.parametrize("kind,R,W,seed", par.FRONTIER_STATE_CASES)
def test_states(oracle_lib, fmask_on, kind, R, W, seed):
    par.test_frontiers_on_states(oracle_lib, kind, R, W, seed)


def test_band_halos(oracle_lib, fmask_on):
    par.test_frontier_band_with_halo(oracle_lib)


def test_auto_switch_rebuilds_stale_records(oracle_lib, monkeypatch):
    """8192 x 8192 explored map: every one of its 16384 tiles is listed, so
    the second pass switches fmask on; the batch integrated in between (with
    fmask off) made the records stale, so the switch rebuilds them first."""
    monkeypatch.setenv("DM_FMASK", "auto")
    from dm import synth

    W = H = 8192
    res = 0.05
    half = W * res / 2
    world = synth.make_world(3, -half, -half, half, half)
    st = synth.explored_state(world, W, H, res, -half, -half, seed=3)
    p = cases.make_params(W, H, resolution=res)
    stream = synth.ScanStream(world, 16, 1024, 77, region=(-half + 1, -half + 1, half - 1, half - 1))
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(1024))
    # the same start on both sides: L from the state (set_state's mapping)
    L0 = np.where(st == 100, np.float32(p.l_occ), np.where(st == 0, np.float32(p.l_free), np.float32(0)))
    om = oracle_lib.OracleMap(p)
    om.L[...] = L0
    om.state[...] = st
    with dm.OccupancyMapper(p) as m:
        m.set_logodds(L0)
        np.testing.assert_array_equal(m.state(), st)
        for k in range(3):
            fr = m.frontiers()
            np.testing.assert_array_equal(fr.clusters, om.frontiers(want_mask=False, want_labels=False)[2])
            assert m.last_stats()["frontier_tiles"] >= 8192
            poses, ranges = stream.next_batch()
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
        fr = m.frontiers()
        np.testing.assert_array_equal(fr.clusters, om.frontiers(want_mask=False, want_labels=False)[2])
