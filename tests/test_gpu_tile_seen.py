"""GPU: the frontier bit rows take a never-written neighbour tile's facing
cells as unknown without loading them (tile_seen): maps whose
free regions end exactly at tile edges, at the ragged last tile column / row
and at the map's edge, set in bulk (k_recount sets tile_seen from the state)
and then grown by integrate calls (k_tile_accum sets it), against the oracle."""
import numpy as np
import pytest

import cases
import dm
from test_gpu_parity import assert_frontiers_equal, assert_map_equal

pytestmark = pytest.mark.gpu


def _tile_edge_state(H, W):
    st = np.full((H, W), -1, np.int8)
    st[64:128, 64:128] = 0            # one whole tile: all four edges face unseen tiles
    st[384:448, 448:W] = 0            # the ragged last tile column (W % 64 != 0)
    st[128:192, 200:300] = 0          # a strip ending exactly at a tile row boundary (row 191)
    st[190:192, 250:252] = 100        # occupied cells on that boundary
    st[200:260, W - 40:W] = 0         # free up to the map's right edge
    st[H - 10:H, 0:64] = 0            # free up to the ragged last tile row
    st[300:301, 0:W] = 0              # one free row across every tile column
    return st


@pytest.mark.parametrize("W,H", [(500, 460), (512, 512)])
def test_frontiers_next_to_unseen_tiles(oracle_lib, W, H):
    p = cases.make_params(W, H)
    st = _tile_edge_state(H, W)
    L0 = np.where(st == 100, np.float32(p.l_occ), np.where(st == 0, np.float32(p.l_free), np.float32(0)))
    om = oracle_lib.OracleMap(p)
    om.L[...] = L0
    om.state[...] = st
    with dm.OccupancyMapper(p) as m:
        m.set_logodds(L0)
        np.testing.assert_array_equal(m.state(), st)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())
        # rays grow the map into tiles that were never written (tile_seen set
        # by the accumulation), synchronous and pipelined passes
        m.set_overlap(True)
        for k in range(3):
            poses, ranges, amin, inc = cases.random_scans(900 + k, p, 3, 360, spread=0.6)
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            m.frontiers_begin()
            fr = m.frontiers_end()
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, om.frontiers(want_mask=False, want_labels=False)[2])
        assert_map_equal(m, om)
        fr = m.frontiers(want_mask=True, want_labels=True)
        assert_frontiers_equal(fr, *om.frontiers())


def test_reset_clears_seen_tiles(oracle_lib):
    """After dm_reset every tile is unseen again: a map rebuilt by rays alone
    (no bulk write) still matches the oracle."""
    W, H = 448, 384
    p = cases.make_params(W, H)
    with dm.OccupancyMapper(p) as m:
        st = _tile_edge_state(H, W)
        m.set_state(st)
        m.frontiers()
        m.reset()
        om = oracle_lib.OracleMap(p)
        for k in range(2):
            poses, ranges, amin, inc = cases.random_scans(950 + k, p, 2, 200, spread=0.4)
            m.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            fr = m.frontiers(want_mask=True, want_labels=True)
            assert_frontiers_equal(fr, *om.frontiers())
        assert_map_equal(m, om)


def _band_edge_state(H, W, edge):
    """Free regions that end exactly at a band edge (row `edge`, a multiple of
    64), on either side of it, next to tiles of the other band that were never
    written (their facing cells are halo rows there, not tile_seen skips)."""
    st = np.full((H, W), -1, np.int8)
    st[edge - 64:edge, 0:64] = 0          # band 0's last tile row, below it unseen band-1 tiles
    st[edge:edge + 64, 128:192] = 0       # band 1's first tile row, above it unseen band-0 tiles
    st[edge - 1:edge + 1, 256:300] = 0    # a strip across the edge
    st[edge - 1, 320:384] = 0             # one free row on band 0's side only
    st[edge, 400:W] = 0                   # one free row on band 1's side, to the ragged map edge
    st[edge - 30:edge + 30, 200:202] = 100
    return st


@pytest.mark.parametrize("fmask", ["off", "on"])
def test_band_edge_tiles_with_and_without_fmask(oracle_lib, monkeypatch, fmask):
    """tile_seen next to band halos, with the bit rows read from
    the state bytes (DM_FMASK=off) and from fmask (on): a sharded handle's
    bands (ty == 0 / ty == TY-1 tiles read the halo rows), bulk-written and
    then grown by rays, against the oracle."""
    monkeypatch.setenv("DM_FMASK", fmask)
    W, H, edge = 470, 512, 256
    p = cases.make_params(W, H)
    st = _band_edge_state(H, W, edge)
    L0 = np.where(st == 100, np.float32(p.l_occ), np.where(st == 0, np.float32(p.l_free), np.float32(0)))
    om = oracle_lib.OracleMap(p)
    om.L[...] = L0
    om.state[...] = st
    with dm.OccupancyMapper(p, devices=[0, 0]) as sh:
        sh.set_logodds(L0)
        np.testing.assert_array_equal(sh.state(), st)
        assert_frontiers_equal(sh.frontiers(want_mask=True, want_labels=True), *om.frontiers())
        for k in range(3):
            poses, ranges, amin, inc = cases.random_scans(950 + k, p, 3, 360, spread=0.5)
            sh.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            fr = sh.frontiers(want_mask=True, want_labels=True)
            assert_frontiers_equal(fr, *om.frontiers())
        assert_map_equal(sh, om)
