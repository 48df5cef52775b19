"""GPU: the device-resident cross-band exchange (dm_frontiers_export_device +
dm_merge_bands, csrc/dm_merge.hip) gives exactly the 1-GPU frontier clusters.

One process plays all P bands (P band handles on cuda:0); the all-gather is
a plain concatenation of the export records in rank order, which is what
RCCL's all_gather_into_tensor produces (dm/sharded.py).  The multi-process
protocol itself is covered by tests/test_sharded.py (gloo, CPU)."""
import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu


def _bands(p, P):
    import dm
    from dm.sharded import band_params

    return [dm.OccupancyMapper(band_params(p, P, r), device=0) for r in range(P)]


def _set_halos(bands):
    edges = [b.edge_rows() for b in bands]
    P = len(bands)
    for r, b in enumerate(bands):
        b.set_halo(edges[r - 1][1] if r > 0 else None, edges[r + 1][0] if r + 1 < P else None)


def _export_all(bands, rec_cap):
    import torch

    P = len(bands)
    nb = bands[0].export_bytes(rec_cap)
    g = torch.zeros(P * nb, dtype=torch.uint8, device="cuda:0")
    for r, b in enumerate(bands):
        b.frontiers_export_device(g.data_ptr() + r * nb, rec_cap)
        b.synchronize()
    return g, nb


def _check_export_record(band, rec_bytes, rec_cap):
    """Header, edge indices -> records whose labels are the band's edge labels."""
    W = band.width
    raw = rec_bytes.cpu().numpy()
    hdr = raw[:64].view(np.int64)
    K = int(hdr[0])
    assert hdr[1] == 0 and hdr[2] == band.row0 and hdr[3] == band.rows and hdr[4] == W
    edge = raw[64:64 + 8 * W].view(np.int32).reshape(2, W)
    rec = raw[64 + 8 * W:64 + 8 * W + 32 * rec_cap].view(np.int64).reshape(rec_cap, 4)[:K]
    assert np.all(np.diff(rec[:, 0]) > 0)  # sorted, unique labels
    first, last = band.edge_labels()
    for e, lab in ((edge[0], first), (edge[1], last)):
        np.testing.assert_array_equal(e >= 0, lab >= 0)
        np.testing.assert_array_equal(rec[e[e >= 0], 0], lab[lab >= 0])


@pytest.mark.parametrize("P,W,H,seed,min_size", [(2, 300, 640, 3, 1), (3, 400, 700, 5, 4),
                                                 (4, 1000, 1024, 7, 1)])
def test_device_merge_scans(P, W, H, seed, min_size):
    import dm

    p = cases.make_params(W, H, min_frontier_size=min_size)
    bands = _bands(p, P)
    with dm.OccupancyMapper(p, device=0) as single:
        for k in range(3):
            poses, ranges, amin, inc = cases.random_scans(seed + k, p, 8, 400)
            single.integrate(poses, ranges, amin, inc)
            for b in bands:
                b.integrate(poses, ranges, amin, inc)
        exp = single.frontiers().clusters
    _set_halos(bands)
    rec_cap = 2048
    g, nb = _export_all(bands, rec_cap)
    for r, b in enumerate(bands):
        _check_export_record(b, g[r * nb:(r + 1) * nb], rec_cap)
    got, _ = bands[0].merge_bands(g.data_ptr(), P, rec_cap, min_size)
    assert len(exp) > 0
    np.testing.assert_array_equal(got, exp)
    for b in bands:
        b.close()


@pytest.mark.parametrize("P,R,W,seed,min_size", [(2, 512, 700, 11, 1), (4, 1024, 1100, 12, 3),
                                                 (8, 2048, 2048, 13, 1)])
def test_device_merge_blobs(P, R, W, seed, min_size):
    """Winding frontiers that cross every band edge many times."""
    import dm

    st = cases.blob_state(seed, R, W, n_blobs=40)
    p = cases.make_params(W, R, min_frontier_size=min_size)
    bands = _bands(p, P)
    with dm.OccupancyMapper(p, device=0) as single:
        single.set_state(st)
        exp = single.frontiers().clusters
    for b in bands:
        b.set_state(st[b.row0:b.row0 + b.rows])
    _set_halos(bands)
    rec_cap = 4096
    g, nb = _export_all(bands, rec_cap)
    got, _ = bands[0].merge_bands(g.data_ptr(), P, rec_cap, min_size)
    assert len(exp) > 0
    np.testing.assert_array_equal(got, exp)
    # every rank merges the same bytes: any band handle gives the same list
    got_last, _ = bands[-1].merge_bands(g.data_ptr(), P, rec_cap, min_size)
    np.testing.assert_array_equal(got_last, exp)
    for b in bands:
        b.close()


def test_device_merge_incomplete_record():
    """A band with more clusters than rec_cap flags its record; the merge
    reports DM_ERR_INCOMPLETE with the largest band K (all ranks see it)."""
    import dm

    st = cases.random_state(21, 256, 256, p_free=0.3, p_occ=0.1)
    p = cases.make_params(256, 256)
    bands = _bands(p, 2)
    for b in bands:
        b.set_state(st[b.row0:b.row0 + b.rows])
    _set_halos(bands)
    g, nb = _export_all(bands, 4)
    got, max_k = bands[0].merge_bands(g.data_ptr(), 2, 4, 1)
    assert got is None and max_k > 4
    with dm.OccupancyMapper(p, device=0) as single:
        single.set_state(st)
        exp = single.frontiers().clusters
    g, nb = _export_all(bands, 1 << 15)
    got, _ = bands[0].merge_bands(g.data_ptr(), 2, 1 << 15, 1)
    np.testing.assert_array_equal(got, exp)
    for b in bands:
        b.close()


def test_single_band_merge_is_identity():
    """P = 1: the merge of one record is that band's cluster list."""
    import dm

    st = cases.blob_state(31, 300, 500)
    p = cases.make_params(500, 300, min_frontier_size=2)
    bp = cases.make_params(500, 300, min_frontier_size=1)
    with dm.OccupancyMapper(p, device=0) as single, dm.OccupancyMapper(bp, device=0) as band:
        single.set_state(st)
        band.set_state(st)
        exp = single.frontiers().clusters
        g, nb = _export_all([band], 8192)
        got, _ = band.merge_bands(g.data_ptr(), 1, 8192, 2)
    np.testing.assert_array_equal(got, exp)
