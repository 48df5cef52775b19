"""GPU: the cluster sort at every cluster count.

The frontier pipeline orders its cluster records by label with one of three
device sorts (csrc/dm_frontier.hip): the O(K^2) rank sort, or, once the last
collected pass of the handle had more than sort_min (4096) clusters, the
row-bucket sort (k_rs_count / k_rs_scan / k_rs_place / k_rs_rank).
Either must give the oracle's list bit for bit whatever the count of the pass
it actually sorts, including a small pass sorted by the bucket path after a
large one, the pipelined begin/end passes and the cross-band merge.
"""
import numpy as np
import pytest

import cases
from test_gpu_parity import assert_frontiers_equal

pytestmark = pytest.mark.gpu


def sparse_state(seed, R, W, step=3, p_free=0.9):
    """Isolated free cells in unknown space: about R*W/step^2 clusters."""
    rng = np.random.Generator(np.random.PCG64(seed))
    st = np.full((R, W), -1, np.int8)
    st[::step, ::step] = np.where(rng.random(st[::step, ::step].shape) < p_free, 0, -1)
    return st


def _oracle_clusters(oracle_lib, p, st):
    om = oracle_lib.OracleMap(p)
    om.state[...] = st
    return om.frontiers()


# K: 26k (> kBucketSortMin, < the rank sort's 65536 cap), 105k (> both)
@pytest.mark.parametrize("R,W,seed", [(512, 512, 1), (1024, 1024, 2)])
def test_bucket_sort_band(oracle_lib, monkeypatch, R, W, seed):
    import dm

    big = sparse_state(seed, R, W)
    small = cases.blob_state(seed, R, W, n_blobs=40)      # a few dozen clusters
    mid = cases.random_state(seed + 7, R, W)              # a few thousand
    p = cases.make_params(W, R)
    exp_big = _oracle_clusters(oracle_lib, p, big)
    assert len(exp_big[2]) > 4096
    with dm.OccupancyMapper(p) as m:
        m.set_state(big)
        for _ in range(3):  # rank sort / host sort, then the bucket sort
            assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *exp_big)
        for st in (small, mid, big, small):  # bucket path at any count, then back
            m.set_state(st)
            assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True),
                                   *_oracle_clusters(oracle_lib, p, st))
        # pipelined passes (dm_frontiers_begin / _end) through the same sorts
        m.set_state(big)
        m.frontiers()
        m.frontiers_begin()
        m.frontiers_begin()
        for _ in range(2):
            fr = m.frontiers_end()
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, exp_big[2])


def test_bucket_sort_min_size_filter(oracle_lib, monkeypatch):
    import dm

    st = cases.random_state(5, 768, 640, p_free=0.45, p_occ=0.05)
    p = cases.make_params(640, 768, min_frontier_size=3)
    exp = _oracle_clusters(oracle_lib, p, st)
    with dm.OccupancyMapper(p) as m:
        m.set_state(sparse_state(9, 768, 640))
        m.frontiers()  # a large pass: the next pass takes the bucket path
        m.set_state(st)
        assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), *exp)


@pytest.mark.parametrize("P", [2, 4])
def test_bucket_sort_merge(oracle_lib, monkeypatch, P):
    """Cross-band merge of ~105k clusters: rank sort cap exceeded first (host
    sort), then the bucket sort over global rows."""
    import dm
    import torch
    from dm.sharded import band_params

    R, W = 1024, 1024
    st = sparse_state(2, R, W)
    p = cases.make_params(W, R)
    exp = _oracle_clusters(oracle_lib, p, st)[2]
    bands = [dm.OccupancyMapper(band_params(p, P, r), device=0) for r in range(P)]
    try:
        for b in bands:
            b.set_state(st[b.row0:b.row0 + b.rows])
        edges = [b.edge_rows() for b in bands]
        for r, b in enumerate(bands):
            b.set_halo(edges[r - 1][1] if r > 0 else None, edges[r + 1][0] if r + 1 < P else None)
        rec_cap = 1 << 17
        nb = bands[0].export_bytes(rec_cap)
        g = torch.zeros(P * nb, dtype=torch.uint8, device="cuda:0")

        def export_all():
            for r, b in enumerate(bands):
                b.frontiers_export_device(g.data_ptr() + r * nb, rec_cap)
                b.synchronize()

        export_all()
        # ~52 k tile-local components per band against the initial 65 536
        # slots in 32 shard regions: which tiles share a region depends on
        # the order the big-tile kernel takes them, so a region can overflow
        # (flag 1, no result).  dm/sharded.py then falls back to the bands'
        # synchronous passes, which grow the slot arrays: the same here.
        if bands[0].merge_bands(g.data_ptr(), P, rec_cap, 1)[0] is None:
            for b in bands:
                b.frontiers()
            export_all()
        for _ in range(3):
            got, _ = bands[0].merge_bands(g.data_ptr(), P, rec_cap, 1)
            np.testing.assert_array_equal(got, exp)
    finally:
        for b in bands:
            b.close()


@pytest.mark.parametrize("R,W,rows", [(64, 65536, 3), (2048, 16384, 1)])
def test_row_sort_clusters_packed_in_few_rows(oracle_lib, monkeypatch, R, W, rows):
    """Clusters packed in a few rows (the round-2 bucket sort's worst case:
    one label bucket holding most records; for the row sort, rows of 8-32 k
    records: its O(b^2) worst case, slow but exact) and a wide label range;
    the second pass is sorted by the large-K path (hint from the first)."""
    import dm

    st = np.full((R, W), -1, np.int8)
    for k in range(rows):
        st[R // 2 + 2 * k, ::2] = 0  # isolated free cells: W / 2 clusters per row
    p = cases.make_params(W, R)
    mask, labels, clusters = _oracle_clusters(oracle_lib, p, st)
    assert len(clusters) > 4096
    with dm.OccupancyMapper(p) as m:
        m.set_state(st)
        for _ in range(2):
            assert_frontiers_equal(m.frontiers(want_mask=True, want_labels=True), mask, labels, clusters)
