"""CPU: the row-bucket cluster sort (csrc/dm_frontier.hip k_rs_count ->
k_rs_scan -> k_rs_place -> k_rs_rank) restated step by step in NumPy with
the kernels' index arithmetic (8192-row scan workgroups of 256 threads x 32
rows that publish their totals, arrival slots inside a row, rank = smaller
keys of the same row), checked against a plain sort of the labels.  The GPU
kernels themselves are checked against the oracle in tests/test_gpu_sort.py;
this pins the algorithm and its edge cases (rows not a multiple of a scan
workgroup, a row holding most records, a band that does not start at row 0)
without a GPU."""
import numpy as np
import pytest

RS_PER = 32
RS_CHUNK = 256 * RS_PER


def row_bucket_sort(labels, base, rows, W, rng):
    K = len(labels)
    keys = (labels - base).astype(np.uint64)
    row = (keys // np.uint64(W)).astype(np.int64)
    assert row.min() >= 0 and row.max() < rows
    # k_rs_count: arrival order inside a row is whatever the atomics give
    order = rng.permutation(K)
    row_cnt = np.zeros(rows, np.int64)
    slot = np.empty(K, np.int64)
    for i in order:
        slot[i] = row_cnt[row[i]]
        row_cnt[row[i]] += 1
    # k_rs_scan: workgroup b scans rows [b*8192, +8192) in registers and adds
    # the published totals of every earlier workgroup
    nsb = (rows + RS_CHUNK - 1) // RS_CHUNK
    totals = [int(row_cnt[b * RS_CHUNK:(b + 1) * RS_CHUNK].sum()) for b in range(nsb)]
    row_off = np.empty(rows + 1, np.int64)
    for b in range(nsb):
        pre = sum(totals[:b])
        seg = row_cnt[b * RS_CHUNK:(b + 1) * RS_CHUNK]
        row_off[b * RS_CHUNK:b * RS_CHUNK + len(seg)] = pre + np.cumsum(seg) - seg
        if b == nsb - 1:
            row_off[rows] = pre + totals[b]
    assert row_off[rows] == K
    # k_rs_place
    placed_keys = np.empty(K, np.uint64)
    placed_idx = np.empty(K, np.int64)
    p = row_off[row] + slot
    placed_keys[p] = keys
    placed_idx[p] = np.arange(K)
    # k_rs_rank: position p's final place = its row's offset + smaller keys of the row
    out = np.empty(K, np.int64)
    for q in range(K):
        r = int(placed_keys[q] // np.uint64(W))
        lo, hi = row_off[r], row_off[r + 1]
        rank = int(np.count_nonzero(placed_keys[lo:hi] < placed_keys[q]))
        out[lo + rank] = placed_idx[q]
    return out


@pytest.mark.parametrize("rows,W,K,row0,skew", [
    (2560, 65536, 3000, 30720, False),     # a C5 band: one partial scan workgroup
    (20000, 1000, 5000, 0, False),         # 3 scan workgroups, the last partial
    (8192, 4096, 4000, 0, True),           # most records in one row
    (64, 65536, 2000, 0, False),           # fewer rows than a workgroup's
])
def test_row_bucket_sort_matches_sort(rows, W, K, row0, skew):
    rng = np.random.Generator(np.random.PCG64(rows + K))
    base = row0 * W
    if skew:
        hot = np.arange(0, W, 2)[:K // 2]
        cells = np.concatenate([hot + 4000 * W, rng.choice(rows * W, K - len(hot), replace=False)])
        cells = np.unique(cells)
    else:
        cells = rng.choice(rows * W, K, replace=False)
    labels = base + rng.permutation(cells).astype(np.int64)  # unique, as components' first cells are
    out = row_bucket_sort(labels, base, rows, W, rng)
    np.testing.assert_array_equal(labels[out], np.sort(labels))
