"""GPU: BASELINE config C5 at full size — ONE 65536² @ 1 cm handle (2^32
cells, 21 GiB of HBM: L, state, fmask), the map bench.py's C5 sweep times.

C5's resolution and range are the reference's slam_config.yaml:26-27 values
at the north star's 1 cm (max_laser_range 12 m = 1200 cells per ray).  Sixty-
four robots in eight groups are placed where the full-size map has its edge
cases: along the top edge (rays reach rows >= 64512, where the min-index
labels exceed 65536 * 64512 and uint32 sentinels would collide), in the
top-right and bottom-left corners and along the right and left edges (rays
leave the grid; some robots stand outside it), straddling band boundaries of
the 2560-row decomposition, and a dense cluster around the origin.

The CPU oracle cannot hold a 2^32-cell frontier pass (≈ 100 GiB of work
arrays), so it runs band-wise, as the sharded layer does:
26 oracle bands of 2560 rows (the last 1536), each fed the scans whose
max-range disk reaches it, with the neighbours' edge rows as halos; their
clusters are merged with dm.sharded.merge_clusters (CPU-tested against the
single-map oracle in tests/test_sharded.py).  Checked bit for bit:
  (a) U / T of every call, L and state of every row, the frontier mask of
      every row and the clusters of the full handle against that oracle;
  (b) the full handle's clusters against 26 band handles on the same GPU
      exchanging through dm_frontiers_export_device + dm_merge_bands (the
      RCCL all-gather replaced by concatenation in rank order), with the
      multi-process layer's retry protocol for fresh bands;
  (c) one sharded handle over those 26 bands (dm_create_sharded, devices
      {0, ..., 0}): U / T, L (digest per band), state, mask and clusters,
      synchronous and pipelined.
The oracle bands run in a thread pool (ctypes releases the GIL)."""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

W = H = 65536
RES = 0.01
BAND = 2560
P = -(-H // BAND)  # 26 bands: 25 x 2560 rows + 1536
TOP_LABEL = 65536 * 64512  # labels at or above this lie in the last 1024 rows


def _regions(half):
    """Eight robot groups (metres): x0, y0, x1, y1 (ScanStream keeps 1 m inside)."""
    def row_y(r):
        return -half + r * RES
    return [
        (-200.0, half - 8.0, 200.0, half + 1.0),              # top edge (some outside the map)
        (half - 8.0, half - 8.0, half + 2.0, half + 2.0),      # top-right corner
        (half - 6.0, -100.0, half + 1.0, 100.0),               # right edge
        (-half - 2.0, -half - 2.0, -half + 8.0, -half + 8.0),  # bottom-left corner
        (-50.0, row_y(13 * BAND) - 2.0, 50.0, row_y(13 * BAND) + 2.0),  # band 12 | 13 boundary
        (-300.0, row_y(25 * BAND) - 2.0, 300.0, row_y(25 * BAND) + 2.0),  # band 24 | 25 boundary
        (-half - 2.0, -300.0, -half + 6.0, 300.0),             # left edge
        (-3.0, -3.0, 3.0, 3.0),                                # dense cluster at the origin
    ]


def _c5_batches(n_beams, n_batches, seed):
    from dm import synth

    half = W * RES / 2.0
    # obstacles 5 m beyond the map on every side: rays cross the map edge
    world = synth.make_world(seed, -half - 5.0, -half - 5.0, half + 5.0, half + 5.0)
    streams = [synth.ScanStream(world, 8, n_beams, seed + 1 + i, region=r)
               for i, r in enumerate(_regions(half))]
    batches = []
    for _ in range(n_batches):
        parts = [s.next_batch() for s in streams]
        batches.append((np.concatenate([q for q, _ in parts]), np.concatenate([r for _, r in parts])))
    p = cases.make_params(W, H, resolution=RES, origin=(-half, -half))
    return p, batches, float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(n_beams))


def _reaches(p, poses, row0, rows):
    """Scans whose max-range disk reaches rows [row0, row0 + rows)."""
    reach = float(p.range_max) + 2 * p.resolution
    y = poses[:, 1]
    return ~((y < p.origin_y + row0 * p.resolution - reach) |
             (y > p.origin_y + (row0 + rows) * p.resolution + reach))


def _band_list():
    return [(r0, min(BAND, H - r0)) for r0 in range(0, H, BAND)]


def _oracle_band_maps(oracle_lib, p, batches, amin, inc):
    """One oracle map per band after every batch; per-call (U, T) per band."""
    def run(band):
        r0, rows = band
        bp = cases.make_params(W, H, resolution=RES, origin=(p.origin_x, p.origin_y),
                               band_row0=r0, band_rows=rows)
        om = oracle_lib.OracleMap(bp)
        counts = []
        for poses, ranges in batches:
            keep = _reaches(p, poses, r0, rows)
            counts.append(om.integrate(poses[keep], ranges[keep], amin, inc) if keep.any() else (0, 0))
        return om, counts

    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(run, _band_list()))


def _oracle_band_frontiers(oracle_lib, bands, st):
    """Band frontiers with halo rows from the (already verified) full state:
    mask, cluster records and edge labels per band."""
    def run(k):
        om = bands[k][0]
        r0, rows = _band_list()[k]
        hb = st[r0 - 1] if r0 > 0 else None
        ha = st[r0 + rows] if r0 + rows < H else None
        mask, labels, clusters = om.frontiers(hb, ha, want_mask=True, want_labels=True)
        rec = np.stack([clusters["label"], clusters["size"], clusters["sum_x"], clusters["sum_y"]],
                       1).astype(np.int64) if len(clusters) else np.zeros((0, 4), np.int64)
        return mask, rec, (labels[0].copy(), labels[-1].copy())

    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(run, range(len(bands))))


def _device_exchange(handles, rec_cap):
    """dm/sharded.py's device exchange for all band handles in one process."""
    import torch

    n = len(handles)
    w = handles[0].width
    grows = torch.empty(n * 2 * w, dtype=torch.int8, device="cuda:0")
    g0 = grows.data_ptr()
    for r, b in enumerate(handles):
        b.edge_rows_device(g0 + r * 2 * w, g0 + r * 2 * w + w)
        b.synchronize()
    for r, b in enumerate(handles):
        b.set_halo_device(g0 + (r - 1) * 2 * w + w if r > 0 else None,
                          g0 + (r + 1) * 2 * w if r + 1 < n else None)
    nb = handles[0].export_bytes(rec_cap)
    gexp = torch.zeros(n * nb, dtype=torch.uint8, device="cuda:0")
    for r, b in enumerate(handles):
        b.frontiers_export_device(gexp.data_ptr() + r * nb, rec_cap)
        b.synchronize()
    got, max_k = handles[0].merge_bands(gexp.data_ptr(), n, rec_cap, 1)
    got_last, _ = handles[-1].merge_bands(gexp.data_ptr(), n, rec_cap, 1)
    return got, got_last, max_k


def _exchange_like_sharded_mapper(handles, rec_cap):
    """The multi-process layer's protocol (dm/sharded.py) on fresh band
    handles: slot arrays are sized for the map at dm_create and the record
    capacity for the band (a cluster per two tiles, as ShardedMapper does),
    so the FIRST device exchange must succeed — no incomplete record, no host
    fallback."""
    got, got_last, max_k = _device_exchange(handles, rec_cap)
    assert got is not None, ("device exchange fell back", getattr(handles[0], "last_incomplete", None), rec_cap,
                             [h.last_stats()["frontier_slots"] for h in handles])
    return got, got_last, max_k


def _digest(a):
    import hashlib

    return hashlib.blake2b(memoryview(np.ascontiguousarray(a)).cast("B"), digest_size=16).hexdigest()


@pytest.mark.parametrize("n_beams,n_batches", [(48, 8), (4096, 2)])
def test_c5_full_map_vs_band_oracle_and_band_handles(oracle_lib, n_beams, n_batches):
    import dm
    from dm.sharded import band_params, merge_clusters

    p, batches, amin, inc = _c5_batches(n_beams, n_batches, 9100 + n_beams)
    S = batches[0][0].shape[0]
    assert S == 64
    oracle_bands = _oracle_band_maps(oracle_lib, p, batches, amin, inc)

    full = dm.OccupancyMapper(p, device=0)
    try:
        # (a) U / T of every call: the bands' sums (each update lies in one band)
        for k, (poses, ranges) in enumerate(batches):
            got = full.integrate(poses, ranges, amin, inc)
            exp = tuple(sum(ob[1][k][i] for ob in oracle_bands) for i in (0, 1))
            assert got == exp, (k, got, exp)
            assert exp[0] > 0
        # L and state, every row
        L = full.logodds()
        L_digest = []
        for (r0, rows), (om, _) in zip(_band_list(), oracle_bands):
            np.testing.assert_array_equal(L[r0:r0 + rows].view(np.uint32), om.L.view(np.uint32),
                                          err_msg=f"L rows {r0}..{r0 + rows}")
            L_digest.append(_digest(L[r0:r0 + rows]))
            om.L = None  # free the band's L (16 GiB over all bands)
        del L
        st = full.state()
        assert st.shape == (H, W)
        for (r0, rows), (om, _) in zip(_band_list(), oracle_bands):
            np.testing.assert_array_equal(st[r0:r0 + rows], om.state, err_msg=f"state rows {r0}..{r0 + rows}")
        # rays reached the last 1024 rows and the last columns
        assert (st[64512:] == 0).any() and (st[:, 65000:] == 0).any() and (st[:, :500] == 0).any()

        # frontiers: mask of every row, clusters merged over the band oracle
        fr = full.frontiers(want_mask=True)
        ofr = _oracle_band_frontiers(oracle_lib, oracle_bands, st)
        band_masks = []
        for (r0, rows), (mask, _, _) in zip(_band_list(), ofr):
            np.testing.assert_array_equal(fr.mask[r0:r0 + rows], mask, err_msg=f"mask rows {r0}..{r0 + rows}")
            band_masks.append(_digest(mask))
        exp_clusters = merge_clusters([o[1] for o in ofr], [o[2] for o in ofr], p, 1)
        assert len(exp_clusters) > 50
        np.testing.assert_array_equal(fr.clusters, exp_clusters)
        assert (fr.clusters["label"] >= TOP_LABEL).any()  # labels in the last 1024 rows (near 2^32)
        # several bands hold frontier pieces joined across band edges
        assert sum(1 for o in ofr if len(o[1])) >= 8
        del fr, ofr
        for ob in oracle_bands:
            ob[0].state = None
    finally:
        full.close()

    # (b) 26 band handles on the same GPU, device export + dm_merge_bands
    handles = [dm.OccupancyMapper(band_params(p, P, r), device=0) for r in range(P)]
    try:
        assert [(h.row0, h.rows) for h in handles] == _band_list()
        for poses, ranges in batches:
            for h in handles:
                keep = _reaches(p, poses, h.row0, h.rows)
                if keep.any():
                    h.integrate(poses[keep], ranges[keep], amin, inc)
        for r, h in enumerate(handles):
            np.testing.assert_array_equal(h.state(), st[h.row0:h.row0 + h.rows], err_msg=f"band {r}")
        tiles = -(-handles[0].width // 64) * -(-handles[0].rows // 64)
        rec_cap = 1 << 14
        while rec_cap < tiles:  # ShardedMapper's up-front sizing
            rec_cap *= 2
        got, got_last, max_k = _exchange_like_sharded_mapper(handles, rec_cap)
        assert got is not None, max_k
        np.testing.assert_array_equal(got, exp_clusters)
        np.testing.assert_array_equal(got_last, exp_clusters)
    finally:
        for h in handles:
            h.close()

    # (c) the same 26 bands behind ONE sharded handle (dm_create_sharded with
    # devices {0, ..., 0}): the drop-in's calls, the exchange inside libdm
    sh = dm.OccupancyMapper(p, devices=[0] * P)
    try:
        for k, (poses, ranges) in enumerate(batches):
            exp = tuple(sum(ob[1][k][i] for ob in oracle_bands) for i in (0, 1))
            assert sh.integrate(poses, ranges, amin, inc) == exp
        L = sh.logodds()
        assert [_digest(L[r0:r0 + rows]) for r0, rows in _band_list()] == L_digest
        del L
        np.testing.assert_array_equal(sh.state(), st)
        fr = sh.frontiers(want_mask=True)  # the first pass grows the fresh bands' capacities itself
        np.testing.assert_array_equal(fr.clusters, exp_clusters)
        for (r0, rows), mask in zip(_band_list(), band_masks):
            assert _digest(fr.mask[r0:r0 + rows]) == mask, f"mask rows {r0}..{r0 + rows}"
        del fr
        sh.frontiers_begin()
        sh.frontiers_begin()
        for _ in range(2):
            fr = sh.frontiers_end()
            assert fr is not None, sh.last_incomplete
            np.testing.assert_array_equal(fr.clusters, exp_clusters)
    finally:
        sh.close()
