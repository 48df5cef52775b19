"""GPU: BASELINE config C4 at full geometry — one 32768² map @ 5 cm shared by
32 robots (32 x 4096-beam scans per batch), split into 8 row bands of 4096
rows.

The 8 band handles live on cuda:0 (8-GPU runs are the driver's); the
device-resident exchange runs as dm/sharded.py runs it on a node, with the
RCCL all-gathers replaced by concatenation in rank order (which is what
all_gather_into_tensor produces): edge rows copied on the device
(dm_get_edge_rows_device) and installed as halos from the gathered buffer
(dm_set_halo_device), dm_frontiers_export_device per band, dm_merge_bands.
Checked bit for bit against a single 32768² handle on the same GPU and
against the CPU oracle over the whole map (the oracle needs ~30 GB of host
memory for a 2^30-cell frontier pass: the GPU box has it)."""
import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

P = 8


@pytest.fixture(scope="module")
def c4_batches():
    from dm import synth

    world, W, H, res, ox, oy = synth.config_world("C4", 0)
    stream = synth.ScanStream(world, 32, 4096, 4500, region=(ox + 1.0, oy + 1.0, -ox - 1.0, -oy - 1.0))
    batches = [stream.next_batch() for _ in range(2)]
    p = cases.make_params(W, H, resolution=res, origin=(ox, oy))
    return p, batches, float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(4096))


def _device_exchange(bands, rec_cap, min_size):
    """dm/sharded.py's _device_enqueue + merge for all bands in one process."""
    import torch

    W = bands[0].width
    grows = torch.empty(P * 2 * W, dtype=torch.int8, device="cuda:0")
    g0 = grows.data_ptr()
    for r, b in enumerate(bands):
        b.edge_rows_device(g0 + r * 2 * W, g0 + r * 2 * W + W)
        b.synchronize()
    for r, b in enumerate(bands):
        b.set_halo_device(g0 + (r - 1) * 2 * W + W if r > 0 else None,
                          g0 + (r + 1) * 2 * W if r + 1 < P else None)
    nb = bands[0].export_bytes(rec_cap)
    gexp = torch.zeros(P * nb, dtype=torch.uint8, device="cuda:0")
    for r, b in enumerate(bands):
        b.frontiers_export_device(gexp.data_ptr() + r * nb, rec_cap)
        b.synchronize()
    # every rank merges the same bytes: the first and the last band handle
    got, max_k = bands[0].merge_bands(gexp.data_ptr(), P, rec_cap, min_size)
    got_last, _ = bands[-1].merge_bands(gexp.data_ptr(), P, rec_cap, min_size)
    return got, got_last, max_k


def test_c4_eight_bands_vs_single_map_and_oracle(oracle_lib, c4_batches):
    import dm
    from dm.sharded import band_params

    p, batches, amin, inc = c4_batches
    om = oracle_lib.OracleMap(p)
    single = dm.OccupancyMapper(p, device=0)
    bands = [dm.OccupancyMapper(band_params(p, P, r), device=0) for r in range(P)]
    try:
        assert [b.rows for b in bands] == [4096] * P
        for poses, ranges in batches:
            exp = om.integrate(poses, ranges, amin, inc)
            assert single.integrate(poses, ranges, amin, inc) == exp
            # every band clips the rays to its rows: each update counted once
            U = sum(b.integrate(poses, ranges, amin, inc)[0] for b in bands)
            assert U == exp[0] and exp[0] > 5_000_000
        # the map: single handle vs oracle (bit for bit), bands vs its rows
        L = single.logodds()
        np.testing.assert_array_equal(L.view(np.uint32), om.L.view(np.uint32))
        st = single.state()
        np.testing.assert_array_equal(st, om.state)
        for b in bands:
            np.testing.assert_array_equal(b.state(), st[b.row0:b.row0 + b.rows])
        del L
        exp_clusters = om.frontiers(want_mask=False, want_labels=False)[2]
        assert len(exp_clusters) > 100
        np.testing.assert_array_equal(single.frontiers().clusters, exp_clusters)
        got, got_last, _ = _device_exchange(bands, 1 << 14, 1)
        np.testing.assert_array_equal(got, exp_clusters)
        np.testing.assert_array_equal(got_last, exp_clusters)
        # min_size applies to merged clusters: filter the oracle's list
        got5, _, _ = _device_exchange(bands, 1 << 14, 5)
        np.testing.assert_array_equal(got5, exp_clusters[exp_clusters["size"] >= 5])
    finally:
        single.close()
        for b in bands:
            b.close()


def test_c4_explored_map_eight_bands(oracle_lib):
    """The same exchange on a mostly explored C4 map (free space with walls,
    unknown pockets behind obstacles): frontiers cross band edges at many
    places, and nearly every tile of every band is visited."""
    import dm
    from dm import synth
    from dm.sharded import band_params

    world, W, H, res, ox, oy = synth.config_world("C4", 0)
    st = synth.explored_state(world, W, H, res, ox, oy, seed=4)
    p = cases.make_params(W, H, resolution=res, origin=(ox, oy))
    om = oracle_lib.OracleMap(p)
    om.state[...] = st
    exp_clusters = om.frontiers(want_mask=False, want_labels=False)[2]
    assert len(exp_clusters) > 1000
    bands = [dm.OccupancyMapper(band_params(p, P, r), device=0) for r in range(P)]
    try:
        for b in bands:
            b.set_state(st[b.row0:b.row0 + b.rows])
        got, got_last, max_k = _device_exchange(bands, 1 << 15, 1)
        assert got is not None, max_k
        np.testing.assert_array_equal(got, exp_clusters)
        np.testing.assert_array_equal(got_last, exp_clusters)
    finally:
        for b in bands:
            b.close()
