"""GPU: pipelined frontier passes and the overlapped integrate front-end
(dm_frontiers_begin / _end, dm_merge_bands_begin / _end, dm_set_overlap).

Every pass collected with frontiers_end() must equal the CPU oracle's
frontiers on the map as it was after that pass's own batch, although the next
batch's integrate call (front-end on the overlap stream) was enqueued before
the pass was collected; the final map must equal the oracle's bit for bit."""
import numpy as np
import pytest

import cases
import dm
from test_gpu_parity import assert_map_equal

pytestmark = pytest.mark.gpu


def _device_batches(batches):
    import torch
    from dm import synth

    out = [(torch.from_numpy(synth.pose4(p)).cuda(), torch.from_numpy(np.ascontiguousarray(r)).cuda())
           for p, r in batches]
    torch.cuda.synchronize()  # overlap mode: device inputs complete at call time
    return out


def _oracle_steps(oracle_lib, p, batches, amin, inc):
    om = oracle_lib.OracleMap(p)
    clusters = []
    for poses, ranges in batches:
        om.integrate(poses, ranges, amin, inc)
        clusters.append(om.frontiers(want_mask=False, want_labels=False)[2])
    return om, clusters


@pytest.mark.parametrize("W,H,S,N,nb,seed", [(2048, 2048, 8, 1024, 6, 41), (640, 480, 3, 720, 5, 42),
                                             (1000, 700, 16, 2048, 4, 43)])
def test_pipelined_steps_match_oracle(oracle_lib, W, H, S, N, nb, seed):
    p, batches, amin, inc = cases.world_case(seed, W, H, 0.05, S, N, nb, region_frac=0.6)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    dev = _device_batches(batches)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        got = []
        for k, (pose4, rng) in enumerate(dev):
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), N, amin, inc)
            if k > 0:
                got.append(m.frontiers_end())
            m.frontiers_begin()
        got.append(m.frontiers_end())
        for k, fr in enumerate(got):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, expect[k])
        assert_map_equal(m, om)
        m.set_overlap(False)
        np.testing.assert_array_equal(m.frontiers().clusters, expect[-1])


def test_overlap_host_integrate_and_sync_frontiers(oracle_lib):
    """Overlap mode with the host-input entry point (uploads on the front-end
    stream) and synchronous frontiers between calls."""
    p, batches, amin, inc = cases.world_case(44, 900, 900, 0.05, 4, 900, 5, region_frac=0.7)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        for k, (poses, ranges) in enumerate(batches):
            m.integrate(poses, ranges, amin, inc)
            np.testing.assert_array_equal(m.frontiers().clusters, expect[k])
        assert_map_equal(m, om)


def test_frontiers_end_protocol():
    import ctypes

    from dm import _ffi

    p, batches, amin, inc = cases.world_case(45, 512, 512, 0.05, 4, 720, 2, region_frac=0.7)
    with dm.OccupancyMapper(p) as m:
        for poses, ranges in batches:
            m.integrate(poses, ranges, amin, inc)
        ref = m.frontiers().clusters
        assert len(ref) > 2
        lib, h = m._lib, m._handle()
        n = ctypes.c_int64(-1)
        # end without begin; two passes may be in flight, a third is refused
        assert lib.dm_frontiers_end(h, None, 0, ctypes.byref(n)) == _ffi.DM_ERR_INVALID_ARG
        assert lib.dm_frontiers_begin(h) == 0
        assert lib.dm_frontiers_begin(h) == 0
        assert lib.dm_frontiers_begin(h) == _ffi.DM_ERR_INVALID_ARG
        # a synchronous pass while two are pending uses its own readback slot
        np.testing.assert_array_equal(m.frontiers().clusters, ref)
        # a merge end while the oldest pending pass is a frontier pass
        assert lib.dm_merge_bands_end(h, None, 0, ctypes.byref(n)) == _ffi.DM_ERR_INVALID_ARG
        buf2 = np.empty(len(ref), dtype=np.dtype(dm.CLUSTER_DTYPE))
        assert lib.dm_frontiers_end(h, buf2.ctypes.data_as(ctypes.c_void_p), len(ref), ctypes.byref(n)) == 0
        np.testing.assert_array_equal(buf2, ref)
        # too small a buffer: DM_ERR_CAPACITY with the count, the pass stays pending
        assert lib.dm_frontiers_end(h, None, 0, ctypes.byref(n)) == _ffi.DM_ERR_CAPACITY
        assert n.value == len(ref)
        buf = np.empty(len(ref), dtype=np.dtype(dm.CLUSTER_DTYPE))
        assert lib.dm_frontiers_end(h, buf.ctypes.data_as(ctypes.c_void_p), len(ref), ctypes.byref(n)) == 0
        np.testing.assert_array_equal(buf, ref)
        # the pass is over now
        assert lib.dm_frontiers_end(h, None, 0, ctypes.byref(n)) == _ffi.DM_ERR_INVALID_ARG
        # the Python wrapper grows its buffer itself
        m._cap = 1
        m.frontiers_begin()
        np.testing.assert_array_equal(m.frontiers_end().clusters, ref)


def test_sharded_single_band_pipelined(oracle_lib):
    from dm.sharded import ShardedMapper

    p, batches, amin, inc = cases.world_case(46, 700, 600, 0.05, 4, 900, 4, region_frac=0.7)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    sm = ShardedMapper(p)
    try:
        sm.set_overlap(True)
        got = []
        for k, (poses, ranges) in enumerate(batches):
            sm.integrate(poses, ranges, amin, inc)
            if k > 0:
                got.append(sm.frontiers_end())
            sm.frontiers_begin()
        got.append(sm.frontiers_end())
        for k, fr in enumerate(got):
            np.testing.assert_array_equal(fr.clusters, expect[k])
    finally:
        sm.close()


@pytest.mark.parametrize("W,H,S,N,nb,seed", [(1500, 1500, 8, 1024, 7, 47), (700, 500, 3, 720, 6, 48)])
def test_two_passes_in_flight_match_oracle(oracle_lib, W, H, S, N, nb, seed):
    """Depth-2 pipelining: pass k is collected after batch k+2's integrate was
    enqueued (two frontier passes in flight); each equals the oracle's
    frontiers after batch k."""
    p, batches, amin, inc = cases.world_case(seed, W, H, 0.05, S, N, nb, region_frac=0.6)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    dev = _device_batches(batches)
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(True)
        got = []
        for k, (pose4, rng) in enumerate(dev):
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), N, amin, inc)
            if k > 1:
                got.append(m.frontiers_end())
            m.frontiers_begin()
        got.append(m.frontiers_end())
        got.append(m.frontiers_end())
        assert len(got) == len(expect)
        for k, fr in enumerate(got):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, expect[k])
        assert_map_equal(m, om)


@pytest.mark.parametrize("P,W,H,seed", [(2, 300, 640, 3), (4, 1000, 1024, 7)])
def test_merge_bands_begin_end_matches_sync(P, W, H, seed):
    from test_gpu_merge import _bands, _export_all, _set_halos

    p, batches, amin, inc = cases.world_case(seed, W, H, 0.05, 6, 900, 2, region_frac=0.8)
    bands = _bands(p, P)
    try:
        for poses, ranges in batches:
            for b in bands:
                b.integrate(poses, ranges, amin, inc)
        _set_halos(bands)
        rec_cap = 4096
        g, nb = _export_all(bands, rec_cap)
        sync, k = bands[0].merge_bands(g.data_ptr(), P, rec_cap, 1)
        assert k is None and len(sync) > 0
        bands[1].merge_bands_begin(g.data_ptr(), P, rec_cap, 1)
        bands[1]._mbuf = np.empty(1, dtype=np.dtype(dm.CLUSTER_DTYPE))  # forces the pending re-read
        got, k = bands[1].merge_bands_end()
        assert k is None
        np.testing.assert_array_equal(got, sync)
    finally:
        for b in bands:
            b.close()


@pytest.mark.parametrize("overlap", [True, False])
def test_async_host_inputs_pipelined(oracle_lib, overlap):
    """dm_integrate_async from pinned host buffers (the PCIe-inclusive form of
    the bench step): each call is enqueued without waiting, its ranges buffer
    reused only two calls later; every pipelined pass equals the oracle's
    frontiers after its own batch and the final map is bit-exact."""
    import torch

    p, batches, amin, inc = cases.world_case(49, 1200, 1100, 0.05, 6, 1024, 7, region_frac=0.6)
    om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
    S, N = batches[0][1].shape
    pinned = [torch.empty((S, N), dtype=torch.float32).pin_memory() for _ in range(2)]
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(overlap)
        got = []
        for k, (poses, ranges) in enumerate(batches):
            buf = pinned[k % 2]  # free again: its copy was two calls ago
            buf.numpy()[...] = ranges
            m.integrate_async(poses, buf.data_ptr(), S, N, amin, inc)
            if k > 0:
                got.append(m.frontiers_end())
            m.frontiers_begin()
        got.append(m.frontiers_end())
        for k, fr in enumerate(got):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, expect[k])
        assert_map_equal(m, om)
        om2 = oracle_lib.OracleMap(p)
        assert m.last_counts() == om2.integrate(*batches[-1], amin, inc)  # U, T of the last call


@pytest.mark.parametrize("overlap", [False, True])
def test_async_host_inputs_reused_without_sync(oracle_lib, overlap):
    """dm.h's staging contract without any synchronising call in between:
    each pinned ranges buffer is overwritten as soon as the second
    dm_integrate_async after the one that used it has returned (no
    frontiers_end, no dm_synchronize in between), so a copy still pending
    then would read a later batch's ranges; the final map must equal the
    oracle's (the staging event once covered only the pose copy)."""
    import torch

    p, batches, amin, inc = cases.world_case(53, 1200, 1100, 0.05, 8, 1024, 9, region_frac=0.6)
    om = oracle_lib.OracleMap(p)
    for poses, ranges in batches:
        om.integrate(poses, ranges, amin, inc)
    S, N = batches[0][1].shape
    # three buffers: call k's ranges must stay unchanged until call k+2 has
    # returned, so pinned[k % 3] (last read by call k-3) is free once call k-1
    # has returned; a copy of call k-3 still pending would read batch k
    pinned = [torch.empty((S, N), dtype=torch.float32).pin_memory() for _ in range(3)]
    with dm.OccupancyMapper(p) as m:
        m.set_overlap(overlap)
        for k, (poses, ranges) in enumerate(batches):
            buf = pinned[k % 3]
            buf.numpy()[...] = ranges
            m.integrate_async(poses, buf.data_ptr(), S, N, amin, inc)
        m.synchronize()  # the contract's other release point
        for b in pinned:
            b.numpy()[...] = np.nan
        assert_map_equal(m, om)


@pytest.mark.parametrize("overlap", [True, False])
def test_host_pose_ring_matches_device_inputs(overlap):
    """k_beam_prep reads the poses of a host-input call straight
    from the mapped staging ring (kPoseRing slots, rewritten at the same
    address every other call).  Ten host-input calls with a different pose
    set each (both slots reused four times, no synchronising call in between)
    must give exactly the map, U and T of the same batches fed as device
    inputs: a stale pose read from a cached slot would move a scan's rays."""
    import torch

    p, batches, amin, inc = cases.world_case(57, 1500, 1300, 0.05, 6, 1024, 10, region_frac=0.7)
    S, N = batches[0][1].shape
    dev = _device_batches(batches)
    pinned = [torch.empty((S, N), dtype=torch.float32).pin_memory() for _ in range(3)]
    with dm.OccupancyMapper(p) as a, dm.OccupancyMapper(p) as b:
        a.set_overlap(overlap)
        b.set_overlap(overlap)
        for k, (poses, ranges) in enumerate(batches):
            buf = pinned[k % 3]  # free again: call k-3 was two calls ago
            buf.numpy()[...] = ranges
            a.integrate_async(poses, buf.data_ptr(), S, N, amin, inc)
            pz, rz = dev[k]
            b.integrate_device(pz.data_ptr(), S, rz.data_ptr(), N, amin, inc)
        a.synchronize()
        b.synchronize()
        assert a.last_counts() == b.last_counts()
        np.testing.assert_array_equal(a.logodds().view(np.uint32), b.logodds().view(np.uint32))
        np.testing.assert_array_equal(a.state(), b.state())


def test_front_end_gate_timeout_is_a_sticky_error(oracle_lib, monkeypatch):
    """A timed-out front-end hand-off (fault injection: DM_FAULT_GATE=1 makes
    the gate wait for a sequence number that never comes, ~10 us) must not
    apply the previous workspace's items: the map stays unchanged, every
    result-reading call reports DM_ERR_PIPELINE, and dm_reset clears it."""
    from dm import _ffi

    p, batches, amin, inc = cases.world_case(49, 600, 500, 0.05, 4, 720, 2, region_frac=0.7)
    dev = _device_batches(batches)
    monkeypatch.setenv("DM_FAULT_GATE", "1")
    with dm.OccupancyMapper(p) as m:
        monkeypatch.delenv("DM_FAULT_GATE")
        # a first call without overlap fills workspace set 0; the faulted
        # calls then find stale items in both sets
        pose4, rng = dev[0]
        m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), 720, amin, inc)
        m.synchronize()
        before = m.state().copy()
        m.set_overlap(True)
        for pose4, rng in dev:
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), 720, amin, inc)
        m.frontiers_begin()
        with pytest.raises(_ffi.DmError) as e:
            m.frontiers_end()
        assert e.value.code == _ffi.DM_ERR_PIPELINE
        with pytest.raises(_ffi.DmError) as e:
            m.frontiers()
        assert e.value.code == _ffi.DM_ERR_PIPELINE
        with pytest.raises(_ffi.DmError) as e:
            m.last_stats()
        assert e.value.code == _ffi.DM_ERR_PIPELINE
        np.testing.assert_array_equal(m.state(), before)  # no stale re-application
        m.set_overlap(False)
        m.reset()
        om, expect = _oracle_steps(oracle_lib, p, batches, amin, inc)
        for pose4, rng in dev:  # no gate without overlap: the handle works again
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), 720, amin, inc)
        np.testing.assert_array_equal(m.frontiers().clusters, expect[-1])
        assert_map_equal(m, om)
