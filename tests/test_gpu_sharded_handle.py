"""GPU: one map sharded in row bands behind ONE handle (dm_create_sharded,
include/dm.h; SURVEY.md §8(b) "sharded variants ... with the same calls").

The bands live on cuda:0 (devices {0, 0, ...}: 8-GPU runs are the driver's);
the exchange is the same code path as on several devices (peer copies
degenerate to device copies).  Every call is checked against one dm_create
handle of the same params fed the same scans, and against the CPU oracle:
U / T, L bit for bit, state, mask, global min-index labels, clusters,
pipelined passes, goals, the /map-image pixels, checkpoints, device inputs."""
import ctypes

import numpy as np
import pytest

import cases
import dm
from dm import _ffi, synth

pytestmark = pytest.mark.gpu


def _world(seed, W, H, S=6, N=720, nb=3):
    p = cases.make_params(W, H)
    half_w, half_h = W * p.resolution / 2, H * p.resolution / 2
    world = synth.make_world(seed, -half_w, -half_h, half_w, half_h)
    stream = synth.ScanStream(world, S, N, seed + 1, region=(-half_w * 0.9, -half_h * 0.9, half_w * 0.9,
                                                              half_h * 0.9))
    return p, [stream.next_batch() for _ in range(nb)], float(synth.LD06_ANGLE_MIN), \
        float(synth.ld06_angle_increment(N))


@pytest.mark.parametrize("P,W,H,seed", [(1, 300, 200, 1), (2, 640, 700, 2), (3, 500, 900, 3),
                                        (5, 700, 1200, 4)])
def test_sharded_handle_equals_single_handle_and_oracle(oracle_lib, P, W, H, seed):
    p, batches, amin, inc = _world(seed, W, H)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p) as single, dm.OccupancyMapper(p, devices=[0] * P) as sh:
        assert sh.rows == H and sh.row0 == 0
        for poses, ranges in batches:
            exp = om.integrate(poses, ranges, amin, inc)
            assert single.integrate(poses, ranges, amin, inc) == exp
            assert sh.integrate(poses, ranges, amin, inc) == exp
        np.testing.assert_array_equal(sh.logodds().view(np.uint32), om.L.view(np.uint32))
        np.testing.assert_array_equal(sh.state(), om.state)
        mask, labels, clusters = om.frontiers()
        assert len(clusters) > 3
        fr = sh.frontiers(want_mask=True, want_labels=True)
        np.testing.assert_array_equal(fr.mask, mask)
        np.testing.assert_array_equal(fr.labels, labels)  # global min-index labels
        np.testing.assert_array_equal(fr.clusters, clusters)
        np.testing.assert_array_equal(sh.frontiers().clusters, clusters)
        np.testing.assert_array_equal(sh.map_image(), single.map_image())
        # goals over the last collected result
        robots = [tuple(q[:2]) for q in batches[-1][0][:3]]
        single.frontiers()
        assert sh.assign_goals(robots, min_size=2) == single.assign_goals(robots, min_size=2)


def test_sharded_pipelined_passes_and_poll(oracle_lib):
    p, batches, amin, inc = _world(11, 800, 1100, S=8, N=1024, nb=5)
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p, devices=[0, 0, 0, 0]) as sh:
        sh.set_overlap(True)
        got, expect = [], []
        for k, (poses, ranges) in enumerate(batches):
            sh.integrate(poses, ranges, amin, inc)
            om.integrate(poses, ranges, amin, inc)
            expect.append(om.frontiers(want_mask=False, want_labels=False)[2])
            if k > 1:
                got.append(sh.frontiers_end())
            sh.frontiers_begin()
        while not sh.frontiers_ready():
            pass
        got.append(sh.frontiers_end())
        got.append(sh.frontiers_end())
        assert len(got) == len(expect)
        for fr, exp in zip(got, expect):
            assert fr is not None
            np.testing.assert_array_equal(fr.clusters, exp)
        # a synchronous pass with two passes in flight
        sh.frontiers_begin()
        sh.frontiers_begin()
        np.testing.assert_array_equal(sh.frontiers().clusters, expect[-1])
        np.testing.assert_array_equal(sh.frontiers_end().clusters, expect[-1])
        np.testing.assert_array_equal(sh.frontiers_end().clusters, expect[-1])


def test_sharded_min_size_device_inputs_and_checkpoint(oracle_lib, tmp_path):
    import torch

    p, batches, amin, inc = _world(21, 600, 800, S=5, N=900, nb=3)
    p.min_frontier_size = 6
    om = oracle_lib.OracleMap(p)
    with dm.OccupancyMapper(p, devices=[0, 0, 0]) as sh:
        for poses, ranges in batches:
            pose4 = torch.from_numpy(synth.pose4(poses)).cuda()
            rng = torch.from_numpy(np.ascontiguousarray(ranges)).cuda()
            torch.cuda.synchronize()
            sh.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), ranges.shape[1], amin, inc)
            assert sh.last_counts() == om.integrate(poses, ranges, amin, inc)
        clusters = om.frontiers(want_mask=False, want_labels=False)[2]
        assert (clusters["size"] >= 6).all() and len(clusters) > 0
        np.testing.assert_array_equal(sh.frontiers().clusters, clusters)
        # the checkpoint format of one full-map handle, both ways
        path = str(tmp_path / "sharded.dmap")
        sh.save(path)
        with dm.OccupancyMapper(p) as single:
            single.load(path)
            np.testing.assert_array_equal(single.logodds().view(np.uint32), om.L.view(np.uint32))
            single.reset()
            single.integrate(*batches[0], amin, inc)
            single.save(path)
        sh.load(path)
        om2 = oracle_lib.OracleMap(p)
        om2.integrate(*batches[0], amin, inc)
        np.testing.assert_array_equal(sh.state(), om2.state)
        sh.reset()
        assert (sh.state() == -1).all()


def test_sharded_refuses_the_multi_process_building_blocks():
    p = cases.make_params(256, 512)
    with dm.OccupancyMapper(p, devices=[0, 0]) as sh:
        lib, h = sh._lib, sh._handle()
        n = ctypes.c_int64(0)
        assert lib.dm_export_bytes(h, 16, ctypes.byref(n)) == _ffi.DM_ERR_INVALID_ARG
        assert lib.dm_set_halo(h, None, None) == _ffi.DM_ERR_INVALID_ARG
        assert lib.dm_set_stream(h, None) == _ffi.DM_ERR_INVALID_ARG
        assert lib.dm_frontiers_end(h, None, 0, ctypes.byref(n)) == _ffi.DM_ERR_INVALID_ARG
        nr, cap = ctypes.c_int32(0), ctypes.c_int64(0)
        assert lib.dm_sharded_info(h, ctypes.byref(nr), ctypes.byref(cap)) == 0 and nr.value == 2
    # a band per device entry needs rows: 2 tiles of rows cannot make 3 bands
    with pytest.raises(dm.DmError):
        dm.OccupancyMapper(cases.make_params(100, 128), devices=[0, 0, 0])


def test_mapping_node_shards_over_dm_devices(oracle_lib):
    """The drop-in: MappingNode(dm_devices="0,0,0") builds one sharded
    handle; its /map equals the oracle's over the same scans."""
    from dm.ros_node import LaserScan, MappingNode

    p, batches, amin, inc = _world(31, 400, 600, S=1, N=450, nb=6)
    poses_by_scan = {}
    node = MappingNode(dm_width=400, dm_height=600, dm_devices="0,0,0", gate=False,
                       pose_provider=lambda m: poses_by_scan[id(m)], clock=lambda: 5.0)
    om = oracle_lib.OracleMap(p)
    try:
        assert node.mapper.devices == [0, 0, 0]
        for poses, ranges in batches:
            msg = LaserScan(angle_min=amin, angle_increment=inc, ranges=ranges[0])
            poses_by_scan[id(msg)] = tuple(poses[0])
            node.scan_cb(msg)
            om.integrate(poses, ranges, amin, inc)
        node.timer_cb()
        assert node.poll_frontiers(wait=True)
        data = np.frombuffer(node.map_pub.messages[-1].data, np.int8).reshape(600, 400)
        np.testing.assert_array_equal(data, om.state)
        exp = om.frontiers(want_mask=False, want_labels=False)[2]
        assert [c.label for c in node.frontier_pub.messages[-1]] == exp["label"].tolist()
    finally:
        node.destroy_node()


def test_sharded_ld06_device_then_integrate_device_without_host_sync(oracle_lib):
    """dm_ld06_to_scans_device writes the scans on band 0's stream; the next
    dm_integrate_device must order every band's reads after it (ADVICE r3:
    bands 1..P-1 run on their own streams).  No host synchronisation between
    the two calls; the ranges buffer starts with values the LD06 kernel
    overwrites, so a band that read early would integrate them."""
    import torch

    p = cases.make_params(500, 1200)
    world = synth.make_world(5, -12.5, -30.0, 12.5, 30.0)
    rng = np.random.Generator(np.random.PCG64(8))
    S, N = 24, 450
    poses = np.array([[rng.uniform(-10, 10), rng.uniform(-28, 28), rng.uniform(-3, 3)] for _ in range(S)])
    revs = [synth.ld06_points(world, x, y, yaw, rng) for x, y, yaw in poses]
    pts = np.ascontiguousarray(np.concatenate(revs), dtype=np.dtype(_ffi.LD06_POINT_DTYPE))
    off = np.cumsum([0] + [len(r) for r in revs]).astype(np.int64)
    inc = float(synth.ld06_angle_increment(N))
    er, _ = oracle_lib.ld06_to_scans(pts, off, N, True)
    om = oracle_lib.OracleMap(p)
    om.integrate(poses, er, 0.0, inc)
    d_pts = torch.from_numpy(pts.view(np.uint8).copy()).cuda()
    d_off = torch.from_numpy(off).cuda()
    d_pose4 = torch.from_numpy(synth.pose4(poses)).cuda()
    for devices in ([0, 0, 0], [0, 0, 0, 0, 0]):
        d_rng = torch.full((S, N), 5.0, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        with dm.OccupancyMapper(p, devices=devices) as sh:
            sh.set_overlap(True)
            lib, h = sh._lib, sh._handle()
            assert lib.dm_ld06_to_scans_device(h, S, ctypes.c_void_p(d_pts.data_ptr()),
                                               ctypes.c_void_p(d_off.data_ptr()), N, 1,
                                               ctypes.c_void_p(d_rng.data_ptr()), None) == 0
            sh.integrate_device(d_pose4.data_ptr(), S, d_rng.data_ptr(), N, 0.0, inc)
            np.testing.assert_array_equal(sh.state(), om.state)
            np.testing.assert_array_equal(sh.logodds().view(np.uint32), om.L.view(np.uint32))
