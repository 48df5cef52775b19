"""GPU: the exact configuration the bench line times, at full size
(VERDICT r4 item 1).  bench.py's C3 sequence on one MI355X: a 16384² map,
the pool of 6 batches of 64 x 4096 beams (synth.c3_pool, the batches bench.py
replays), the untimed counts loop, band.reset(), overlap on, then 5 + 20
pipelined depth-2 steps (integrate_device + frontiers_begin / _end), so the
tile-list rebuilds after 1, 2, 4, 8 and 16 passes and the hint-sized
accumulation / frontier grids all run.  Every collected pass must equal the
oracle's clusters after its own batch, and the final map must equal the
oracle's bit for bit.  Plus the work-hint undershoot: a tiny call, then a
full C3 batch whose accumulation grid is sized from the tiny call's work.

Anchor: the /map consumer the clusters feed,
/root/reference/server/thymio_project/thymio_project/main.py:80-81."""
import os

import numpy as np
import pytest

import dm
from dm import synth
from test_gpu_parity import assert_map_equal

pytestmark = pytest.mark.gpu

G, S, N, POOL = 16384, 64, 4096, 6


def _threads():
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(env)) if env.isdigit() and int(env) > 0 else n


@pytest.fixture(scope="module")
def c3():
    import torch

    world, (ox, oy), pool = synth.c3_pool(0, G, S, N, POOL)
    p = dm.default_params(G, G, resolution=0.05)
    p.origin_x, p.origin_y = ox, oy
    amin = float(synth.LD06_ANGLE_MIN)
    inc = float(synth.ld06_angle_increment(N))
    dpool = [(torch.from_numpy(synth.pose4(q)).cuda(), torch.from_numpy(np.ascontiguousarray(r)).cuda())
             for q, r in pool]
    torch.cuda.synchronize()
    return p, pool, dpool, amin, inc


def test_bench_c3_sequence_pipelined_matches_oracle(oracle_lib, c3):
    """bench.py main(): counts loop, reset, warm-up run_steps(0, 5), timed
    run_steps(5, 20); depth 2, order 'eb'."""
    p, pool, dpool, amin, inc = c3
    warmup, steps, depth = 5, 20, 2
    with dm.OccupancyMapper(p) as m:
        def integrate(k):
            pose4, rng = dpool[k % len(dpool)]
            m.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), N, amin, inc)

        for k in range(len(dpool)):  # the counts loop (before overlap is switched on)
            integrate(k)
            m.last_stats()
        m.reset()
        m.set_overlap(True)
        got = []

        def run_steps(k0, n):
            for k in range(n):
                integrate(k0 + k)
                if k >= depth:
                    got.append(m.frontiers_end())
                m.frontiers_begin()
            for _ in range(min(depth, n)):
                got.append(m.frontiers_end())

        run_steps(0, warmup)
        run_steps(warmup, steps)
        m.synchronize()
        assert len(got) == warmup + steps
        om = oracle_lib.OracleMapMT(p, threads=_threads())
        for k, fr in enumerate(got):
            poses, ranges = pool[k % POOL]
            om.integrate(poses, ranges, amin, inc)
            _, _, clusters = om.frontiers(want_mask=False, want_labels=False)
            assert fr is not None, f"pass {k}: no result"
            np.testing.assert_array_equal(fr.clusters, clusters, err_msg=f"pass {k}")
            assert len(clusters) > 100
        m.set_overlap(False)
        assert_map_equal(m, om)


def test_hint_undershoot_then_full_batch(oracle_lib, c3):
    """A one-scan call leaves a tiny work hint; the next call (a full C3
    batch, ~3.8k work items) launches its accumulation and fmask grids sized
    from it (the kernels grid-stride, and sparse items wrap around the grid)
    and its frontier pass after a pass over the tiny map.  Synchronous and
    pipelined."""
    p, pool, dpool, amin, inc = c3
    om = oracle_lib.OracleMapMT(p, threads=_threads())
    with dm.OccupancyMapper(p) as m:
        for overlap in (False, True):
            m.reset()
            om.L[:] = 0.0
            om.state[:] = -1
            m.set_overlap(overlap)
            seq = [(pool[0][0][:1], pool[0][1][:1]), pool[1], (pool[2][0][:1], pool[2][1][:1]), pool[3],
                   (pool[4][0][:2, :], pool[4][1][:2, :360]), pool[5]]
            for poses, ranges in seq:
                n = ranges.shape[1]
                inc_n = float(synth.ld06_angle_increment(n))
                got = m.integrate(poses, ranges, amin, inc_n)
                exp = om.integrate(poses, ranges, amin, inc_n)
                assert got == exp, (overlap, got, exp)
                fr = m.frontiers()
                _, _, clusters = om.frontiers(want_mask=False, want_labels=False)
                np.testing.assert_array_equal(fr.clusters, clusters)
            m.set_overlap(False)
            assert_map_equal(m, om)
