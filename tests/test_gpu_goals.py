"""GPU: frontier goal selection on the device (dm_assign_goals, csrc/dm_goals.hip,
SURVEY.md §8(f) f4) against its host restatement dm.goals.assign_goals on
the same cluster list: chosen indices equal, centroids bit for bit.

Cases: clusters of a real mapped world (few thousand clusters, one 4096-record
chunk or two), a random sparse map with ~10^5 single-cell clusters (many
chunks, merge rounds), all-equal utilities (distance_weight 0 and unit sizes:
every choice is a tie, decided by the smaller label), 1 to 256 robots,
min_size / min_distance filters, and the error paths."""
import numpy as np
import pytest

import cases
import dm
from dm.goals import assign_goals

pytestmark = pytest.mark.gpu


def _check(m, clusters, robots, **kw):
    got = m.assign_goals(robots, **kw)
    exp = assign_goals(clusters, robots, **kw)
    assert len(got) == len(exp) == len(robots)
    for g, e in zip(got, exp):
        if e is None:
            assert g is None
        else:
            assert g is not None and g[0] == e[0]
            assert g[1] == e[1]  # same record: the same doubles
    return got


def test_goals_on_mapped_world():
    p, batches, amin, inc = cases.world_case(51, 1024, 1024, 0.05, 16, 1440, 3, region_frac=0.7)
    m = dm.OccupancyMapper(p)
    try:
        for poses, ranges in batches:
            m.integrate(poses, ranges, amin, inc)
        fr = m.frontiers()
        cl = fr.clusters
        assert len(cl) > 20
        rng = np.random.default_rng(5)
        half = 0.5 * 1024 * 0.05
        for R in (1, 8, 64):
            robots = rng.uniform(-half, half, (R, 2))
            _check(m, cl, robots, min_size=8)
            _check(m, cl, robots, min_size=1, distance_weight=0.25, min_distance=1.0)
        # more robots than eligible clusters: the rest get None
        got = _check(m, cl, rng.uniform(-half, half, (256, 2)), min_size=40)
        assert any(g is None for g in got)
    finally:
        m.close()


def test_goals_many_clusters_and_ties():
    W = H = 2048
    p = cases.make_params(W, H)
    rng = np.random.default_rng(9)
    st = np.full((H, W), -1, np.int8)
    # isolated free cells in unknown space: one single-cell cluster each
    ys = rng.integers(0, H // 2, 60000) * 2
    xs = rng.integers(0, W // 2, 60000) * 2
    st[ys, xs] = 0
    st[rng.random((H, W)) < 0.01] = 100
    m = dm.OccupancyMapper(p)
    try:
        m.set_state(st)
        cl = m.frontiers().clusters
        assert len(cl) > 40000  # > 10 chunks of 4096 records: merge rounds
        robots = rng.uniform(-50.0, 50.0, (200, 2))
        _check(m, cl, robots, min_size=1)
        # all utilities equal (unit sizes, no distance term): ties everywhere,
        # each robot takes the smallest label not taken yet
        got = _check(m, cl, robots, min_size=1, distance_weight=0.0)
        assert [g[0] for g in got] == list(range(200))
    finally:
        m.close()


def test_goals_need_a_collected_result():
    p = cases.make_params(256, 256)
    m = dm.OccupancyMapper(p)
    try:
        with pytest.raises(dm.DmError):
            m.assign_goals([(0.0, 0.0)])
        m.frontiers()  # empty map: no clusters
        assert m.assign_goals([(0.0, 0.0), (1.0, 1.0)]) == [None, None]
        with pytest.raises(dm.DmError):
            m.assign_goals(np.zeros((257, 2)))
        # util ranks by IEEE bits, valid for util > 0 only: w < 0 is refused
        # (the host restatement refuses it the same way)
        with pytest.raises(dm.DmError):
            m.assign_goals([(0.0, 0.0)], distance_weight=-0.5)
    finally:
        m.close()
