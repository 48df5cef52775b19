"""CPU: frontier goal selection (dm/goals.py)."""
import numpy as np

from dm._ffi import CLUSTER_DTYPE
from dm.goals import assign_goals, select_goal


def clusters(rows):
    a = np.zeros(len(rows), dtype=np.dtype(CLUSTER_DTYPE))
    for i, (label, size, x, y) in enumerate(rows):
        a[i] = (label, size, 0, 0, x, y)
    return a


def test_select_prefers_big_and_near():
    c = clusters([(10, 5, 1.0, 0.0), (20, 50, 2.0, 0.0), (30, 50, 20.0, 0.0)])
    assert select_goal(c, (0.0, 0.0), min_size=8)[0] == 1
    assert select_goal(c, (0.0, 0.0), min_size=100) is None
    assert select_goal(clusters([]), (0, 0)) is None


def test_ties_break_on_label_and_min_distance():
    c = clusters([(7, 10, 1.0, 0.0), (3, 10, -1.0, 0.0)])
    assert select_goal(c, (0.0, 0.0), min_size=1)[0] == 1  # label 3 < 7
    assert select_goal(c, (0.9, 0.0), min_size=1, min_distance=0.5)[0] == 1


def test_assign_distinct_goals():
    c = clusters([(1, 40, 0.0, 5.0), (2, 40, 0.0, -5.0), (3, 1, 9.0, 9.0)])
    goals = assign_goals(c, [(0.0, 4.0), (0.0, -4.0), (0.0, 0.0)], min_size=8)
    assert goals[0][0] == 0 and goals[1][0] == 1 and goals[2] is None


def test_negative_distance_weight_refused():
    """A negative weight makes util negative or infinite; dm_assign_goals
    refuses it (its device keys order positive utils only), and so does the
    host restatement."""
    import pytest

    c = clusters([(10, 5, 1.0, 1.0)])
    with pytest.raises(ValueError):
        assign_goals(c, [(0.0, 0.0)], distance_weight=-1.0)
