"""Generate tests/golden/oracle_golden.npz: small seeded hot-path cases with
the C oracle's outputs, cross-checked against the NumPy restatement before
they are written.  Inputs + expected outputs only (no code).

    python tests/golden/make_oracle_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path[:0] = [TESTS, os.path.join(os.path.dirname(TESTS), "oracle"),
                os.path.join(os.path.dirname(TESTS), "distributed-autonomous-exploration-and-mapping_amd")]

import cases  # noqa: E402
import np_oracle  # noqa: E402
import oracle  # noqa: E402
from golden_io import dump_case  # noqa: E402


def run(name, p, batches, amin, inc, arrays):
    m = oracle.OracleMap(p)
    R, W = m.L.shape
    L = np.zeros((R, W), np.float32)
    st = np.full((R, W), -1, np.int8)
    counts = []
    for poses, ranges in batches:
        c = m.integrate(poses, ranges, amin, inc)
        c2 = np_oracle.integrate(p, L, st, poses, ranges, amin, inc)
        assert c == c2, (name, c, c2)
        counts.append(c)
    assert np.array_equal(m.L.view(np.uint32), L.view(np.uint32)) and np.array_equal(m.state, st)
    mask, labels, clusters = m.frontiers()
    F, lab, clu = np_oracle.frontiers(p, m.state)
    assert np.array_equal(mask, F) and np.array_equal(labels, lab) and len(clu) == len(clusters)
    dump_case(arrays, name, p, batches, amin, inc, counts, m.L, m.state, mask, labels, clusters)
    print(f"{name}: {R}x{W}, {len(batches)} batches, U={sum(c[0] for c in counts)}, "
          f"clusters={len(clusters)}")


def main():
    oracle.build()
    arrays = {}
    p = cases.make_params(64, 64)
    run("tiny64", p, [cases.random_scans(100 + k, p, 3, 90)[:2] for k in range(3)],
        0.0, float(np.float32(2 * np.pi / 89)), arrays)
    p, batches, amin, inc = cases.world_case(1, 400, 400, 0.05, 1, 360, 12)
    run("c1_room", p, batches, amin, inc, arrays)
    p = cases.make_params(130, 70)
    run("ragged", p, [cases.random_scans(200 + k, p, 4, 200)[:2] for k in range(2)],
        0.0, float(np.float32(2 * np.pi / 199)), arrays)
    p = cases.make_params(96, 96, resolution=0.1)
    run("offgrid", p, [cases.random_scans(300 + k, p, 6, 64, spread=4.0)[:2] for k in range(2)],
        0.0, float(np.float32(2 * np.pi / 63)), arrays)
    out = os.path.join(HERE, "oracle_golden.npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
