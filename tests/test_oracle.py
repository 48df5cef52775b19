"""CPU: pin the C oracle (oracle/dm_oracle.c) against an independent
NumPy/scipy restatement (oracle/np_oracle.py) and against the committed
golden fixtures.  No GPU needed."""
import os

import numpy as np
import pytest

import cases
import np_oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_line_matches_numpy(oracle_lib):
    rng = np.random.Generator(np.random.PCG64(0))
    for _ in range(300):
        sx, sy = (int(v) for v in rng.integers(-50, 50, 2))
        ex, ey = sx + int(rng.integers(-80, 80)), sy + int(rng.integers(-80, 80))
        a = oracle_lib.line_cells(sx, sy, ex, ey)
        b = np.array(np_oracle.line(sx, sy, ex, ey))
        np.testing.assert_array_equal(a, b)
        # endpoints, one cell per step of the major axis, 8-connected
        assert tuple(a[0]) == (sx, sy) and tuple(a[-1]) == (ex, ey)
        assert len(a) == max(abs(ex - sx), abs(ey - sy)) + 1
        if len(a) > 1:
            assert np.abs(np.diff(a, axis=0)).max() <= 1


def test_endpoints_match_numpy(oracle_lib):
    p = cases.make_params(96, 80)
    poses, ranges, amin, inc = cases.random_scans(1, p, 4, 200)
    cells, flags = oracle_lib.endpoints(p, poses, ranges, amin, inc)
    ref = np_oracle.endpoints(p, poses, ranges, amin, inc)
    valid = np.nonzero(flags & 1)[0]
    assert list(valid) == [r[0] for r in ref]
    for (b, sx, sy, ex, ey, hit) in ref:
        assert tuple(cells[b]) == (sx, sy, ex, ey)
        assert bool(flags[b] & 2) == hit


@pytest.mark.parametrize("seed,W,H,S,N", [(2, 64, 64, 3, 90), (3, 100, 70, 5, 120), (4, 130, 150, 2, 360)])
def test_integrate_matches_numpy(oracle_lib, seed, W, H, S, N):
    p = cases.make_params(W, H)
    m = oracle_lib.OracleMap(p)
    L = np.zeros((H, W), np.float32)
    st = np.full((H, W), -1, np.int8)
    for k in range(3):
        poses, ranges, amin, inc = cases.random_scans(seed * 10 + k, p, S, N)
        U1, T1 = m.integrate(poses, ranges, amin, inc)
        U2, T2 = np_oracle.integrate(p, L, st, poses, ranges, amin, inc)
        assert (U1, T1) == (U2, T2)
        np.testing.assert_array_equal(m.L.view(np.uint32), L.view(np.uint32))
        np.testing.assert_array_equal(m.state, st)


def test_integrate_band_matches_full(oracle_lib):
    """A row band integrates exactly the full map's rows (sharding basis)."""
    W, H = 90, 200
    p = cases.make_params(W, H)
    full = oracle_lib.OracleMap(p)
    bands = [oracle_lib.OracleMap(cases.make_params(W, H, band_row0=r0, band_rows=min(64, H - r0)))
             for r0 in range(0, H, 64)]
    for k in range(3):
        poses, ranges, amin, inc = cases.random_scans(40 + k, p, 4, 150)
        U, T = full.integrate(poses, ranges, amin, inc)
        us = [b.integrate(poses, ranges, amin, inc) for b in bands]
        assert sum(u for u, _ in us) == U and sum(t for _, t in us) == T
    np.testing.assert_array_equal(np.concatenate([b.L for b in bands]), full.L)
    np.testing.assert_array_equal(np.concatenate([b.state for b in bands]), full.state)


@pytest.mark.parametrize("seed,R,W,kind", [(5, 64, 64, "random"), (6, 77, 131, "random"),
                                          (7, 150, 120, "blob"), (8, 1, 50, "random"),
                                          (9, 40, 1, "random")])
def test_frontiers_match_scipy(oracle_lib, seed, R, W, kind):
    p = cases.make_params(W, R)
    st = cases.random_state(seed, R, W) if kind == "random" else cases.blob_state(seed, R, W)
    m = oracle_lib.OracleMap(p)
    m.state[...] = st
    mask, labels, clusters = m.frontiers()
    F, lab, clu = np_oracle.frontiers(p, st)
    np.testing.assert_array_equal(mask, F)
    np.testing.assert_array_equal(labels, lab)
    assert len(clusters) == len(clu)
    for a, b in zip(clusters, clu):
        assert tuple(int(v) for v in list(a)[:4]) == b[:4]
        assert a["cx_m"] == b[4] and a["cy_m"] == b[5]


def test_frontiers_halo_and_min_size(oracle_lib):
    R, W = 30, 40
    p = cases.make_params(W, 100, band_row0=64, band_rows=R, min_frontier_size=3)
    st = cases.random_state(11, R, W, p_free=0.7, p_occ=0.05)
    hb = cases.random_state(12, 1, W)[0]
    ha = cases.random_state(13, 1, W)[0]
    m = oracle_lib.OracleMap(p)
    m.state[...] = st
    mask, labels, clusters = m.frontiers(hb, ha)
    F, lab, clu = np_oracle.frontiers(p, st, hb, ha)
    np.testing.assert_array_equal(mask, F)
    np.testing.assert_array_equal(labels, lab)
    assert [tuple(int(v) for v in list(a)[:4]) for a in clusters] == [c[:4] for c in clu]
    assert all(c[1] >= 3 for c in clu)


def test_map_image_matches_reference_golden(oracle_lib):
    """get_map_image's pixels, produced by the reference itself
    (tests/golden/make_map_image_golden.py)."""
    d = np.load(os.path.join(GOLD, "map_image_golden.npz"))
    n = len([k for k in d.files if k.startswith("state_")])
    assert n >= 5
    for i in range(n):
        st = d[f"state_{i}"]
        np.testing.assert_array_equal(np_oracle.map_image(st), d[f"image_{i}"])
        m = oracle_lib.OracleMap(cases.make_params(st.shape[1], st.shape[0]))
        m.state[...] = st
        np.testing.assert_array_equal(m.map_image(), d[f"image_{i}"])


def test_oracle_golden_fixtures(oracle_lib):
    """The committed hot-path fixtures (tests/golden/make_oracle_golden.py)
    still reproduce: guards the SPEC against silent drift."""
    path = os.path.join(GOLD, "oracle_golden.npz")
    d = np.load(path)
    names = sorted({k.split("__")[0] for k in d.files})
    assert names
    from golden_io import load_case
    for name in names:
        c = load_case(d, name)
        m = oracle_lib.OracleMap(c["params"])
        for k, (poses, ranges) in enumerate(c["batches"]):
            U, T = m.integrate(poses, ranges, c["amin"], c["inc"])
            assert (U, T) == tuple(c["counts"][k])
        np.testing.assert_array_equal(m.L.view(np.uint32), c["L"].view(np.uint32))
        np.testing.assert_array_equal(m.state, c["state"])
        mask, labels, clusters = m.frontiers()
        np.testing.assert_array_equal(mask, c["mask"])
        np.testing.assert_array_equal(labels, c["labels"])
        np.testing.assert_array_equal(clusters, c["clusters"])


@pytest.mark.parametrize("seed,W,H,S,N,threads", [(31, 300, 260, 8, 720, 4), (32, 1000, 700, 16, 2048, 8),
                                                  (33, 130, 70, 5, 500, 3)])
def test_openmp_restatement_equals_single_thread(oracle_lib, seed, W, H, S, N, threads):
    """dm_oracle_mt.c (bench.py's strong-CPU line) gives dm_oracle.c's
    results bit for bit: U / T, L, state, mask, labels, clusters; also on a
    band with halo rows and with a size filter."""
    p = cases.make_params(W, H, min_frontier_size=1 + seed % 3)
    one = oracle_lib.OracleMap(p)
    mt = oracle_lib.OracleMapMT(p, threads=threads)
    assert mt.threads == threads
    for k in range(3):
        poses, ranges, amin, inc = cases.random_scans(seed * 10 + k, p, S, N)
        assert mt.integrate(poses, ranges, amin, inc) == one.integrate(poses, ranges, amin, inc)
    np.testing.assert_array_equal(mt.L.view(np.uint32), one.L.view(np.uint32))
    np.testing.assert_array_equal(mt.state, one.state)
    for a, b in zip(mt.frontiers(), one.frontiers()):
        np.testing.assert_array_equal(a, b)
    # a band of the same map with halo rows
    bp = cases.make_params(W, H, band_row0=64, band_rows=min(128, H - 64))
    ob, mb = oracle_lib.OracleMap(bp), oracle_lib.OracleMapMT(bp, threads=threads)
    st = one.state
    ob.state[...] = st[64:64 + ob.state.shape[0]]
    mb.state[...] = ob.state
    ha = st[64 + ob.state.shape[0]] if 64 + ob.state.shape[0] < H else None
    for a, b in zip(mb.frontiers(st[63], ha), ob.frontiers(st[63], ha)):
        np.testing.assert_array_equal(a, b)
