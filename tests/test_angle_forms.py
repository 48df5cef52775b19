"""How often the SPEC's angle-addition beam direction (DESIGN.md §2.1:
dcx = cos(yaw)·cos(φ) − sin(yaw)·sin(φ), each product rounded) lands the
endpoint in a different cell than SURVEY.md §8 a4's literal form
cos(yaw + φ) (yaw + φ rounded to double first), on C3 inputs and on a 1 cm
map (C5 geometry, 12 m rays = 1200 cells, where a ULP of the direction is
worth the most cells).

The endpoint cell decides the whole Bresenham line, so a beam whose
endpoint cell agrees under both forms updates exactly the same cells.
Measured here (seeded, deterministic): 8 batches of 64 × 4096 beams each
for C3 (5 cm) and C5 (1 cm), beams with a return or a max-range miss; the
counts are printed and asserted.  Both forms are evaluated with the C
library's cos/sin (Python's math.cos / math.sin call glibc, as libdm's host
side and the oracle do; NumPy's vectorised np.cos may differ from glibc by an
ulp) and IEEE double products/sums without FMA: this measures
the spec choice, not a device kernel."""
import math

import numpy as np

import dm  # noqa: F401  (package path set up by conftest)
from dm import synth


def _cells(poses, ranges, amin, inc, ox, oy, res, rmax, form):
    n = ranges.shape[1]
    phi = np.float64(amin) + np.arange(n, dtype=np.float64) * np.float64(inc)
    x = poses[:, 0:1]
    y = poses[:, 1:2]
    yaw = poses[:, 2:3]
    r = ranges.astype(np.float32)
    ok = np.isfinite(r) & (r >= np.float32(0.02))
    rr = np.where(r <= np.float32(rmax), r.astype(np.float64), np.float64(rmax))
    cos, sin = np.frompyfunc(math.cos, 1, 1), np.frompyfunc(math.sin, 1, 1)  # glibc, per element
    if form == "spec":
        cy, sy = cos(yaw).astype(np.float64), sin(yaw).astype(np.float64)
        cphi, sphi = cos(phi).astype(np.float64)[None, :], sin(phi).astype(np.float64)[None, :]
        dcx = cy * cphi - sy * sphi
        dcy = sy * cphi + cy * sphi
    else:
        th = yaw + phi[None, :]
        dcx, dcy = cos(th).astype(np.float64), sin(th).astype(np.float64)
    ex = x + rr * dcx
    ey = y + rr * dcy
    cx = np.floor((ex - ox) / res)
    cy_ = np.floor((ey - oy) / res)
    return cx, cy_, ok


def _count(cfg, n_beams, seed):
    world, W, H, res, ox, oy = synth.config_world(cfg, seed)
    half_x, half_y = -ox, -oy
    st = synth.ScanStream(world, 64, n_beams, seed * 1000 + 11,
                          region=(ox + 1.0, oy + 1.0, half_x - 1.0, half_y - 1.0))
    amin = float(synth.LD06_ANGLE_MIN)
    inc = float(synth.ld06_angle_increment(n_beams))
    rmax = 12.0
    beams = diff = 0
    for _ in range(8):
        poses, ranges = st.next_batch()
        a = _cells(poses, ranges, amin, inc, ox, oy, res, rmax, "spec")
        b = _cells(poses, ranges, amin, inc, ox, oy, res, rmax, "sum")
        ok = a[2]
        beams += int(ok.sum())
        diff += int((ok & ((a[0] != b[0]) | (a[1] != b[1]))).sum())
    return beams, diff


def test_angle_addition_vs_sum_form_c3():
    beams, diff = _count("C3", 4096, 0)
    print(f"C3: {diff} of {beams} endpoint cells differ ({diff / beams:.2e})")
    assert beams > 800_000
    # a direction ULP moves a 12 m endpoint by ~1e-15 m: only endpoints within
    # that of a cell boundary can flip; measured: none
    assert diff == 0


def test_angle_addition_vs_sum_form_c5_1cm():
    beams, diff = _count("C5", 4096, 0)
    print(f"C5 (1 cm): {diff} of {beams} endpoint cells differ ({diff / beams:.2e})")
    assert beams > 800_000
    assert diff == 0  # measured
