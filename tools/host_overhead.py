"""Host-side cost of the bench step (C3, one GPU): wall time of the Python
wrapper calls vs the raw ctypes calls vs the GPU span, to see where the
step's non-GPU time goes.  Diagnostic only."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dm  # noqa: E402
from dm import synth  # noqa: E402


def med(f, n=30):
    ts = []
    for _ in range(n):
        a = time.perf_counter()
        f()
        ts.append(time.perf_counter() - a)
    return 1e6 * float(np.median(ts))


def main():
    G, res, S, N = 16384, 0.05, 64, 4096
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    st = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    pool = [st.next_batch() for _ in range(3)]
    dev = torch.device("cuda", 0)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(r).to(dev)) for p, r in pool]
    torch.cuda.synchronize()
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(N))
    m = dm.OccupancyMapper(dm.default_params(G, G, resolution=res))
    lib, h = m._lib, m._h
    k = [0]

    def integ():
        p4, r = dpool[k[0] % 3]
        k[0] += 1
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)

    for _ in range(8):
        integ()
        m.frontiers()
    buf = np.empty(1 << 14, dtype=np.dtype(dm._ffi.CLUSTER_DTYPE))
    n = ctypes.c_int64(0)
    out = {"ctypes_noop_us": med(lambda: lib.dm_last_error(), 200)}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    acc = {k: [] for k in ("integ_enqueue", "integ_total", "fr_wrapper", "fr_ctypes", "step")}
    for rep in range(30):
        m.synchronize()
        a = time.perf_counter()
        integ()
        b = time.perf_counter()
        m.synchronize()
        c = time.perf_counter()
        acc["integ_enqueue"].append(b - a)
        acc["integ_total"].append(c - a)
        a = time.perf_counter()
        m.frontiers()
        acc["fr_wrapper"].append(time.perf_counter() - a)
        a = time.perf_counter()
        lib.dm_frontiers(h, None, None, buf.ctypes.data_as(ctypes.c_void_p), buf.shape[0], ctypes.byref(n))
        acc["fr_ctypes"].append(time.perf_counter() - a)
        a = time.perf_counter()
        integ()
        m.frontiers()
        acc["step"].append(time.perf_counter() - a)
    for key, v in acc.items():
        out[key + "_us"] = 1e6 * float(np.median(v))
    for key, v in out.items():
        print(f"{key:28s} {v:9.1f}")
    m.close()


if __name__ == "__main__":
    main()
