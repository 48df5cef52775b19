"""Host-side timing of the pipelined bench loop (C3, one GPU): per step, the
wall time spent in the integrate call, in frontiers_end (waiting for the
previous pass + copying its clusters) and in frontiers_begin (enqueueing the
pass).  Diagnostic only.  usage: python tools/pipeline_probe.py [c5 N]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dm  # noqa: E402
from dm import synth  # noqa: E402


def main():
    G, res, S, N = 16384, 0.05, 64, 4096
    if len(sys.argv) > 1 and sys.argv[1] == "c5":  # "c5 N": 65536^2 @ 1 cm, 64 robots x N beams
        G, res, N = 65536, 0.01, int(sys.argv[2]) if len(sys.argv) > 2 else 48
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    st = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    pool = [st.next_batch() for _ in range(4)]
    dev = torch.device("cuda", 0)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(r).to(dev)) for p, r in pool]
    torch.cuda.synchronize()
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(N))
    m = dm.OccupancyMapper(dm.default_params(G, G, resolution=res))
    m.set_overlap(True)

    def integrate(k):
        p4, r = dpool[k % len(dpool)]
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)

    # raw ctypes calls (no Python wrapper): the C-ABI's own host cost
    import ctypes
    lib, h = m._lib, m._handle()
    buf = np.empty(1 << 16, dtype=np.dtype(dm.CLUSTER_DTYPE))
    bp, bc = buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(buf.shape[0])
    nout = ctypes.c_int64(0)
    raw_args = [(ctypes.c_void_p(p4.data_ptr()), ctypes.c_int32(S), ctypes.c_void_p(r.data_ptr()),
                 ctypes.c_int32(N), ctypes.c_float(amin), ctypes.c_float(inc)) for p4, r in dpool]
    for rep in range(2):
        ti, te, tb = [], [], []
        t0 = time.perf_counter()
        steps, depth = 200, 2
        for k in range(steps):
            a = time.perf_counter()
            pp, ss, rr, nn, am, ic = raw_args[k % len(raw_args)]
            lib.dm_integrate_device(h, ss, pp, nn, rr, am, ic)
            b = time.perf_counter()
            if k >= depth:
                lib.dm_frontiers_end(h, bp, bc, ctypes.byref(nout))
            c = time.perf_counter()
            lib.dm_frontiers_begin(h)
            d = time.perf_counter()
            ti.append(b - a)
            te.append(c - b)
            tb.append(d - c)
        for _ in range(depth):
            lib.dm_frontiers_end(h, bp, bc, ctypes.byref(nout))
        el = time.perf_counter() - t0
        f = lambda v: 1e6 * float(np.median(v[depth:]))
        print(f"raw C-ABI depth 2: {1e6 * el / steps:.1f} us/step; integrate call {f(ti):.1f}, "
              f"frontiers_end {f(te):.1f}, frontiers_begin {f(tb):.1f} us (medians)", flush=True)

    for depth in (1, 2, 1, 2):
        ti, te, tb = [], [], []
        t0 = time.perf_counter()
        steps = 60
        for k in range(steps):
            a = time.perf_counter()
            integrate(k)
            b = time.perf_counter()
            if k >= depth:
                m.frontiers_end()
            c = time.perf_counter()
            m.frontiers_begin()
            d = time.perf_counter()
            ti.append(b - a)
            te.append(c - b)
            tb.append(d - c)
        for _ in range(depth):
            m.frontiers_end()
        el = time.perf_counter() - t0
        f = lambda v: 1e6 * float(np.median(v[depth:]))
        print(f"depth {depth}: {1e6 * el / steps:.1f} us/step; integrate call {f(ti):.1f}, "
              f"frontiers_end {f(te):.1f}, frontiers_begin {f(tb):.1f} us (medians)", flush=True)
    m.close()


if __name__ == "__main__":
    main()
