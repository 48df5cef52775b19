"""Step-cycle probe (C3 workload, one GPU): where the pipelined step's time
goes.  Times K steps of
  full   integrate + frontier pass, pipelined as bench.py (overlap on, depth 2)
  int    integrate only, overlap on (front-end on its own stream)
  int1   integrate only, overlap off (one stream)
  pass4  integrate every step, a frontier pass every 4th step
Prints us per step for each mode.  Diagnostic only (never the bench line).
Usage: python tools/cycle_probe.py [steps]"""
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    G, res, S, N = 16384, 0.05, 64, 4096
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    st = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    pool = [st.next_batch() for _ in range(6)]
    dev = torch.device("cuda", 0)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(np.ascontiguousarray(r)).to(dev))
             for p, r in pool]
    torch.cuda.synchronize()
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(N))
    params = dm.default_params(G, G, resolution=res)
    params.origin_x = -half
    params.origin_y = -half
    m = dm.OccupancyMapper(params, device=0)

    def integ(k):
        p4, r = dpool[k % len(dpool)]
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)

    def run(mode, n):
        if mode == "int1":
            m.set_overlap(False)
        else:
            m.set_overlap(True)
        inflight = 0
        for k in range(n):
            integ(k)
            if mode in ("full", "pass4") and (mode == "full" or k % 4 == 0):
                if inflight >= 2:
                    m.frontiers_end()
                    inflight -= 1
                m.frontiers_begin()
                inflight += 1
        while inflight:
            m.frontiers_end()
            inflight -= 1
        m.synchronize()

    for mode in ("full", "int", "int1", "pass4", "full", "int"):
        run(mode, 30)
        t0 = time.perf_counter()
        run(mode, steps)
        dt = (time.perf_counter() - t0) / steps
        print(f"{mode:6s} {dt * 1e6:8.1f} us/step", flush=True)
    m.close()


if __name__ == "__main__":
    main()
