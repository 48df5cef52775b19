#!/usr/bin/env python3
"""Frontier passes alone over a C3-sized (16384²) map, for rocprofv3 runs
(kernel stats and PMC passes of the `C3-explored` workload):

  --map explored   synth.explored_state: free space, obstacle outlines with
                   unknown interiors, unknown pockets (>= 90 % of the tiles hold
                   free cells: the pass's worst case, every tile read)

Prints one JSON line (median wall ms per pass, per-kernel HIP-event ms)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", default="explored", choices=["explored"])
    ap.add_argument("--grid", type=int, default=16384)
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import numpy as np

    import dm
    from dm import synth

    res = 0.05
    G = a.grid
    half = G * res / 2.0
    world = synth.make_world(a.seed * 1000, -half, -half, half, half)
    st = synth.explored_state(world, G, G, res, -half, -half, seed=a.seed * 1000 + 77)
    p = dm.default_params(G, G, resolution=res)
    with dm.OccupancyMapper(p) as m:
        m.set_state(st)
        del st
        m.frontiers()
        ts = []
        for _ in range(a.passes):
            t0 = time.perf_counter()
            fr = m.frontiers()
            ts.append(time.perf_counter() - t0)
        st_ = m.last_stats()
        m.profile(True)
        m.profile_reset()
        for _ in range(5):
            m.frontiers()
        k = m.profile_read()
    print(json.dumps({"map": a.map, "grid": G, "frontier_ms": float(np.median(ts)) * 1e3,
                      "clusters": len(fr), "frontier_cells": int(fr.clusters["size"].sum()),
                      "tiles_visited": st_["frontier_tiles"],
                      "kernel_avg_ms": {n: t / max(1, c) for n, (c, t) in k.items()}}), flush=True)


if __name__ == "__main__":
    main()
