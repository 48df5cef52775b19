"""Diagnostic: the C5 test's 26-band sharded handle (tests/test_gpu_c5_full.py
workload), many pipelined passes compared with the synchronous result;
prints every pass without a result and its message."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"),
          os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import dm  # noqa: E402
import test_gpu_c5_full as t5  # noqa: E402

n_beams = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p, batches, amin, inc = t5._c5_batches(n_beams, 2, 9100 + n_beams)
sh = dm.OccupancyMapper(p, devices=[0] * t5.P)
for poses, ranges in batches:
    sh.integrate(poses, ranges, amin, inc)
ref = sh.frontiers(want_mask=True).clusters
print("clusters", len(ref), flush=True)
bad = 0
for it in range(iters):
    sh.frontiers_begin()
    sh.frontiers_begin()
    for j in range(2):
        fr = sh.frontiers_end()
        if fr is None or not np.array_equal(fr.clusters, ref):
            bad += 1
            print("iter", it, j, "no result" if fr is None else "DIFFERENT", sh.last_incomplete, flush=True)
    if it % 5 == 0:
        fr = sh.frontiers()
        print("iter", it, "sync ok" if np.array_equal(fr.clusters, ref) else "sync DIFFERENT", flush=True)
print("bad", bad, "of", 2 * iters, flush=True)
sh.close()
