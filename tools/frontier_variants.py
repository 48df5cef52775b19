#!/usr/bin/env python3
"""A/B timing of libdm builds on the frontier pass (experiment tool, not the
bench): for each library given (csrc `make variant V=...` ->
dm/libdm_V.so), a fresh process builds the C3 bench map (6 batches of
64 x 4096 beams, bench.py's seeds) and the explored map, and times
synchronous frontier passes on both (median wall ms, per-kernel HIP-event
ms).  Usage: python tools/frontier_variants.py dm/libdm.so dm/libdm_a.so ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd")


def child():
    sys.path.insert(0, PKG)
    import time

    import numpy as np
    import torch

    import dm
    from dm import synth

    G, res, S, N = 16384, 0.05, 64, 4096
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    st = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    pool = [st.next_batch() for _ in range(6)]
    dev = torch.device("cuda", 0)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(r).to(dev)) for p, r in pool]
    torch.cuda.synchronize()
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(N))
    m = dm.OccupancyMapper(dm.default_params(G, G, resolution=res))
    out = {"lib": os.path.basename(os.environ.get("DM_LIB", "")),
           "env": {k: v for k, v in os.environ.items() if k.startswith("DM_") and k != "DM_LIB"}}

    def passes(tag, n=20):
        m.frontiers()
        ts = []
        for _ in range(n):
            a = time.perf_counter()
            fr = m.frontiers()
            ts.append(time.perf_counter() - a)
        m.profile(True)
        m.profile_reset()
        for _ in range(10):
            m.frontiers()
        k = m.profile_read()
        m.profile(False)
        out[tag] = {"wall_ms": float(np.median(ts)) * 1e3, "clusters": len(fr),
                    "kernels_us": {n_: round(t / max(1, c) * 1e3, 1) for n_, (c, t) in k.items()}}

    for p4, r in dpool:
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)
    m.synchronize()
    # integrate alone (the pool replayed), then frontier passes on that map
    ti = []
    for k in range(20):
        p4, r = dpool[k % len(dpool)]
        a = time.perf_counter()
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)
        m.synchronize()
        ti.append(time.perf_counter() - a)
    m.profile(True)
    m.profile_reset()
    for k in range(12):
        p4, r = dpool[k % len(dpool)]
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)
    k = m.profile_read()
    m.profile(False)
    out["integrate"] = {"wall_ms": float(np.median(ti)) * 1e3,
                        "kernels_us": {n_: round(t / max(1, c) * 1e3, 1) for n_, (c, t) in k.items()}}
    passes("c3")
    m.set_state(synth.explored_state(world, G, G, res, -half, -half, seed=77))
    passes("explored")
    m.close()
    print(json.dumps(out), flush=True)


def main():
    if sys.argv[1:2] == ["--child"]:
        return child()
    for spec in sys.argv[1:]:
        # LIB[:ENV=VAL,...]
        lib, _, envs = spec.partition(":")
        env = dict(os.environ, DM_LIB=os.path.abspath(os.path.join(PKG, lib) if not os.path.isabs(lib) else lib))
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else json.dumps({"lib": spec, "rc": r.returncode, "err": r.stderr[-800:]}),
              flush=True)
        if r.returncode != 0:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
