"""Per-workgroup timeline of k_tile_accum at C3, from the
opt-in timing build (csrc `make phase` -> dm/libdm_phase.so, DM_TL_* in
dm_phase.h).  Runs the bench's pipelined steps (integrate + frontier pass,
overlap on), then reads the last launch's record of every workgroup: start and
end (100 MHz wall clock), XCC / CU, items it ran, and the heavy finisher's span.

Prints the launch span, when workgroups were dispatched (start histogram),
how many were resident over time (the concurrency curve against the chip's
7 x 256 slots), the item-carrying workgroups' durations, and what ran in the
tail.  Diagnostic only; never part of the product path.

usage: python tools/accum_timeline.py [steps] [--json OUT]
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd")
os.environ.setdefault("DM_LIB", os.path.join(PKG, "dm", "libdm_phase.so"))
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dm  # noqa: E402
from dm import synth  # noqa: E402

TICK_US = 0.01  # wall_clock64: 100 MHz


def run(steps, overlap=True):
    G, res, S, N = 16384, 0.05, 64, 4096
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    st = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    pool = [st.next_batch() for _ in range(4)]
    dev = torch.device("cuda", 0)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(r).to(dev)) for p, r in pool]
    torch.cuda.synchronize()
    amin, inc = float(synth.LD06_ANGLE_MIN), float(synth.ld06_angle_increment(N))
    lib = dm._ffi.load_library()
    rd = lib.dm_debug_timeline_accum
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    m = dm.OccupancyMapper(dm.default_params(G, G, resolution=res))
    m.set_overlap(overlap)
    pending = 0
    for k in range(steps):
        p4, r = dpool[k % len(dpool)]
        m.integrate_device(p4.data_ptr(), S, r.data_ptr(), N, amin, inc)
        if pending == 2:
            m.frontiers_end()
            pending -= 1
        m.frontiers_begin()
        pending += 1
    while pending:
        m.frontiers_end()
        pending -= 1
    m.synchronize()
    n_wg = 16384
    buf = np.zeros(4 * n_wg, np.uint64)
    assert rd(buf.ctypes.data, n_wg) == 0
    m.close()
    return buf.reshape(n_wg, 4)


def summarise(tl):
    t0 = tl[:, 0].astype(np.int64)
    t1 = tl[:, 1].astype(np.int64)
    ok = (t1 >= t0) & (t0 > 0)
    # the grid follows the work (dm_integrate.hip: the mapped work hint), so
    # records past this launch's grid are older launches': keep the last one's
    ok &= t0 >= t0[ok].max() - 50000  # 500 us
    t0, t1, hw, word = t0[ok], t1[ok], tl[ok, 2], tl[ok, 3]
    base = t0.min()
    s = (t0 - base) * TICK_US
    e = (t1 - base) * TICK_US
    dense = (word & 0xFFFF).astype(np.int64)
    sparse = ((word >> 16) & 0xFFFF).astype(np.int64)
    fin = (word >> 32).astype(np.int64) * TICK_US
    xcc = (hw >> 32).astype(np.int64)
    busy = (dense + sparse) > 0
    span = e.max()
    out = {"workgroups": int(ok.sum()), "with_items": int(busy.sum()), "span_us": float(span),
           "last_start_us": float(s.max()), "last_idle_start_us": float(s[~busy].max()) if (~busy).any() else None}
    # dispatch histogram and residency (workgroups alive) in 1 us bins
    bins = np.arange(0.0, span + 1.0, 1.0)
    out["starts_per_us"] = np.histogram(s, bins)[0].tolist()
    out["item_starts_per_us"] = np.histogram(s[busy], bins)[0].tolist()
    alive = [int(((s <= b) & (e > b)).sum()) for b in bins[:-1]]
    alive_items = [int(((s <= b) & (e > b) & busy).sum()) for b in bins[:-1]]
    out["resident"] = alive
    out["resident_with_items"] = alive_items
    d = e[busy] - s[busy]
    out["item_wg_duration_us"] = {"p10": float(np.percentile(d, 10)), "p50": float(np.percentile(d, 50)),
                                  "p90": float(np.percentile(d, 90)), "max": float(d.max()),
                                  "mean": float(d.mean())}
    out["item_wg_end_us"] = {"p50": float(np.percentile(e[busy], 50)), "p90": float(np.percentile(e[busy], 90)),
                             "p99": float(np.percentile(e[busy], 99)), "max": float(e[busy].max())}
    out["idle_wg_duration_us_mean"] = float((e[~busy] - s[~busy]).mean()) if (~busy).any() else None
    out["finishers"] = {"n": int((fin > 0).sum()), "mean_us": float(fin[fin > 0].mean()) if (fin > 0).any() else 0,
                        "max_us": float(fin.max())}
    # tail: the workgroups still running in the last 20 % of the span
    tail = e > 0.8 * span
    out["tail"] = {"n": int(tail.sum()), "heavy_finishers": int((tail & (fin > 0)).sum()),
                   "sparse_wgs": int((tail & (sparse > 0)).sum()), "dense_only": int((tail & (sparse == 0) & busy).sum()),
                   "start_us_p50": float(np.percentile(s[tail], 50)) if tail.any() else None}
    out["per_xcc_end_us"] = {int(x): float(e[xcc == x].max()) for x in np.unique(xcc)}
    out["per_xcc_items"] = {int(x): int((dense + sparse)[xcc == x].sum()) for x in np.unique(xcc)}
    return out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 30
    js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    res = {}
    for pm in ("pipelined", "alone"):
        if True:
            mode = pm
            tl = run(steps, overlap=(pm == "pipelined"))
            res[mode] = summarise(tl)
            r = res[mode]
            print(f"[{mode}] workgroups {r['workgroups']} (with items {r['with_items']}), span {r['span_us']:.1f} us, "
                  f"last start {r['last_start_us']:.1f} us, idle wgs last start {r['last_idle_start_us']}")
            print(f"  item wg duration {r['item_wg_duration_us']}")
            print(f"  item wg end      {r['item_wg_end_us']}")
            print(f"  idle wg mean duration {r['idle_wg_duration_us_mean']}")
            print(f"  heavy finishers {r['finishers']}")
            print(f"  tail {r['tail']}")
            print(f"  per-XCC end {r['per_xcc_end_us']}")
            print(f"  per-XCC items {r['per_xcc_items']}")
            print("  us : starts / item starts / resident / resident with items")
            for b in range(len(r["resident"])):
                print(f"  {b:3d}: {r['starts_per_us'][b]:5d} {r['item_starts_per_us'][b]:5d} {r['resident'][b]:5d} "
                      f"{r['resident_with_items'][b]:5d}")
    if js:
        with open(js, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
