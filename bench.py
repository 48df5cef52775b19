#!/usr/bin/env python3
"""Benchmark: beam-cell updates/s + frontier-extract ms (BASELINE.json metric).

Workload (per GPU): BASELINE config C3 — a 16384 x 16384 grid at 5 cm,
64 robots random-walking in a seeded synthetic world, 64-scan x 4096-beam
LD06-format batches.  One step = integrate one 64-scan batch (inputs already
resident in HBM, dm_integrate_device) + full frontier extraction
(mask + CCL + clusters, clusters copied to the host).  Steps are pipelined
by default: step k's frontier pass (dm_frontiers_begin) is collected
(dm_frontiers_end) after step k+1's integrate call was enqueued, and with
dm_set_overlap step k+1's ray front-end (beam prep, tile planning, piece
scatter) runs beside it; the map update of step k+1 still waits for step k's
frontier pass.  --no-overlap runs the steps back to back.

N GPUs (weak scaling): rank r owns a 16384-row band of a 16384 x 16384*N map
with its own 64 robots anywhere in the band (plus the neighbours' scans that
reach across the band edge); frontiers are merged across bands on the device
(halo rows sent to the two neighbour bands with one batched RCCL send /
receive, RCCL all-gather of the export records over the same communicator,
dm_merge_bands; dm/sharded.py).

Prints ONE JSON line on rank 0.  See DESIGN.md §5 for every field.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd")
sys.path[:0] = [PKG]

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md §Chip-level parameters
TILE_APPLY_BYTES_PER_UPDATE = 8.0   # one 4 B counter RMW per update
TILE_APPLY_BYTES_PER_TOUCHED = 25.0  # read h,m,L; write L, state; zero h,m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=16384, help="cells per side of each GPU's band")
    ap.add_argument("--robots", type=int, default=64)
    ap.add_argument("--beams", type=int, default=4096)
    ap.add_argument("--pool", type=int, default=6, help="distinct pre-generated batches")
    ap.add_argument("--profile-steps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="budget for the CPU-oracle baseline sample (0 disables)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--depth", type=int, default=None,
                    help="frontier passes in flight in the pipelined steps (1 or 2; libdm keeps 2 readback "
                         "slots); default 2, and 1 for the 400² one-scan replay C1 (depth 2 measured no "
                         "faster there and less steady: profiles/r06_depth_ab.log)")
    ap.add_argument("--pin-host", default="auto", choices=["auto", "off"],
                    help="auto: the host thread on the CPUs of the GPU's NUMA node (pin_host_near_gpu)")
    ap.add_argument("--order", default="eb", choices=["eb", "be"],
                    help="host order per pipelined step after integrate(k): 'eb' collects pass "
                         "k-depth then starts pass k; 'be' starts pass k then collects pass "
                         "k-depth (depth + 1 passes in flight)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the steps back to back without overlapping step k+1's integrate "
                         "front-end with step k's frontier pass")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1")
    ap.add_argument("--records-comm", default="shared", choices=["shared", "separate"],
                    help="N>1: all-gather the export records over the halo exchange's communicator "
                         "(shared, default) or over a second one (separate; dm/sharded.py)")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="N>1: seconds a collective may take before the job fails (DM_ERR_COLLECTIVE)")
    ap.add_argument("--device-override", type=int, default=None,
                    help="put every rank on this GPU (rehearsal with --backend gloo)")
    ap.add_argument("--config", default="C3", choices=["C3", "C1", "C2", "C4", "C5"],
                    help="C3 (default, the bench line): 16384² batches; C1 / C2: 400² / 4096² "
                         "single-robot scan-by-scan replay; C4: one 32768² map shared by 32 robots, "
                         "row bands over the ranks (strong scaling); C5: 65536² @1cm "
                         "beam-density sweep (single GPU)")
    ap.add_argument("--scans", type=int, default=None,
                    help="C1 / C2: scans in the replay (default 1000 / 10000)")
    ap.add_argument("--sweep", default="12,48,192,768,4096", help="C5: beams per scan")
    ap.add_argument("--no-explored", action="store_true",
                    help="skip the explored-map frontier measurement (frontier_ms_explored)")
    ap.add_argument("--no-host-inputs", action="store_true",
                    help="skip the PCIe-inclusive measurement (value_host_inputs)")
    ap.add_argument("--step-trace", default=None,
                    help="C3 / C4: write every timed step's host start-to-start time (us) to this JSON file")
    args = ap.parse_args()
    if args.depth is None:
        args.depth = 1 if args.config == "C1" else 2
    return args


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start N rank
    processes of this same script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment, exactly what
    torch.distributed.run would give them) and wait for them.  This process
    never touches the GPU (no torch import), so the children are fresh
    processes, not an exec of a GPU-initialised one.  Rank 0 prints the JSON
    line on the inherited stdout; the first rank that fails ends the others
    (their own PIDs) and its exit code is returned."""
    import subprocess

    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   DM_BENCH_LAUNCHER="bench.py --gpus N (self-spawned ranks)")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a failed rank: end the others (exact PIDs)
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 128 - rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args))
    if args.config not in ("C3", "C4"):
        return run_config(args)
    c4 = args.config == "C4"
    import numpy as np
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}: launch N ranks with "
                         "torch.distributed.run or let bench.py spawn them (no WORLD_SIZE)")
    if args.device_override is not None:
        local_rank = args.device_override
    torch.cuda.set_device(local_rank)
    host_cpus = pin_host_near_gpu(torch, local_rank, args.pin_host)
    if world_size > 1:
        import datetime

        # a dead peer ends the job with an error instead of a hang: the
        # process-group timeout bounds RCCL's watchdog, ShardedMapper's own
        # deadline (DM_ERR_COLLECTIVE) bounds every exchange it waits for
        pg_timeout = datetime.timedelta(seconds=args.collective_timeout)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=pg_timeout)
        else:
            dist.init_process_group(args.backend, timeout=pg_timeout)

    import dm
    from dm import synth
    from dm.sharded import ShardedMapper

    ring = int(dm.load_library().dm_max_passes_in_flight())
    if args.order == "be" and args.depth + 1 > ring:
        # 'be' starts pass k before collecting pass k-depth: depth + 1 in flight
        raise SystemExit(f"--order be --depth {args.depth} needs {args.depth + 1} readback slots; "
                         f"libdm has {ring} (DM_RB_SLOTS): use --depth {ring - 1} or more slots")

    res = 0.05
    if c4:  # BASELINE C4: one 32768² map, 32 robots anywhere in it, bands = ranks
        G = H_total = 32768
        args.robots = 32
    else:   # C3 per GPU: a 16384-row band per rank (weak scaling)
        G = args.grid
        H_total = G * world_size
    half_w = G * res / 2.0
    oy_global = -H_total * res / 2.0
    from dm.sharded import band_rows as _band_rows
    b_row0, b_rows = _band_rows(H_total, world_size, rank) if world_size > 1 else (0, H_total)
    # Scans near a band edge also reach the neighbouring band: each rank
    # integrates its own robots' scans plus the neighbours' scans whose
    # max-range disk reaches its band (host-side replication of the scan
    # stream); libdm clips every ray to the band, so each
    # cell update is counted by exactly one rank.  C4: every rank replays the
    # same 32-robot stream and keeps the scans that reach its band.
    t_gen = time.perf_counter()
    if c4:
        # one world over the whole map (every rank builds the same one)
        world = synth.make_world(args.seed * 1000, -half_w, oy_global, half_w, -oy_global)
        reach = 12.0 + 2 * res
        ylo = oy_global + b_row0 * res - reach
        yhi = oy_global + (b_row0 + b_rows) * res + reach
        st = synth.ScanStream(world, args.robots, args.beams, args.seed * 1000 + 500,
                              region=(-half_w + 1.0, oy_global + 1.0, half_w - 1.0, -oy_global - 1.0))
        pool = []
        for _ in range(args.pool):
            p_, r_ = st.next_batch()
            keep = (p_[:, 1] >= ylo) & (p_[:, 1] <= yhi)
            pool.append((p_[keep], r_[keep]))
    else:
        # rank r's robots random-walk anywhere in r's band (synth.c3_pool:
        # the same batches the GPU test of the timed configuration replays)
        world, _, pool = synth.c3_pool(args.seed, G, args.robots, args.beams, args.pool, world_size, rank, res)
    t_gen = time.perf_counter() - t_gen
    amin = float(synth.LD06_ANGLE_MIN)
    inc = float(synth.ld06_angle_increment(args.beams))
    dev = torch.device("cuda", local_rank)
    dpool = [(torch.from_numpy(synth.pose4(p)).to(dev), torch.from_numpy(np.ascontiguousarray(r)).to(dev))
             for p, r in pool]
    torch.cuda.synchronize()

    params = dm.default_params(G, H_total, resolution=res)
    params.origin_x = -half_w
    params.origin_y = oy_global
    mapper = ShardedMapper(params, rank=rank, world_size=world_size, device=local_rank,
                           group=dist.group.WORLD if world_size > 1 else None,
                           timeout=args.collective_timeout, records_comm=args.records_comm)
    band = mapper.band
    S, N = args.robots, args.beams

    def integrate(k):
        pose4, rng = dpool[k % len(dpool)]
        band.integrate_device(pose4.data_ptr(), pose4.shape[0], rng.data_ptr(), N, amin, inc)

    # per-batch U and T are properties of the batch (not of the map state):
    # measure them once, untimed
    counts, stats = [], []
    for k in range(len(dpool)):
        integrate(k)
        st = band.last_stats()
        stats.append(st)
        counts.append((st["updates"], st["touched"]))
    band.reset()

    def step(k):
        integrate(k)
        return mapper.frontiers()

    # Pipelined steps (default): step k's frontier pass is started right
    # after its integrate call and collected after step k+1's integrate call
    # was enqueued, so step k+1's ray front-end (beam prep, tile planning,
    # piece scatter: poses/ranges only) runs beside step k's frontier pass
    # (dm_set_overlap).  Every frontier pass still sees exactly the map after
    # its own batch, every batch is fully integrated: the work per step is
    # unchanged, only independent kernels overlap.
    pipelined = not args.no_overlap

    def run_steps(k0, n, integ=None, marks=None):
        """n steps from batch k0; marks (a list) receives the host clock at
        every step's start and at the end (the step cadence record)."""
        integ = integ or integrate
        if n <= 0:
            return None
        if not pipelined:
            fr = None
            for k in range(n):
                integ(k0 + k)
                fr = mapper.frontiers()
            return fr
        # up to `depth` frontier passes in flight: pass k is collected after
        # batch k + depth was enqueued, so the host never waits for the pass
        # it just started before enqueuing the next batch's front-end
        depth = max(1, min(args.depth, n))
        fr = None
        for k in range(n):
            if marks is not None:
                marks.append(time.perf_counter())
            integ(k0 + k)
            if args.order == "be":
                mapper.frontiers_begin()
                if k >= depth:
                    mapper.frontiers_end()
                continue
            if k >= depth:
                mapper.frontiers_end()
            mapper.frontiers_begin()
        for _ in range(min(depth, n)):
            fr = mapper.frontiers_end()
        if marks is not None:
            marks.append(time.perf_counter())
        # None: the pass overflowed a capacity (grown now); rerun on this map
        return fr if fr is not None else mapper.frontiers()

    if pipelined:
        mapper.set_overlap(True)

    def barrier():
        if world_size > 1:
            dist.barrier()

    # no cyclic-GC pass inside the timed steps (the setup's objects are frozen
    # first): a collection is a host stall of 0.1+ ms that the pipelined step
    # cannot hide (as timeit does; reference counting still frees everything
    # the steps create).  Done BEFORE the warm-up: a collection between the
    # warm-up and the timed steps (~65 ms with torch loaded) left the GPU idle
    # and the host's caches cold, and the first timed step took 175-200 us
    # instead of ~100 (profiles/r05_driver_cmd_*)
    import gc

    gc.collect()
    gc.freeze()
    gc.disable()
    run_steps(0, args.warmup)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    fr = run_steps(args.warmup, args.steps, marks=marks)
    band.synchronize()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    gc.unfreeze()
    if args.step_trace:
        with open(args.step_trace, "w") as f:
            json.dump({"rank": rank, "step_us": (np.diff(np.asarray(marks)) * 1e6).tolist()}, f)
    cdev = dev if args.backend == "nccl" else torch.device("cpu")
    U_rank = sum(counts[(args.warmup + k) % len(counts)][0] for k in range(args.steps))
    U_all = U_rank
    ranks_info = None
    if world_size > 1:
        # per-rank record of the timed region: [elapsed s, updates, exchange
        # fallbacks, step p50 us, step max us], summed into rank order
        cad = _cadence(marks) or {"p50": 0.0, "max": 0.0}
        t = torch.zeros((world_size, 5), dtype=torch.float64, device=cdev)
        t[rank] = torch.tensor([elapsed, float(U_rank), float(getattr(mapper, "fallbacks", 0)),
                                cad["p50"], cad["max"]], dtype=torch.float64)
        dist.all_reduce(t)
        per = t.cpu().numpy()
        elapsed = float(per[:, 0].max())
        U_all = int(round(per[:, 1].sum()))
        ranks_info = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                      "launcher": os.environ.get("DM_BENCH_LAUNCHER", "torch.distributed.run"),
                      "ms_per_step": [float(x) / args.steps * 1e3 for x in per[:, 0]],
                      "updates": [int(round(x)) for x in per[:, 1]],
                      "exchange_fallbacks": [int(x) for x in per[:, 2]],
                      "step_wall_us_p50": [float(x) for x in per[:, 3]],
                      "step_wall_us_max": [float(x) for x in per[:, 4]]}

    # integrate-only and frontier-only timings (untimed w.r.t. `value`)
    reps = max(3, min(args.steps, 20))
    ti = []
    for k in range(reps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        integrate(k)
        band.synchronize()
        ti.append(time.perf_counter() - a)
    tf = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fr = mapper.frontiers()
        tf.append(time.perf_counter() - a)
    fstats = band.last_stats()  # the last pass's visited tiles / slots / clusters
    t_int = float(np.median(ti))
    t_fr = float(np.median(tf))
    U_mean = float(np.mean([c[0] for c in counts]))
    T_mean = float(np.mean([c[1] for c in counts]))

    # live per-kernel timing with HIP events on the library's stream
    band.profile(True)
    band.profile_reset()
    if world_size > 1:
        mapper.set_timing(True)
    for k in range(args.profile_steps):
        step(k)
    kstats = band.profile_read()
    band.profile(False)
    avg = {name: tot / max(1, n) for name, (n, tot) in kstats.items()}
    if world_size > 1:
        # every rank's exchange phases per pass (ms, HIP events): halo
        # send / receive with the two neighbour bands, the band's export, the
        # records all-gather, the merge of all P records
        xt = mapper.exchange_times()
        mapper.set_timing(False)
        ph = [xt["halo_ms"], avg.get("export"), xt["records_gather_ms"], avg.get("merge")]
        t = torch.zeros((world_size, 4), dtype=torch.float64, device=cdev)
        t[rank] = torch.tensor([float("nan") if v is None else float(v) for v in ph], dtype=torch.float64)
        dist.all_reduce(t)
        per = t.cpu().numpy()
        nb = band.export_bytes(mapper.rec_cap)
        ranks_info["exchange_ms_per_pass"] = {
            "halo": [float(x) for x in per[:, 0]], "export": [float(x) for x in per[:, 1]],
            "records_gather": [float(x) for x in per[:, 2]], "merge": [float(x) for x in per[:, 3]],
            "passes_timed": int(xt["passes"]),
            "how": "HIP events: halo = map stream reaching the neighbour send / receive to its "
                   "completion; records_gather = this band's export record written to the all-gather's "
                   "completion; export / merge = libdm's kernel timers (dm_profile) of the record kernel "
                   "(k_export; the band's frontier pipeline before it is timed under its own kernels in "
                   "kernel_avg_ms) and of the merge"}
        ranks_info["exchange_bytes_per_pass"] = {
            "halo_row_bytes": G, "halo_sent_per_interior_rank": 2 * G,
            "records_gathered_per_rank": world_size * nb, "record_bytes": nb, "rec_cap": mapper.rec_cap,
            "model": "halo: W B to each neighbour band; records: P x (64 + 8 W + 32 rec_cap) B "
                     "(include/dm.h export record)"}
        ranks_info["records_comm"] = mapper.records_comm
    dominant = max(kstats, key=lambda n: kstats[n][1]) if kstats else None
    # roofline of the dominant integrate kernel, k_tile_accum: it performs
    # every update (8 B each) and applies every touched cell (25 B each),
    # heavy tiles included
    t_accum_ms = avg.get("tile_accum", float("nan"))
    bytes_accum = TILE_APPLY_BYTES_PER_UPDATE * U_mean + TILE_APPLY_BYTES_PER_TOUCHED * T_mean
    achieved = bytes_accum / (t_accum_ms * 1e-3) / 1e9 if t_accum_ms > 0 else None
    workload = "C4" if c4 else "C3"
    traffic, traffic_src = pmc_traffic("k_tile_accum", workload)
    fr_roof = None
    if world_size == 1:
        F_cells = int(fr.clusters["size"].sum()) if len(fr) else 0
        fr_roof = frontier_roofline(avg, G * H_total, F_cells, len(fr), fstats["frontier_tiles"], workload,
                                    t_fr)

    # PCIe-inclusive rate: the same pipelined steps fed from pinned host
    # buffers through dm_integrate_async (H2D of the ranges on the library's
    # front-end stream, poses read from its mapped staging ring)
    host_inputs = None
    if not args.no_host_inputs:
        pinned = [torch.from_numpy(np.ascontiguousarray(r, np.float32)).pin_memory() for _, r in pool]

        def integrate_host(k):
            poses_k = pool[k % len(pool)][0]
            band.integrate_async(poses_k, pinned[k % len(pool)].data_ptr(), poses_k.shape[0], N, amin, inc)

        band.reset()
        gc.collect()  # as for `value`: no collection inside (or right before) the timed steps
        gc.freeze()
        gc.disable()
        run_steps(0, args.warmup, integrate_host)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_steps(args.warmup, args.steps, integrate_host)
        band.synchronize()
        torch.cuda.synchronize()
        barrier()
        el_h = time.perf_counter() - t0
        gc.enable()
        gc.unfreeze()
        if world_size > 1:
            t = torch.tensor([el_h], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_h = float(t.item())
        host_inputs = {"value": U_all / el_h, "ms_per_step": el_h / args.steps * 1e3,
                       "bytes_per_step": float(np.mean([4 * r.size + 24 * p_.shape[0] for p_, r in pool])),
                       "how": "dm_integrate_async from pinned host buffers (poses as (x, y, yaw): cos/sin "
                              "on the host per call), pipelined like `value`"}

    # atomic throughput of the raycast against the device's measured peak
    # (north star): every beam-cell update is one LDS add
    atom = None
    if rank == 0:
        pk = dm.atomic_peak(local_rank)
        a_ach = U_mean / (t_accum_ms * 1e-3) if t_accum_ms > 0 else None
        atom = {"kernel": "tile_accum", "achieved": a_ach, "peak": pk["lds_add_u32_per_s"],
                "unit": "LDS atomic adds/s", "frac": a_ach / pk["lds_add_u32_per_s"] if a_ach else None,
                "global_peak": pk["global_add_u32_per_s"],
                "ops_model": "one ds_add_u32 per beam-cell update (U per launch); peak = dm_atomic_peak "
                             "(uncontended ds_add_u32, every lane its own bank, 8 workgroups/CU)"}

    # frontier worst case: one pass over a mostly explored map (every tile
    # read), N=1 only (SURVEY.md §8(d) frontier bytes 2*W*H + 16*F + 48*K)
    explored = None
    if world_size == 1 and not args.no_explored and not c4:
        explored = explored_frontier(band, mapper, synth, world, G, H_total, res, -half_w, oy_global,
                                     args.seed, reps, np)

    result = None
    if rank == 0:
        cpu = None
        if world_size == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(params, pool, amin, inc, args.cpu_seconds)
        fr_clusters = int(len(fr))
        result = {
            "metric": ("beam-cell updates/sec + frontier-extract ms (C4: 32768² shared map)" if c4
                       else "beam-cell updates/sec + frontier-extract ms on 16384² grid"),
            "value": U_all / elapsed,
            "unit": "beam-cell updates/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if c4 else "weak",
            "vs_baseline": None,
            "dtype": "int32/u32 ray math + fp32 log-odds (fp64 endpoints)",
            "data": "synthetic: seeded rectangle world, random-walk robots, LD06-format scans",
            "config": {
                "workload": ("C4: one 32768² grid @5cm shared by 32 robots (32 x 4096-beam scans "
                             "per step), row bands over the ranks, integrate + full frontier "
                             "extraction per step" if c4 else
                             "C3: 16384² grid @5cm per GPU, 64-scan x 4096-beam batch "
                             "integrate + full frontier extraction per step"),
                "grid": [G, H_total],
                "resolution_m": res,
                "scans_per_batch": S,
                "beams_per_scan": N,
                "batch_pool": len(pool),
                "parallelism": f"row-bands x{world_size}" if world_size > 1 else "single GPU",
            },
            "frontier_ms": t_fr * 1e3,
            "integrate_ms": t_int * 1e3,
            "integrate_updates_per_s": U_mean / t_int,
            "updates_per_batch": U_mean,
            "touched_cells_per_batch": T_mean,
            "clusters": fr_clusters,
            "kernel_avg_ms": avg,
            "roofline": {
                # bytes the DRAM actually moved (PMC) lead: the model's 8 B per
                # update stay in LDS, so `frac` (the contract's algorithmic
                # fraction) credits bytes that never reach HBM
                "frac_traffic": (traffic / (t_accum_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
                                 if traffic and t_accum_ms > 0 else None),
                "traffic": traffic,
                "kernel": "tile_accum",
                "dominant_kernel": dominant,
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBPS) if achieved else None,
                "traffic_source": traffic_src,
                "avg_launch_ms": t_accum_ms,
                "algorithmic_bytes_per_launch": bytes_accum,
                "bytes_model": "8*U + 25*T per call (SURVEY.md §8(d) per-unit figures)",
                **hbm_model({k: float(np.mean([st[k] for st in stats]))
                             for k in ("active_tiles", "pieces", "sparse_items")},
                            t_accum_ms, T_mean),
                "atomics": atom,
                "frontier": fr_roof,
            },
            "value_host_inputs": host_inputs["value"] if host_inputs else None,
            "host_inputs": host_inputs,
            "frontier_ms_explored": explored["frontier_ms"] if explored else None,
            "frontier_explored": explored,
            "stage_stats": {k: float(np.mean([st[k] for st in stats])) for k in stats[0]},
            "scans_per_rank_batch": float(np.mean([p.shape[0] for p, _ in pool])),
            "exchange": (f"device: halo rows sent to / received from the two neighbour bands (batched "
                         f"{'RCCL' if args.backend == 'nccl' else args.backend} send / receive), export "
                         f"records all-gathered ({args.records_comm} communicator), dm_merge_bands on "
                         f"every rank" if world_size > 1 else None),
            "exchange_fallbacks": (sum(ranks_info["exchange_fallbacks"]) if ranks_info
                                   else getattr(mapper, "fallbacks", 0)),
            # N > 1: the world size the process group reports, the launcher,
            # and every rank's own timed region (value uses the slowest)
            "ranks": ranks_info,
            "pipelined": (f"step k+1's integrate front-end overlaps step k's frontier pass "
                          f"(dm_set_overlap + dm_frontiers_begin/_end), {args.depth} passes in flight")
            if pipelined else None,
            "cpu_baseline": cpu,
            "host_cpus": host_cpus,
            "gen_seconds": t_gen,
            # host-side start-to-start time of each timed step (rank 0): a
            # host stall shows here as a long tail, kernel time in `roofline`
            "step_wall_us": _cadence(marks),
        }
        print(json.dumps(result), flush=True)
    mapper.close()
    if world_size > 1:
        dist.destroy_process_group()
    return result


def pmc_summary(workload):
    """The committed PMC summary of `workload` (tools/pmc_passes.sh +
    tools/pmc_summary.py -> profiles/pmc_latest.json, keyed by workload), only
    if it was measured on the same libdm sources; else (None, reason)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    try:
        from src_hash import src_hash
        summ = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))
    except (OSError, ValueError, ImportError):
        return None, None
    if summ.get("src_hash") != src_hash():
        return None, "profiles/pmc_latest.json is from other sources"
    w = summ.get("workloads", {}).get(workload)
    if w is None:
        return None, f"profiles/pmc_latest.json has no {workload} workload"
    return w, (f"profiles/pmc_latest.json [{workload}] (FETCH_SIZE, WRITE_SIZE KiB x per-shape factors of "
               f"profiles/fetch_calibration.json, tools/pmc_summary.py)")


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` measured on `workload`, or None."""
    w, src = pmc_summary(workload)
    if w is None:
        return None, src
    return w.get("kernels", {}).get(kernel, {}).get("traffic_bytes"), src


# the pass's kernels in stream order; frontier_big runs on its own stream
# beside frontier_tile, so the pass's device time counts the
# longer of the two
FRONTIER_KERNELS = ("frontier_bits", "frontier_tile", "frontier_big", "frontier_resolve",
                    "frontier_compact", "sort_clusters")
PMC_FRONTIER_KERNELS = ("k_frontier_bits", "k_frontier_tile", "k_frontier_tile_big",
                        "k_frontier_resolve", "k_frontier_compact", "k_rank_sort", "k_rs_count", "k_rs_scan",
                        "k_rs_place", "k_rs_rank")


def frontier_device_ms(avg):
    """Device time of a pass from per-kernel averages: the kernels in stream
    order, with frontier_tile and frontier_big (concurrent) as the longer."""
    serial = sum(avg.get(k, 0.0) for k in FRONTIER_KERNELS if k not in ("frontier_tile", "frontier_big"))
    return serial + max(avg.get("frontier_tile", 0.0), avg.get("frontier_big", 0.0))


def frontier_roofline(avg, cells, F, K, tiles_visited, workload, wall_s=None):
    """Frontier pass vs the HBM roofline, over the sum of its kernels'
    HIP-event averages (device time).  SURVEY.md §8(d) prices a pass at
    B_fr = 2*W*H (read state, write a byte mask) + 16*F (int64 label write +
    read per frontier cell) + 48*K (cluster records); the kernels read only
    the tiles holding a free cell, so `frac` is that model
    over the tiles the pass actually lists (4096 state bytes + 260 halo bytes
    + a 4096-byte mask each: `visited_bytes`) and `frac_traffic` the
    PMC-measured bytes (listed first: what the DRAM really moved).  No
    whole-map fraction: a pass reads only the listed tiles."""
    t_ms = frontier_device_ms(avg)
    # frac_traffic (PMC bytes moved) is filled in first below when measured
    out = {"frac_traffic": None, "traffic": None,
           "bound": "hbm", "bytes_model": "(4096 + 260 + 4096)*tiles_visited + 16*F + 48*K per pass "
                                          "(SURVEY.md §8(d)'s 2*W*H + 16*F + 48*K over the listed tiles)",
           "frontier_cells": F, "clusters": K, "device_ms": t_ms,
           "peak": HBM_PEAK_GBPS, "unit": "GB/s",
           "kernels_ms": {k: avg[k] for k in FRONTIER_KERNELS if k in avg}}
    if wall_s:
        out["wall_ms"] = wall_s * 1e3
    vb = (4096.0 + 260.0 + 4096.0) * (tiles_visited or 0) + 16.0 * F + 48.0 * K
    ach = vb / (t_ms * 1e-3) / 1e9 if t_ms > 0 else None
    out.update({"tiles_visited": tiles_visited, "algorithmic_bytes": vb, "achieved": ach,
                "frac": ach / HBM_PEAK_GBPS if ach else None})
    w, src = pmc_summary(workload)
    out["traffic_source"] = src
    if w is not None:
        ks = w.get("kernels", {})
        tr = [ks[k]["traffic_bytes"] for k in PMC_FRONTIER_KERNELS if "traffic_bytes" in ks.get(k, {})]
        out["traffic"] = sum(tr) if tr else None
        if out["traffic"] and t_ms > 0:
            out["frac_traffic"] = out["traffic"] / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    return out


def explored_frontier(band, mapper, synth, world, W, H, res, ox, oy, seed, reps, np):
    """frontier_ms on a mostly explored W x H map (synth.explored_state:
    free space, obstacle outlines, unknown pockets; >= 90 % of the tiles hold
    free cells, so the pass reads the whole map): median wall time of `reps`
    synchronous passes, per-kernel HIP-event times and the roofline."""
    a = time.perf_counter()
    st = synth.explored_state(world, W, H, res, ox, oy, seed=seed * 1000 + 77)
    t_gen = time.perf_counter() - a
    tiles = st.reshape(-1, 64, W // 64, 64)
    tiles_free = float((tiles == 0).any(axis=(1, 3)).mean())
    del tiles
    band.reset()
    band.set_state(st)
    del st
    mapper.set_overlap(False)
    fr = mapper.frontiers()
    tf = []
    for _ in range(reps):
        a = time.perf_counter()
        fr = mapper.frontiers()
        tf.append(time.perf_counter() - a)
    fst = band.last_stats()
    band.profile(True)
    band.profile_reset()
    for _ in range(reps):
        mapper.frontiers()
    kst = band.profile_read()
    band.profile(False)
    avg = {name: tot / max(1, n) for name, (n, tot) in kst.items()}
    F = int(fr.clusters["size"].sum()) if len(fr) else 0
    t = float(np.median(tf))
    return {"frontier_ms": t * 1e3, "grid": [W, H], "tiles_with_free_cells": tiles_free,
            "tiles_visited": fst["frontier_tiles"], "frontier_slots": fst["frontier_slots"],
            "clusters": len(fr), "frontier_cells": F, "gen_seconds": t_gen,
            "roofline": frontier_roofline(avg, W * H, F, len(fr), fst["frontier_tiles"], "C3-explored", t)}


def cpu_baseline(params, pool, amin, inc, budget_s):
    """The CPU restatement (oracle/, a port of the SPEC; single thread) on a
    bounded sample of the same workload: integrate as many pool batches as
    fit in ~budget_s into a fresh map, then one frontier extraction."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    oracle.build()
    om = oracle.OracleMap(params)
    U = 0
    t_int = 0.0
    done = 0
    for poses, ranges in pool:
        a = time.perf_counter()
        u, _ = om.integrate(poses, ranges, amin, inc)
        t_int += time.perf_counter() - a
        U += u
        done += 1
        if t_int > budget_s * 0.6:
            break
    a = time.perf_counter()
    om.frontiers(want_mask=False, want_labels=False)
    t_fr = time.perf_counter() - a
    del om
    return {
        "value": U / t_int,
        "unit": "beam-cell updates/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{done} batch(es) of {pool[0][1].shape[0]}x{pool[0][1].shape[1]} beams into a fresh "
                   f"{params.width}x{params.height} map + 1 frontier pass"),
        "frontier_ms": t_fr * 1e3,
        "cpu": _cpu_model(),
        "strong": cpu_baseline_strong(params, pool, amin, inc, budget_s),
    }


def host_threads():
    """Host cores this process may use: the CPU share the GPU box gives a
    job (OMP_NUM_THREADS is set to it there) within the affinity mask."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(env)) if env.isdigit() and int(env) > 0 else n


def cpu_baseline_strong(params, pool, amin, inc, budget_s):
    """The "strong CPU" line: the same SPEC restated with
    OpenMP on every host core this job may use (oracle/dm_oracle_mt.c, -O3;
    the build's own code, bit-identical to the 1-thread port by
    tests/test_oracle.py), on the same bounded sample."""
    import oracle

    threads = host_threads()
    om = oracle.OracleMapMT(params, threads=threads)
    om.integrate(*pool[0], amin, inc)  # warm-up (untimed): first-touch page faults of the map and counters
    U = 0
    t_int = 0.0
    done = 0
    for k in range(1, max(1, len(pool)) * 8):
        poses, ranges = pool[k % len(pool)]
        a = time.perf_counter()
        u, _ = om.integrate(poses, ranges, amin, inc)
        t_int += time.perf_counter() - a
        U += u
        done += 1
        if t_int > budget_s * 0.3:
            break
    a = time.perf_counter()
    om.frontiers(want_mask=False, want_labels=False)
    t_fr = time.perf_counter() - a
    return {"value": U / t_int, "unit": "beam-cell updates/s", "cores": om.threads, "kind": "port (OpenMP)",
            "sample": (f"{done} batch(es) after 1 untimed warm-up batch into a fresh {params.width}x"
                       f"{params.height} map + 1 frontier pass"),
            "frontier_ms": t_fr * 1e3}


def pin_host_near_gpu(torch, dev_i, mode):
    """--pin-host auto: run this process's host thread (the one that launches,
    polls and reads back) on the CPUs of the GPU's own NUMA node, from the
    GPU's PCI address in sysfs, intersected with the CPUs the process may use.
    The library's pinned host buffers (pose ring, readback) are allocated
    after this, so they land in that node's memory too.  Unpinned, a process
    on a two-socket box runs where the scheduler puts it: the GPU then reads
    the mapped buffers and the host polls across the socket link.  Returns
    what was done (for the JSON line)."""
    if mode == "off":
        return {"pinned": False, "why": "--pin-host off"}
    try:
        p = torch.cuda.get_device_properties(dev_i)
        addr = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        base = f"/sys/bus/pci/devices/{addr}"
        text = open(base + "/local_cpulist").read().strip()
        node = open(base + "/numa_node").read().strip()
        local = set()
        for part in text.split(","):
            lo, _, hi = part.partition("-")
            local.update(range(int(lo), int(hi or lo) + 1))
        cpus = local & os.sched_getaffinity(0)
        if not cpus:
            return {"pinned": False, "why": f"no allowed CPU on the GPU's node {node}"}
        os.sched_setaffinity(0, cpus)
        return {"pinned": True, "gpu_pci": addr, "numa_node": int(node), "cpus": len(cpus)}
    except (OSError, ValueError, AttributeError) as e:
        return {"pinned": False, "why": f"{type(e).__name__}: {e}"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


# ---------------------------------------------------------------------------
# Secondary BASELINE configs (single GPU, not the bench line): C2 replay and
# the C5 beam-density sweep.  Same step definition as C3 (integrate + full
# frontier extraction, pipelined), same roofline bookkeeping.
# ---------------------------------------------------------------------------

def _cadence(marks):
    """p50 / p90 / max of the gaps between consecutive host clock marks (us)."""
    import numpy as np

    if len(marks) < 2:
        return None
    d = np.diff(np.asarray(marks)) * 1e6
    return {"p50": float(np.percentile(d, 50)), "p90": float(np.percentile(d, 90)),
            "max": float(d.max()), "n": int(d.size)}


HBM_MODEL_NOTE = ("bytes k_tile_accum moves from HBM by the design: 10 B per cell of every dense item's "
                  "64x64 tile (L and state read and written, whole tiles at line granularity) + 16 B per "
                  "packed piece read; sparse items (<= 15 pieces, C5's sparse scans) load and store only "
                  "their touched 4-cell groups, at most 40 B per touched cell, which frac_hbm_touched "
                  "(10 B per touched cell + pieces) bounds from below. The hit / miss counts (the 8*U of "
                  "`frac`) stay in LDS and are in neither, so frac (the SURVEY.md §8(d) model) reads ~2x "
                  "(C3) to ~3x+ (C5-4096) above the bytes moved; frac_traffic (PMC) is the measured figure. "
                  "When more than half the active tiles are sparse items (C5 12-768 beams) their scattered "
                  "4-cell groups move whole lines that neither model counts, and frac_hbm_model is null")


def hbm_model(stats_mean, t_ms, T_mean=None):
    """frac_hbm_model: the design's own HBM bytes per
    k_tile_accum launch (HBM_MODEL_NOTE) over its launch time, beside `frac`
    (SURVEY.md §8(d)'s 8 U + 25 T, which counts LDS-resident counter bytes)."""
    act, pieces = stats_mean.get("active_tiles"), stats_mean.get("pieces")
    if not act or not t_ms or t_ms <= 0:
        return {"frac_hbm_model": None, "hbm_model_bytes_per_launch": None, "frac_hbm_touched": None,
                "hbm_model": HBM_MODEL_NOTE}
    sparse = stats_mean.get("sparse_items") or 0.0
    dense = act - sparse  # a tile is one dense or one sparse item
    b = 10.0 * 4096.0 * dense + 16.0 * pieces
    bt = 10.0 * T_mean + 16.0 * pieces if T_mean else None
    rate = lambda x: x / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS  # noqa: E731
    # a call whose tiles are mostly sparse items moves line-granular bytes of
    # scattered 4-cell groups that neither model counts: no model fraction
    applies = sparse <= 0.5 * act
    return {"frac_hbm_model": rate(b) if applies else None, "hbm_model_bytes_per_launch": b if applies else None,
            "frac_hbm_touched": rate(bt) if bt else None, "hbm_model_applies": applies,
            "hbm_model": HBM_MODEL_NOTE}


def _profiled_roofline(band, run, U_mean, T_mean, stats_mean=None):
    """Per-kernel average launch time (HIP events on the library's stream)
    over `run()`, and the k_tile_accum roofline (SURVEY.md §8(d) bytes)."""
    band.profile(True)
    band.profile_reset()
    run()
    kstats = band.profile_read()
    band.profile(False)
    avg = {name: tot / max(1, n) for name, (n, tot) in kstats.items()}
    t_ms = avg.get("tile_accum", float("nan"))
    bytes_accum = TILE_APPLY_BYTES_PER_UPDATE * U_mean + TILE_APPLY_BYTES_PER_TOUCHED * T_mean
    achieved = bytes_accum / (t_ms * 1e-3) / 1e9 if t_ms > 0 else None
    return avg, {
        "kernel": "tile_accum", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
        "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBPS) if achieved else None,
        "traffic": None, "avg_launch_ms": t_ms, "algorithmic_bytes_per_launch": bytes_accum,
        "bytes_model": "8*U + 25*T per call (SURVEY.md §8(d) per-unit figures)",
        **hbm_model(stats_mean or {}, t_ms, T_mean),
    }


def _pipelined(mapper, integrate, ks, depth=2):
    """integrate(k) + frontier pass per k, as the C3 bench's run_steps: up to
    `depth` passes in flight, pass k collected after batch k + depth was
    enqueued (depth 1: after batch k + 1), then the passes still in flight.
    Returns the last pass's frontiers."""
    ks = list(ks)
    if not ks:
        return None
    depth = max(1, min(depth, len(ks)))
    fr = None
    for i, k in enumerate(ks):
        integrate(k)
        if i >= depth:
            mapper.frontiers_end()
        mapper.frontiers_begin()
    for _ in range(depth):
        fr = mapper.frontiers_end()
    # None: the pass overflowed a capacity (grown now); rerun on this map
    return fr if fr is not None else mapper.frontiers()


def run_config(args):
    import numpy as np
    import torch

    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        raise SystemExit(f"--config {args.config} is a single-GPU measurement")
    dev_i = args.device_override or 0
    torch.cuda.set_device(dev_i)
    host_cpus = pin_host_near_gpu(torch, dev_i, args.pin_host)
    dev = torch.device("cuda", dev_i)
    import dm
    from dm import synth

    world, W, H, res, ox, oy = synth.config_world(args.config, args.seed)
    params = dm.default_params(W, H, resolution=res)
    params.origin_x, params.origin_y = ox, oy
    amin = float(synth.LD06_ANGLE_MIN)
    base = {
        "metric": f"beam-cell updates/sec + frontier-extract ms ({args.config})",
        "unit": "beam-cell updates/s", "n_gpus": 1, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32/u32 ray math + fp32 log-odds (fp64 endpoints)",
        "data": "synthetic: seeded rectangle world, random-walk robots, LD06-format scans",
    }
    mapper = dm.OccupancyMapper(params, device=dev_i)
    mapper.set_overlap(not args.no_overlap)  # PMC passes: --no-overlap (one dispatch at a time)
    try:
        if args.config in ("C1", "C2"):
            out = _run_replay(args, np, torch, synth, mapper, params, amin, dev)
        else:
            out = _run_c5(args, np, torch, synth, mapper, params, amin, dev, world)
    finally:
        mapper.close()
    out = {**base, **out, "host_cpus": host_cpus}
    print(json.dumps(out), flush=True)
    return out


def _run_replay(args, np, torch, synth, m, params, amin, dev):
    """C1 (400²) / C2 (4096²) @5 cm, one robot, N=360, scan-by-scan replay
    (S=1): every scan is integrated and followed by a full frontier
    extraction.  CPU baseline: C1 the NumPy restatement (the reference's
    Python idiom, BASELINE config C1), C2 the C restatement."""
    cfg = args.config
    N = 360
    n = args.scans if args.scans is not None else (1000 if cfg == "C1" else 10000)
    inc = float(synth.ld06_angle_increment(N))
    world, G = synth.config_world(cfg, args.seed)[:2]
    stream = synth.ScanStream(world, 1, N, args.seed * 1000 + 2)
    t_gen = time.perf_counter()
    batches = [stream.next_batch() for _ in range(n)]
    t_gen = time.perf_counter() - t_gen
    poses = np.concatenate([b[0] for b in batches])
    ranges = np.ascontiguousarray(np.concatenate([b[1] for b in batches]), np.float32)
    d_pose = torch.from_numpy(synth.pose4(poses)).to(dev)
    d_rng = torch.from_numpy(ranges).to(dev)
    torch.cuda.synchronize()
    p0, r0 = d_pose.data_ptr(), d_rng.data_ptr()

    def integrate(k):
        m.integrate_device(p0 + 32 * k, 1, r0 + 4 * N * k, N, amin, inc)

    # per-scan U / T (properties of the scan, not of the map), untimed
    U = T = 0
    for k in range(n):
        integrate(k)
        st = m.last_stats()
        U += st["updates"]
        T += st["touched"]
    m.reset()
    _pipelined(m, integrate, range(min(args.warmup * 20, n)), args.depth)
    m.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fr = _pipelined(m, integrate, range(n), args.depth)
    m.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    reps = min(200, n)
    ti, tf = [], []
    for k in range(reps):
        a = time.perf_counter()
        integrate(k)
        m.synchronize()
        ti.append(time.perf_counter() - a)
    for _ in range(reps):
        a = time.perf_counter()
        m.frontiers()
        tf.append(time.perf_counter() - a)
    avg, roof = _profiled_roofline(m, lambda: [(integrate(k), m.frontiers()) for k in range(reps)],
                                   U / n, T / n)
    cpu = None
    if args.cpu_seconds > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        if cfg == "C1":
            import np_oracle

            L = np.zeros((params.height, params.width), np.float32)
            st = np.full((params.height, params.width), -1, np.int8)
            integ = lambda k: np_oracle.integrate(params, L, st, poses[k:k + 1], ranges[k:k + 1],  # noqa: E731
                                                  amin, inc)[0]
            front = lambda: np_oracle.frontiers(params, st)  # noqa: E731
            impl = "NumPy restatement (oracle/np_oracle.py)"
        else:
            import oracle

            oracle.build()
            om = oracle.OracleMap(params)
            integ = lambda k: om.integrate(poses[k:k + 1], ranges[k:k + 1], amin, inc)[0]  # noqa: E731
            front = lambda: om.frontiers(want_mask=False, want_labels=False)  # noqa: E731
            impl = "C restatement (oracle/dm_oracle.c)"
        u_c, t_i, t_f, done = 0, 0.0, [], 0
        for k in range(n):
            a = time.perf_counter()
            u_c += integ(k)
            t_i += time.perf_counter() - a
            a = time.perf_counter()
            front()
            t_f.append(time.perf_counter() - a)
            done += 1
            if t_i + sum(t_f) > args.cpu_seconds:
                break
        cpu = {"value": u_c / t_i, "unit": "beam-cell updates/s", "cores": 1, "kind": "port",
               "sample": f"first {done} scans of the replay, integrate + frontier pass per scan, {impl}",
               "scans_per_s": done / (t_i + sum(t_f)), "frontier_ms": float(np.median(t_f)) * 1e3,
               "cpu": _cpu_model()}
    return {
        "value": U / elapsed, "steps": n, "warmup": min(args.warmup * 20, n),
        "ms_per_step": elapsed / n * 1e3, "scans_per_s": n / elapsed,
        "config": {"workload": f"{cfg}: {G}² grid @5cm, single robot, {n}-scan replay x {N} beams, "
                               "integrate + full frontier extraction per scan (S=1)",
                   "grid": [G, G], "resolution_m": 0.05, "scans_per_batch": 1,
                   "beams_per_scan": N, "parallelism": "single GPU"},
        "updates_total": U, "touched_total": T,
        "integrate_ms": float(np.median(ti)) * 1e3, "frontier_ms": float(np.median(tf)) * 1e3,
        "clusters": len(fr) if fr is not None else None, "kernel_avg_ms": avg, "roofline": roof,
        "pipelined": f"scan k+1's integrate front-end overlaps scan k's frontier pass, {args.depth} passes in flight",
        "cpu_baseline": cpu, "gen_seconds": t_gen,
    }


def _run_c5(args, np, torch, synth, m, params, amin, dev, world):
    """C5: 65536² @1 cm (12 m = 1200 cells), 64 robots, beam-density sweep:
    for each N, K pipelined steps of integrate(64 x N) + frontier pass on a
    fresh map."""
    S = args.robots
    sweep = [int(x) for x in args.sweep.split(",") if x]
    rows, cpu = [], None
    for N in sweep:
        inc = float(synth.ld06_angle_increment(N))
        stream = synth.ScanStream(world, S, N, args.seed * 1000 + 7 + N)
        pool = [stream.next_batch() for _ in range(max(2, min(args.pool, 4)))]
        dpool = [(torch.from_numpy(synth.pose4(p)).to(dev),
                  torch.from_numpy(np.ascontiguousarray(r, np.float32)).to(dev)) for p, r in pool]
        torch.cuda.synchronize()

        def integrate(k):
            pp, rr = dpool[k % len(dpool)]
            m.integrate_device(pp.data_ptr(), pp.shape[0], rr.data_ptr(), N, amin, inc)

        stats = []
        for k in range(len(dpool)):
            integrate(k)
            stats.append(m.last_stats())
        m.reset()
        _pipelined(m, integrate, range(args.warmup), args.depth)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fr = _pipelined(m, integrate, range(args.warmup, args.warmup + args.steps), args.depth)
        m.synchronize()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        U = sum(stats[k % len(stats)]["updates"] for k in range(args.warmup, args.warmup + args.steps))
        ti, tf = [], []
        for k in range(max(3, min(args.steps, 10))):
            a = time.perf_counter()
            integrate(k)
            m.synchronize()
            ti.append(time.perf_counter() - a)
            a = time.perf_counter()
            m.frontiers()
            tf.append(time.perf_counter() - a)
        fst = m.last_stats()  # the last pass's listed tiles, tile-local components, clusters
        mean = lambda key: float(np.mean([st[key] for st in stats]))  # noqa: E731
        avg, roof = _profiled_roofline(m, lambda: [(integrate(k), m.frontiers()) for k in range(5)],
                                       mean("updates"), mean("touched"),
                                       {k: mean(k) for k in ("active_tiles", "pieces", "sparse_items")})
        # PMC traffic of this sweep point (tools/pmc_passes.sh over
        # `bench.py --config C5 --sweep N`, workload "C5-N"), when measured
        # on these sources
        wl = f"C5-{N}"
        traffic, tsrc = pmc_traffic("k_tile_accum", wl)
        roof["traffic"], roof["traffic_source"] = traffic, tsrc
        if traffic and roof["avg_launch_ms"] > 0:
            roof["frac_traffic"] = traffic / (roof["avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS
        F_cells = int(fr.clusters["size"].sum()) if fr is not None and len(fr) else 0
        roof["frontier"] = frontier_roofline(avg, 65536 * 65536, F_cells, len(fr) if fr is not None else 0,
                                             fst["frontier_tiles"], wl, float(np.median(tf)))
        rows.append({"beams_per_scan": N, "value": U / elapsed,
                     "ms_per_step": elapsed / args.steps * 1e3,
                     "integrate_ms": float(np.median(ti)) * 1e3,
                     "frontier_ms": float(np.median(tf)) * 1e3,
                     "integrate_updates_per_s": mean("updates") / float(np.median(ti)),
                     "updates_per_batch": mean("updates"), "touched_cells_per_batch": mean("touched"),
                     "clusters": len(fr) if fr is not None else None,
                     "stage_stats": {k: mean(k) for k in ("pieces", "active_tiles", "work_items", "heavy_tiles",
                                                          "sparse_items")},
                     "frontier_tiles": fst["frontier_tiles"], "frontier_slots": fst["frontier_slots"],
                     "kernel_avg_ms": avg, "roofline": roof})
        if N == sweep[-1] and args.cpu_seconds > 0:
            # CPU restatement, integrate only: its frontier pass over 2^32
            # cells needs 64 GiB of int64 work arrays
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle

            oracle.build()
            om = oracle.OracleMap(params)
            u_c, t_c, done = 0, 0.0, 0
            for p_, r_ in pool:
                a = time.perf_counter()
                u_c += om.integrate(p_, r_, amin, inc)[0]
                t_c += time.perf_counter() - a
                done += 1
                if t_c > args.cpu_seconds:
                    break
            del om
            cpu = {"value": u_c / t_c, "unit": "beam-cell updates/s", "cores": 1, "kind": "port",
                   "sample": f"{done} batch(es) of {S}x{N} beams into a fresh 65536² map "
                             "(integrate only)", "cpu": _cpu_model()}
        m.reset()
        del dpool
    head = rows[-1]
    return {
        "value": head["value"], "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "config": {"workload": f"C5: 65536² grid @1cm, {S}-scan batches, beam-density sweep "
                               f"{sweep}; integrate + full frontier extraction per step "
                               "(value = last sweep point)",
                   "grid": [65536, 65536], "resolution_m": 0.01, "scans_per_batch": S,
                   "beams_per_scan": sweep, "parallelism": "single GPU"},
        "frontier_ms": head["frontier_ms"], "roofline": head["roofline"], "sweep": rows,
        "pipelined": f"step k+1's integrate front-end overlaps step k's frontier pass, {args.depth} passes in flight",
        "cpu_baseline": cpu,
    }


if __name__ == "__main__":
    main()
