"""Row-band sharding of one map over the GPUs of a node.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" for CPU tests).  Rank r owns rows [row0_r, row0_r + rows_r) of
the global map, rows_r a multiple of 64 except for the last band.

* Integration is embarrassingly parallel: every rank integrates the scans
  whose max-range disk reaches its band; libdm clips rays to the band, so
  cell writes are disjoint and the union of the bands equals a 1-GPU map
  bit for bit (tests/test_sharded.py).
* Frontier extraction has the only real exchange steps.  On GPUs they are
  device-resident (one host synchronisation per call, as on one GPU): each
  band's first / last rows go to its two neighbours only, received straight
  into their halos (one batched RCCL send / receive; 2 W bytes each way,
  exchange_neighbour_rows), every band
  writes an export record (include/dm.h: its edge components as indices into
  its sorted cluster list, and the clusters), the records are all-gathered
  with RCCL and every rank merges them with libdm's merge kernels
  (dm_merge_bands, csrc/dm_merge.hip).  The host path below is the
  restatement the CPU tests run (and the fallback when a band's record
  overflows its capacity):
  1. halo rows: each band's first/last state rows are sent to the
     neighbouring bands (W bytes per edge) and installed as their halos, so
     the 8-neighbour frontier test sees across band edges;
  2. label merge: each band's first/last-row labels (band-local min-index
     labels, int64) are all-gathered; every rank forms the cross-edge
     equivalence pairs (8-connectivity: x-1, x, x+1) and resolves them with
     the same connected-components pass, so the global label = min over the
     component, identical to the 1-GPU result;
  3. cluster all-gather: per-band (label, size, sum_x, sum_y) records are
     all-gathered (counts first, then padded records), merged by final
     label with exact int64 sums, filtered by min_frontier_size and sorted.
All messages are KB-MB: latency-bound on xGMI, no ring all-reduce needed.

Failure handling (the reference's analogue is the bounded
connect thread, pi/src/thymio_project/thymio_project/main.py:138-148): every
collective is issued with ``async_op=True`` and waited for at most
``timeout`` seconds; on the device path the host polls an event recorded
after the collectives instead of blocking in the merge's synchronisation.
A peer that died, raised or stalled therefore surfaces on every other rank
as ``DmError(DM_ERR_COLLECTIVE)`` within the timeout, never as a hang; the
error is sticky (the communicator may hold a half-finished collective), so
every later call on that mapper raises it again.
"""
from __future__ import annotations

import collections
import time
from datetime import timedelta

import numpy as np

from ._ffi import CLUSTER_DTYPE, DM_ERR_COLLECTIVE, DM_TILE, DmError, DmParams, load_library
from .grid import Frontiers, OccupancyMapper


def band_rows(height: int, world_size: int, rank: int):
    """(row0, rows) of rank's band: equal multiples of 64, last band ragged."""
    tiles = -(-height // DM_TILE)
    per = -(-tiles // world_size) * DM_TILE
    row0 = min(rank * per, height)
    rows = max(0, min(per, height - row0))
    return row0, rows


def group_ranks(dist, group=None) -> list[int]:
    """Global ranks of `group` (None: the default group) in group-rank order:
    the member list a second communicator over the same processes needs."""
    if group is None or group is dist.group.WORLD:
        return list(range(dist.get_world_size()))
    return [int(r) for r in dist.get_process_group_ranks(group)]


def exchange_neighbour_rows(dist, group, peers, rank: int, world_size: int, first, last, before, after):
    """Post the band-edge exchange with the two neighbour bands only (SURVEY.md
    §8(e)): `first` (this band's first row) goes to rank - 1 and `last` to
    rank + 1; `before` receives rank - 1's last row and `after` rank + 1's
    first row (None at the map's top / bottom band).  `peers`: the group's
    global ranks.  Returns the works to wait for (one batched RCCL launch, or
    gloo's per-op requests)."""
    ops = []
    if rank > 0:
        ops.append(dist.P2POp(dist.isend, first, peers[rank - 1], group))
        ops.append(dist.P2POp(dist.irecv, before, peers[rank - 1], group))
    if rank + 1 < world_size:
        ops.append(dist.P2POp(dist.isend, last, peers[rank + 1], group))
        ops.append(dist.P2POp(dist.irecv, after, peers[rank + 1], group))
    return dist.batch_isend_irecv(ops) if ops else []


def band_params(params: DmParams, world_size: int, rank: int) -> DmParams:
    bp = DmParams.from_buffer_copy(params)
    row0, rows = band_rows(int(params.height), world_size, rank)
    if rows <= 0:
        raise ValueError(f"rank {rank}: no rows left for this band (height {params.height}, "
                         f"{world_size} ranks)")
    bp.band_row0 = row0
    bp.band_rows = rows
    bp.min_frontier_size = 1  # the size filter applies to merged, global clusters
    return bp


def resolve_labels(records: list[np.ndarray], edges: list[tuple[np.ndarray, np.ndarray]]):
    """Union band-local labels across band edges.

    records[r]: int64 [K_r, 4] (label, size, sum_x, sum_y) of band r
    edges[r]:   (first_row_labels, last_row_labels) int64 [W] of band r
    Returns (allrec [K,4], uniq labels (sorted), comp id per uniq label,
    final label per comp id = min label of the component)."""
    recs = [np.asarray(r, np.int64).reshape(-1, 4) for r in records]
    allrec = np.concatenate(recs, 0) if recs else np.zeros((0, 4), np.int64)
    uniq = np.unique(allrec[:, 0])
    comp = np.arange(uniq.shape[0])
    pa, pb = [], []
    for b in range(len(edges) - 1):  # band b's last row vs band b+1's first row
        last = np.asarray(edges[b][1], np.int64)
        first = np.asarray(edges[b + 1][0], np.int64)
        W = last.shape[0]
        for d in (-1, 0, 1):
            lo, hi = max(0, -d), min(W, W - d)
            a = last[lo:hi]
            c = first[lo + d:hi + d]
            ok = (a >= 0) & (c >= 0)
            pa.append(a[ok])
            pb.append(c[ok])
    A = np.concatenate(pa) if pa else np.zeros(0, np.int64)
    B = np.concatenate(pb) if pb else np.zeros(0, np.int64)
    if A.size and uniq.size:
        from scipy.sparse import coo_matrix
        from scipy.sparse.csgraph import connected_components

        ia = np.searchsorted(uniq, A)
        ib = np.searchsorted(uniq, B)
        n = uniq.shape[0]
        g = coo_matrix((np.ones(ia.size, np.int8), (ia, ib)), shape=(n, n))
        _, comp = connected_components(g, directed=False)
    ncomp = int(comp.max()) + 1 if comp.size else 0
    final = np.full(ncomp, np.iinfo(np.int64).max, np.int64)
    if ncomp:
        np.minimum.at(final, comp, uniq)
    return allrec, uniq, comp, final


def merge_clusters(records: list[np.ndarray], edges: list[tuple[np.ndarray, np.ndarray]],
                   params: DmParams, min_size: int) -> np.ndarray:
    """Merge per-band cluster records into global clusters: a CLUSTER_DTYPE
    array sorted by label, exact int64 sums."""
    allrec, uniq, comp, final = resolve_labels(records, edges)
    if allrec.shape[0] == 0:
        return np.zeros(0, dtype=np.dtype(CLUSTER_DTYPE))
    ncomp = final.shape[0]
    rec_comp = comp[np.searchsorted(uniq, allrec[:, 0])]
    size = np.zeros(ncomp, np.int64)
    sx = np.zeros(ncomp, np.int64)
    sy = np.zeros(ncomp, np.int64)
    np.add.at(size, rec_comp, allrec[:, 1])
    np.add.at(sx, rec_comp, allrec[:, 2])
    np.add.at(sy, rec_comp, allrec[:, 3])
    keep = size >= max(1, int(min_size))
    order = np.argsort(final[keep], kind="stable")
    out = np.zeros(int(keep.sum()), dtype=np.dtype(CLUSTER_DTYPE))
    out["label"] = final[keep][order]
    out["size"] = size[keep][order]
    out["sum_x"] = sx[keep][order]
    out["sum_y"] = sy[keep][order]
    # same double formula as libdm / the SPEC: one division, then + 0.5, * res
    mx = out["sum_x"].astype(np.float64) / out["size"].astype(np.float64)
    my = out["sum_y"].astype(np.float64) / out["size"].astype(np.float64)
    out["cx_m"] = params.origin_x + (mx + 0.5) * params.resolution
    out["cy_m"] = params.origin_y + (my + 0.5) * params.resolution
    return out


def relabel(band_labels: np.ndarray, records, edges) -> np.ndarray:
    """Band-local label image -> global labels (parity / debug output)."""
    _, uniq, comp, final = resolve_labels(records, edges)
    out = band_labels.copy()
    m = out >= 0
    if m.any():
        out[m] = final[comp[np.searchsorted(uniq, out[m])]]
    return out


class ShardedMapper:
    """A map split in row bands over `world_size` ranks; this object is
    rank `rank`'s part.  With world_size == 1 it is a plain OccupancyMapper."""

    def __init__(self, params: DmParams, rank: int = 0, world_size: int = 1, device: int = 0,
                 group=None, band=None, timeout: float = 300.0, force_exchange: bool = False,
                 records_comm: str = "shared"):
        """`timeout`: seconds any collective (or the device work queued behind
        one) may take before this rank gives up with DM_ERR_COLLECTIVE.
        `force_exchange`: with world_size 1, run the multi-rank exchange
        anyway (halo exchange, export record, records gather, device merge)
        over `group` (a 1-rank process group): the RCCL path on one GPU.
        `records_comm`: "shared" (default) all-gathers the export records over
        `group`, the halo exchange's own communicator, so every collective of
        the mapper runs in one issue order on one communicator; "separate"
        builds a second communicator for them (dist.new_group over the same
        ranks), so a records gather waiting for a pass's labelling does not
        hold up the next pass's halo exchange.  Two communicators driven from
        two streams at once have run on one GPU only (tests/test_gpu_nccl.py),
        never across devices, hence the default."""
        self.params = DmParams.from_buffer_copy(params)
        self.rank, self.world_size, self.group = rank, world_size, group
        self._exchange = world_size > 1 or bool(force_exchange)
        self.timeout = float(timeout)
        self.failed = None  # sticky DM_ERR_COLLECTIVE message
        self.min_size = int(params.min_frontier_size)
        if not self._exchange:
            bp = DmParams.from_buffer_copy(params)
        else:
            bp = band_params(params, world_size, rank)
        self.band = band if band is not None else OccupancyMapper(bp, device)
        self.row0, self.rows = int(bp.band_row0), int(bp.band_rows or params.height)
        self.W = int(params.width)
        self._device = None
        self._dev_path = False
        if records_comm not in ("shared", "separate"):
            raise ValueError(f"records_comm must be 'shared' or 'separate', not {records_comm!r}")
        self.records_comm = records_comm
        self.timing = False  # set_timing(): HIP-event times of the exchange phases
        # (halo start, halo end, gather start, gather end) per timed pass; the
        # most recent 4096 are kept (a mapper left timing does not grow)
        self._tev = collections.deque(maxlen=4096)
        self._pending = collections.deque()  # frontiers_begin() passes in flight, oldest first
        try:
            self.max_in_flight = int(load_library().dm_max_passes_in_flight())
        except Exception:  # a non-libdm band (CPU tests): libdm's default ring
            self.max_in_flight = 2
        if self._exchange:
            import torch.distributed as dist

            self._dist = dist
            self._nccl = dist.get_backend(group) == "nccl"
            self._group_ranks = group_ranks(dist, group)
            if self._nccl:
                import torch

                self._device = torch.device("cuda", device)
            # device-resident exchange when the band is a libdm handle
            self._dev_path = hasattr(self.band, "frontiers_export_device")
            if self._dev_path:
                import torch

                self._torch = torch
                self._tdev = torch.device("cuda", device)
                # the band's map stream: its map kernels and the halo-row
                # exchange between them (RCCL orders itself against it)
                # (high priority, as libdm's own map stream: the front-end
                # stream fills what the map chain leaves idle)
                self.stream = torch.cuda.Stream(device=self._tdev, priority=-1)
                self.band.set_stream(self.stream.cuda_stream)
                # the export records are all-gathered on the band's exchange
                # stream (its pass stream with overlap on).  "shared": over
                # the mapper's group, the halo's communicator (one issue
                # order for every collective; a gather waiting for pass k's
                # labelling delays pass k+1's halo exchange behind it).
                # "separate": over a second communicator, so that gather
                # never holds up the next halo exchange on the map stream.
                # Built over the mapper's own group's ranks (a subgroup's
                # ranks are not 0..P-1 globally); new_group is collective
                # over the default group, so every process of it constructs
                # its mappers in the same order.
                self.rec_group = (dist.new_group(self._group_ranks) if records_comm == "separate"
                                  else group)
                self._xstreams = {}
                # records per band export: sized for the band up front (a
                # cluster per tile: C5's 4096-beam fans reach 0.81), then to
                # twice the largest band K seen (_size_rec_cap; grown on an
                # incomplete record)
                tiles = -(-self.W // DM_TILE) * -(-self.rows // DM_TILE)
                self.rec_cap = 16384
                while self.rec_cap < tiles:
                    self.rec_cap *= 2
                self._bufs = {}
                self.fallbacks = 0

    # -- collective failure handling ----------------------------------------
    def _check(self):
        if self.failed is not None:
            raise DmError(DM_ERR_COLLECTIVE, self.failed)

    def _fail(self, what: str):
        self.failed = f"rank {self.rank}/{self.world_size}: {what} (sharded map unusable; recreate it)"
        raise DmError(DM_ERR_COLLECTIVE, self.failed)

    def _wait(self, work, what: str):
        """Wait for one async collective at most self.timeout seconds (gloo:
        host-side; RCCL: orders the current stream only — the host deadline is
        enforced by _poll / _drain on an event recorded after it.  An RCCL
        work's wait(timeout) would block the host until the collective and
        every kernel queued before it had finished, which serialises the
        pipelined passes)."""
        try:
            if self._nccl:
                work.wait()
                return
            ok = work.wait(timeout=timedelta(seconds=self.timeout))
        except Exception as e:  # gloo: a timed-out or aborted peer raises here
            self._fail(f"{what} failed: {e}")
        if ok is False:
            self._fail(f"{what} did not complete within {self.timeout:g} s")

    def _all_gather(self, out, t, what: str, group=None):
        self._check()
        try:
            work = self._dist.all_gather_into_tensor(out, t, group=group if group is not None else self.group,
                                                     async_op=True)
        except Exception as e:
            self._fail(f"{what} failed: {e}")
        self._wait(work, what)

    def _poll(self, ev, what: str):
        """Wait (host side, at most self.timeout) for a CUDA/HIP event recorded
        after collectives, so no later blocking synchronisation can wait on a
        collective a dead peer never joins."""
        t0 = time.monotonic()
        deadline = t0 + self.timeout
        while not ev.query():
            now = time.monotonic()
            if now > deadline:
                self._fail(f"{what}: device exchange did not complete within {self.timeout:g} s")
            # poll without sleeping for the first 2 ms: a pipelined pass ends
            # tens of microseconds after the host starts waiting, and a sleep
            # of 20 us oversleeps by ~50 us (the kernel's timer slack)
            if now - t0 > 2e-3:
                time.sleep(2e-5)

    def _drain(self, what: str, stream=None):
        import torch

        ev = torch.cuda.Event()
        ev.record(stream if stream is not None else self.stream)
        self._poll(ev, what)

    # -- integration ------------------------------------------------------
    def scan_mask(self, poses) -> np.ndarray:
        """Scans whose max-range disk reaches this band's rows."""
        poses = np.asarray(poses, np.float64).reshape(-1, 3)
        p = self.params
        reach = float(p.range_max) + 2 * p.resolution
        y = poses[:, 1]
        ylo = p.origin_y + self.row0 * p.resolution - reach
        yhi = p.origin_y + (self.row0 + self.rows) * p.resolution + reach
        return ~((y < ylo) | (y > yhi))  # NaN poses are kept (libdm skips them)

    def integrate(self, poses, ranges, angle_min, angle_increment):
        self._check()
        poses = np.asarray(poses, np.float64).reshape(-1, 3)
        ranges = np.asarray(ranges, np.float32)
        if ranges.ndim != 2:
            ranges = ranges.reshape(poses.shape[0], -1)
        if self._exchange:
            keep = self.scan_mask(poses)
            poses, ranges = poses[keep], ranges[keep]
        return self.band.integrate(poses, ranges, angle_min, angle_increment)

    # -- frontiers --------------------------------------------------------
    def _allgather(self, arr: np.ndarray) -> np.ndarray:
        """all-gather a same-shape array from every rank -> [P, ...]."""
        import torch

        t = torch.from_numpy(np.ascontiguousarray(arr))
        if self._nccl:
            t = t.to(self._device)
        t = t.reshape(1, -1)
        out = torch.empty((self.world_size, t.shape[1]), dtype=t.dtype, device=t.device)
        self._all_gather(out, t, "all-gather")
        if self._nccl:
            self._drain("all-gather", torch.cuda.current_stream(self._device))
        return out.cpu().numpy().reshape((self.world_size,) + arr.shape)

    def exchange_halos(self):
        """Host path: the halo rows from the two neighbour bands
        (exchange_neighbour_rows), set on the band."""
        import torch

        first, last = (torch.from_numpy(np.ascontiguousarray(a, np.int8)) for a in self.band.edge_rows())
        dev = self._device if self._nccl else None
        if dev is not None:
            first, last = first.to(dev), last.to(dev)
        W, r, P = first.numel(), self.rank, self.world_size
        before = torch.empty(W, dtype=torch.int8, device=dev) if r > 0 else None
        after = torch.empty(W, dtype=torch.int8, device=dev) if r + 1 < P else None
        self._exchange_rows(first, last, before, after)
        if dev is not None:
            self._drain("halo exchange", torch.cuda.current_stream(dev))
        self.band.set_halo(None if before is None else before.cpu().numpy(),
                           None if after is None else after.cpu().numpy())

    # -- device-resident exchange (RCCL + dm_merge_bands) -------------------
    def _buf(self, name, n, dtype):
        t = self._bufs.get(name)
        if t is None or t.numel() != n:
            if t is not None:
                # a pass in flight may still read the old buffer on another
                # stream (capacities only change after an incomplete pass)
                self._torch.cuda.synchronize(self._tdev)
            t = self._torch.empty(n, dtype=dtype, device=self._tdev)
            self._bufs[name] = t
        return t

    def _gather_dev(self, t, out, group=None):
        """all-gather a device tensor into out ([P * n], rank order), ordered
        on the current stream."""
        if self._nccl:
            self._all_gather(out, t, "device all-gather", group)
        else:  # gloo rehearsal on GPUs: host-staged
            o = self._torch.empty(out.numel(), dtype=t.dtype)
            self._all_gather(o, t.cpu(), "all-gather", group)
            out.copy_(o)

    def _halo_dev(self, rows):
        """The band's halo rows from its two neighbours only, ordered on the
        current stream (exchange_neighbour_rows: 2 W bytes each way instead of
        an all-gather of every band's 2 W).  Returns the (before, after)
        device rows, None at the map's top / bottom band."""
        torch = self._torch
        W, P, r = self.W, self.world_size, self.rank
        before = self._buf("halo_before", W, torch.int8) if r > 0 else None
        after = self._buf("halo_after", W, torch.int8) if r + 1 < P else None
        if before is None and after is None:
            return None, None
        first, last = rows[:W], rows[W:]
        if self._nccl:
            dst = (before, after)
        else:  # gloo (the on-GPU rehearsal) exchanges host copies
            first, last = first.cpu(), last.cpu()
            dst = tuple(None if b is None else torch.empty(W, dtype=torch.int8) for b in (before, after))
        self._exchange_rows(first, last, *dst)
        if not self._nccl:
            for b, h in zip((before, after), dst):
                if b is not None:
                    b.copy_(h)
        return before, after

    def _exchange_rows(self, first, last, before, after):
        self._check()
        try:
            works = exchange_neighbour_rows(self._dist, self.group, self._group_ranks, self.rank,
                                            self.world_size, first, last, before, after)
        except Exception as e:
            self._fail(f"halo exchange failed: {e}")
        for w in works:
            self._wait(w, "halo exchange")

    def _xstream(self):
        """The band's exchange stream (dm_exchange_stream) as a torch stream."""
        ptr = self.band.exchange_stream()
        if ptr == self.stream.cuda_stream:
            return self.stream
        xs = self._xstreams.get(ptr)
        if xs is None:
            xs = self._torch.cuda.ExternalStream(ptr, device=self._tdev)
            self._xstreams[ptr] = xs
        return xs

    def _device_enqueue(self):
        """Neighbour halo exchange (map stream), band frontiers + export record, and
        the records' all-gather on the band's exchange stream (no host wait).
        Returns the gathered buffer and the exchange stream the merge runs on."""
        torch = self._torch
        W, P, r = self.W, self.world_size, self.rank
        tev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if self.timing else None
        with torch.cuda.stream(self.stream):
            rows = self._buf("rows", 2 * W, torch.int8)
            self.band.edge_rows_device(rows.data_ptr(), rows.data_ptr() + W)
            if tev:
                tev[0].record(self.stream)
            before, after = self._halo_dev(rows)
            if tev:  # the map stream waits for the exchange's completion here
                tev[1].record(self.stream)
            self.band.set_halo_device(before.data_ptr() if before is not None else None,
                                      after.data_ptr() if after is not None else None)
            nb = self.band.export_bytes(self.rec_cap)
            exp = self._buf("exp", nb, torch.uint8)
            gexp = self._buf("gexp", P * nb, torch.uint8)
            self.band.frontiers_export_device(exp.data_ptr(), self.rec_cap)
        xs = self._xstream()
        with torch.cuda.stream(xs):
            if tev:  # reached once this band's export record is written
                tev[2].record(xs)
            self._gather_dev(exp, gexp, self.rec_group)
            if tev:
                tev[3].record(xs)
        if tev:
            self._tev.append(tev)
        return gexp, xs

    # -- exchange timing (bench.py's N > 1 line) ------------------------------
    def set_timing(self, on: bool = True):
        """Record HIP events around this rank's halo exchange (map stream) and
        records all-gather (exchange stream) of every following pass; the
        export and merge kernels are timed by libdm's own profile."""
        self.timing = bool(on) and self._dev_path
        self._tev.clear()

    def exchange_times(self) -> dict:
        """Mean ms per pass since set_timing(True): `halo_ms` from the map
        stream reaching the halo exchange to its completion (the peers' rows
        included: a late neighbour shows here), `records_gather_ms` from this
        band's export record being written to the all-gather's completion
        (waits for the slowest rank's record), and the passes counted."""
        if not self._tev:
            return {"passes": 0, "halo_ms": None, "records_gather_ms": None}
        self._torch.cuda.synchronize(self._tdev)
        halo = [t[0].elapsed_time(t[1]) for t in self._tev]
        gath = [t[2].elapsed_time(t[3]) for t in self._tev]
        return {"passes": len(self._tev), "halo_ms": float(np.mean(halo)),
                "records_gather_ms": float(np.mean(gath))}

    def _device_finish(self, result) -> Frontiers | None:
        """Frontiers from a device merge result, or None when a band's export
        record was incomplete (every rank merged the same gathered headers, so
        all ranks see that together).  The record capacity is grown for the
        next pass; the caller decides what to rerun (frontiers() falls back to
        the host exchange on the map as it is now, frontiers_end() returns None
        because a rerun would describe a later map than the pass it collects)."""
        clusters, max_k = result
        if clusters is not None:
            self._size_rec_cap(self.band.merge_max_band_k())
            return Frontiers(clusters=clusters)
        self.fallbacks += 1
        while self.rec_cap < max_k:
            self.rec_cap *= 2
        return None

    def _size_rec_cap(self, max_k: int):
        """Records per band export for the next passes, from the largest band
        K of the pass just collected (the same value on every rank: all merged
        the same bytes): twice that, a power of two >= 1024, changed only when
        the band K nears the capacity (grown before it overflows) or the
        capacity is 4x what is needed (the record is all-gathered every pass:
        rec_cap x 32 B per rank)."""
        target = 1024
        while target < 2 * max_k:
            target *= 2
        if max_k > (3 * self.rec_cap) // 4 or self.rec_cap >= 4 * target:
            self.rec_cap = target

    def _frontiers_device(self):
        gexp, xs = self._device_enqueue()
        self._drain("frontier exchange", xs)
        with self._torch.cuda.stream(xs):  # libdm merges on the exchange stream
            res = self.band.merge_bands(gexp.data_ptr(), self.world_size, self.rec_cap, self.min_size)
        fr = self._device_finish(res)
        # incomplete record (capacity grown now): this call is synchronous, so
        # the host exchange over the map as it is now is the same map
        return fr if fr is not None else self._frontiers_host(False, False)

    def frontiers(self, want_mask=False, want_labels=False) -> Frontiers:
        """Frontiers of the map as it is now (synchronous; passes started with
        frontiers_begin() may still be in flight)."""
        self._check()
        if not self._exchange:
            return self.band.frontiers(want_mask=want_mask, want_labels=want_labels)
        if self._dev_path and not (want_mask or want_labels):
            return self._frontiers_device()
        return self._frontiers_host(want_mask, want_labels)

    # -- pipelined frontier passes -----------------------------------------
    def set_overlap(self, on: bool = True):
        """Let the next integrate calls' ray front-end run beside an in-flight
        frontier pass (dm_set_overlap; results unchanged)."""
        if hasattr(self.band, "set_overlap"):
            self.band.set_overlap(on)

    def frontiers_begin(self):
        """Start a clusters-only frontier pass over the map as it is now and
        return; frontiers_end() returns its clusters (the same as frontiers()
        would have), and integrate calls may be made in between.  Up to
        dm_max_passes_in_flight() passes may be in flight (libdm's readback
        ring); frontiers_end() collects the oldest."""
        self._check()
        if len(self._pending) >= self.max_in_flight:
            raise RuntimeError(f"{len(self._pending)} frontiers_begin() passes are in flight: "
                               "call frontiers_end() first")
        if not self._exchange and hasattr(self.band, "frontiers_begin"):
            self.band.frontiers_begin()
            self._pending.append(("band", None))
        elif self._exchange and self._dev_path:
            gexp, xs = self._device_enqueue()
            with self._torch.cuda.stream(xs):  # libdm merges on the exchange stream
                self.band.merge_bands_begin(gexp.data_ptr(), self.world_size, self.rec_cap, self.min_size)
            ev = self._torch.cuda.Event()
            ev.record(xs)  # after this pass's collectives and merge
            self._pending.append(("merge", ev))
        else:  # host exchange (or a non-libdm band): computed now
            self._pending.append(("done", self.frontiers()))

    def frontiers_end(self) -> Frontiers | None:
        """Clusters of the oldest pass started with frontiers_begin(), exactly
        as frontiers() would have returned them when the pass started; None if
        that pass has no result (the library's slot arrays or a band's export
        record overflowed: capacities are grown now).  A None pass is not
        recomputed here — the map may have changed since it started; call
        frontiers() for the map as it is now."""
        self._check()
        kind, res = self._pending.popleft()
        if kind == "band":
            return self.band.frontiers_end()
        if kind == "merge":
            self._poll(res, "frontier exchange")
            return self._device_finish(self.band.merge_bands_end())
        return res

    def _frontiers_host(self, want_mask, want_labels) -> Frontiers:
        if self._dev_path:
            self._torch.cuda.synchronize(self._tdev)
        self.exchange_halos()
        local = self.band.frontiers(want_mask=want_mask, want_labels=want_labels)
        first, last = self.band.edge_labels()
        edges = self._allgather(np.stack([first, last]))
        rec = np.stack([local.clusters["label"], local.clusters["size"], local.clusters["sum_x"],
                        local.clusters["sum_y"]], 1).astype(np.int64) if len(local) else \
            np.zeros((0, 4), np.int64)
        counts = self._allgather(np.array([rec.shape[0]], np.int64))[:, 0]
        kmax = int(counts.max()) if counts.size else 0
        pad = np.zeros((kmax, 4), np.int64)
        pad[:rec.shape[0]] = rec
        allrec = self._allgather(pad) if kmax else np.zeros((self.world_size, 0, 4), np.int64)
        records = [allrec[r, :int(counts[r])] for r in range(self.world_size)]
        merged = merge_clusters(records, [(edges[r, 0], edges[r, 1]) for r in range(self.world_size)],
                                self.params, self.min_size)
        labels = None
        if want_labels and local.labels is not None:
            labels = relabel(local.labels, records, [(edges[r, 0], edges[r, 1]) for r in range(self.world_size)])
        return Frontiers(clusters=merged, mask=local.mask, labels=labels)

    def close(self):
        self.band.close()


__all__ = ["ShardedMapper", "band_rows", "band_params", "exchange_neighbour_rows", "merge_clusters", "relabel",
           "resolve_labels"]
