// dm_sharded.cpp — one map sharded in row bands over the HIP devices of ONE
// process (dm_create_sharded; SURVEY.md §8(b) "sharded variants ... with the
// same calls", §8(e) row bands).
//
// The handle dm_create_sharded returns is a parent whose bands are ordinary
// band handles (dm_create with band_row0 / band_rows, one per device entry).
// Every public call on the parent is dispatched here (dm_api.cpp: DM_SHARDED)
// and runs on the bands, so the reference's caller — the ROS node wired at
// server/thymio_project/launch/pc_server.launch.py:12-19 — shards a map by
// passing a device list, with no code of its own for the exchange:
//
// * integrate: every band gets the scans whose max-range disk reaches its rows
//   (the band clips the rays itself, so each beam-cell update is counted by
//   exactly one band); bands on different devices run concurrently;
// * frontiers: the exchange of dm/sharded.py, device-resident and inside
//   libdm: each band copies its first / last state rows into an exchange
//   buffer on its device; each band's halo rows arrive by peer copies from
//   its neighbours' devices (hipMemcpyPeerAsync over xGMI; a plain device
//   copy when both bands share a device), ordered by events; every band
//   writes its export record (dm_frontiers_export_device); the records are
//   peer-copied in band order into one gathered buffer on band 0's device
//   and dm_merge_bands resolves the labels there.  The result equals a single
//   handle's bit for bit (min-index labels, exact int64 sums).
//   A process-local device exchange needs no collective library: peer copies
//   are what RCCL would issue for these KB-MB messages.  Multi-process
//   sharding (one process per GPU) stays in dm/sharded.py over RCCL.
//
// Buffers the exchange writes are double-buffered by pass parity: at most
// kRbSlots asynchronous passes are in flight (band 0's readback ring), and a
// parity set is rewritten only after the pass that used it was collected.
#include <string.h>

#include <algorithm>
#include <new>
#include <numeric>
#include <vector>

#include "dm_internal.h"

namespace {

constexpr int kSets = 2;

struct Staging {  // pinned host copies of one band's scan subset (a ring of 3)
  double* poses = nullptr;
  float* ranges = nullptr;
  int64_t pose_cap = 0, ranges_cap = 0;
};

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

template <class T>
int dev_alloc_on(int dev, T** p, int64_t count, const char* what) {
  (void)hipSetDevice(dev);
  if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (count <= 0) count = 1;
  const hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    *p = nullptr;
    return dm_set_error(e == hipErrorOutOfMemory ? DM_ERR_OOM : DM_ERR_HIP, "hipMalloc(%s): %s", what,
                        hipGetErrorString(e));
  }
  return DM_OK;
}

}  // namespace

struct dm_shard_set {
  int P = 0;
  std::vector<dm_grid*> band;
  std::vector<int> dev;
  std::vector<int64_t> row0, rows;
  int64_t W = 0, H = 0;
  int64_t min_size = 1;
  // exchange buffers [set][band] on the band's device
  std::vector<int8_t*> erows[kSets], halo[kSets];  // [2W]: own first / last rows; neighbours' rows
  std::vector<uint8_t*> exp[kSets];                 // export record of the band
  uint8_t* gathered[kSets] = {nullptr, nullptr};    // P records on band 0's device
  std::vector<hipEvent_t> ev_rows, ev_exp;
  // dm_sh_ld06_to_scans_device writes its scans on band 0's stream: the next
  // dm_sh_integrate_device orders every band's input reads after ev_in
  hipEvent_t ev_in = nullptr;
  bool in_pending = false;
  int64_t rec_cap = 0, want_rec_cap = 0, nb = 0;
  bool refresh = false;  // run a synchronous pass on every band before the next exchange
  int set = 0;       // parity of the next pass
  int pending = 0;   // asynchronous passes in flight
  // integrate staging and the bands integrated by the last call
  std::vector<Staging> stage[3];
  std::vector<int> stage_head;  // per band: its own calls, so slot j % 3 is free at its call j
  std::vector<char> active;
  // device-input copies for bands on another device than the inputs
  std::vector<double*> d_pose;
  std::vector<float*> d_ranges;
  std::vector<int64_t> d_pose_cap, d_ranges_cap;
};

namespace {

int sh_alloc_exchange(dm_shard_set* s, int64_t rec_cap) {
  for (int k = 0; k < kSets; ++k) {
    for (int r = 0; r < s->P; ++r) {
      int rc = dev_alloc_on(s->dev[r], &s->erows[k][r], 2 * s->W, "sharded edge rows");
      if (!rc) rc = dev_alloc_on(s->dev[r], &s->halo[k][r], 2 * s->W, "sharded halo rows");
      if (rc) return rc;
    }
  }
  int64_t nb = 0;
  int rc = dm_export_bytes(s->band[0], rec_cap, &nb);
  if (rc) return rc;
  for (int k = 0; k < kSets; ++k) {
    for (int r = 0; r < s->P; ++r)
      if ((rc = dev_alloc_on(s->dev[r], &s->exp[k][r], nb, "sharded export record"))) return rc;
    if ((rc = dev_alloc_on(s->dev[0], &s->gathered[k], nb * s->P, "sharded gathered records"))) return rc;
  }
  s->rec_cap = rec_cap;
  s->nb = nb;
  return DM_OK;
}

int sh_sync(dm_shard_set* s) {
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_synchronize(s->band[r])) return rc;
  return DM_OK;
}

// Grow the export capacity after an incomplete record.  The exchange
// buffers may be reallocated once the device work of every pass in flight is
// done (their results live in band 0's readback slots, not in these
// buffers): `synced` says the caller just waited for the bands; otherwise
// growth waits until no pass is in flight.
int sh_apply_growth(dm_shard_set* s, bool synced) {
  if (s->want_rec_cap <= s->rec_cap || (s->pending && !synced)) return DM_OK;
  if (int rc = sh_sync(s)) return rc;
  return sh_alloc_exchange(s, s->want_rec_cap);
}

// After an incomplete merge (band 0's merge counters say why): a record
// with more clusters than rec_cap grows the records; a band whose slot arrays
// overflowed or whose clusters were too many for the sort it chose runs one
// synchronous pass of its own before the next exchange (dm_frontiers grows
// its slots and sets its sort hint).  A union-find bound is an error.
int sh_note_incomplete(dm_shard_set* s, int64_t max_k) {
  const unsigned long long flags = s->band[0]->h_mcnt[1];
  if (flags & 32ull)
    return dm_set_error(DM_ERR_INCOMPLETE, "frontier union-find did not converge within its bound");
  if (flags & 2ull) s->want_rec_cap = std::max<int64_t>(2 * s->rec_cap, max_k + max_k / 4 + 64);
  if (flags & (1ull | 4ull)) s->refresh = true;
  if (!(flags & (1ull | 2ull | 4ull))) s->refresh = true;  // unknown cause: refresh anyway
  return DM_OK;
}

int sh_refresh_bands(dm_shard_set* s, bool synced) {
  if (!s->refresh) return sh_apply_growth(s, synced);
  // band 0's own pass would become its goal source (dm_assign_goals reads
  // the last collected result): keep the last merged result's instead
  dm_grid* b0 = s->band[0];
  const int goal_slot = b0->goal_slot, goal_kind = b0->goal_kind;
  const uint64_t goal_epoch = b0->goal_epoch, goal_gen = b0->goal_gen;
  const int64_t goal_n = b0->goal_n;
  for (int r = 0; r < s->P; ++r) {
    int64_t n = 0;
    const int rc = dm_frontiers(s->band[(size_t)r], nullptr, nullptr, nullptr, 0, &n);
    if (rc && rc != DM_ERR_CAPACITY) return rc;
  }
  b0->goal_slot = goal_slot;
  b0->goal_kind = goal_kind;
  b0->goal_epoch = goal_epoch;
  b0->goal_gen = goal_gen;
  b0->goal_n = goal_n;
  s->refresh = false;
  return sh_apply_growth(s, synced);
}

// One exchange copy on `st`: a peer copy over xGMI between two devices, a
// device copy when both are the same (hipMemcpyPeerAsync takes both, so the
// bands-on-one-GPU tests drive this same call).
hipError_t peer_copy(void* dst, int ddev, const void* src, int sdev, size_t n, hipStream_t st) {
  return hipMemcpyPeerAsync(dst, ddev, src, sdev, n, st);
}

// Halo rows, band exports and the gather into band 0's buffer, all enqueued
// (no host wait), on exchange set `k`.
int sh_enqueue_exchange(dm_shard_set* s, int k) {
  const int P = s->P;
  const int64_t W = s->W;
  int rc = 0;
  for (int r = 0; r < P; ++r) {
    if ((rc = dm_get_edge_rows_device(s->band[r], s->erows[k][r], s->erows[k][r] + W))) return rc;
    DM_HIP(hipEventRecord(s->ev_rows[r], s->band[r]->stream));
  }
  for (int r = 0; r < P; ++r) {
    dm_grid* b = s->band[r];
    DM_HIP(hipSetDevice(s->dev[r]));
    if (r > 0) {  // the row above the band = band r-1's last row
      DM_HIP(hipStreamWaitEvent(b->stream, s->ev_rows[r - 1], 0));
      DM_HIP(peer_copy(s->halo[k][r], s->dev[r], s->erows[k][r - 1] + W, s->dev[r - 1], (size_t)W, b->stream));
    }
    if (r + 1 < P) {  // the row below = band r+1's first row
      DM_HIP(hipStreamWaitEvent(b->stream, s->ev_rows[r + 1], 0));
      DM_HIP(peer_copy(s->halo[k][r] + W, s->dev[r], s->erows[k][r + 1], s->dev[r + 1], (size_t)W, b->stream));
    }
    if ((rc = dm_set_halo_device(b, r > 0 ? s->halo[k][r] : nullptr, r + 1 < P ? s->halo[k][r] + W : nullptr)))
      return rc;
    if ((rc = dm_frontiers_export_device(b, s->exp[k][r], s->rec_cap))) return rc;
    // the record is complete on the band's exchange stream (its pass
    // stream with overlap on: the split pass)
    DM_HIP(hipEventRecord(s->ev_exp[r], dm_exchange_stream_of(b)));
  }
  // gathered on band 0's exchange stream, where its merge runs
  dm_grid* b0 = s->band[0];
  DM_HIP(hipSetDevice(s->dev[0]));
  hipStream_t ms = dm_exchange_stream_of(b0);
  for (int r = 0; r < P; ++r) {
    DM_HIP(hipStreamWaitEvent(ms, s->ev_exp[r], 0));
    DM_HIP(peer_copy(s->gathered[k] + (size_t)r * (size_t)s->nb, s->dev[0], s->exp[k][r], s->dev[r],
                     (size_t)s->nb, ms));
  }
  return DM_OK;
}

// Host merge of per-band cluster lists for the labels output: band r's
// records (label-sorted) and its first / last-row labels -> the final label
// of every record (the min label of its cross-band component).
struct HostMerge {
  std::vector<std::vector<int64_t>> labels;  // per band, sorted
  std::vector<int64_t> base;                 // element offset of each band
  std::vector<int64_t> parent, final_label;

  int64_t find(int64_t a) {
    while (parent[(size_t)a] != a) {
      parent[(size_t)a] = parent[(size_t)parent[(size_t)a]];
      a = parent[(size_t)a];
    }
    return a;
  }
  void unite(int64_t a, int64_t b) {
    a = find(a);
    b = find(b);
    if (a == b) return;
    if (final_label[(size_t)a] <= final_label[(size_t)b]) parent[(size_t)b] = a;
    else parent[(size_t)a] = b;
  }
  int64_t elem(int r, int64_t label) const {
    const auto& v = labels[(size_t)r];
    const auto it = std::lower_bound(v.begin(), v.end(), label);
    return (it != v.end() && *it == label) ? base[(size_t)r] + (int64_t)(it - v.begin()) : -1;
  }
};

}  // namespace

int dm_sh_destroy(dm_grid* g) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r) {
    if (!s->band[r]) continue;
    (void)hipSetDevice(s->dev[r]);
    (void)dm_synchronize(s->band[r]);
    for (int k = 0; k < kSets; ++k) {
      if (s->erows[k][r]) (void)hipFree(s->erows[k][r]);
      if (s->halo[k][r]) (void)hipFree(s->halo[k][r]);
      if (s->exp[k][r]) (void)hipFree(s->exp[k][r]);
    }
    if (s->d_pose[r]) (void)hipFree(s->d_pose[r]);
    if (s->d_ranges[r]) (void)hipFree(s->d_ranges[r]);
    if (s->ev_rows[r]) (void)hipEventDestroy(s->ev_rows[r]);
    if (s->ev_exp[r]) (void)hipEventDestroy(s->ev_exp[r]);
    for (auto& st : s->stage) {
      if (st[(size_t)r].poses) (void)hipHostFree(st[(size_t)r].poses);
      if (st[(size_t)r].ranges) (void)hipHostFree(st[(size_t)r].ranges);
    }
  }
  if (s->P > 0 && s->band[0]) {
    (void)hipSetDevice(s->dev[0]);
    for (auto* p : s->gathered)
      if (p) (void)hipFree(p);
    if (s->ev_in) (void)hipEventDestroy(s->ev_in);
  }
  for (int r = 0; r < s->P; ++r) (void)dm_destroy(s->band[r]);
  delete s;
  g->sh = nullptr;
  delete g;
  return DM_OK;
}

extern "C" int dm_sharded_band_rows(int64_t height, int32_t nranks, int32_t rank, int64_t* row0,
                                    int64_t* rows) {
  if (height <= 0 || nranks < 1 || rank < 0 || rank >= nranks || !row0 || !rows)
    return dm_set_error(DM_ERR_INVALID_ARG, "need height > 0, 0 <= rank < nranks, row0 / rows");
  const int64_t per = ceil_div(ceil_div(height, DM_TILE), nranks) * DM_TILE;
  *row0 = std::min<int64_t>((int64_t)rank * per, height);
  *rows = std::max<int64_t>(0, std::min<int64_t>(per, height - *row0));
  return DM_OK;
}

extern "C" int dm_create_sharded(dm_grid** out, const dm_params* p, int32_t nranks, const int32_t* devices) {
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  if (!p) return dm_set_error(DM_ERR_INVALID_ARG, "params is NULL");
  if (nranks < 1 || nranks > 64 || !devices)
    return dm_set_error(DM_ERR_INVALID_ARG, "need 1 <= nranks <= 64 and a device list");
  if (p->band_row0 != 0 || (p->band_rows != 0 && p->band_rows != p->height))
    return dm_set_error(DM_ERR_INVALID_ARG, "a sharded map covers the whole grid: band_row0 = 0, band_rows = 0");
  dm_grid* g = new (std::nothrow) dm_grid();
  dm_shard_set* s = new (std::nothrow) dm_shard_set();
  if (!g || !s) {
    delete g;
    delete s;
    return dm_set_error(DM_ERR_OOM, "host allocation failed");
  }
  g->sh = s;
  g->p = *p;
  g->p.band_row0 = 0;
  g->p.band_rows = p->height;
  g->device = devices[0];
  g->W = p->width;
  g->H = g->R = p->height;
  s->P = nranks;
  s->W = p->width;
  s->H = p->height;
  s->min_size = p->min_frontier_size;
  s->band.assign((size_t)nranks, nullptr);
  s->dev.assign(devices, devices + nranks);
  s->row0.assign((size_t)nranks, 0);
  s->rows.assign((size_t)nranks, 0);
  for (int k = 0; k < kSets; ++k) {
    s->erows[k].assign((size_t)nranks, nullptr);
    s->halo[k].assign((size_t)nranks, nullptr);
    s->exp[k].assign((size_t)nranks, nullptr);
  }
  s->ev_rows.assign((size_t)nranks, nullptr);
  s->ev_exp.assign((size_t)nranks, nullptr);
  for (auto& st : s->stage) st.assign((size_t)nranks, Staging());
  s->active.assign((size_t)nranks, 0);
  s->stage_head.assign((size_t)nranks, 0);
  s->d_pose.assign((size_t)nranks, nullptr);
  s->d_ranges.assign((size_t)nranks, nullptr);
  s->d_pose_cap.assign((size_t)nranks, 0);
  s->d_ranges_cap.assign((size_t)nranks, 0);
  auto fail = [&](int code) {
    dm_sh_destroy(g);
    return code;
  };
  for (int r = 0; r < nranks; ++r) {
    int64_t r0 = 0, rows = 0;
    int rc = dm_sharded_band_rows(p->height, nranks, r, &r0, &rows);
    if (rc) return fail(rc);
    if (rows <= 0)
      return fail(dm_set_error(DM_ERR_INVALID_ARG, "band %d has no rows (height %lld over %d bands)", r,
                               (long long)p->height, nranks));
    dm_params bp = *p;
    bp.band_row0 = r0;
    bp.band_rows = rows;
    bp.min_frontier_size = 1;  // the size filter applies to merged clusters
    if ((rc = dm_create(&s->band[(size_t)r], &bp, devices[r]))) return fail(rc);
    s->row0[(size_t)r] = r0;
    s->rows[(size_t)r] = rows;
    (void)hipSetDevice(devices[r]);
    for (hipEvent_t* ev : {&s->ev_rows[(size_t)r], &s->ev_exp[(size_t)r]}) {
      const hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
      if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
    }
  }
  (void)hipSetDevice(devices[0]);
  {
    const hipError_t e = hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
  }
  // peer access between the bands' devices where the platform offers it
  // (the copies work either way; with access they go device to device)
  for (int a = 0; a < nranks; ++a)
    for (int b = 0; b < nranks; ++b) {
      if (devices[a] == devices[b]) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[a], devices[b]) == hipSuccess && can) {
        (void)hipSetDevice(devices[a]);
        const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(dm_hip_check(e, "peer access"));
        (void)hipGetLastError();
      }
    }
  // records per band export, sized for the band up front (an export that
  // overflows has no result): a cluster per two tiles of the band (C5's
  // sparsest rays: ~0.2); the exchange copies stay on the node's xGMI
  int64_t rec_cap = 16384;
  while (rec_cap < ceil_div(p->width, DM_TILE) * ceil_div(s->rows[0], DM_TILE)) rec_cap *= 2;
  if (int rc = sh_alloc_exchange(s, rec_cap)) return fail(rc);
  *out = g;
  return DM_OK;
}

// ---- integrate -----------------------------------------------------------

namespace {

// Stage band r's scans (those whose max-range disk reaches its rows) in the
// current staging slot; returns the count.
int sh_stage(dm_shard_set* s, const dm_params& p, int r, int32_t S, const double* poses, int32_t N,
             const float* ranges, int32_t* S_out) {
  Staging& st = s->stage[s->stage_head[(size_t)r]][(size_t)r];
  if ((int64_t)S * 3 > st.pose_cap) {
    if (st.poses) (void)hipHostFree(st.poses);
    st.poses = nullptr;
    st.pose_cap = 0;
    DM_HIP(hipHostMalloc((void**)&st.poses, sizeof(double) * 3 * (size_t)std::max(S, 1), hipHostMallocDefault));
    st.pose_cap = (int64_t)std::max(S, 1) * 3;
  }
  if ((int64_t)S * N > st.ranges_cap) {
    if (st.ranges) (void)hipHostFree(st.ranges);
    st.ranges = nullptr;
    st.ranges_cap = 0;
    const int64_t n = std::max<int64_t>((int64_t)S * N, 1);
    DM_HIP(hipHostMalloc((void**)&st.ranges, sizeof(float) * (size_t)n, hipHostMallocDefault));
    st.ranges_cap = n;
  }
  const double reach = (double)p.range_max + 2.0 * p.resolution;
  const double ylo = p.origin_y + (double)s->row0[(size_t)r] * p.resolution - reach;
  const double yhi = p.origin_y + (double)(s->row0[(size_t)r] + s->rows[(size_t)r]) * p.resolution + reach;
  int32_t k = 0;
  for (int32_t i = 0; i < S; ++i) {
    const double y = poses[3 * i + 1];
    if (y < ylo || y > yhi) continue;  // NaN poses are kept (the band skips them)
    memcpy(st.poses + 3 * (size_t)k, poses + 3 * (size_t)i, 3 * sizeof(double));
    memcpy(st.ranges + (size_t)k * (size_t)N, ranges + (size_t)i * (size_t)N, sizeof(float) * (size_t)N);
    ++k;
  }
  *S_out = k;
  return DM_OK;
}

}  // namespace

int dm_sh_integrate_async(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges,
                          float amin, float inc) {
  dm_shard_set* s = g->sh;
  if (S < 0 || N < 0) return dm_set_error(DM_ERR_SHAPE, "S and N must be >= 0");
  if ((int64_t)S * N > 0 && (!poses || !ranges)) return dm_set_error(DM_ERR_INVALID_ARG, "poses/ranges is NULL");
  int rc = 0;
  for (int r = 0; r < s->P; ++r) {
    int32_t k = 0;
    if ((rc = sh_stage(s, g->p, r, S, poses, N, ranges, &k))) return rc;
    s->active[(size_t)r] = k > 0;
    if (!k) continue;
    int& head = s->stage_head[(size_t)r];
    const Staging& st = s->stage[head][(size_t)r];
    if ((rc = dm_integrate_async(s->band[(size_t)r], k, st.poses, N, st.ranges, amin, inc))) return rc;
    // the band's slot j % 3 is rewritten at its call j + 3: its call j + 2
    // has returned by then, which waited for the copies of its call j
    // (dm_integrate_async's staging contract)
    head = (head + 1) % 3;
  }
  return DM_OK;
}

int dm_sh_last_counts(dm_grid* g, uint64_t* U, uint64_t* T) {
  dm_shard_set* s = g->sh;
  uint64_t su = 0, st = 0;
  for (int r = 0; r < s->P; ++r) {
    if (!s->active[(size_t)r]) continue;
    uint64_t u = 0, t = 0;
    if (int rc = dm_last_counts(s->band[(size_t)r], &u, &t)) return rc;
    su += u;
    st += t;
  }
  if (U) *U = su;
  if (T) *T = st;
  return DM_OK;
}

int dm_sh_integrate(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges, float amin,
                    float inc, uint64_t* U, uint64_t* T) {
  if (int rc = dm_sh_integrate_async(g, S, poses, N, ranges, amin, inc)) return rc;
  return dm_sh_last_counts(g, U, T);
}

int dm_sh_integrate_device(dm_grid* g, int32_t S, const double* d_pose4, int32_t N, const float* d_ranges,
                           float amin, float inc) {
  dm_shard_set* s = g->sh;
  if (S < 0 || N < 0) return dm_set_error(DM_ERR_SHAPE, "S and N must be >= 0");
  const int64_t nb = (int64_t)S * N;
  if (nb > 0 && (!d_pose4 || !d_ranges)) return dm_set_error(DM_ERR_INVALID_ARG, "poses/ranges is NULL");
  int src = s->dev[0];
  if (nb > 0) {
    hipPointerAttribute_t a;
    DM_HIP(hipPointerGetAttributes(&a, d_ranges));
    src = a.device;
  }
  // scans written by dm_sh_ld06_to_scans_device on band 0's stream: every
  // band reads them after that kernel (each band's front-end runs on its own
  // stream, and with overlap on a stream of its own again)
  const bool wait_in = s->in_pending;
  s->in_pending = false;
  for (int r = 0; r < s->P; ++r) {
    dm_grid* b = s->band[(size_t)r];
    const int d = s->dev[(size_t)r];
    const double* pp = d_pose4;
    const float* rp = d_ranges;
    // the stream the band's front-end (the only reader of the inputs) runs on
    hipStream_t fs = b->overlap ? dm_fe_stream_of(b, dm_next_set(b)) : b->stream;
    DM_HIP(hipSetDevice(d));
    if (wait_in) DM_HIP(hipStreamWaitEvent(fs, s->ev_in, 0));
    if (nb > 0 && d != src) {  // inputs on another device: a copy the band owns
      if ((int64_t)S * 4 > s->d_pose_cap[(size_t)r] || nb > s->d_ranges_cap[(size_t)r]) {
        // a call in flight may still read the old copy
        if (int rc = dm_synchronize(b)) return rc;
      }
      if ((int64_t)S * 4 > s->d_pose_cap[(size_t)r]) {
        if (int rc = dev_alloc_on(d, &s->d_pose[(size_t)r], (int64_t)S * 4, "sharded poses")) return rc;
        s->d_pose_cap[(size_t)r] = (int64_t)S * 4;
      }
      if (nb > s->d_ranges_cap[(size_t)r]) {
        if (int rc = dev_alloc_on(d, &s->d_ranges[(size_t)r], nb, "sharded ranges")) return rc;
        s->d_ranges_cap[(size_t)r] = nb;
      }
      // on the front-end's stream: after the previous call's front-end read
      // the last copy (on another stream when front-ends alternate between
      // two: ev_fe_end), before this call's reads it
      if (dm_grid::kFeStreams > 1 && b->overlap) DM_HIP(hipStreamWaitEvent(fs, b->ev_fe_end[b->iw_cur % 2], 0));
      DM_HIP(hipMemcpyPeerAsync(s->d_pose[(size_t)r], d, d_pose4, src, sizeof(double) * 4 * (size_t)S, fs));
      DM_HIP(hipMemcpyPeerAsync(s->d_ranges[(size_t)r], d, d_ranges, src, sizeof(float) * (size_t)nb, fs));
      pp = s->d_pose[(size_t)r];
      rp = s->d_ranges[(size_t)r];
    }
    if (int rc = dm_integrate_device(b, S, pp, N, rp, amin, inc)) return rc;
    s->active[(size_t)r] = 1;
  }
  return DM_OK;
}

// ---- map access -------------------------------------------------------------

int dm_sh_get_state(dm_grid* g, int8_t* out) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_get_state(s->band[(size_t)r], out + s->row0[(size_t)r] * s->W)) return rc;
  return DM_OK;
}

int dm_sh_get_logodds(dm_grid* g, float* out) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_get_logodds(s->band[(size_t)r], out + s->row0[(size_t)r] * s->W)) return rc;
  return DM_OK;
}

int dm_sh_set_logodds(dm_grid* g, const float* in) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_set_logodds(s->band[(size_t)r], in + s->row0[(size_t)r] * s->W)) return rc;
  return DM_OK;
}

int dm_sh_set_state(dm_grid* g, const int8_t* in) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_set_state(s->band[(size_t)r], in + s->row0[(size_t)r] * s->W)) return rc;
  return DM_OK;
}

int dm_sh_map_image(dm_grid* g, uint8_t* out) {
  // flipud per band: band rows [row0, row0 + rows) land on image rows
  // [H - row0 - rows, H - row0)
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_map_image(s->band[(size_t)r], out + (s->H - s->row0[(size_t)r] - s->rows[(size_t)r]) * s->W))
      return rc;
  return DM_OK;
}

int dm_sh_reset(dm_grid* g) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_reset(s->band[(size_t)r])) return rc;
  return DM_OK;
}

int dm_sh_synchronize(dm_grid* g) { return sh_sync(g->sh); }

int dm_sh_set_overlap(dm_grid* g, int32_t on) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_set_overlap(s->band[(size_t)r], on)) return rc;
  return DM_OK;
}

int dm_sh_last_stats(dm_grid* g, uint64_t* out, int32_t cap, int32_t* n_out) {
  dm_shard_set* s = g->sh;
  if (cap > 0 && !out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  // [0, 7): the last integrate call's counters, over the bands it ran on;
  // the frontier pass's over every band
  uint64_t sum[kNStats] = {0};
  for (int r = 0; r < s->P; ++r) {
    uint64_t v[kNStats] = {0};
    int32_t n = 0;
    if (int rc = dm_last_stats(s->band[(size_t)r], v, kNStats, &n)) return rc;
    // a band without scans in the last call contributes its frontier stats only
    for (int i = 0; i < kNStats; ++i)
      if (s->active[(size_t)r] || dm_stat_is_frontier(i)) sum[i] += v[i];
  }
  for (int32_t i = 0; i < cap && i < kNStats; ++i) out[i] = sum[i];
  if (n_out) *n_out = kNStats;
  return DM_OK;
}

int dm_sh_profile_enable(dm_grid* g, int enable) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_profile_enable(s->band[(size_t)r], enable)) return rc;
  return DM_OK;
}

int dm_sh_profile_read(dm_grid* g, dm_kernel_stat* out, int32_t cap, int32_t* n_out) {
  // per kernel name, summed over the bands
  dm_shard_set* s = g->sh;
  std::vector<dm_kernel_stat> all;
  for (int r = 0; r < s->P; ++r) {
    int32_t n = 0;
    if (int rc = dm_profile_read(s->band[(size_t)r], nullptr, 0, &n)) return rc;
    std::vector<dm_kernel_stat> v((size_t)std::max(n, 1));
    if (int rc = dm_profile_read(s->band[(size_t)r], v.data(), n, &n)) return rc;
    for (int32_t i = 0; i < n; ++i) {
      auto it = std::find_if(all.begin(), all.end(),
                             [&](const dm_kernel_stat& e) { return !strcmp(e.name, v[(size_t)i].name); });
      if (it == all.end()) {
        all.push_back(v[(size_t)i]);
      } else {
        it->launches += v[(size_t)i].launches;
        it->total_ms += v[(size_t)i].total_ms;
      }
    }
  }
  for (int32_t i = 0; i < cap && i < (int32_t)all.size(); ++i) out[i] = all[(size_t)i];
  if (n_out) *n_out = (int32_t)all.size();
  return DM_OK;
}

int dm_sh_profile_reset(dm_grid* g) {
  dm_shard_set* s = g->sh;
  for (int r = 0; r < s->P; ++r)
    if (int rc = dm_profile_reset(s->band[(size_t)r])) return rc;
  return DM_OK;
}

// ---- frontiers ------------------------------------------------------------

namespace {

// Per-cell labels of a sharded map: each band's labels (band-local
// min-index), then every label mapped to its cross-band component's min.
int sh_labels(dm_shard_set* s, uint8_t* mask, int64_t* labels) {
  const int P = s->P;
  const int64_t W = s->W;
  HostMerge hm;
  hm.labels.resize((size_t)P);
  hm.base.resize((size_t)P);
  int64_t total = 0;
  for (int r = 0; r < P; ++r) {
    const int64_t off = s->row0[(size_t)r] * W;
    std::vector<dm_cluster> c(4096);
    int64_t n = 0;
    int rc = 0;
    while (true) {  // mask, labels and the band's label-sorted records
      rc = dm_frontiers(s->band[(size_t)r], mask ? mask + off : nullptr, labels ? labels + off : nullptr, c.data(),
                        (int64_t)c.size(), &n);
      if (rc != DM_ERR_CAPACITY) break;
      c.resize((size_t)n);
    }
    if (rc) return rc;
    if (!labels) continue;
    hm.base[(size_t)r] = total;
    auto& v = hm.labels[(size_t)r];
    v.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) v[(size_t)i] = c[(size_t)i].label;
    total += n;
  }
  if (!labels) return DM_OK;
  hm.parent.resize((size_t)total);
  hm.final_label.resize((size_t)total);
  for (int r = 0; r < P; ++r)
    for (size_t i = 0; i < hm.labels[(size_t)r].size(); ++i) {
      const int64_t e = hm.base[(size_t)r] + (int64_t)i;
      hm.parent[(size_t)e] = e;
      hm.final_label[(size_t)e] = hm.labels[(size_t)r][i];
    }
  // band r's last row vs band r+1's first row, 8-connected
  for (int r = 0; r + 1 < P; ++r) {
    const int64_t* last = labels + (s->row0[(size_t)r] + s->rows[(size_t)r] - 1) * W;
    const int64_t* first = labels + s->row0[(size_t)r + 1] * W;
    for (int64_t x = 0; x < W; ++x) {
      if (last[x] < 0) continue;
      const int64_t a = hm.elem(r, last[x]);
      for (int64_t d = -1; d <= 1; ++d) {
        const int64_t y = x + d;
        if (y < 0 || y >= W || first[y] < 0) continue;
        const int64_t b = hm.elem(r + 1, first[y]);
        if (a >= 0 && b >= 0) hm.unite(a, b);
      }
    }
  }
  for (int r = 0; r < P; ++r) {
    int64_t* lab = labels + s->row0[(size_t)r] * W;
    const int64_t cells = s->rows[(size_t)r] * W;
    for (int64_t i = 0; i < cells; ++i) {
      if (lab[i] < 0) continue;
      const int64_t e = hm.elem(r, lab[i]);
      if (e >= 0) lab[i] = hm.final_label[(size_t)hm.find(e)];
    }
  }
  return DM_OK;
}

}  // namespace

int dm_sh_frontiers(dm_grid* g, uint8_t* mask, int64_t* labels, dm_cluster* out, int64_t cap, int64_t* n_out) {
  dm_shard_set* s = g->sh;
  if (cap < 0 || (cap > 0 && !out)) return dm_set_error(DM_ERR_INVALID_ARG, "bad cluster buffer");
  int rc = 0;
  int k = s->set;
  for (int attempt = 0;; ++attempt) {
    // a synchronous pass reuses exchange set s->set: wait for the passes in
    // flight first (one of them may still read it)
    const bool synced = s->pending > 0;
    if (synced && (rc = sh_sync(s))) return rc;
    if ((rc = sh_refresh_bands(s, synced))) return rc;
    k = s->set;
    if ((rc = sh_enqueue_exchange(s, k))) return rc;
    DM_HIP(hipSetDevice(s->dev[0]));
    int64_t n = 0;
    rc = dm_merge_bands(s->band[0], s->gathered[k], s->P, s->rec_cap, s->min_size, out, cap, &n);
    if (n_out) *n_out = n;
    if (rc != DM_ERR_INCOMPLETE) break;
    if (attempt == 4) return dm_set_error(DM_ERR_INCOMPLETE, "band exports stayed incomplete after growing");
    if ((rc = sh_note_incomplete(s, n))) return rc;
  }
  if (rc && rc != DM_ERR_CAPACITY) return rc;
  const int rc_clusters = rc;
  if (mask || labels) {
    if (int r2 = sh_sync(s)) return r2;
    if (int r2 = sh_labels(s, mask, labels)) return r2;
    // the bands' own passes replaced band 0's last collected result (the
    // one dm_assign_goals reads): merge the same gathered records again
    int64_t n = 0;
    DM_HIP(hipSetDevice(s->dev[0]));
    const int r2 = dm_merge_bands(s->band[0], s->gathered[k], s->P, s->rec_cap, s->min_size, nullptr, 0, &n);
    if (r2 && r2 != DM_ERR_CAPACITY) return r2;
  }
  return rc_clusters;
}

int dm_sh_frontiers_begin(dm_grid* g) {
  dm_shard_set* s = g->sh;
  if (s->pending >= dm_grid::kRbSlots)
    return dm_set_error(DM_ERR_INVALID_ARG, "%d passes in flight: end the oldest first", dm_grid::kRbSlots);
  int rc = sh_refresh_bands(s, false);
  if (rc) return rc;
  const int k = s->set;
  if ((rc = sh_enqueue_exchange(s, k))) return rc;
  DM_HIP(hipSetDevice(s->dev[0]));
  if ((rc = dm_merge_bands_begin(s->band[0], s->gathered[k], s->P, s->rec_cap, s->min_size))) return rc;
  s->set = (s->set + 1) % kSets;
  ++s->pending;
  return DM_OK;
}

int dm_sh_frontiers_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out) {
  dm_shard_set* s = g->sh;
  if (!s->pending) return dm_set_error(DM_ERR_INVALID_ARG, "no dm_frontiers_begin pass in flight");
  DM_HIP(hipSetDevice(s->dev[0]));
  const int rc = dm_merge_bands_end(s->band[0], out, cap, n_out);
  if (rc == DM_ERR_CAPACITY) return rc;  // the pass stays pending
  --s->pending;
  if (rc == DM_ERR_INCOMPLETE) {  // this pass has no result; the next one will
    if (int r2 = sh_note_incomplete(s, n_out ? *n_out : 0)) return r2;
    if (n_out) *n_out = 0;
    return dm_set_error(DM_ERR_INCOMPLETE, "a band export of this pass was incomplete (capacities grown for "
                                           "the next pass): run dm_frontiers");
  }
  return rc;
}

int dm_sh_frontiers_poll(dm_grid* g, int32_t* ready) {
  dm_shard_set* s = g->sh;
  if (!ready) return dm_set_error(DM_ERR_INVALID_ARG, "ready is NULL");
  if (!s->pending) return dm_set_error(DM_ERR_INVALID_ARG, "no dm_frontiers_begin pass in flight");
  return dm_frontiers_poll(s->band[0], ready);
}

int dm_sh_assign_goals(dm_grid* g, const double* robots_xy, int32_t n_robots, int64_t min_size, double w,
                       double min_distance, int64_t* out_index, double* out_xy) {
  return dm_assign_goals(g->sh->band[0], robots_xy, n_robots, min_size, w, min_distance, out_index, out_xy);
}

int dm_sh_ld06_to_scans(dm_grid* g, int32_t S, const dm_ld06_point* points, const int64_t* offsets, int32_t N,
                        int dir, float* ranges, float* intensities) {
  return dm_ld06_to_scans(g->sh->band[0], S, points, offsets, N, dir, ranges, intensities);
}

int dm_sh_ld06_to_scans_device(dm_grid* g, int32_t S, const dm_ld06_point* d_points, const int64_t* d_offsets,
                               int32_t N, int dir, float* d_ranges, float* d_intensities) {
  dm_shard_set* s = g->sh;
  if (int rc = dm_ld06_to_scans_device(s->band[0], S, d_points, d_offsets, N, dir, d_ranges, d_intensities))
    return rc;
  DM_HIP(hipSetDevice(s->dev[0]));
  DM_HIP(hipEventRecord(s->ev_in, s->band[0]->stream));
  s->in_pending = true;
  return DM_OK;
}

extern "C" int dm_sharded_info(const dm_grid* g, int32_t* nranks, int64_t* rec_cap) {
  if (!g) return dm_set_error(DM_ERR_INVALID_ARG, "grid handle is NULL");
  if (nranks) *nranks = g->sh ? g->sh->P : 1;
  if (rec_cap) *rec_cap = g->sh ? g->sh->rec_cap : 0;
  return DM_OK;
}
