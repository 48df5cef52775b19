// dm_api.cpp — the C-ABI of libdm.so (include/dm.h): handle lifetime,
// validation, error codes, host<->device staging, checkpoints, profiling.
//
// Contract from SURVEY.md §8(b): device memory is owned by the handle; host
// pointers are borrowed for the call; synchronous functions return after
// outputs are in host memory; errors are negative codes + a thread-local
// message, never an abort or an exception across the ABI.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "dm_internal.h"

#include <stdlib.h>

// Wait for all three streams; nothing of this handle is in flight afterwards.
hipError_t dm_sync_all(dm_grid* g) {
  for (hipStream_t s : {g->stream, g->fe_streams[0], g->fe_streams[1], g->pass_stream, g->big_stream}) {
    if (!s) continue;
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
  }
  g->p_pending = false;
  for (auto& f : g->fw) f.busy_pending = false;
  return hipSuccess;
}

hipError_t dm_copy_shards(dm_grid* g) {
  const size_t bytes = sizeof(unsigned long long) * kShards * kShardWords;
  hipError_t e = hipMemcpyAsync(g->h_sh, g->iw[g->iw_cur].sh, bytes, hipMemcpyDeviceToHost, g->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->h_sh + kShards * kShardWords, g->fsh, bytes, hipMemcpyDeviceToHost, g->stream);
  return e;
}

namespace {
thread_local std::string t_err;

bool dm_env_on(const char* name) {  // opt-in A/B switches: NAME=1
  const char* v = getenv(name);
  return v && v[0] == '1';
}


struct HostCluster {
  long long label, size, sum_x, sum_y;
};

template <class T>
int dev_alloc(T** p, int64_t count, const char* what) {
  if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (count <= 0) count = 1;
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    *p = nullptr;
    return dm_set_error(e == hipErrorOutOfMemory ? DM_ERR_OOM : DM_ERR_HIP,
                        "hipMalloc(%s, %lld bytes): %s", what,
                        (long long)(sizeof(T) * (size_t)count), hipGetErrorString(e));
  }
  return DM_OK;
}

template <class T>
void dev_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int validate_params(const dm_params* p) {
  if (!p) return dm_set_error(DM_ERR_INVALID_ARG, "params is NULL");
  if (p->width <= 0 || p->height <= 0 || p->width > (1ll << 30) || p->height > (1ll << 30))
    return dm_set_error(DM_ERR_INVALID_ARG, "width/height must be in [1, 2^30] (got %lld x %lld)",
                        (long long)p->width, (long long)p->height);
  if (!(p->resolution > 0.0) || !isfinite(p->resolution))
    return dm_set_error(DM_ERR_INVALID_ARG, "resolution must be finite and > 0");
  if (!isfinite(p->origin_x) || !isfinite(p->origin_y))
    return dm_set_error(DM_ERR_INVALID_ARG, "origin must be finite");
  if (!(p->range_min >= 0.0f) || !(p->range_max > 0.0f) || !isfinite(p->range_max))
    return dm_set_error(DM_ERR_INVALID_ARG, "need 0 <= range_min and finite range_max > 0");
  if ((double)p->range_max / p->resolution > 16384.0)
    return dm_set_error(DM_ERR_INVALID_ARG,
                        "range_max / resolution must be <= 16384 cells (rays longer than that "
                        "are outside the kernels' integer bounds)");
  if (!isfinite(p->l_occ) || !isfinite(p->l_free) || !isfinite(p->l_min) || !isfinite(p->l_max) ||
      !(p->l_min <= p->l_max))
    return dm_set_error(DM_ERR_INVALID_ARG, "log-odds constants must be finite with l_min <= l_max");
  if (p->band_row0 < 0 || p->band_row0 >= p->height || p->band_row0 % DM_TILE != 0)
    return dm_set_error(DM_ERR_INVALID_ARG, "band_row0 must be in [0, height) and a multiple of %d",
                        DM_TILE);
  int64_t R = p->band_rows > 0 ? p->band_rows : p->height - p->band_row0;
  if (R <= 0 || p->band_row0 + R > p->height)
    return dm_set_error(DM_ERR_INVALID_ARG, "band_rows out of range");
  if (ceil_div(p->width, DM_TILE) * ceil_div(R, DM_TILE) > (1ll << 30))
    return dm_set_error(DM_ERR_INVALID_ARG, "too many tiles");
  if (p->min_frontier_size < 0) return dm_set_error(DM_ERR_INVALID_ARG, "min_frontier_size < 0");
  return DM_OK;
}

int grow_integrate(dm_grid* g, int32_t S, int32_t N) {
  const int64_t nb = (int64_t)S * N;
  const int64_t chunks = dm_integrate_chunks(g, nb);
  // pieces per beam: <= 2 per 64 steps + 8, and every chunk adds <= 3
  const int64_t per_beam = 2 * (g->nmax / DM_TILE) + 8 + 4 * chunks;
  const int64_t blocks = ceil_div(nb * chunks, 256);  // k_beam_prep / k_scatter workgroups
  if (nb > g->beams_cap || blocks > g->blk_cap) {
    const int64_t nbc = std::max<int64_t>(nb, g->beams_cap);
    const int64_t bc = std::max<int64_t>(blocks, g->blk_cap);
    int rc = 0;
    for (auto& w : g->iw) {
      if (!rc) rc = dev_alloc(&w.beams, nbc, "beams");
      if (!rc) rc = dev_alloc(&w.blk_hist, bc * 1024, "per-block tile histograms");
      if (!rc) rc = dev_alloc(&w.blk_n, bc, "per-block histogram sizes");
    }
    if (rc) { g->beams_cap = g->blk_cap = 0; return rc; }
    g->beams_cap = nbc;
    g->blk_cap = bc;
  }
  const int64_t segs = nb * per_beam;
  if (segs > g->segs_cap) {
    for (auto& w : g->iw) {
      int rc = dev_alloc(&w.pieces, segs, "ray pieces");
      if (rc) { g->segs_cap = 0; return rc; }
    }
    g->segs_cap = segs;
  }
  const int64_t side = ceil_div(2 * (int64_t)g->nmax + 1, DM_TILE) + 1;
  int64_t act = std::min<int64_t>(g->NT, std::min<int64_t>(segs, (int64_t)S * side * side));
  if (act < 1) act = 1;
  if (act > g->act_cap) {
    int rc = 0;
    for (auto& w : g->iw) {
      if (!rc) rc = dev_alloc(&w.act_raw, act * kShards, "first-touch lists");
      if (!rc) rc = dev_alloc(&w.litems, act, "light work items");
    }
    if (rc) { g->act_cap = 0; return rc; }
    g->act_cap = act;
  }
  // work items of medium and heavy tiles (exact bounds: such a tile has
  // more than kIntegrateChunk pieces, its items ceil(pieces / chunk) <=
  // pieces / chunk + 1), heavy tiles (more than kIntegrateMedium pieces)
  const int64_t chunk = kIntegrateChunk;
  const int64_t heavy = std::max<int64_t>(1, std::min<int64_t>(g->act_cap, segs / (kIntegrateMedium + 1) + 1));
  const int64_t hitems = segs / chunk + segs / (chunk + 1) + 2;
  if (hitems > g->hitem_cap) {
    for (auto& w : g->iw) {
      int rc = dev_alloc(&w.hitems, hitems, "heavy work items");
      if (rc) { g->hitem_cap = 0; return rc; }
    }
    g->hitem_cap = hitems;
  }
  if (heavy > g->heavy_cap) {
    for (auto& w : g->iw) {
      int rc = dev_alloc(&w.heavy_list, heavy, "heavy tiles");
      if (!rc) rc = dev_alloc(&w.slabs, heavy * 2 * DM_TILE * DM_TILE, "heavy-tile slabs");
      if (!rc) rc = dev_alloc(&w.heavy_done, heavy, "heavy-tile item tickets");
      if (rc) { g->heavy_cap = 0; return rc; }
      DM_HIP(hipMemset(w.slabs, 0, sizeof(uint32_t) * (size_t)(heavy * 2 * DM_TILE * DM_TILE)));
      DM_HIP(hipMemset(w.heavy_done, 0, sizeof(int32_t) * (size_t)heavy));
    }
    g->heavy_cap = heavy;
  }
  if (2 * (int64_t)N > g->trig_cap) {
    int rc = dev_alloc(&g->trig, 2 * (int64_t)N, "trig table");
    if (rc) return rc;
    g->trig_cap = 2 * (int64_t)N;
    g->trig_n = -1;
  }
  return DM_OK;
}

int ensure_trig(dm_grid* g, int32_t N, float amin, float inc) {
  if (N == g->trig_n && amin == g->trig_amin && inc == g->trig_inc) return DM_OK;
  // the table may still be read by an in-flight call
  DM_HIP(dm_sync_all(g));
  std::vector<double> t(2 * (size_t)std::max(N, 1));
  for (int32_t i = 0; i < N; ++i) {
    const double phi = (double)amin + (double)i * (double)inc;
    t[2 * i] = cos(phi);
    t[2 * i + 1] = sin(phi);
  }
  if (N > 0) DM_HIP(hipMemcpy(g->trig, t.data(), sizeof(double) * 2 * N, hipMemcpyHostToDevice));
  g->trig_n = N;
  g->trig_amin = amin;
  g->trig_inc = inc;
  return DM_OK;
}

}  // namespace

// Record workspace of the row-bucket sort (k_bs_*): >= every record count a
// sort may be asked to order (band slot_cap, merge m_cap).
int dm_grow_bucket_sort(dm_grid* g, int64_t n) {
  if (n <= g->bs_cap) return DM_OK;
  int rc = dev_alloc(&g->bs_key, n, "row-sort keys");
  if (!rc) rc = dev_alloc(&g->bs_key2, n, "row-sort keys");
  if (!rc) rc = dev_alloc(&g->bs_idx, n, "row-sort indices");
  if (!rc) rc = dev_alloc(&g->bs_idx2, n, "row-sort indices");
  if (!rc && g->rs_rows < g->H) {  // rows of the whole map (merges sort over H rows)
    rc = dev_alloc(&g->rs_cnt, g->H, "row-sort counters");
    if (!rc) rc = dev_alloc(&g->rs_off, g->H + 1, "row-sort offsets");
    if (!rc) rc = dev_alloc(&g->rs_status, g->H / 8192 + 2, "row-sort workgroup totals");
    if (!rc) {
      DM_HIP(hipMemset(g->rs_cnt, 0, sizeof(int32_t) * (size_t)g->H));
      g->rs_rows = g->H;
    }
  }
  if (rc) { g->bs_cap = 0; return rc; }
  g->bs_cap = n;
  return DM_OK;
}

namespace {

int grow_slots(dm_grid* g, int64_t need) {
  int64_t cap = std::max<int64_t>(need, 2 * g->slot_cap);
  if (cap < (1 << 16)) cap = 1 << 16;
  cap = ceil_div(cap, kShards) * kShards;  // kShards equal regions (k_frontier_tile)
  int rc = dev_alloc(&g->slot_label, cap, "slot labels");
  for (auto& f : g->fw)
    if (!rc) rc = dev_alloc(&f.slot_parent, cap, "slot parents");
  g->slot_parent = g->fw[g->fparity].slot_parent;
  if (!rc) rc = dev_alloc(&g->slot_root, cap, "slot roots");
  if (!rc) rc = dev_alloc(&g->slot_own, 3 * cap, "slot sums");
  if (!rc) rc = dev_alloc(&g->slot_acc, 3 * cap, "slot totals");
  if (!rc) rc = dev_alloc(&g->clusters, 4 * cap, "clusters");
  for (int sl = 0; sl <= dm_grid::kRbSlots && !rc; ++sl) {  // one per readback slot
    dm_cluster* base = g->rb[sl].out_clu ? g->rb[sl].out_clu - kRbRecords : nullptr;
    rc = dev_alloc(&base, cap + kRbRecords, "sorted clusters");
    g->rb[sl].out_clu = base ? base + kRbRecords : nullptr;
  }
  ++g->rb_gen;
  g->out_clu = g->rb[g->rb_head].out_clu;
  if (!rc) rc = dev_alloc(&g->slot_k, cap, "slot cluster index");
  if (!rc) rc = dev_alloc(&g->rank_of, cap, "cluster sorted position");
  if (!rc) rc = dm_grow_bucket_sort(g, cap);
  if (rc) return rc;
  g->slot_cap = cap;
  return DM_OK;
}

// Grow readback slot `slot`'s mapped buffer (no pass of that slot in flight).
int grow_host_out(dm_grid* g, int slot, int64_t need) {
  dm_grid::RbSlot& r = g->rb[slot];
  if (need <= r.h_out_cap) return DM_OK;
  int64_t cap = std::max<int64_t>(need, 2 * r.h_out_cap);
  if (r.h_out) (void)hipHostFree(r.h_out - kRbHostRecords);
  r.h_out = nullptr;
  r.h_out_cap = 0;
  // mapped + coherent: k_rank_sort writes the readback header and the first
  // records (32 bytes each) straight into it over PCIe (no D2H copy command
  // per call)
  dm_raw_record* base = nullptr;
  DM_HIP(hipHostMalloc((void**)&base, sizeof(dm_raw_record) * (size_t)(cap + kRbHostRecords),
                       hipHostMallocMapped | hipHostMallocCoherent));
  dm_raw_record* dbase = nullptr;
  const hipError_t e = hipHostGetDevicePointer((void**)&dbase, base, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(base);
    return dm_hip_check(e, "hipHostGetDevicePointer(cluster readback)");
  }
  r.h_out = base + kRbHostRecords;
  r.h_out_dev = dbase + kRbHostRecords;
  r.h_out_cap = cap;
  return DM_OK;
}

// Copy nw sorted cluster records to `out`: the first `have` are already in
// g->h_out (32-byte records that arrived with the counters: the centroids
// are added here, dm_centroid); the rest come from d_sorted.  When the device
// could not sort (too many records), sort the n raw records of d_raw ([n][4]
// int64) here and compute the centroids with the same formula.
int copy_clusters(dm_grid* g, bool sorted, int64_t n, int64_t nw, int64_t have,
                  const dm_cluster* d_sorted, const long long* d_raw, dm_cluster* out) {
  if (sorted) {
    have = std::min<int64_t>(have, nw);
    const double ox = g->p.origin_x, oy = g->p.origin_y, res = g->p.resolution;
    for (int64_t i = 0; i < have; ++i) {
      const dm_raw_record& q = g->h_out[i];
      dm_cluster& c = out[i];
      c.label = q.label;
      c.size = q.size;
      c.sum_x = q.sum_x;
      c.sum_y = q.sum_y;
      c.cx_m = dm_centroid(ox, q.sum_x, q.size, res);
      c.cy_m = dm_centroid(oy, q.sum_y, q.size, res);
    }
    if (nw > have)
      DM_HIP(hipMemcpy(out + have, d_sorted + have, sizeof(dm_cluster) * (size_t)(nw - have),
                       hipMemcpyDeviceToHost));
    return DM_OK;
  }
  std::vector<HostCluster> hc((size_t)n);
  if (n > 0) DM_HIP(hipMemcpy(hc.data(), d_raw, sizeof(HostCluster) * (size_t)n, hipMemcpyDeviceToHost));
  std::sort(hc.begin(), hc.end(), [](const HostCluster& a, const HostCluster& b) { return a.label < b.label; });
  for (int64_t i = 0; i < nw; ++i) {
    dm_cluster& c = out[i];
    c.label = hc[i].label;
    c.size = hc[i].size;
    c.sum_x = hc[i].sum_x;
    c.sum_y = hc[i].sum_y;
    c.cx_m = dm_centroid(g->p.origin_x, c.sum_x, c.size, g->p.resolution);
    c.cy_m = dm_centroid(g->p.origin_y, c.sum_y, c.size, g->p.resolution);
  }
  return DM_OK;
}

// The label-sorted device records of a collected result (slot's out_clu for
// kind 1, m_out for kind 2), n records; n < 0: not sorted on the device.
void note_goal_source(dm_grid* g, int slot, int kind, int64_t n) {
  g->goal_slot = n >= 0 ? slot : -1;
  g->goal_kind = kind;
  g->goal_n = n;
  g->goal_epoch = kind == 1 ? g->rb[slot].wepoch : g->rb[slot].mepoch;
  g->goal_gen = g->rb_gen;
}

int grow_merge(dm_grid* g, int64_t n) {
  if (n <= g->m_cap) return DM_OK;
  int rc = dev_alloc(&g->m_parent, n, "merge parents");
  if (!rc) rc = dev_alloc(&g->m_label, n, "merge labels");
  if (!rc) rc = dev_alloc(&g->m_acc, 3 * n, "merge sums");
  if (!rc) rc = dev_alloc(&g->m_clu, 4 * n, "merged clusters");
  for (int sl = 0; sl <= dm_grid::kRbSlots && !rc; ++sl)
    rc = dev_alloc(&g->rb[sl].m_out, n, "merged clusters (sorted)");
  ++g->rb_gen;
  if (!rc) rc = dm_grow_bucket_sort(g, n);
  if (rc) { g->m_cap = 0; return rc; }
  g->m_cap = n;
  return DM_OK;
}

int check_grid(const dm_grid* g) {
  if (!g) return dm_set_error(DM_ERR_INVALID_ARG, "grid handle is NULL");
  return DM_OK;
}

// The building blocks of the multi-process exchange are not calls of a
// sharded parent: it runs that exchange itself (dm_sharded.cpp).
int not_on_sharded(const dm_grid* g, const char* what) {
  if (g && g->sh)
    return dm_set_error(DM_ERR_INVALID_ARG, "%s is not available on a sharded handle (dm_create_sharded runs "
                                            "the band exchange itself)", what);
  return DM_OK;
}

int use_device(const dm_grid* g) {
  DM_HIP(hipSetDevice(g->device));
  return DM_OK;
}

int check_integrate_args(int32_t S, int32_t N, const void* poses, const void* ranges) {
  if (S < 0 || N < 0) return dm_set_error(DM_ERR_SHAPE, "S and N must be >= 0");
  if ((int64_t)S * N > (1ll << 31) - 1) return dm_set_error(DM_ERR_SHAPE, "S*N must be < 2^31");
  if (N > 65535) return dm_set_error(DM_ERR_SHAPE, "N must be <= 65535");
  if ((int64_t)S * N > 0 && (!poses || !ranges))
    return dm_set_error(DM_ERR_INVALID_ARG, "poses/ranges is NULL");
  return DM_OK;
}

// Copies both counter blocks (frontier, then the last integrate call's) and
// both shard blocks into the pinned mirrors and waits for them.
int read_counters(dm_grid* g) {
  DM_HIP(dm_join_pass_stream(g));
  DM_HIP(hipMemcpyAsync(g->h_cnt, g->cnt, sizeof(unsigned long long) * CNT_N,
                        hipMemcpyDeviceToHost, g->stream));
  DM_HIP(hipMemcpyAsync(g->h_cnt + CNT_N, g->iw[g->iw_cur].cnt, sizeof(unsigned long long) * CNT_N,
                        hipMemcpyDeviceToHost, g->stream));
  DM_HIP(hipMemcpyAsync(g->h_cnt + 2 * CNT_N, g->fe_flag + kHaltWord, sizeof(unsigned long long),
                        hipMemcpyDeviceToHost, g->stream));
  DM_HIP(dm_copy_shards(g));
  DM_HIP(hipStreamSynchronize(g->stream));
  if (g->h_cnt[2 * CNT_N])
    return dm_set_error(DM_ERR_PIPELINE, "the overlapped pipeline's front-end hand-off timed out: a map "
                        "update was skipped; dm_reset the handle");
  return DM_OK;
}

int finish_counts(dm_grid* g, uint64_t* U, uint64_t* T) {
  int rc = read_counters(g);
  if (rc) return rc;
  const unsigned long long* ic = g->h_cnt + CNT_N;
  if (ic[CNT_IOVERFLOW]) {
    // cannot happen with the bounds in grow_integrate; keep the map consistent anyway
    (void)hipMemset(g->iw[g->iw_cur].tile_count, 0, sizeof(int32_t) * (size_t)g->NT);
    return dm_set_error(DM_ERR_CAPACITY, "integrate workspace overflow (flags %llu: 1 first-touch "
                        "list, 2 pieces, 4 work lists)",
                        (unsigned long long)ic[CNT_IOVERFLOW]);
  }
  if (U) *U = dm_shard_sum(g->h_sh, SH_U);
  if (T) *T = dm_shard_sum(g->h_sh, SH_T);
  return DM_OK;
}

}  // namespace

int dm_set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

int dm_hip_check(hipError_t e, const char* what) {
  return dm_set_error(e == hipErrorOutOfMemory ? DM_ERR_OOM : DM_ERR_HIP, "%s: %s (%d)", what,
                      hipGetErrorString(e), (int)e);
}

void dm_timer_begin(dm_grid* g, const char* name, KernelTimer* t, hipStream_t s) {
  if (!g->profile) return;
  t->name = name;
  t->stream = s ? s : g->stream;
  (void)hipEventCreate(&t->start);
  (void)hipEventCreate(&t->stop);
  (void)hipEventRecord(t->start, t->stream);
}

void dm_timer_end(dm_grid* g, KernelTimer* t) {
  if (!g->profile) return;
  (void)hipEventRecord(t->stop, t->stream);
  g->pending.push_back(*t);
  if (g->pending.size() > 4096) {
    int32_t n = 0;
    (void)dm_profile_read(g, nullptr, 0, &n);
  }
}

extern "C" {

const char* dm_last_error(void) { return t_err.c_str(); }
const char* dm_version(void) { return "dm 0.1.0 (gfx950, HIP)"; }
int dm_max_passes_in_flight(void) { return dm_grid::kRbSlots; }

int dm_default_params(dm_params* p, int64_t width, int64_t height) {
  if (!p) return dm_set_error(DM_ERR_INVALID_ARG, "params is NULL");
  memset(p, 0, sizeof *p);
  p->width = width;
  p->height = height;
  p->resolution = 0.05;                      // slam_config.yaml:26
  p->origin_x = -0.5 * (double)width * p->resolution;
  p->origin_y = -0.5 * (double)height * p->resolution;
  p->range_min = 0.02f;                      // LD06 driver rodata 0xbc840
  p->range_max = 12.0f;                      // slam_config.yaml:27
  p->l_occ = 0.85f;
  p->l_free = -0.4f;
  p->l_min = -2.0f;
  p->l_max = 3.5f;
  p->occ_thresh = 0.0f;
  p->free_thresh = 0.0f;
  p->min_frontier_size = 1;
  p->band_row0 = 0;
  p->band_rows = 0;
  return DM_OK;
}

int dm_create(dm_grid** out, const dm_params* p, int device) {
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int rc = validate_params(p);
  if (rc) return rc;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0)
    return dm_set_error(DM_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= ndev)
    return dm_set_error(DM_ERR_INVALID_ARG, "device %d out of range [0, %d)", device, ndev);
  DM_HIP(hipSetDevice(device));
  dm_grid* g = new (std::nothrow) dm_grid();
  if (!g) return dm_set_error(DM_ERR_OOM, "host allocation failed");
  g->p = *p;
  if (g->p.band_rows <= 0) g->p.band_rows = p->height - p->band_row0;
  g->device = device;
  g->W = p->width;
  g->H = p->height;
  g->row0 = p->band_row0;
  g->R = g->p.band_rows;
  g->TX = ceil_div(g->W, DM_TILE);
  g->TY = ceil_div(g->R, DM_TILE);
  g->NT = g->TX * g->TY;
  g->nmax = (int32_t)ceil((double)p->range_max / p->resolution) + 2;
  const int64_t cells = g->W * g->R;
  auto fail = [&](int code) {
    dm_destroy(g);
    return code;
  };
  if ((rc = dev_alloc(&g->L, cells, "log-odds"))) return fail(rc);
  if ((rc = dev_alloc(&g->state, cells, "state"))) return fail(rc);
  for (auto& w : g->iw) {
    if ((rc = dev_alloc(&w.tile_count, g->NT, "tile counts"))) return fail(rc);
    if ((rc = dev_alloc(&w.tile_cur, g->NT, "tile bin cursors"))) return fail(rc);
    if ((rc = dev_alloc(&w.cnt, CNT_N, "integrate counters"))) return fail(rc);
    if ((rc = dev_alloc(&w.sh, kShards * kShardWords, "integrate shard counters"))) return fail(rc);
    DM_HIP(hipMemset(w.cnt, 0, sizeof(unsigned long long) * CNT_N));
    DM_HIP(hipMemset(w.sh, 0, sizeof(unsigned long long) * kShards * kShardWords));
  }
  if ((rc = dev_alloc(&g->tile_free, g->NT, "tile free counts"))) return fail(rc);
  if ((rc = dev_alloc(&g->fmask, g->NT * DM_TILE * 16, "tile free / unknown bit rows"))) return fail(rc);
  if ((rc = dev_alloc(&g->fedge, g->NT * 4, "tile unknown edge words"))) return fail(rc);
  if ((rc = dev_alloc(&g->tile_seen, g->NT, "tile seen flags"))) return fail(rc);
  // The five run-time switches (read once, here): DM_SPARSE_PIECES (0: no
  // sparse work items), DM_FMASK=on|off (fmask maintenance forced either way),
  // DM_FRONTIER_KERNEL=wave|wg (one frontier tile kernel for every pass),
  // DM_SORT_MIN (cluster count above which the row sort runs) and
  // DM_FAULT_GATE=1 (fault injection: the front-end hand-off never arrives).
  // Each selects between paths the default also runs, so tests can drive
  // every path on small maps; none changes a result.
  if (const char* sp = getenv("DM_SPARSE_PIECES")) g->sparse_pieces = std::max(0, atoi(sp));
  const char* fm = getenv("DM_FMASK");
  g->fmask_mode = fm && !strcmp(fm, "on") ? 1 : (fm && !strcmp(fm, "off") ? 2 : 0);
  const char* fk = getenv("DM_FRONTIER_KERNEL");
  g->frontier_kernel = fk && !strcmp(fk, "wave") ? 1 : (fk && !strcmp(fk, "wg") ? 2 : 0);
  if (const char* sm = getenv("DM_SORT_MIN")) g->sort_min = std::max<int64_t>(0, atoll(sm));
  g->fault_gate = dm_env_on("DM_FAULT_GATE");
  for (auto& f : g->fw) {
    e = hipEventCreateWithFlags(&f.ev_split, hipEventDisableTiming | hipEventDisableSystemFence);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
    if ((rc = dev_alloc(&f.cnt, CNT_N, "frontier counters"))) return fail(rc);
    DM_HIP(hipMemset(f.cnt, 0, sizeof(unsigned long long) * CNT_N));
    if ((rc = dev_alloc(&f.fsh, kShards * kShardWords, "frontier shard counters"))) return fail(rc);
    DM_HIP(hipMemset(f.fsh, 0, sizeof(unsigned long long) * kShards * kShardWords));
    if ((rc = dev_alloc(&f.big_tiles, g->NT, "frontier big tiles"))) return fail(rc);
    if ((rc = dev_alloc(&f.fbits, g->NT * DM_TILE, "frontier bit rows"))) return fail(rc);
    if ((rc = dev_alloc(&f.edge_slot, 2 * g->W, "edge slots"))) return fail(rc);
  }
  if ((rc = dev_alloc(&g->fl_n, 48, "frontier list lengths"))) return fail(rc);
  for (int i = 0; i < 2; ++i) {
    if ((rc = dev_alloc(&g->flist[i], g->NT, "frontier tile list"))) return fail(rc);
    if ((rc = dev_alloc(&g->flist_n[i], 16, "frontier tile list length"))) return fail(rc);
    DM_HIP(hipMemset(g->flist_n[i], 0, sizeof(unsigned long long) * 16));
  }
  g->ftiles = g->flist[0];
  g->ftiles_n = g->flist_n[0];
  DM_HIP(hipMemset(g->fl_n, 0, sizeof(unsigned long long) * 48));
  if ((rc = dev_alloc(&g->bits_flag, 16, "bit-row hand-off word"))) return fail(rc);
  DM_HIP(hipMemset(g->bits_flag, 0, sizeof(unsigned long long) * 16));
  if ((rc = dev_alloc(&g->fe_flag, 32, "front-end completion words"))) return fail(rc);
  DM_HIP(hipMemset(g->fe_flag, 0, sizeof(unsigned long long) * 32));
  if ((rc = dev_alloc(&g->border, g->NT * 256, "frontier borders"))) return fail(rc);
  // [0, 4 NT): the dense passes' pair hand-off words; [4 NT, 8 NT): the
  // sparse passes' per-edge stamps (dm_frontier.hip, EDGE tile kernels)
  if ((rc = dev_alloc(&g->rel, 8 * g->NT, "tile-edge hand-off words"))) return fail(rc);
  DM_HIP(hipMemset(g->rel, 0, sizeof(unsigned long long) * 8 * (size_t)g->NT));
  if ((rc = dev_alloc(&g->edge_label, 2 * g->W, "edge labels"))) return fail(rc);
  if ((rc = dev_alloc(&g->halo, 2 * g->W, "halo rows"))) return fail(rc);
  // slot arrays sized for the map up front (a pass that overflows them has
  // no result and must be rerun): kSlotsPerTile tile-local components per
  // tile, ~276 B each (C3: 72 MB; a 65536^2 map: 1.2 GB of its 288 GB).  A
  // C5 row band under 64 x 4096-beam fans holds 0.81 clusters per tile and
  // more than two slots per tile (test_gpu_c5_full.py).
  if ((rc = grow_slots(g, std::max<int64_t>(1 << 16, kSlotsPerTile * g->NT)))) return fail(rc);
  dm_select_fw(g, g->fparity);
  for (int sl = 0; sl <= dm_grid::kRbSlots; ++sl)
    if ((rc = grow_host_out(g, sl, 1 << 14))) return fail(rc);
  dm_select_slot(g, 0);
  e = hipHostMalloc((void**)&g->h_cnt, sizeof(unsigned long long) * (2 * CNT_N + 1), hipHostMallocDefault);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipHostMalloc(counters)"));
  e = hipHostMalloc((void**)&g->h_sh, sizeof(unsigned long long) * 2 * kShards * kShardWords,
                    hipHostMallocDefault);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipHostMalloc(shard counters)"));
  if ((rc = dev_alloc(&g->m_cnt, 4, "merge counters"))) return fail(rc);
  e = hipHostMalloc((void**)&g->h_mcnt, sizeof(unsigned long long) * 4, hipHostMallocDefault);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipHostMalloc(merge counters)"));
  e = hipHostMalloc((void**)&g->h_hint, sizeof(unsigned long long) * 16, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipHostMalloc(work hint)"));
  memset(g->h_hint, 0, sizeof(unsigned long long) * 16);
  e = hipHostGetDevicePointer((void**)&g->d_hint, g->h_hint, 0);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipHostGetDevicePointer(work hint)"));
  e = hipDeviceGetAttribute(&g->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipDeviceGetAttribute(multiprocessor count)"));
  // Stream priorities: the map chain (accumulation, frontier bit rows) and
  // the pass's labelling streams high, the integrate front-end low,
  // so a front-end enqueued early fills what the map chain leaves idle instead
  // of competing with the accumulation for its CUs (round-2/3 A/B of every
  // combination and of CU-masked streams: DESIGN.md §3.3).
  // (DM_PRIO_GRID / _FE / _PASS: 1 high, 0 low -- A/B builds only)
#ifndef DM_PRIO_GRID
#define DM_PRIO_GRID 1
#endif
#ifndef DM_PRIO_FE
#define DM_PRIO_FE 0
#endif
#ifndef DM_PRIO_PASS
#define DM_PRIO_PASS 1
#endif

  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  e = hipStreamCreateWithPriority(&g->stream, hipStreamNonBlocking, DM_PRIO_GRID ? prio_hi : prio_lo);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipStreamCreate"));
  g->own_stream = true;
  for (int i = 0; i < dm_grid::kFeStreams; ++i) {
    e = hipStreamCreateWithPriority(&g->fe_streams[i], hipStreamNonBlocking, DM_PRIO_FE ? prio_hi : prio_lo);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipStreamCreate(front-end)"));
  }
  e = hipStreamCreateWithPriority(&g->pass_stream, hipStreamNonBlocking, DM_PRIO_PASS ? prio_hi : prio_lo);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipStreamCreate(pass)"));
  e = hipStreamCreateWithPriority(&g->big_stream, hipStreamNonBlocking, DM_PRIO_PASS ? prio_hi : prio_lo);
  if (e != hipSuccess) return fail(dm_hip_check(e, "hipStreamCreate(big)"));
  // ev_fe / ev_free only order the two streams on the device: no system-
  // scope fence (no host-visible cache writeback at every step).  The host
  // waits on a readback slot's event and then reads mapped host memory:
  // default fences.
  for (hipEvent_t* ev : {&g->ev_fe, &g->ev_bits[0], &g->ev_bits[1], &g->iw[0].ev_free, &g->iw[1].ev_free,
                         &g->ev_bigfork, &g->ev_big, &g->flist_ev[0], &g->flist_ev[1], &g->ev_fe_end[0],
                         &g->ev_fe_end[1]}) {
    e = hipEventCreateWithFlags(ev, hipEventDisableTiming | hipEventDisableSystemFence);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
  }
  for (auto& r : g->rb) {
    e = hipEventCreateWithFlags(&r.ev, hipEventDisableTiming);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
  }
  for (hipEvent_t& ev : g->ev_pose) {  // host waits on these before reusing a staging buffer
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return fail(dm_hip_check(e, "hipEventCreate"));
  }

  if ((rc = dm_reset(g))) return fail(rc);
  *out = g;
  return DM_OK;
}

int dm_destroy(dm_grid* g) {
  if (g && g->sh) return dm_sh_destroy(g);
  if (!g) return DM_OK;
  (void)hipSetDevice(g->device);
  (void)dm_sync_all(g);
  for (auto& t : g->pending) { (void)hipEventDestroy(t.start); (void)hipEventDestroy(t.stop); }
  for (hipEvent_t ev : {g->ev_fe, g->ev_bits[0], g->ev_bits[1], g->iw[0].ev_free, g->iw[1].ev_free,
                        g->ev_bigfork, g->ev_big, g->flist_ev[0], g->flist_ev[1], g->ev_fe_end[0],
                        g->ev_fe_end[1]})
    if (ev) (void)hipEventDestroy(ev);
  for (auto& r : g->rb) {
    if (r.ev) (void)hipEventDestroy(r.ev);
    if (r.out_clu) (void)hipFree(r.out_clu - kRbRecords);
    if (r.h_out) (void)hipHostFree(r.h_out - kRbHostRecords);
    dev_free(r.m_out);
  }
  for (hipStream_t& fs : g->fe_streams)
    if (fs) (void)hipStreamDestroy(fs);
  if (g->pass_stream) (void)hipStreamDestroy(g->pass_stream);
  if (g->big_stream) (void)hipStreamDestroy(g->big_stream);
  for (auto& f : g->fw) {
    if (f.ev_split) (void)hipEventDestroy(f.ev_split);
    dev_free(f.cnt); dev_free(f.fsh); dev_free(f.big_tiles); dev_free(f.fbits);
    dev_free(f.edge_slot); dev_free(f.slot_parent);
  }
  dev_free(g->fl_n); dev_free(g->bits_flag);
  for (int i = 0; i < 2; ++i) { dev_free(g->flist[i]); dev_free(g->flist_n[i]); }
  for (int b = 0; b < 2; ++b) { dev_free(g->goal_k[b]); dev_free(g->goal_i[b]); }
  dev_free(g->goal_io); dev_free(g->goal_idx);
  for (auto& w : g->iw) {
    dev_free(w.pieces); dev_free(w.hitems); dev_free(w.litems); dev_free(w.heavy_list); dev_free(w.slabs);
    dev_free(w.heavy_done); dev_free(w.tile_count); dev_free(w.tile_cur); dev_free(w.cnt); dev_free(w.sh);
    dev_free(w.pose4); dev_free(w.ranges);
    dev_free(w.beams); dev_free(w.blk_hist); dev_free(w.blk_n); dev_free(w.act_raw);
  }
  dev_free(g->L); dev_free(g->state); dev_free(g->fmask); dev_free(g->fedge); dev_free(g->tile_seen);
  dev_free(g->tile_free);
  dev_free(g->trig);
  dev_free(g->bs_key); dev_free(g->bs_key2); dev_free(g->bs_idx); dev_free(g->bs_idx2);
  dev_free(g->rs_cnt); dev_free(g->rs_off); dev_free(g->rs_status);
  dev_free(g->border); dev_free(g->rel); dev_free(g->slot_label); dev_free(g->slot_root);
  dev_free(g->slot_own); dev_free(g->slot_acc); dev_free(g->clusters); dev_free(g->cell_slot);
  dev_free(g->edge_label); dev_free(g->mask); dev_free(g->labels);
  dev_free(g->halo); dev_free(g->fe_flag);
  dev_free(g->slot_k); dev_free(g->rank_of); dev_free(g->m_parent); dev_free(g->m_label);
  dev_free(g->m_acc); dev_free(g->m_clu); dev_free(g->m_cnt);
  if (g->h_mcnt) (void)hipHostFree(g->h_mcnt);
  if (g->h_hint) (void)hipHostFree(g->h_hint);
  if (g->h_cnt) (void)hipHostFree(g->h_cnt);
  if (g->h_sh) (void)hipHostFree(g->h_sh);
  for (int i = 0; i < dm_grid::kPoseRing; ++i) {
    if (g->h_pose4[i]) (void)hipHostFree(g->h_pose4[i]);
    if (g->ev_pose[i]) (void)hipEventDestroy(g->ev_pose[i]);
  }
  if (g->stream && g->own_stream) (void)hipStreamDestroy(g->stream);
  delete g;
  return DM_OK;
}

int dm_reset(dm_grid* g) {
  if (g && g->sh) return dm_sh_reset(g);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  const int64_t cells = g->W * g->R;
  DM_HIP(hipMemsetAsync(g->L, 0, sizeof(float) * (size_t)cells, g->stream));
  DM_HIP(hipMemsetAsync(g->state, 0xFF, (size_t)cells, g->stream));
  DM_HIP(dm_sync_all(g));
  for (auto& w : g->iw) DM_HIP(hipMemsetAsync(w.tile_count, 0, sizeof(int32_t) * (size_t)g->NT, g->stream));
  DM_HIP(hipMemsetAsync(g->tile_free, 0, sizeof(int32_t) * (size_t)g->NT, g->stream));
  if ((rc = dm_launch_recount(g))) return rc;  // fmask: every in-grid cell unknown
  for (auto& f : g->fw) DM_HIP(hipMemsetAsync(f.cnt, 0, sizeof(unsigned long long) * CNT_N, g->stream));
  DM_HIP(hipMemsetAsync(g->fe_flag + kHaltWord, 0, sizeof(unsigned long long), g->stream));  // sticky error
  DM_HIP(hipStreamSynchronize(g->stream));
  return DM_OK;
}

int dm_get_params(const dm_grid* g, dm_params* out) {
  int rc = check_grid(g);
  if (rc) return rc;
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  *out = g->p;
  return DM_OK;
}

}  // extern "C"

namespace {

// Host inputs -> device: poses to (x, y, cos yaw, sin yaw) with the C
// library (as the oracle) into the next pinned staging buffer of the ring,
// then the ranges H2D copy on the front-end stream (k_beam_prep reads the
// poses from the mapped staging buffer), then the integrate launch.
// Nothing here waits for the device except a staging buffer whose copy (two
// calls ago) has not finished yet.
int enqueue_host_integrate(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges,
                           float angle_min, float angle_increment) {
  int rc = 0;
  if ((rc = check_integrate_args(S, N, poses, ranges))) return rc;
  if ((rc = grow_integrate(g, S, N))) return rc;
  if ((rc = ensure_trig(g, N, angle_min, angle_increment))) return rc;
  const int64_t nb = (int64_t)S * N;
  hipStream_t fs = g->overlap ? dm_fe_stream_of(g, dm_next_set(g)) : g->stream;
  // the ranges copy goes to the device buffer of the workspace set this call
  // will use (dm_launch_integrate alternates them); with overlap the front-end
  // stream first waits until that set is free (its last accumulation, which
  // may read its inputs, is done).  The copy stays at the head of this call's
  // front-end: on a stream of its own (waiting for the set, the front-end
  // waiting for it) host-input steps took 1.6x as long.
  dm_grid::IntWs& w = g->iw[dm_next_set(g)];
  if (g->overlap) {
    DM_HIP(dm_mark_ws_free(g));
    DM_HIP(hipStreamWaitEvent(fs, w.free_wait ? w.free_wait : w.ev_free, 0));
  }
  if ((int64_t)S * 4 > w.pose_cap || nb > w.ranges_cap || (int64_t)S * 4 > g->h_pose_cap) {
    // the device buffers may still feed an in-flight call
    DM_HIP(dm_sync_all(g));
  }
  if ((int64_t)S * 4 > w.pose_cap) {
    if ((rc = dev_alloc(&w.pose4, (int64_t)S * 4, "poses"))) return rc;
    w.pose_cap = (int64_t)S * 4;
  }
  if (nb > w.ranges_cap) {
    if ((rc = dev_alloc(&w.ranges, nb, "ranges"))) return rc;
    w.ranges_cap = nb;
  }
  if ((int64_t)S * 4 > g->h_pose_cap) {
    for (int i = 0; i < dm_grid::kPoseRing; ++i) {
      if (g->h_pose4[i]) (void)hipHostFree(g->h_pose4[i]);
      g->h_pose4[i] = nullptr;
    }
    g->h_pose_cap = 0;
    for (int i = 0; i < dm_grid::kPoseRing; ++i) {
      // Coherent: k_beam_prep reads the slot through its device address and
      // the slot is rewritten every kPoseRing calls at the same address, so
      // the GPU must not keep it in L2 (non-coherent host memory may be
      // cached there; the other mapped buffers the device reads are
      // Mapped | Coherent too)
#ifndef DM_POSE_COHERENT
#define DM_POSE_COHERENT 1  // 0: Mapped only (the round-5 allocation; A/B builds)
#endif
      DM_HIP(hipHostMalloc((void**)&g->h_pose4[i], sizeof(double) * 4 * (size_t)std::max(S, 1),
                           hipHostMallocMapped | (DM_POSE_COHERENT ? hipHostMallocCoherent : 0u)));
      DM_HIP(hipHostGetDevicePointer((void**)&g->h_pose4_dev[i], g->h_pose4[i], 0));
    }
    g->h_pose_cap = (int64_t)std::max(S, 1) * 4;
  }
  const int slot = g->pose_head;
  g->pose_head = (g->pose_head + 1) % dm_grid::kPoseRing;
  DM_HIP(hipEventSynchronize(g->ev_pose[slot]));  // its last reader (two calls ago) is done
  double* hp = g->h_pose4[slot];
  for (int32_t s = 0; s < S; ++s) {
    const double x = poses[3 * s], y = poses[3 * s + 1], yaw = poses[3 * s + 2];
    hp[4 * s + 0] = x;
    hp[4 * s + 1] = y;
    hp[4 * s + 2] = cos(yaw);  // C library, as the oracle
    hp[4 * s + 3] = sin(yaw);
  }
  // into the set's buffers: their last readers (the front-end of the set's
  // previous call, on fs) are done (above: that front-end precedes the set's
  // last accumulation).  DM_HOST_POSE: no pose copy, k_beam_prep reads the
  // mapped staging buffer (a 2 KB copy is a blit kernel, which waits for the
  // accumulation's CUs and adds a compute -> copy-engine hand-off)
  const double* d_pose = w.pose4;
  if (DM_HOST_POSE) {
    d_pose = g->h_pose4_dev[slot];
  } else if (S > 0) {
    DM_HIP(hipMemcpyAsync(w.pose4, hp, sizeof(double) * 4 * (size_t)S, hipMemcpyHostToDevice, fs));
  }
  if (nb > 0)
    DM_HIP(hipMemcpyAsync(w.ranges, ranges, sizeof(float) * (size_t)nb, hipMemcpyHostToDevice, fs));
  if ((rc = dm_launch_integrate(g, S, d_pose, N, w.ranges, g->trig))) return rc;
  // after the front-end (which read the staging buffer) and so after the
  // ranges copy: two calls later this event proves the caller's ranges
  // buffer has been read too (dm.h: reusable after the second call that follows)
  DM_HIP(hipEventRecord(g->ev_pose[slot], fs));
  g->last_S = S;
  g->last_N = N;
  g->frontier_valid = false;
  ++g->integrate_seq;
  return DM_OK;
}

}  // namespace

extern "C" {

int dm_integrate(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges,
                 float angle_min, float angle_increment, uint64_t* out_updates,
                 uint64_t* out_touched) {
  if (g && g->sh) return dm_sh_integrate(g, S, poses, N, ranges, angle_min, angle_increment, out_updates, out_touched);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if ((rc = enqueue_host_integrate(g, S, poses, N, ranges, angle_min, angle_increment))) return rc;
  return finish_counts(g, out_updates, out_touched);
}

int dm_integrate_async(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges,
                       float angle_min, float angle_increment) {
  if (g && g->sh) return dm_sh_integrate_async(g, S, poses, N, ranges, angle_min, angle_increment);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  return enqueue_host_integrate(g, S, poses, N, ranges, angle_min, angle_increment);
}

int dm_integrate_device(dm_grid* g, int32_t S, const double* d_pose4, int32_t N,
                        const float* d_ranges, float angle_min, float angle_increment) {
  if (g && g->sh) return dm_sh_integrate_device(g, S, d_pose4, N, d_ranges, angle_min, angle_increment);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if ((rc = check_integrate_args(S, N, d_pose4, d_ranges))) return rc;
  if ((rc = grow_integrate(g, S, N))) return rc;
  if ((rc = ensure_trig(g, N, angle_min, angle_increment))) return rc;
  if ((rc = dm_launch_integrate(g, S, d_pose4, N, d_ranges, g->trig))) return rc;
  g->last_S = S;
  g->last_N = N;
  g->frontier_valid = false;
  ++g->integrate_seq;
  return DM_OK;
}

int dm_last_counts(dm_grid* g, uint64_t* updates, uint64_t* touched) {
  if (g && g->sh) return dm_sh_last_counts(g, updates, touched);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  return finish_counts(g, updates, touched);
}

int dm_last_stats(dm_grid* g, uint64_t* out, int32_t cap, int32_t* n_out) {
  if (g && g->sh) return dm_sh_last_stats(g, out, cap, n_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (cap > 0 && !out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  if ((rc = read_counters(g))) return rc;
  const unsigned long long* fs = g->h_sh + kShards * kShardWords;
  const unsigned long long* ic = g->h_cnt + CNT_N;  // the last integrate call's counters
  const uint64_t items = ic[CNT_ITEMS] + ic[CNT_LITEMS] + ic[CNT_SITEMS];  // heavy + light + sparse items
  const uint64_t pieces = ic[CNT_SEGS];
  const uint64_t v[kNStats] = {dm_shard_sum(g->h_sh, SH_U),  dm_shard_sum(g->h_sh, SH_T),
                               dm_shard_sum(g->h_sh, SH_TH), pieces,
                               ic[CNT_ACTIVE],               items,
                               ic[CNT_HEAVY],                g->h_cnt[CNT_FL0],
                               dm_shard_sum(fs, SH_SLOT),    g->h_cnt[CNT_CLUSTERS],
                               ic[CNT_SITEMS]};
  for (int32_t i = 0; i < cap && i < kNStats; ++i) out[i] = v[i];
  if (n_out) *n_out = kNStats;
  return DM_OK;
}

int dm_get_state(dm_grid* g, int8_t* out) {
  if (g && g->sh) return (out ? dm_sh_get_state(g, out) : dm_set_error(DM_ERR_INVALID_ARG, "out is NULL"));
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  DM_HIP(hipMemcpyAsync(out, g->state, (size_t)(g->W * g->R), hipMemcpyDeviceToHost, g->stream));
  DM_HIP(hipStreamSynchronize(g->stream));
  return DM_OK;
}

int dm_get_logodds(dm_grid* g, float* out) {
  if (g && g->sh) return (out ? dm_sh_get_logodds(g, out) : dm_set_error(DM_ERR_INVALID_ARG, "out is NULL"));
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  DM_HIP(hipMemcpyAsync(out, g->L, sizeof(float) * (size_t)(g->W * g->R), hipMemcpyDeviceToHost,
                        g->stream));
  DM_HIP(hipStreamSynchronize(g->stream));
  return DM_OK;
}

int dm_set_logodds(dm_grid* g, const float* in) {
  if (g && g->sh) return (in ? dm_sh_set_logodds(g, in) : dm_set_error(DM_ERR_INVALID_ARG, "in is NULL"));
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!in) return dm_set_error(DM_ERR_INVALID_ARG, "in is NULL");
  DM_HIP(hipStreamSynchronize(g->stream));
  DM_HIP(hipMemcpy(g->L, in, sizeof(float) * (size_t)(g->W * g->R), hipMemcpyHostToDevice));
  if ((rc = dm_launch_state_from_logodds(g))) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  g->frontier_valid = false;
  ++g->integrate_seq;
  return DM_OK;
}

int dm_set_state(dm_grid* g, const int8_t* in) {
  if (g && g->sh) return (in ? dm_sh_set_state(g, in) : dm_set_error(DM_ERR_INVALID_ARG, "in is NULL"));
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!in) return dm_set_error(DM_ERR_INVALID_ARG, "in is NULL");
  const int64_t cells = g->W * g->R;
  int8_t* d = nullptr;
  if ((rc = dev_alloc(&d, cells, "state staging"))) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  hipError_t e = hipMemcpy(d, in, (size_t)cells, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    rc = dm_launch_set_state(g, d);
    if (!rc) e = hipStreamSynchronize(g->stream);
  }
  (void)hipFree(d);
  if (e != hipSuccess) return dm_hip_check(e, "dm_set_state");
  g->frontier_valid = false;
  ++g->integrate_seq;
  return rc;
}

int dm_frontiers(dm_grid* g, uint8_t* mask, int64_t* labels, dm_cluster* out, int64_t cap,
                 int64_t* n_out) {
  if (g && g->sh) return dm_sh_frontiers(g, mask, labels, out, cap, n_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (cap < 0 || (cap > 0 && !out)) return dm_set_error(DM_ERR_INVALID_ARG, "bad cluster buffer");
  const int64_t cells = g->W * g->R;
  if (mask && !g->mask && (rc = dev_alloc(&g->mask, cells, "dense mask"))) return rc;
  if (labels && !g->cell_slot) {
    if ((rc = dev_alloc(&g->cell_slot, cells, "dense cell slots"))) return rc;
    if ((rc = dev_alloc(&g->labels, cells, "dense labels"))) return rc;
  }
  // its own readback slot: asynchronous passes may be in flight (this pass
  // runs after them in stream order and sees the map as it is now)
  const int slot = dm_grid::kRbSync;
  dm_select_slot(g, slot);
  int64_t n = 0, copied = 0;
  for (int attempt = 0; attempt < 8; ++attempt) {
    rc = dm_launch_frontiers(g, mask != nullptr, labels != nullptr, &n, &copied);
    if (rc != DM_ERR_CAPACITY) break;
    if ((rc = grow_slots(g, n + n / 2 + 1024))) return rc;
    rc = DM_ERR_CAPACITY;
  }
  if (rc) return rc == DM_ERR_CAPACITY ? dm_set_error(rc, "frontier slot arrays kept overflowing") : rc;
  g->frontier_valid = true;
  const int64_t nw = std::min<int64_t>(n, cap);
  note_goal_source(g, slot, 1, g->h_cnt[CNT_SORTED] != 0 ? n : -1);
  if ((rc = copy_clusters(g, g->h_cnt[CNT_SORTED] != 0, n, nw, copied, g->out_clu, g->clusters, out)))
    return rc;
  if ((rc = grow_host_out(g, slot, n + n / 4 + 64))) return rc;
  if (mask) DM_HIP(hipMemcpy(mask, g->mask, (size_t)cells, hipMemcpyDeviceToHost));
  if (labels) DM_HIP(hipMemcpy(labels, g->labels, sizeof(int64_t) * (size_t)cells, hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  if (n > cap) return dm_set_error(DM_ERR_CAPACITY, "%lld clusters, capacity %lld", (long long)n,
                                   (long long)cap);
  return DM_OK;
}

int dm_export_bytes(const dm_grid* g, int64_t rec_cap, int64_t* bytes) {
  if (int rc0 = not_on_sharded(g, "dm_export_bytes")) return rc0;
  int rc = check_grid(g);
  if (rc) return rc;
  if (!bytes || rec_cap < 0) return dm_set_error(DM_ERR_INVALID_ARG, "bytes is NULL or rec_cap < 0");
  *bytes = dm_export_nbytes(g->W, rec_cap);
  return DM_OK;
}

int dm_frontiers_export_device(dm_grid* g, void* d_export, int64_t rec_cap) {
  if (int rc0 = not_on_sharded(g, "dm_frontiers_export_device")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!d_export || rec_cap < 0) return dm_set_error(DM_ERR_INVALID_ARG, "d_export is NULL or rec_cap < 0");
  if (g->p.min_frontier_size > 1)
    return dm_set_error(DM_ERR_INVALID_ARG,
                        "export needs a band handle with min_frontier_size <= 1 (the size filter "
                        "applies to merged clusters)");
  // the band's sorted records go to a readback slot no pending pass holds
  // (the synchronous slot when the ring is full: a merge of a sharded parent
  // can have every ring slot pending on its band 0)
  dm_select_slot(g, g->rb_count < dm_grid::kRbSlots ? (g->rb_head + g->rb_count) % dm_grid::kRbSlots
                                                    : dm_grid::kRbSync);
  // with overlap, split as dm_frontiers_begin: the labelling, sort and
  // export on the pass stream, beside the next batch's map update
  hipStream_t es = g->stream;
  if ((rc = dm_enqueue_frontiers(g, false, false, g->overlap, &es))) return rc;
  if ((rc = dm_launch_export(g, es, d_export, rec_cap))) return rc;
  if (es != g->stream) {
    // the parity set is free again, and the grid stream may use the shared
    // pass arrays, once the pass stream is past this export
    dm_grid::FrWs& f = g->fw[g->fparity];
    DM_HIP(hipEventRecord(f.ev_split, es));
    f.busy = f.ev_split;
    f.busy_pending = true;
    f.busy_pass = g->fr_pass;
    g->p_tail = f.ev_split;
    g->p_pending = true;
    g->p_tail_pass = g->fr_pass;
  } else {
    DM_HIP(dm_mark_ws_free(g));
  }
  g->frontier_valid = true;
  return DM_OK;
}

int dm_exchange_stream(dm_grid* g, void** stream) {
  if (int rc0 = not_on_sharded(g, "dm_exchange_stream")) return rc0;
  int rc = check_grid(g);
  if (rc) return rc;
  if (!stream) return dm_set_error(DM_ERR_INVALID_ARG, "stream is NULL");
  *stream = (void*)dm_exchange_stream_of(g);
  return DM_OK;
}

namespace {

// Claim the next readback slot for an asynchronous pass (selected as the
// current slot), or fail if every slot holds a pass not collected yet.
int claim_slot(dm_grid* g, int* slot) {
  if (g->rb_count == dm_grid::kRbSlots)
    return dm_set_error(DM_ERR_INVALID_ARG, "%d passes in flight: end the oldest first", dm_grid::kRbSlots);
  *slot = (g->rb_head + g->rb_count) % dm_grid::kRbSlots;
  dm_select_slot(g, *slot);
  return DM_OK;
}

// The oldest pending pass, if it is of `kind`: wait for it, select its slot.
int wait_oldest(dm_grid* g, int kind, const char* what) {
  if (!g->rb_count || g->rb[g->rb_head].kind != kind)
    return dm_set_error(DM_ERR_INVALID_ARG, "the oldest pass in flight is not a %s pass", what);
  DM_HIP(dm_event_wait(g->rb[g->rb_head].ev));
  if (kind == 1) {  // passes end in order: this one and every earlier one are done
    const uint64_t pass = g->rb[g->rb_head].pass;
    for (auto& f : g->fw)
      if (f.busy_pending && f.busy_pass <= pass) f.busy_pending = false;
    if (g->p_pending && g->p_tail_pass <= pass) g->p_pending = false;
  }
  dm_select_slot(g, g->rb_head);
  return DM_OK;
}

void retire_oldest(dm_grid* g) {
  g->rb[g->rb_head].kind = 0;
  g->rb_head = (g->rb_head + 1) % dm_grid::kRbSlots;
  --g->rb_count;
}

// A completed merge in readback slot `slot` (selected): header -> result.
int merge_readback(dm_grid* g, int slot, int64_t n, dm_cluster* out, int64_t cap, int64_t* n_out) {
  dm_select_slot(g, slot);
  // the merge's sort kernel wrote the merge counters and the first h_out_cap
  // records into the slot's mapped readback buffer: no copy command
  const int64_t hint = std::min<int64_t>(g->h_out_cap, n);
  memcpy(g->h_mcnt, dm_rb_header(g->h_out), sizeof(unsigned long long) * 4);
  // the band exports (dm_frontiers_export_device) never pass through
  // dm_frontiers_readback: the largest band's K hints the next export's sort
  g->sort_hint = (int64_t)g->h_mcnt[3];
  if (g->h_mcnt[1]) {
    if (n_out) *n_out = (int64_t)g->h_mcnt[3];
    return dm_set_error(DM_ERR_INCOMPLETE,
                        "a band export is incomplete (flags %llu: 1 slot overflow, 2 K > rec_cap, "
                        "4 unsorted, 8 width mismatch, 16 bands not contiguous, 32 union-find bound); largest band K %llu",
                        (unsigned long long)g->h_mcnt[1], (unsigned long long)g->h_mcnt[3]);
  }
  const int64_t K = (int64_t)g->h_mcnt[0];
  g->msort_hint = K;
  if (n_out) *n_out = K;
  if (K > cap)
    return dm_set_error(DM_ERR_CAPACITY, "%lld clusters, capacity %lld", (long long)K, (long long)cap);
  if (K > hint && slot != dm_grid::kRbSync &&
      (g->rb[slot].gen != g->rb_gen || (!g->h_mcnt[2] && g->rb[slot].pass != g->m_pass)))
    return dm_set_error(DM_ERR_INCOMPLETE, "merge result lost to a workspace reallocation or a later "
                                           "unsorted merge: rerun");
  note_goal_source(g, slot, 2, g->h_mcnt[2] != 0 ? K : -1);
  int rc = copy_clusters(g, g->h_mcnt[2] != 0, K, K, hint, g->m_out, g->m_clu, out);
  if (rc) return rc;
  return grow_host_out(g, slot, K + K / 4 + 64);
}

}  // namespace

int dm_merge_bands_begin(dm_grid* g, const void* d_gathered, int32_t nranks, int64_t rec_cap,
                         int64_t min_size) {
  if (int rc0 = not_on_sharded(g, "dm_merge_bands_begin")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!d_gathered || nranks < 1 || rec_cap < 1)
    return dm_set_error(DM_ERR_INVALID_ARG, "need d_gathered, nranks >= 1, rec_cap >= 1");
  const int64_t n = (int64_t)nranks * rec_cap;
  if (n >= (1ll << 31)) return dm_set_error(DM_ERR_SHAPE, "nranks * rec_cap must be < 2^31");
  int slot = 0;
  if ((rc = grow_merge(g, n)) || (rc = claim_slot(g, &slot))) return rc;
  // on the exchange stream: the grid stream's with overlap off (after the
  // pass stream: the sort workspace is shared with the frontier passes), the
  // pass stream's with overlap on (the exports' own order)
  hipStream_t ms = dm_exchange_stream_of(g);
  if (ms == g->stream) DM_HIP(dm_join_pass_stream(g));
  if ((rc = dm_launch_merge(g, ms, d_gathered, nranks, rec_cap, min_size))) return rc;
  dm_grid::RbSlot& r = g->rb[slot];
  DM_HIP(hipEventRecord(r.ev, ms));
  if (ms != g->stream) {
    g->p_tail = r.ev;
    g->p_pending = true;
    // no band pass's completion implies this merge's: only an explicit join
    // (dm_join_pass_stream) clears it, never wait_oldest of a kind-1 pass
    // (the merge reads the shared sort workspace a later pass would reuse)
    g->p_tail_pass = UINT64_MAX;
  }
  r.kind = 2;
  r.merge_n = n;
  r.gen = g->rb_gen;
  r.pass = g->m_pass;
  ++g->rb_count;
  return DM_OK;
}

int dm_merge_bands_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out) {
  if (int rc0 = not_on_sharded(g, "dm_merge_bands_end")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (cap < 0 || (cap > 0 && !out)) return dm_set_error(DM_ERR_INVALID_ARG, "bad cluster buffer");
  if ((rc = wait_oldest(g, 2, "dm_merge_bands_begin"))) return rc;
  const int slot = g->rb_head;
  rc = merge_readback(g, slot, g->rb[slot].merge_n, out, cap, n_out);
  if (rc != DM_ERR_CAPACITY) retire_oldest(g);  // on a capacity error the result stays pending
  return rc;
}

int dm_merge_bands(dm_grid* g, const void* d_gathered, int32_t nranks, int64_t rec_cap, int64_t min_size,
                   dm_cluster* out, int64_t cap, int64_t* n_out) {
  if (int rc0 = not_on_sharded(g, "dm_merge_bands")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!d_gathered || nranks < 1 || rec_cap < 1)
    return dm_set_error(DM_ERR_INVALID_ARG, "need d_gathered, nranks >= 1, rec_cap >= 1");
  if (cap < 0 || (cap > 0 && !out)) return dm_set_error(DM_ERR_INVALID_ARG, "bad cluster buffer");
  const int64_t n = (int64_t)nranks * rec_cap;
  if (n >= (1ll << 31)) return dm_set_error(DM_ERR_SHAPE, "nranks * rec_cap must be < 2^31");
  if ((rc = grow_merge(g, n))) return rc;
  dm_select_slot(g, dm_grid::kRbSync);  // its own slot: asynchronous passes may be in flight
  hipStream_t ms = dm_exchange_stream_of(g);  // as dm_merge_bands_begin
  if (ms == g->stream) DM_HIP(dm_join_pass_stream(g));
  if ((rc = dm_launch_merge(g, ms, d_gathered, nranks, rec_cap, min_size))) return rc;
  DM_HIP(hipStreamSynchronize(ms));
  return merge_readback(g, dm_grid::kRbSync, n, out, cap, n_out);
}

int dm_merge_max_band_k(const dm_grid* g, int64_t* max_k) {
  if (int rc0 = not_on_sharded(g, "dm_merge_max_band_k")) return rc0;
  int rc = check_grid(g);
  if (rc) return rc;
  if (!max_k) return dm_set_error(DM_ERR_INVALID_ARG, "max_k is NULL");
  *max_k = (int64_t)g->h_mcnt[3];  // the header merge_readback copied (M_MAXK)
  return DM_OK;
}

int dm_frontiers_begin(dm_grid* g) {
  if (g && g->sh) return dm_sh_frontiers_begin(g);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  int slot = 0;
  if ((rc = claim_slot(g, &slot))) return rc;
  // with overlap, the pass's labelling half runs on the pass stream, beside
  // the next batch's map update (dm_enqueue_frontiers)
  hipStream_t es = g->stream;
  if ((rc = dm_enqueue_frontiers(g, false, false, g->overlap, &es))) return rc;
  dm_grid::RbSlot& r = g->rb[slot];
  DM_HIP(hipEventRecord(r.ev, es));
  dm_grid::FrWs& f = g->fw[g->fparity];
  f.busy = r.ev;  // the set is free again once this pass ended
  f.busy_pending = true;
  f.busy_pass = g->fr_pass;
  if (es != g->stream) {
    g->p_tail = r.ev;
    g->p_pending = true;
    g->p_tail_pass = g->fr_pass;
  }
  // the integrate workspaces' accumulations are ahead of this event: it
  // frees them (a marker right behind the write-heavy map update would cost
  // the stream several microseconds)
  DM_HIP(dm_mark_ws_free(g, r.ev));
  r.kind = 1;
  r.seq = g->integrate_seq;
  r.gen = g->rb_gen;
  r.pass = g->fr_pass;
  ++g->rb_count;
  return DM_OK;
}

int dm_frontiers_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out) {
  if (g && g->sh) return dm_sh_frontiers_end(g, out, cap, n_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (cap < 0 || (cap > 0 && !out)) return dm_set_error(DM_ERR_INVALID_ARG, "bad cluster buffer");
  if ((rc = wait_oldest(g, 1, "dm_frontiers_begin"))) return rc;
  const int slot = g->rb_head;
  const dm_grid::RbSlot& r = g->rb[slot];
  int64_t n = 0, copied = 0;
  rc = dm_frontiers_readback(g, &n, &copied);
  if (rc == DM_ERR_CAPACITY) {
    retire_oldest(g);
    if ((rc = grow_slots(g, n + n / 2 + 1024))) return rc;
    if (n_out) *n_out = 0;
    return dm_set_error(DM_ERR_INCOMPLETE, "frontier slot arrays overflowed (grown now): this pass "
                                           "has no result, run dm_frontiers");
  }
  if (rc) {
    retire_oldest(g);
    return rc;
  }
  if (n_out) *n_out = n;
  if (n > cap)  // the result stays pending: call again with cap >= n
    return dm_set_error(DM_ERR_CAPACITY, "%lld clusters, capacity %lld", (long long)n, (long long)cap);
  // the device records were reallocated meanwhile, or the result is unsorted
  // (raw records, shared by every pass) and a later pass overwrote them
  const bool sorted = g->h_cnt[CNT_SORTED] != 0;
  if ((n > copied && r.gen != g->rb_gen) || (!sorted && r.pass != g->fr_pass)) {
    retire_oldest(g);
    return dm_set_error(DM_ERR_INCOMPLETE, "frontier result lost to a workspace reallocation or a "
                                           "later pass: rerun");
  }
  // the slot data (dm_get_edge_labels) describes the map only if this was
  // the last pass and no map change came in between
  g->frontier_valid = g->rb_count == 1 && r.seq == g->integrate_seq;
  note_goal_source(g, slot, 1, sorted ? n : -1);
  rc = copy_clusters(g, sorted, n, n, copied, g->out_clu, g->clusters, out);
  retire_oldest(g);
  if (rc) return rc;
  return grow_host_out(g, slot, n + n / 4 + 64);
}

int dm_frontiers_poll(dm_grid* g, int32_t* ready) {
  if (g && g->sh) return dm_sh_frontiers_poll(g, ready);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!ready) return dm_set_error(DM_ERR_INVALID_ARG, "ready is NULL");
  *ready = 0;
  if (!g->rb_count) return dm_set_error(DM_ERR_INVALID_ARG, "no asynchronous pass in flight");
  const hipError_t e = hipEventQuery(g->rb[g->rb_head].ev);
  if (e == hipSuccess) {
    *ready = 1;
    return DM_OK;
  }
  if (e == hipErrorNotReady) return DM_OK;
  DM_HIP(e);
  return DM_OK;
}

int dm_assign_goals(dm_grid* g, const double* robots_xy, int32_t n_robots, int64_t min_size,
                    double distance_weight, double min_distance, int64_t* out_index, double* out_xy) {
  if (g && g->sh) return dm_sh_assign_goals(g, robots_xy, n_robots, min_size, distance_weight, min_distance, out_index, out_xy);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (n_robots < 0 || n_robots > 256)
    return dm_set_error(DM_ERR_INVALID_ARG, "n_robots must be in [0, 256] (got %d)", n_robots);
  if (n_robots > 0 && (!robots_xy || !out_index || !out_xy))
    return dm_set_error(DM_ERR_INVALID_ARG, "robots_xy / out_index / out_xy is NULL");
  if (!isfinite(distance_weight) || !isfinite(min_distance))
    return dm_set_error(DM_ERR_INVALID_ARG, "distance_weight / min_distance must be finite");
  // the device ranks by the util's IEEE bits, an order that holds for util > 0
  // only: w >= 0 keeps util = size / (1 + w*dist) positive and finite
  if (distance_weight < 0.0)
    return dm_set_error(DM_ERR_INVALID_ARG, "distance_weight must be >= 0");
  const int s = g->goal_slot;
  if (s < 0 || g->goal_gen != g->rb_gen ||
      (g->goal_kind == 1 ? g->rb[s].wepoch : g->rb[s].mepoch) != g->goal_epoch)
    return dm_set_error(DM_ERR_INVALID_ARG, "no collected frontier result on the device (call dm_frontiers, "
                                            "dm_frontiers_end or dm_merge_bands first; a later pass may have "
                                            "reused its readback slot)");
  if (n_robots == 0) return DM_OK;
  const dm_cluster* recs = g->goal_kind == 1 ? g->rb[s].out_clu : g->rb[s].m_out;
  const int64_t K = g->goal_n;
  if (!g->goal_io) {
    DM_HIP(hipMalloc((void**)&g->goal_io, sizeof(double) * 4 * 256));
    DM_HIP(hipMalloc((void**)&g->goal_idx, sizeof(int64_t) * 256));
  }
  DM_HIP(dm_join_pass_stream(g));
  const int32_t R = n_robots, T = n_robots;
  DM_HIP(hipMemcpyAsync(g->goal_io, robots_xy, sizeof(double) * 2 * (size_t)R, hipMemcpyHostToDevice,
                        g->stream));
  std::vector<int64_t> idx((size_t)R, -1);
  if (K > 0) {
    const unsigned long long* dk = nullptr;
    const uint32_t* di = nullptr;
    if ((rc = dm_launch_goal_topk(g, recs, K, g->goal_io, R, T, min_size, distance_weight, min_distance, &dk,
                                  &di)))
      return rc;
    std::vector<unsigned long long> hk((size_t)R * T);
    std::vector<uint32_t> hi((size_t)R * T);
    DM_HIP(hipMemcpyAsync(hk.data(), dk, sizeof(unsigned long long) * hk.size(), hipMemcpyDeviceToHost,
                          g->stream));
    DM_HIP(hipMemcpyAsync(hi.data(), di, sizeof(uint32_t) * hi.size(), hipMemcpyDeviceToHost, g->stream));
    DM_HIP(hipStreamSynchronize(g->stream));
    // greedy in robot order over each robot's best-first list (its choice is
    // within its first r + 1 entries: r clusters are taken before its turn)
    for (int32_t r = 0; r < R; ++r) {
      for (int32_t t = 0; t < T; ++t) {
        if (hk[(size_t)r * T + t] == 0ull) break;  // no eligible cluster left in the list
        const int64_t c = hi[(size_t)r * T + t];
        if (std::find(idx.begin(), idx.begin() + r, c) != idx.begin() + r) continue;
        idx[(size_t)r] = c;
        break;
      }
    }
  }
  DM_HIP(hipMemcpyAsync(g->goal_idx, idx.data(), sizeof(int64_t) * (size_t)R, hipMemcpyHostToDevice,
                        g->stream));
  if ((rc = dm_launch_goal_gather(g, recs, g->goal_idx, R, g->goal_io + 2 * 256))) return rc;
  DM_HIP(hipMemcpyAsync(out_xy, g->goal_io + 2 * 256, sizeof(double) * 2 * (size_t)R, hipMemcpyDeviceToHost,
                        g->stream));
  DM_HIP(hipStreamSynchronize(g->stream));
  memcpy(out_index, idx.data(), sizeof(int64_t) * (size_t)R);
  return DM_OK;
}

int dm_set_overlap(dm_grid* g, int32_t on) {
  if (g && g->sh) return dm_sh_set_overlap(g, on);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  DM_HIP(dm_sync_all(g));
  g->overlap = on != 0;
  for (auto& w : g->iw) {
    w.free_owed = false;
    w.free_wait = nullptr;
  }
  return DM_OK;
}

int dm_set_halo(dm_grid* g, const int8_t* before, const int8_t* after) {
  if (int rc0 = not_on_sharded(g, "dm_set_halo")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  if (before) DM_HIP(hipMemcpy(g->halo, before, (size_t)g->W, hipMemcpyHostToDevice));
  if (after) DM_HIP(hipMemcpy(g->halo + g->W, after, (size_t)g->W, hipMemcpyHostToDevice));
  g->has_halo[0] = before != nullptr;
  g->has_halo[1] = after != nullptr;
  g->frontier_valid = false;
  ++g->integrate_seq;
  return DM_OK;
}

int dm_set_halo_device(dm_grid* g, const int8_t* before, const int8_t* after) {
  if (int rc0 = not_on_sharded(g, "dm_set_halo_device")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (before) DM_HIP(hipMemcpyAsync(g->halo, before, (size_t)g->W, hipMemcpyDeviceToDevice, g->stream));
  if (after)
    DM_HIP(hipMemcpyAsync(g->halo + g->W, after, (size_t)g->W, hipMemcpyDeviceToDevice, g->stream));
  g->has_halo[0] = before != nullptr;
  g->has_halo[1] = after != nullptr;
  g->frontier_valid = false;
  ++g->integrate_seq;
  return DM_OK;
}

int dm_get_edge_rows(dm_grid* g, int8_t* first_row, int8_t* last_row) {
  if (int rc0 = not_on_sharded(g, "dm_get_edge_rows")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (first_row)
    DM_HIP(hipMemcpyAsync(first_row, g->state, (size_t)g->W, hipMemcpyDeviceToHost, g->stream));
  if (last_row)
    DM_HIP(hipMemcpyAsync(last_row, g->state + (g->R - 1) * g->W, (size_t)g->W,
                          hipMemcpyDeviceToHost, g->stream));
  DM_HIP(hipStreamSynchronize(g->stream));
  return DM_OK;
}

int dm_get_edge_rows_device(dm_grid* g, int8_t* first_row, int8_t* last_row) {
  if (int rc0 = not_on_sharded(g, "dm_get_edge_rows_device")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (first_row)
    DM_HIP(hipMemcpyAsync(first_row, g->state, (size_t)g->W, hipMemcpyDeviceToDevice, g->stream));
  if (last_row)
    DM_HIP(hipMemcpyAsync(last_row, g->state + (g->R - 1) * g->W, (size_t)g->W,
                          hipMemcpyDeviceToDevice, g->stream));
  return DM_OK;
}

int dm_get_edge_labels(dm_grid* g, int64_t* first_row, int64_t* last_row) {
  if (int rc0 = not_on_sharded(g, "dm_get_edge_labels")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!g->frontier_valid)
    return dm_set_error(DM_ERR_STATE, "call dm_frontiers first (map or halo changed since)");
  DM_HIP(dm_join_pass_stream(g));
  if ((rc = dm_launch_edge_labels(g))) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  if (first_row)
    DM_HIP(hipMemcpy(first_row, g->edge_label, sizeof(int64_t) * (size_t)g->W, hipMemcpyDeviceToHost));
  if (last_row)
    DM_HIP(hipMemcpy(last_row, g->edge_label + g->W, sizeof(int64_t) * (size_t)g->W,
                     hipMemcpyDeviceToHost));
  return DM_OK;
}

static int check_ld06_args(int32_t S, int32_t N, const void* pts, const void* off, const void* out) {
  if (S < 0) return dm_set_error(DM_ERR_SHAPE, "S must be >= 0");
  if (N < 2 || N > 8192) return dm_set_error(DM_ERR_SHAPE, "N must be in [2, 8192] (got %d)", N);
  if (S > 0 && (!pts || !off || !out)) return dm_set_error(DM_ERR_INVALID_ARG, "NULL buffer");
  return DM_OK;
}

int dm_ld06_to_scans_device(dm_grid* g, int32_t S, const dm_ld06_point* d_points,
                            const int64_t* d_offsets, int32_t N, int laser_scan_dir,
                            float* d_ranges_out, float* d_intensities_out) {
  if (g && g->sh) return dm_sh_ld06_to_scans_device(g, S, d_points, d_offsets, N, laser_scan_dir, d_ranges_out, d_intensities_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if ((rc = check_ld06_args(S, N, d_points, d_offsets, d_ranges_out))) return rc;
  return dm_launch_ld06(g, S, d_points, d_offsets, N, laser_scan_dir ? 1 : 0, d_ranges_out,
                        d_intensities_out);
}

int dm_ld06_to_scans(dm_grid* g, int32_t S, const dm_ld06_point* points, const int64_t* offsets,
                     int32_t N, int laser_scan_dir, float* ranges_out, float* intensities_out) {
  if (g && g->sh) return dm_sh_ld06_to_scans(g, S, points, offsets, N, laser_scan_dir, ranges_out, intensities_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if ((rc = check_ld06_args(S, N, points, offsets, ranges_out))) return rc;
  if (S == 0) return DM_OK;
  const int64_t np = offsets[S];
  if (np < 0 || offsets[0] != 0) return dm_set_error(DM_ERR_SHAPE, "offsets must start at 0");
  for (int32_t s = 0; s < S; ++s)
    if (offsets[s + 1] < offsets[s]) return dm_set_error(DM_ERR_SHAPE, "offsets must be non-decreasing");
  dm_ld06_point* dp = nullptr;
  int64_t* doff = nullptr;
  float* dr = nullptr;
  float* di = nullptr;
  auto cleanup = [&]() { dev_free(dp); dev_free(doff); dev_free(dr); dev_free(di); };
  if ((rc = dev_alloc(&dp, np, "ld06 points")) || (rc = dev_alloc(&doff, S + 1, "ld06 offsets")) ||
      (rc = dev_alloc(&dr, (int64_t)S * N, "ld06 ranges")) ||
      (intensities_out && (rc = dev_alloc(&di, (int64_t)S * N, "ld06 intensities")))) {
    cleanup();
    return rc;
  }
  hipError_t e = hipMemcpyAsync(dp, points, sizeof(dm_ld06_point) * (size_t)np, hipMemcpyHostToDevice, g->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(doff, offsets, sizeof(int64_t) * (size_t)(S + 1), hipMemcpyHostToDevice, g->stream);
  if (e == hipSuccess) rc = dm_launch_ld06(g, S, dp, doff, N, laser_scan_dir ? 1 : 0, dr, di);
  if (e == hipSuccess && !rc)
    e = hipMemcpyAsync(ranges_out, dr, sizeof(float) * (size_t)S * N, hipMemcpyDeviceToHost, g->stream);
  if (e == hipSuccess && !rc && intensities_out)
    e = hipMemcpyAsync(intensities_out, di, sizeof(float) * (size_t)S * N, hipMemcpyDeviceToHost, g->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
  cleanup();
  if (e != hipSuccess) return dm_hip_check(e, "dm_ld06_to_scans");
  return rc;
}

static const char kMagic[8] = {'D', 'M', 'A', 'P', '0', '0', '0', '1'};

int dm_save(dm_grid* g, const char* path) {
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!path) return dm_set_error(DM_ERR_INVALID_ARG, "path is NULL");
  const int64_t cells = g->W * g->R;
  std::vector<float> L((size_t)cells);
  if ((rc = dm_get_logodds(g, L.data()))) return rc;
  FILE* f = fopen(path, "wb");
  if (!f) return dm_set_error(DM_ERR_IO, "cannot open %s for writing", path);
  bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&g->p, sizeof(dm_params), 1, f) == 1 &&
            fwrite(L.data(), sizeof(float), (size_t)cells, f) == (size_t)cells;
  ok = (fclose(f) == 0) && ok;
  if (!ok) return dm_set_error(DM_ERR_IO, "short write to %s", path);
  return DM_OK;
}

int dm_load(dm_grid* g, const char* path) {
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!path) return dm_set_error(DM_ERR_INVALID_ARG, "path is NULL");
  FILE* f = fopen(path, "rb");
  if (!f) return dm_set_error(DM_ERR_IO, "cannot open %s", path);
  char magic[8];
  dm_params p;
  const int64_t cells = g->W * g->R;
  std::vector<float> L((size_t)cells);
  bool ok = fread(magic, 1, 8, f) == 8 && memcmp(magic, kMagic, 8) == 0 &&
            fread(&p, sizeof p, 1, f) == 1;
  if (ok && (p.width != g->p.width || p.height != g->p.height || p.band_row0 != g->p.band_row0 ||
             p.band_rows != g->p.band_rows || p.resolution != g->p.resolution)) {
    fclose(f);
    return dm_set_error(DM_ERR_SHAPE, "checkpoint %s has a different grid geometry", path);
  }
  ok = ok && fread(L.data(), sizeof(float), (size_t)cells, f) == (size_t)cells;
  fclose(f);
  if (!ok) return dm_set_error(DM_ERR_IO, "%s is not a dm checkpoint or is truncated", path);
  return dm_set_logodds(g, L.data());
}

int dm_set_stream(dm_grid* g, void* stream) {
  if (int rc0 = not_on_sharded(g, "dm_set_stream")) return rc0;
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  DM_HIP(dm_sync_all(g));
  if (stream) {
    if (g->own_stream && g->stream) (void)hipStreamDestroy(g->stream);
    g->stream = (hipStream_t)stream;
    g->own_stream = false;
  } else if (!g->own_stream) {
    DM_HIP(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    g->own_stream = true;
  }
  return DM_OK;
}

int dm_synchronize(dm_grid* g) {
  if (g && g->sh) return dm_sh_synchronize(g);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  DM_HIP(dm_sync_all(g));
  return DM_OK;
}

int dm_profile_enable(dm_grid* g, int enable) {
  if (g && g->sh) return dm_sh_profile_enable(g, enable);
  int rc = check_grid(g);
  if (rc) return rc;
  g->profile = enable != 0;
  return DM_OK;
}

int dm_profile_read(dm_grid* g, dm_kernel_stat* out, int32_t cap, int32_t* n_out) {
  if (g && g->sh) return dm_sh_profile_read(g, out, cap, n_out);
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  for (auto& t : g->pending) {
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, t.start, t.stop);
    (void)hipEventDestroy(t.start);
    (void)hipEventDestroy(t.stop);
    dm_kernel_stat* s = nullptr;
    for (auto& e : g->stats)
      if (t.name == e.name) s = &e;
    if (!s) {
      dm_kernel_stat ns;
      memset(&ns, 0, sizeof ns);
      snprintf(ns.name, sizeof ns.name, "%s", t.name.c_str());
      g->stats.push_back(ns);
      s = &g->stats.back();
    }
    s->launches += 1;
    s->total_ms += ms;
  }
  g->pending.clear();
  const int32_t n = (int32_t)g->stats.size();
  for (int32_t i = 0; i < std::min(n, cap); ++i) out[i] = g->stats[(size_t)i];
  if (n_out) *n_out = n;
  return DM_OK;
}

int dm_profile_reset(dm_grid* g) {
  if (g && g->sh) return dm_sh_profile_reset(g);
  int rc = check_grid(g);
  if (rc) return rc;
  int32_t n = 0;
  if ((rc = dm_profile_read(g, nullptr, 0, &n))) return rc;
  g->stats.clear();
  return DM_OK;
}

int dm_map_image(dm_grid* g, uint8_t* out) {
  if (g && g->sh) return (out ? dm_sh_map_image(g, out) : dm_set_error(DM_ERR_INVALID_ARG, "out is NULL"));
  int rc = check_grid(g);
  if (rc || (rc = use_device(g))) return rc;
  if (!out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  const int64_t cells = g->W * g->R;
  uint8_t* d = nullptr;
  if ((rc = dev_alloc(&d, cells, "image"))) return rc;
  rc = dm_launch_map_image(g, d);
  hipError_t e = hipSuccess;
  if (!rc) e = hipMemcpyAsync(out, d, (size_t)cells, hipMemcpyDeviceToHost, g->stream);
  if (!rc && e == hipSuccess) e = hipStreamSynchronize(g->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return dm_hip_check(e, "dm_map_image");
  return rc;
}

}  // extern "C"
