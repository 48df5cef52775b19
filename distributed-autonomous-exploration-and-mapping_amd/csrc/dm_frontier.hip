// dm_frontier.hip — exploration frontiers on the occupancy grid (gfx950).
//
// The reference has no frontier code (reactive navigation in
// server/thymio_project/thymio_project/main.py:123-188, map-based planning is
// future work in report.pdf p.5 §VI-2).  SPEC rows a8-a10 (SURVEY.md §8(a),
// DESIGN.md §2.4):
//   F[c]    = state[c] == 0 and some in-grid 8-neighbour has state == -1
//   label   = min global row-major index of c's 8-connected component of F
//   cluster = (label, size, sum_x, sum_y), sorted by label (host side).
//
// Pipeline; tiles are the 64x64 tiles of dm_integrate.hip:
//   k_ftile_list    tiles holding >= 1 free cell (tile_free > 0, maintained
//                   incrementally by k_tile_apply) -> visit list + map.  Only
//                   free cells can be frontier cells, so every other tile is
//                   skipped without reading it.
//   k_frontier_tile one workgroup per listed tile: state tile + 1-cell halo
//                   in LDS, frontier test, LDS union-find (atomicMin hooking,
//                   root = min index), per-component sums, one slot per
//                   tile-local component, border slot ids
//   k_frontier_merge unions slots across tile borders (8-connectivity),
//                   lock-free CAS union-find keyed by label
//   k_frontier_resolve / k_frontier_compact  roots, int64 sums, cluster list
#include "dm_internal.h"

namespace {

constexpr int kFT = 256;              // threads per frontier workgroup
constexpr int kHP = DM_TS + 2;        // halo tile pitch (66)
constexpr int kMaxRoots = 1024;       // 8-connected components in a 64x64 tile

struct FGeom {
  int32_t W, R, row0, TX, TY;
  int32_t has_before, has_after;
  int32_t want_mask, want_labels;
  int64_t H;
  int64_t slot_cap;
  int64_t clu_cap;
  int64_t min_size;
};

__global__ __launch_bounds__(256) void k_ftile_list(FGeom g, int64_t NT, const int32_t* __restrict__ tile_free,
                                                    int32_t* __restrict__ ftiles,
                                                    int32_t* __restrict__ fmap,
                                                    unsigned long long* cnt) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < NT;
       t += (int64_t)gridDim.x * blockDim.x) {
    int32_t idx = -1;
    if (tile_free[t] > 0) {
      idx = (int32_t)atomicAdd(&cnt[CNT_FTILES], 1ull);
      ftiles[idx] = (int32_t)t;
    }
    fmap[t] = idx;
  }
}

__device__ inline int32_t lds_find(volatile int32_t* par, int32_t x) {
  int32_t p = par[x];
  while (p != x) {
    x = p;
    p = par[x];
  }
  return x;
}

// Union of the sets of a and b; the root with the larger index is hooked
// under the smaller one, so a root is always its set's minimum index.
__device__ inline void lds_unite(int32_t* par, int32_t a, int32_t b) {
  volatile int32_t* vp = par;
  for (int it = 0; it < 8192; ++it) {
    a = lds_find(vp, a);
    b = lds_find(vp, b);
    if (a == b) return;
    if (a < b) { const int32_t t = a; a = b; b = t; }
    const int32_t old = atomicMin(&par[a], b);
    if (old == a) return;
    a = old;
  }
}

__global__ __launch_bounds__(kFT) void k_frontier_tile(
    FGeom g, const int8_t* __restrict__ state, const int8_t* __restrict__ halo,
    const int32_t* __restrict__ ftiles, int32_t* __restrict__ border,
    long long* __restrict__ slot_label, int32_t* __restrict__ slot_parent,
    long long* __restrict__ slot_own, long long* __restrict__ slot_acc,
    uint8_t* __restrict__ mask, int32_t* __restrict__ cell_slot, int32_t* __restrict__ edge_slot,
    unsigned long long* cnt) {
  __shared__ int8_t st[kHP * kHP];
  __shared__ int32_t par[DM_TS * DM_TS];
  __shared__ int16_t rid[DM_TS * DM_TS];
  __shared__ int16_t rcell[kMaxRoots];
  __shared__ uint32_t ssz[kMaxRoots], ssx[kMaxRoots], ssy[kMaxRoots];
  __shared__ int32_t nroots;
  __shared__ long long sbase;
  const int tid = threadIdx.x;
  const int64_t nft = (int64_t)cnt[CNT_FTILES];
  for (int64_t j = blockIdx.x; j < nft; j += gridDim.x) {
    const int32_t tile = ftiles[j];
    const int32_t tx0 = (tile % g.TX) * DM_TS;
    const int32_t ty0 = (tile / g.TX) * DM_TS;  // band-local
    if (tid == 0) nroots = 0;
    // state tile + halo; out-of-grid (and missing-halo) cells read as 0,
    // which is "not unknown" (out-of-bounds neighbours do not count)
    for (int e = tid; e < kHP * kHP; e += kFT) {
      const int hy = e / kHP, hx = e - hy * kHP;
      const int32_t y = ty0 + hy - 1, x = tx0 + hx - 1;
      int8_t v = 0;
      if (x >= 0 && x < g.W) {
        if (y >= 0 && y < g.R) v = state[(int64_t)y * g.W + x];
        else if (y == -1 && g.has_before) v = halo[x];
        else if (y == g.R && g.has_after) v = halo[g.W + x];
      }
      st[e] = v;
    }
    __syncthreads();
    int any = 0;
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      const int ly = c >> 6, lx = c & 63;
      int f = 0;
      if (tx0 + lx < g.W && ty0 + ly < g.R) {
        const int h = (ly + 1) * kHP + lx + 1;
        if (st[h] == 0) {
          f = (st[h - kHP - 1] == -1) | (st[h - kHP] == -1) | (st[h - kHP + 1] == -1) |
              (st[h - 1] == -1) | (st[h + 1] == -1) | (st[h + kHP - 1] == -1) |
              (st[h + kHP] == -1) | (st[h + kHP + 1] == -1);
        }
      }
      par[c] = f ? c : -1;
      any |= f;
    }
    any = __syncthreads_or(any);
    if (!any) {
      border[j * 256 + tid] = -1;
      __syncthreads();
      continue;
    }
    // union with the already-defined neighbours W, NW, N, NE
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      if (par[c] < 0) continue;
      const int ly = c >> 6, lx = c & 63;
      if (lx > 0 && par[c - 1] >= 0) lds_unite(par, c, c - 1);
      if (ly > 0) {
        if (lx > 0 && par[c - 65] >= 0) lds_unite(par, c, c - 65);
        if (par[c - 64] >= 0) lds_unite(par, c, c - 64);
        if (lx < 63 && par[c - 63] >= 0) lds_unite(par, c, c - 63);
      }
    }
    __syncthreads();
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      if (par[c] >= 0) par[c] = lds_find(par, c);
    }
    __syncthreads();
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      if (par[c] == c) {
        const int r = atomicAdd(&nroots, 1);
        rid[c] = (int16_t)r;
        rcell[r] = (int16_t)c;
      }
    }
    for (int r = tid; r < kMaxRoots; r += kFT) { ssz[r] = 0; ssx[r] = 0; ssy[r] = 0; }
    __syncthreads();
    if (tid == 0) sbase = (long long)atomicAdd(&cnt[CNT_SLOTS], (unsigned long long)nroots);
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      const int32_t p = par[c];
      if (p < 0) continue;
      const int r = rid[p];
      atomicAdd(&ssz[r], 1u);
      atomicAdd(&ssx[r], (uint32_t)(c & 63));
      atomicAdd(&ssy[r], (uint32_t)(c >> 6));
    }
    __syncthreads();
    const long long base = sbase;
    const int nr = nroots;
    for (int r = tid; r < nr; r += kFT) {
      const long long slot = base + r;
      if (slot >= g.slot_cap) { atomicOr(&cnt[CNT_OVERFLOW], 4ull); continue; }
      const int c = rcell[r];
      const long long gy = (long long)g.row0 + ty0 + (c >> 6);
      const long long gx = (long long)tx0 + (c & 63);
      const long long sz = ssz[r];
      slot_label[slot] = gy * g.W + gx;
      slot_parent[slot] = (int32_t)slot;
      const long long sx = sz * tx0 + ssx[r];
      const long long sy = sz * ((long long)g.row0 + ty0) + ssy[r];
      slot_own[3 * slot + 0] = sz; slot_own[3 * slot + 1] = sx; slot_own[3 * slot + 2] = sy;
      slot_acc[3 * slot + 0] = sz; slot_acc[3 * slot + 1] = sx; slot_acc[3 * slot + 2] = sy;
    }
    // border slots: [0] first row, [1] last row, [2] first col, [3] last col
    {
      const int side = tid >> 6, pos = tid & 63;
      const int c = side == 0 ? pos : side == 1 ? (63 * 64 + pos) : side == 2 ? (pos * 64) : (pos * 64 + 63);
      const int32_t p = par[c];
      long long s = p < 0 ? -1 : base + rid[p];
      if (s >= g.slot_cap) s = -1;
      border[j * 256 + tid] = (int32_t)s;
    }
    // band edge rows (for cross-band merging) and optional dense outputs
    for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
      const int ly = c >> 6, lx = c & 63;
      const int32_t y = ty0 + ly, x = tx0 + lx;
      if (x >= g.W || y >= g.R) continue;
      const int32_t p = par[c];
      long long s = p < 0 ? -1 : base + rid[p];
      if (s >= g.slot_cap) s = -1;
      const int64_t gi = (int64_t)y * g.W + x;
      if (g.want_mask) mask[gi] = p >= 0;
      if (g.want_labels) cell_slot[gi] = (int32_t)s;
      if (p >= 0) {
        if (y == 0) edge_slot[x] = (int32_t)s;
        if (y == g.R - 1) edge_slot[g.W + x] = (int32_t)s;
      }
    }
    __syncthreads();
  }
}

__device__ inline int32_t g_load(int32_t* p) { return atomicOr(p, 0); }

__device__ inline int32_t g_find(int32_t* par, int32_t x) {
  for (int it = 0; it < (1 << 22); ++it) {
    const int32_t p = g_load(par + x);
    if (p == x) return x;
    x = p;
  }
  return x;
}

// Lock-free union: hook the root with the larger label under the other.
// Every access to parent[] is an atomic RMW, performed at the device-coherent
// point (per-XCD L2s are not coherent; MI355X_MICROARCH.md §Workgroup dispatch).
__device__ inline void g_unite(int32_t* par, const long long* label, int32_t a, int32_t b) {
  for (int it = 0; it < (1 << 20); ++it) {
    a = g_find(par, a);
    b = g_find(par, b);
    if (a == b) return;
    if (label[a] < label[b]) { const int32_t t = a; a = b; b = t; }
    if (atomicCAS(&par[a], a, b) == a) return;
  }
}

__global__ __launch_bounds__(256) void k_frontier_merge(FGeom g, const int32_t* __restrict__ ftiles,
                                                        const int32_t* __restrict__ fmap,
                                                        const int32_t* __restrict__ border,
                                                        const long long* __restrict__ slot_label,
                                                        int32_t* slot_parent,
                                                        const unsigned long long* cnt) {
  const int tid = threadIdx.x;
  const int64_t nft = (int64_t)cnt[CNT_FTILES];
  for (int64_t j = blockIdx.x; j < nft; j += gridDim.x) {
    const int32_t tile = ftiles[j];
    const int32_t tx = tile % g.TX, ty = tile / g.TX;
    const int32_t* bA = border + j * 256;
    if (tid < 64) {  // right neighbour: our last column vs its first column
      const int32_t sa = bA[3 * 64 + tid];
      if (sa >= 0 && tx + 1 < g.TX) {
        const int32_t fb = fmap[ty * g.TX + tx + 1];
        if (fb >= 0) {
          const int32_t* bB = border + (int64_t)fb * 256;
          for (int d = -1; d <= 1; ++d) {
            const int y2 = tid + d;
            if (y2 < 0 || y2 > 63) continue;
            const int32_t sb = bB[2 * 64 + y2];
            if (sb >= 0) g_unite(slot_parent, slot_label, sa, sb);
          }
        }
      }
    } else if (tid < 128) {  // next tile row: our last row vs its first row
      const int x = tid - 64;
      const int32_t sa = bA[1 * 64 + x];
      if (sa >= 0 && ty + 1 < g.TY) {
        const int32_t fc = fmap[(ty + 1) * g.TX + tx];
        if (fc >= 0) {
          const int32_t* bC = border + (int64_t)fc * 256;
          for (int d = -1; d <= 1; ++d) {
            const int x2 = x + d;
            if (x2 < 0 || x2 > 63) continue;
            const int32_t sb = bC[x2];
            if (sb >= 0) g_unite(slot_parent, slot_label, sa, sb);
          }
        }
      }
    } else if (tid == 128) {  // diagonal: our (63,63) vs (tx+1,ty+1)'s (0,0)
      const int32_t sa = bA[1 * 64 + 63];
      if (sa >= 0 && tx + 1 < g.TX && ty + 1 < g.TY) {
        const int32_t fd = fmap[(ty + 1) * g.TX + tx + 1];
        if (fd >= 0) {
          const int32_t sb = border[(int64_t)fd * 256 + 0];
          if (sb >= 0) g_unite(slot_parent, slot_label, sa, sb);
        }
      }
    } else if (tid == 129) {  // anti-diagonal: our (0,63) vs (tx-1,ty+1)'s (63,0)
      const int32_t sa = bA[1 * 64 + 0];
      if (sa >= 0 && tx > 0 && ty + 1 < g.TY) {
        const int32_t fe = fmap[(ty + 1) * g.TX + tx - 1];
        if (fe >= 0) {
          const int32_t sb = border[(int64_t)fe * 256 + 63];
          if (sb >= 0) g_unite(slot_parent, slot_label, sa, sb);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_frontier_resolve(FGeom g, const int32_t* __restrict__ slot_parent,
                                                          int32_t* __restrict__ slot_root,
                                                          const long long* __restrict__ slot_own,
                                                          long long* slot_acc,
                                                          const unsigned long long* cnt) {
  const int64_t ns = min((int64_t)cnt[CNT_SLOTS], g.slot_cap);
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ns;
       s += (int64_t)gridDim.x * blockDim.x) {
    int32_t r = (int32_t)s;
    for (int it = 0; it < (1 << 22); ++it) {
      const int32_t p = slot_parent[r];
      if (p == r) break;
      r = p;
    }
    slot_root[s] = r;
    if (r != (int32_t)s) {
      atomicAdd((unsigned long long*)&slot_acc[3 * (int64_t)r + 0], (unsigned long long)slot_own[3 * s + 0]);
      atomicAdd((unsigned long long*)&slot_acc[3 * (int64_t)r + 1], (unsigned long long)slot_own[3 * s + 1]);
      atomicAdd((unsigned long long*)&slot_acc[3 * (int64_t)r + 2], (unsigned long long)slot_own[3 * s + 2]);
    }
  }
}

__global__ __launch_bounds__(256) void k_frontier_compact(FGeom g, const int32_t* __restrict__ slot_root,
                                                          const long long* __restrict__ slot_label,
                                                          const long long* __restrict__ slot_acc,
                                                          long long* __restrict__ clusters,
                                                          unsigned long long* cnt) {
  const int64_t ns = min((int64_t)cnt[CNT_SLOTS], g.slot_cap);
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ns;
       s += (int64_t)gridDim.x * blockDim.x) {
    if (slot_root[s] != (int32_t)s) continue;
    const long long sz = slot_acc[3 * s];
    if (sz < g.min_size) continue;
    const unsigned long long k = atomicAdd(&cnt[CNT_CLUSTERS], 1ull);
    if ((int64_t)k >= g.clu_cap) continue;
    clusters[4 * k + 0] = slot_label[s];
    clusters[4 * k + 1] = sz;
    clusters[4 * k + 2] = slot_acc[3 * s + 1];
    clusters[4 * k + 3] = slot_acc[3 * s + 2];
  }
}

__global__ __launch_bounds__(256) void k_slot_labels(int64_t n, const int32_t* __restrict__ cslot,
                                                     const int32_t* __restrict__ slot_root,
                                                     const long long* __restrict__ slot_label,
                                                     long long* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = cslot[i];
    out[i] = s < 0 ? -1 : slot_label[slot_root[s]];
  }
}

int grid_for(int64_t n, int threads, int64_t cap) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

// Runs the frontier pipeline.  Returns DM_ERR_CAPACITY (with *n_clusters set
// to the number of slots needed) when the slot arrays overflowed; the caller
// grows them and reruns.
int dm_launch_frontiers(dm_grid* g, bool want_mask, bool want_labels, int64_t* n_clusters) {
  FGeom fg;
  fg.W = (int32_t)g->W;
  fg.R = (int32_t)g->R;
  fg.row0 = (int32_t)g->row0;
  fg.TX = (int32_t)g->TX;
  fg.TY = (int32_t)g->TY;
  fg.has_before = g->has_halo[0];
  fg.has_after = g->has_halo[1];
  fg.want_mask = want_mask ? 1 : 0;
  fg.want_labels = want_labels ? 1 : 0;
  fg.H = g->H;
  fg.slot_cap = g->slot_cap;
  fg.clu_cap = g->slot_cap;
  fg.min_size = g->p.min_frontier_size;
  const int64_t cells = g->R * g->W;

  DM_HIP(hipMemsetAsync(g->cnt + CNT_FTILES, 0, sizeof(unsigned long long) * 4, g->stream));
  DM_HIP(hipMemsetAsync(g->edge_slot, 0xFF, sizeof(int32_t) * 2 * g->W, g->stream));
  if (want_mask) DM_HIP(hipMemsetAsync(g->mask, 0, (size_t)cells, g->stream));
  if (want_labels) DM_HIP(hipMemsetAsync(g->cell_slot, 0xFF, sizeof(int32_t) * (size_t)cells, g->stream));

  KernelTimer t;
  dm_timer_begin(g, "ftile_list", &t);
  hipLaunchKernelGGL(k_ftile_list, dim3(grid_for(g->NT, 256, 4096)), dim3(256), 0, g->stream, fg,
                     g->NT, g->tile_free, g->ftiles, g->fmap, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  const int nft_grid = grid_for(g->NT, 1, 2048);
  dm_timer_begin(g, "frontier_tile", &t);
  hipLaunchKernelGGL(k_frontier_tile, dim3(nft_grid), dim3(kFT), 0, g->stream, fg, g->state,
                     g->halo, g->ftiles, g->border, g->slot_label, g->slot_parent, g->slot_own,
                     g->slot_acc, g->mask, g->cell_slot, g->edge_slot, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "frontier_merge", &t);
  hipLaunchKernelGGL(k_frontier_merge, dim3(nft_grid), dim3(256), 0, g->stream, fg, g->ftiles,
                     g->fmap, g->border, g->slot_label, g->slot_parent, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  const int sgrid = grid_for(g->slot_cap, 256, 1024);
  dm_timer_begin(g, "frontier_resolve", &t);
  hipLaunchKernelGGL(k_frontier_resolve, dim3(sgrid), dim3(256), 0, g->stream, fg,
                     g->slot_parent, g->slot_root, g->slot_own, g->slot_acc, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "frontier_compact", &t);
  hipLaunchKernelGGL(k_frontier_compact, dim3(sgrid), dim3(256), 0, g->stream, fg,
                     g->slot_root, g->slot_label, g->slot_acc, g->clusters, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_slot_labels, dim3(grid_for(2 * g->W, 256, 1024)), dim3(256), 0, g->stream,
                     2 * g->W, g->edge_slot, g->slot_root, g->slot_label, g->edge_label);
  DM_HIP(hipGetLastError());
  if (want_labels) {
    hipLaunchKernelGGL(k_slot_labels, dim3(grid_for(cells, 256, 8192)), dim3(256), 0, g->stream,
                       cells, g->cell_slot, g->slot_root, g->slot_label, g->labels);
    DM_HIP(hipGetLastError());
  }
  DM_HIP(hipMemcpyAsync(g->h_cnt, g->cnt, sizeof(unsigned long long) * CNT_N, hipMemcpyDeviceToHost,
                        g->stream));
  DM_HIP(hipStreamSynchronize(g->stream));
  const unsigned long long slots = g->h_cnt[CNT_SLOTS];
  if ((int64_t)slots > g->slot_cap || (g->h_cnt[CNT_OVERFLOW] & 4ull)) {
    *n_clusters = (int64_t)slots;
    return DM_ERR_CAPACITY;
  }
  *n_clusters = (int64_t)g->h_cnt[CNT_CLUSTERS];
  return DM_OK;
}
