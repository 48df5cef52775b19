// dm_merge.hip — cross-band frontier exchange for row-band sharded maps
// (export layout in include/dm.h).
//
// A map split into row bands (one per GPU) extracts frontiers per band with
// band-local min-index labels.  A component that crosses a band edge shows
// up in both bands; the global label is the min over its parts.  Instead of
// copying edges and clusters to the host and merging there, every band
// writes one export record (header, its first/last-row components as indices
// into its sorted cluster list, the clusters), the caller all-gathers the
// records over RCCL, and every rank merges all of them on its own device:
//
//   k_export        band: edge cells -> sorted cluster index; records; header
//   k_merge_init    one element per (band, cluster): parent = self, own sums
//   k_merge_pairs   band b's last row vs band b+1's first row, 8-connectivity
//                   (x-1, x, x+1): union keyed by label (dm_uf.h), so the
//                   root of a merged set is its min label = the 1-GPU label
//   k_merge_resolve roots; int64 sums folded into the roots
//   k_merge_compact roots with size >= min_size -> merged records
//   k_rank_sort     (dm_frontier.hip) sorted dm_cluster records + centroids
//
// All ranks merge the same gathered bytes with the same integer arithmetic,
// so every rank holds the same cluster list, bit-identical to a 1-GPU run.
#include "dm_internal.h"
#include "dm_uf.h"

#include <algorithm>

namespace {

constexpr int64_t kHdrWords = 8;

struct ExportView {
  int64_t W, rec_cap, bytes;
  __host__ __device__ int64_t edge_off() const { return kHdrWords * 8; }
  __host__ __device__ int64_t rec_off() const { return kHdrWords * 8 + 8 * W; }
};

__host__ __device__ inline int64_t export_bytes(int64_t W, int64_t rec_cap) {
  return kHdrWords * 8 + 8 * W + 32 * rec_cap;
}

__device__ inline const long long* hdr_of(const uint8_t* base, const ExportView& v, int r) {
  return reinterpret_cast<const long long*>(base + (int64_t)r * v.bytes);
}
__device__ inline const int32_t* edge_of(const uint8_t* base, const ExportView& v, int r) {
  return reinterpret_cast<const int32_t*>(base + (int64_t)r * v.bytes + v.edge_off());
}
__device__ inline const long long* rec_of(const uint8_t* base, const ExportView& v, int r) {
  return reinterpret_cast<const long long*>(base + (int64_t)r * v.bytes + v.rec_off());
}

// Band export.  Edge slot -> root slot -> compact index -> sorted index.
__global__ __launch_bounds__(256) void k_export(ExportView v, int64_t row0, int64_t rows,
                                                const int32_t* __restrict__ edge_slot,
                                                const int32_t* __restrict__ slot_root,
                                                const int32_t* __restrict__ slot_k,
                                                const int32_t* __restrict__ rank_of,
                                                const dm_cluster* __restrict__ out_clu,
                                                const unsigned long long* __restrict__ cnt,
                                                uint8_t* __restrict__ exp) {
  const int64_t K = (int64_t)cnt[CNT_CLUSTERS];
  long long flags = 0;
  if (cnt[CNT_OVERFLOW] & kOvSlots) flags |= 1;
  if (cnt[CNT_OVERFLOW] & kOvUnionFind) flags |= 32;
  if (K > v.rec_cap) flags |= 2;
  if (!cnt[CNT_SORTED]) flags |= 4;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (i0 == 0) {
    long long* h = reinterpret_cast<long long*>(exp);
    h[0] = K; h[1] = flags; h[2] = row0; h[3] = rows; h[4] = v.W;
    h[5] = 0; h[6] = 0; h[7] = 0;
  }
  int32_t* edge = reinterpret_cast<int32_t*>(exp + v.edge_off());
  for (int64_t x = i0; x < 2 * v.W; x += stride) {
    const int32_t s = edge_slot[x];
    int32_t e = -1;
    if (s >= 0 && flags == 0) {
      const int32_t k = slot_k[slot_root[s]];
      if (k >= 0 && k < K) e = rank_of[k];
    }
    edge[x] = e;
  }
  long long* rec = reinterpret_cast<long long*>(exp + v.rec_off());
  const int64_t n = min(K, v.rec_cap);
  for (int64_t i = i0; i < n; i += stride) {
    const dm_cluster c = out_clu[i];
    rec[4 * i + 0] = c.label;
    rec[4 * i + 1] = c.size;
    rec[4 * i + 2] = c.sum_x;
    rec[4 * i + 3] = c.sum_y;
  }
}

struct MGeom {
  ExportView v;
  int32_t P;
  int64_t min_size;
};

enum { M_K = 0, M_FLAGS = 1, M_SORTED = 2, M_MAXK = 3 };

__device__ inline int64_t band_k(const uint8_t* g, const MGeom& m, int r) {
  const long long K = hdr_of(g, m.v, r)[0];
  return K < 0 ? 0 : min((int64_t)K, m.v.rec_cap);
}

// One element per (band r, record k): global index r*rec_cap + k.  Also
// collects the band flags (and band contiguity) and the largest band K.
__global__ __launch_bounds__(256) void k_merge_init(MGeom m, const uint8_t* __restrict__ gat,
                                                    int32_t* __restrict__ parent,
                                                    long long* __restrict__ label,
                                                    long long* __restrict__ acc,
                                                    unsigned long long* mcnt) {
  const int64_t n = (int64_t)m.P * m.v.rec_cap;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 < m.P) {
    const long long* h = hdr_of(gat, m.v, (int)i0);
    unsigned long long f = (unsigned long long)h[1];
    if (h[4] != m.v.W) f |= 8;
    if (i0 + 1 < m.P && h[2] + h[3] != hdr_of(gat, m.v, (int)i0 + 1)[2]) f |= 16;  // not contiguous
    if (f) atomicOr(&mcnt[M_FLAGS], f);
    atomicMax(&mcnt[M_MAXK], (unsigned long long)(h[0] < 0 ? 0 : h[0]));
  }
  for (int64_t i = i0; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / m.v.rec_cap);
    const int64_t k = i - (int64_t)r * m.v.rec_cap;
    parent[i] = (int32_t)i;
    if (k < band_k(gat, m, r)) {
      const long long* rc = rec_of(gat, m.v, r) + 4 * k;
      label[i] = rc[0];
      acc[3 * i + 0] = rc[1];
      acc[3 * i + 1] = rc[2];
      acc[3 * i + 2] = rc[3];
    } else {
      label[i] = -1;  // unused
    }
  }
}

// Band b's last row against band b+1's first row: cell x joins x-1, x, x+1.
// A lane skips the pairs its predecessor lane (cell x-1) already issued: a
// frontier crossing the edge repeats the same pair over consecutive cells.
__global__ __launch_bounds__(256) void k_merge_pairs(MGeom m, const uint8_t* __restrict__ gat,
                                                     int32_t* parent, const long long* __restrict__ label,
                                                     unsigned long long* mcnt) {
  const int64_t W = m.v.W;
  const int64_t n = (int64_t)(m.P - 1) * W;
  const int lane = __lane_id();
  // grid-stride in whole waves so __shfl_up sees the previous cell
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const bool in = i < n;
    const int b = in ? (int)(i / W) : 0;
    const int64_t x = in ? i - (int64_t)b * W : 0;
    int32_t a = -1, c[3] = {-1, -1, -1};
    if (in) {
      const int64_t Ka = band_k(gat, m, b), Kb = band_k(gat, m, b + 1);
      const int32_t ea = edge_of(gat, m.v, b)[W + x];  // band b, last row
      if (ea >= 0 && ea < Ka) {
        a = (int32_t)((int64_t)b * m.v.rec_cap + ea);
        const int32_t* first = edge_of(gat, m.v, b + 1);
        for (int d = -1; d <= 1; ++d) {
          const int64_t xx = x + d;
          if (xx < 0 || xx >= W) continue;
          const int32_t eb = first[xx];
          if (eb >= 0 && eb < Kb) c[d + 1] = (int32_t)((int64_t)(b + 1) * m.v.rec_cap + eb);
        }
      }
    }
    const int32_t pa = __shfl_up(a, 1);
    int32_t pc[3];
    for (int q = 0; q < 3; ++q) pc[q] = __shfl_up(c[q], 1);
    const bool has_prev = lane > 0 && x > 0;
    for (int q = 0; q < 3; ++q) {
      const int32_t bb = c[q];
      if (a < 0 || bb < 0) continue;
      bool dup = false;
      for (int r = 0; r < q; ++r) dup |= c[r] == bb;
      if (has_prev && pa == a) dup |= (pc[0] == bb) | (pc[1] == bb) | (pc[2] == bb);
      if (!dup) dm_uf_unite(parent, label, a, bb, &mcnt[M_FLAGS], 32ull);
    }
  }
}

__global__ __launch_bounds__(256) void k_merge_resolve(MGeom m, const uint8_t* __restrict__ gat,
                                                       const int32_t* __restrict__ parent,
                                                       long long* acc, unsigned long long* mcnt) {
  const int64_t n = (int64_t)m.P * m.v.rec_cap;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / m.v.rec_cap);
    const int64_t k = i - (int64_t)r * m.v.rec_cap;
    if (k >= band_k(gat, m, r)) continue;
    const int32_t root = dm_uf_root(parent, (int32_t)i, &mcnt[M_FLAGS], 32ull);
    if (root == (int32_t)i) continue;
    const long long* rc = rec_of(gat, m.v, r) + 4 * k;
    atomicAdd((unsigned long long*)&acc[3 * (int64_t)root + 0], (unsigned long long)rc[1]);
    atomicAdd((unsigned long long*)&acc[3 * (int64_t)root + 1], (unsigned long long)rc[2]);
    atomicAdd((unsigned long long*)&acc[3 * (int64_t)root + 2], (unsigned long long)rc[3]);
  }
}

__global__ __launch_bounds__(256) void k_merge_compact(MGeom m, const uint8_t* __restrict__ gat,
                                                       const int32_t* __restrict__ parent,
                                                       const long long* __restrict__ label,
                                                       const long long* __restrict__ acc,
                                                       long long* __restrict__ out,
                                                       unsigned long long* mcnt) {
  const int64_t n = (int64_t)m.P * m.v.rec_cap;
  const int lane = __lane_id();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); s0 < n; s0 += stride) {
    const int64_t i = s0 + lane;
    bool keep = false;
    if (i < n) {
      const int r = (int)(i / m.v.rec_cap);
      const int64_t k = i - (int64_t)r * m.v.rec_cap;
      keep = k < band_k(gat, m, r) && parent[i] == (int32_t)i && acc[3 * i] >= m.min_size;
    }
    const unsigned long long bal = __ballot(keep);
    if (!bal) continue;
    const int first = __ffsll(bal) - 1;
    unsigned long long k0 = 0;
    if (lane == first) k0 = atomicAdd(&mcnt[M_K], (unsigned long long)__popcll(bal));
    k0 = __shfl(k0, first);
    if (!keep) continue;
    const unsigned long long k = k0 + __popcll(bal & ((1ull << lane) - 1));
    out[4 * k + 0] = label[i];
    out[4 * k + 1] = acc[3 * i + 0];
    out[4 * k + 2] = acc[3 * i + 1];
    out[4 * k + 3] = acc[3 * i + 2];
  }
}

int grid_for(int64_t n, int threads, int64_t cap) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

int64_t dm_export_nbytes(int64_t W, int64_t rec_cap) { return export_bytes(W, rec_cap); }

int dm_launch_export(dm_grid* g, hipStream_t s, void* d_export, int64_t rec_cap) {
  ExportView v;
  v.W = g->W;
  v.rec_cap = rec_cap;
  v.bytes = export_bytes(g->W, rec_cap);
  KernelTimer t;
  dm_timer_begin(g, "export", &t, s);
  hipLaunchKernelGGL(k_export, dim3(grid_for(std::max<int64_t>(2 * g->W, rec_cap), 256, 256)), dim3(256), 0,
                     s, v, g->row0, g->R, g->edge_slot, g->slot_root, g->slot_k, g->rank_of,
                     g->out_clu, g->cnt, static_cast<uint8_t*>(d_export));
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_merge(dm_grid* g, hipStream_t s, const void* d_gathered, int32_t nranks, int64_t rec_cap,
                    int64_t min_size) {
  ++g->m_pass;
  ++g->rb[g->cur_slot].mepoch;  // this merge rewrites the selected slot's records
  MGeom m;
  m.v.W = g->W;
  m.v.rec_cap = rec_cap;
  m.v.bytes = export_bytes(g->W, rec_cap);
  m.P = nranks;
  m.min_size = min_size < 1 ? 1 : min_size;
  const uint8_t* gat = static_cast<const uint8_t*>(d_gathered);
  const int64_t n = (int64_t)nranks * rec_cap;
  DM_HIP(hipMemsetAsync(g->m_cnt, 0, sizeof(unsigned long long) * 4, s));
  KernelTimer t;
  dm_timer_begin(g, "merge", &t, s);
  const int eg = grid_for(n, 256, 1024);
  hipLaunchKernelGGL(k_merge_init, dim3(eg), dim3(256), 0, s, m, gat, g->m_parent, g->m_label,
                     g->m_acc, g->m_cnt);
  DM_HIP(hipGetLastError());
  if (nranks > 1) {
    hipLaunchKernelGGL(k_merge_pairs, dim3(grid_for((int64_t)(nranks - 1) * g->W, 256, 1024)), dim3(256), 0,
                       s, m, gat, g->m_parent, g->m_label, g->m_cnt);
    DM_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_merge_resolve, dim3(eg), dim3(256), 0, s, m, gat, g->m_parent, g->m_acc,
                     g->m_cnt);
  DM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_merge_compact, dim3(eg), dim3(256), 0, s, m, gat, g->m_parent, g->m_label,
                     g->m_acc, g->m_clu, g->m_cnt);
  DM_HIP(hipGetLastError());
  // merged labels are global row-major indices over the whole map
  const int rc = g->msort_hint > g->sort_min
      ? dm_launch_bucket_sort(g, s, g->m_clu, nullptr, nullptr, g->m_cnt + M_K, n, 0, g->H, g->m_out, nullptr, g->m_cnt + M_SORTED,
                              g->m_cnt, 4, M_SORTED, nullptr, g->h_out_dev, g->h_out_cap)
      : dm_launch_rank_sort(s, g->m_clu, nullptr, nullptr, g->m_cnt + M_K, n, g->p.origin_x, g->p.origin_y,
                            g->p.resolution, g->m_out, nullptr, g->m_cnt + M_SORTED, g->m_cnt, 4,
                            M_SORTED, nullptr, g->h_out_dev, g->h_out_cap, g->msort_hint);
  dm_timer_end(g, &t);
  return rc;
}
