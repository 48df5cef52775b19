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
//   (list)          the persistent tile list: every tile that has held a free
//                   cell, appended by the integrate apply (dm_internal.h,
//                   ftiles); only free cells can be frontier cells, so every
//                   other tile is skipped without reading it
//   k_frontier_bits one wave per listed tile: frontier bit rows (the only
//                   kernel that reads the map), plus the pass's resets
//   k_frontier_tile(_big)  per listed tile: runs, LDS union-find (atomicMin
//                   hooking, root = min index), per-component sums, one slot
//                   per tile-local component; then, in dense passes, the
//                   unions across its edges with the neighbour tiles that
//                   finished before it (the later tile of each edge unites: a
//                   stamped hand-off word per tile pair), lock-free CAS
//                   union-find keyed by slot; in sparse passes it only
//                   publishes its edges
//   k_frontier_edges (sparse passes) the unions across every tile edge and
//                   corner, after the tile kernels
//   k_frontier_resolve / k_frontier_compact  roots, int64 sums and the min
//                   label of each merged set, cluster list
//   k_rank_sort / row sort  records by label, centroids, readback
#include "dm_internal.h"
#include "dm_uf.h"
#include "dm_phase.h"

#include <string.h>

#include <algorithm>

DM_PH_DECL(frontier)
DM_PH_DECL(ftile)

namespace {

constexpr int kFT = 256;              // threads per frontier workgroup
// Tile-edge unions, two ways (template parameter EDGE of the tile kernels):
//  * EDGE = false (dense passes, C3's ray fans): in-kernel, through the
//    stamped hand-off words rel[0, 4 NT) (the tile that arrives second at a
//    pair unites it; rounds 2-5);
//  * EDGE = true (sparse passes: the wave kernel + run-rich tiles beside it,
//    C5): the tile kernels only publish their edges' slot ids and a per-edge
//    stamp (rel[4 NT + 4 tile + side] = pass stamp, a region of its own so
//    the two encodings never meet); k_frontier_edges, launched after them,
//    unites every tile pair across its edges and corners.
// DM_EDGE_KERNEL (A/B builds): 1 the split above, 0 every pass in-kernel,
// 2 every pass with the edge kernel.
#ifndef DM_EDGE_KERNEL
#define DM_EDGE_KERNEL 1
#endif
#ifndef DM_EDGE_HALVE
#define DM_EDGE_HALVE 0
#endif
#if DM_EDGE_HALVE
#define EDGE_UNITE dm_uf_unite_idx_halve
#else
#define EDGE_UNITE dm_uf_unite_idx2
#endif
// waves per SIMD for k_frontier_tile: 7 workgroups per CU (LDS 22.6 KB each,
// <= 72 VGPRs), so a C3 pass's ~3.3k listed tiles run in two rounds of the
// chip's 1792 slots instead of three of 1280
#ifndef DM_FT_OCC
#define DM_FT_OCC 7
#endif
constexpr int kMaxRoots = 1024;       // 8-connected components in a 64x64 tile

struct FGeom {
  int32_t W, R, row0, TX, TY;
  int32_t has_before, has_after;
  int32_t pad_ = 0;  // no implicit padding
  int64_t NT;
  int32_t want_mask, want_labels;
  int64_t H;
  int64_t slot_cap;
  int64_t slot_per;  // slot_cap / kShards: slots of one shard region
  int64_t clu_cap;
  int64_t min_size;
};

// Find with path halving: every other node on the way is re-pointed to its
// grandparent, so later finds (the unions of the next rows, the final
// compression) walk shorter chains.  Only non-roots are re-pointed, to an
// ancestor: a halving store racing an atomicMin hook on the same node can
// drop that hook, but lds_unite then continues with the node's previous
// parent (atomicMin's return value), which is still an ancestor, so no
// union is lost.
__device__ inline int32_t lds_find(volatile int32_t* par, int32_t x) {
  int32_t p = par[x];
  while (p != x) {
    const int32_t gp = par[p];
    if (gp != p) par[x] = gp;
    x = gp;
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

constexpr int kMaxRuns = 2048;        // <= 32 runs per 64-bit row x 64 rows

__device__ inline uint64_t upto_mask(int p) {  // bits 0..p inclusive
  return p >= 63 ? ~0ull : ((2ull << p) - 1ull);
}

// First cells of the runs of a 64-bit frontier row.
__device__ inline uint64_t run_starts(uint64_t F) { return F & ~(F << 1); }

// Last column of the run of row F that starts at column s0.
__device__ inline int run_end(uint64_t F, int s0) {
  const uint64_t rest = ~(F >> s0);
  return rest ? s0 + __ffsll((unsigned long long)rest) - 2 : 63;
}

// Run id of frontier bit p of tile row y (p must be set): runs are numbered
// in row-major order of their first cell.
__device__ inline int run_of(const int32_t* rbase, const uint64_t* rowF, int y, int p) {
  return rbase[y] + __popcll(run_starts(rowF[y]) & upto_mask(p)) - 1;
}

// Component id of root run r: the number of root runs before it (root bits
// in s_root, one 64-bit word per 64 runs, exclusive word prefix in pre).
__device__ inline int root_rank(const uint64_t* s_root, const int32_t* pre, int r) {
  return pre[r >> 6] + __popcll(s_root[r >> 6] & ((1ull << (r & 63)) - 1ull));
}

// One workgroup per listed tile.  Each 64-cell tile row is a 64-bit word:
//  1. the tile's frontier bit rows (k_frontier_bits), one 8-byte load per
//     thread of wave 0;
//  2. runs of set bits, numbered row-major;
//  3. 8-connected CCL on the runs: a run is joined with every run of the row
//     above that overlaps it extended by one cell each side (LDS union-find,
//     atomicMin hooking: a root is its set's first run, whose first cell is
//     the component's min linear index);
//  4. per-component sums from run lengths, one slot per component;
//  5. unions across the tile's edges (below).
// Tiles come from the pass's list (bflag == nullptr: every list position),
// or only the positions bflag marks (k_frontier_bits: too run-rich for the
// wave kernel); a workgroup then gathers the flags of its next 64 positions
// in one load round and works through the marked ones.
template <bool EDGE>
__global__ __launch_bounds__(kFT, DM_FT_OCC) void k_frontier_tile_big(
    FGeom g, const uint64_t* __restrict__ fbits, const int32_t* __restrict__ bflag,
    const int32_t* __restrict__ ftiles, const unsigned long long* __restrict__ list_n,
    int32_t* border, unsigned long long* rel,
    long long* __restrict__ slot_label, int32_t* slot_parent,
    long long* __restrict__ slot_own, long long* __restrict__ slot_acc,
    uint8_t* __restrict__ mask, int32_t* __restrict__ cell_slot, int32_t* __restrict__ edge_slot,
    unsigned long long* cnt, unsigned long long* fsh, int count_stats) {
  const unsigned long long stamp = cnt[CNT_STAMP];  // this pass's (k_frontier_bits)
  __shared__ uint64_t s_F[DM_TS];          // frontier bit rows
  __shared__ int32_t s_rbase[DM_TS + 1];
  __shared__ int32_t r_par[kMaxRuns];
  __shared__ uint8_t r_s[kMaxRuns], r_y[kMaxRuns];  // run end: run_end(s_F[y], s)
  __shared__ uint64_t s_root[kMaxRuns / 64];        // root-run bits
  __shared__ int32_t s_rootpre[kMaxRuns / 64];
  // per-component size << 18 | sum of x (size <= 4096 < 2^13, sum of x <=
  // 4096 * 63 < 2^18: one 32-bit LDS add per run for both) and sum of y
  __shared__ uint32_t szx[kMaxRoots], ssy[kMaxRoots];
  __shared__ int32_t nroots;
  __shared__ long long sbase;
  const int tid = threadIdx.x, lane = __lane_id();
  const int64_t nft = (int64_t)*list_n;
  const int64_t G = gridDim.x;
  __shared__ uint64_t s_todo;
  DM_PH_INIT();
  for (int64_t kb = blockIdx.x; kb < nft; kb += bflag ? 64 * G : G) {  // one tile per workgroup at C3
  uint64_t todo = 1ull;
  if (bflag) {
    if (tid < 64) {
      const int64_t q = kb + (int64_t)tid * G;
      const uint64_t m = __ballot(q < nft && bflag[q] != 0);
      if (tid == 0) s_todo = m;
    }
    __syncthreads();
    todo = s_todo;
    __syncthreads();
  }
  while (todo) {
    const int64_t jj = bflag ? kb + (int64_t)(__ffsll((unsigned long long)todo) - 1) * G : kb;
    todo &= todo - 1;
    const int32_t tile = ftiles[jj];
    const uint64_t F = tid < DM_TS ? fbits[jj * DM_TS + tid] : 0ull;
    const int64_t j = tile;  // border records are indexed by tile
    DM_PH_COUNT(dm_phase_acc_frontier, 16, 1);
    const int32_t tx0 = (tile % g.TX) * DM_TS;
    const int32_t ty0 = (tile / g.TX) * DM_TS;  // band-local
    DM_PH(dm_phase_acc_frontier, 0);
    // ---- 2. runs ----------------------------------------------------------------
    int any = 0;
    if (tid < DM_TS) {
      const int y = tid;
      const uint64_t st = run_starts(F);
      s_F[y] = F;
      any = F != 0ull;
      // exclusive scan of run counts over the 64 rows (wave 0)
      const int c = __popcll(st);
      int incl = c;
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      s_rbase[y] = incl - c;
      if (y == 63) s_rbase[DM_TS] = incl;
    }
    any = __syncthreads_or(any);
    DM_PH(dm_phase_acc_frontier, 1);
    if (!any) {  // nothing to publish: the neighbours never read this tile's edges
      __syncthreads();
      DM_PH(dm_phase_acc_frontier, 8);
      continue;
    }
    {  // enumerate the runs: four threads per row, each the runs starting in its 16 columns
      const int y = tid >> 2, q = tid & 3;
      const uint64_t st_all = run_starts(s_F[y]);
      const uint64_t below = q ? upto_mask(16 * q - 1) : 0ull;
      uint64_t st = st_all & upto_mask(16 * q + 15) & ~below;
      int r = s_rbase[y] + __popcll(st_all & below);
      while (st) {
        const int s0 = __ffsll((unsigned long long)st) - 1;
        r_s[r] = (uint8_t)s0;
        r_y[r] = (uint8_t)y;
        r_par[r] = r;
        ++r;
        st &= st - 1;
      }
    }
    for (int r = tid; r < kMaxRoots; r += kFT) { szx[r] = 0; ssy[r] = 0; }
    __syncthreads();
    const int nruns = s_rbase[DM_TS];
    if (count_stats && tid == 0) {
      atomicAdd(&fsh[(blockIdx.x % kShards) * kShardWords + SH_RUNS], (unsigned long long)nruns);
      atomicAdd(&fsh[(blockIdx.x % kShards) * kShardWords + SH_FTF], 1ull);
    }
    DM_PH(dm_phase_acc_frontier, 2);
    DM_PH_COUNT(dm_phase_acc_frontier, 17, nruns);
    DM_PH_COUNT(dm_phase_acc_frontier, 18, 1);
    // ---- 3. union with overlapping runs of the row above ---------------------
    // (all rows at once: uniting row blocks level by level, 6 barriers, so
    // that finds stay short, measured 1.5x slower at C5)
    for (int r = tid; r < nruns; r += kFT) {
      const int y = r_y[r];
      if (y == 0) continue;
      const int s0 = r_s[r], e0 = run_end(s_F[y], s0);
      const int lo = s0 > 0 ? s0 - 1 : 0;
      const int hi = e0 < 63 ? e0 + 1 : 63;
      const uint64_t M = upto_mask(hi) & ~(lo > 0 ? upto_mask(lo - 1) : 0ull);
      uint64_t P = s_F[y - 1] & M;
      while (P) {
        const int p = __ffsll((unsigned long long)P) - 1;
        lds_unite(r_par, r, run_of(s_rbase, s_F, y - 1, p));
        // skip the rest of that run inside M
        const uint64_t rest = ~(s_F[y - 1] >> p);
        const int len = rest ? __ffsll((unsigned long long)rest) - 1 : 64 - p;
        P &= ~(upto_mask(p + len - 1));
      }
    }
    __syncthreads();
    DM_PH(dm_phase_acc_frontier, 3);
    // compress: every run points at its root.  The finds here only read
    // (no halving), so the only stores are final roots: a find passing
    // through a run already compressed just takes the shortcut.  Lane l of
    // a wave holds run 64 * word + l, so one ballot is the word of root bits.
    for (int r = tid; r < nruns; r += kFT) {
      int32_t x = r, p = r_par[r];
      while (p != x) {
        x = p;
        p = ((volatile int32_t*)r_par)[x];
      }
      r_par[r] = x;
      const uint64_t rb = __ballot(x == r);
      if (lane == 0) s_root[r >> 6] = rb;
    }
    __syncthreads();
    DM_PH(dm_phase_acc_frontier, 4);
    // ---- 4. components, sums, slots ------------------------------------------
    // component id = rank of its root run (row-major order of first cells)
    if (tid < 64) {
      const int nw = (nruns + 63) >> 6;
      const int c = tid < nw ? __popcll(s_root[tid]) : 0;
      int incl = c;
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      if (tid < nw) s_rootpre[tid] = incl - c;
      if (tid == 63) nroots = incl;
    }
    __syncthreads();
    DM_PH(dm_phase_acc_frontier, 5);
    // slots come from this workgroup's shard region [shard*slot_per, +slot_per)
    if (tid == 0)
      sbase = (long long)atomicAdd(&fsh[(blockIdx.x % kShards) * kShardWords + SH_SLOT],
                                   (unsigned long long)nroots);
    for (int r = tid; r < nruns; r += kFT) {
      const int c = root_rank(s_root, s_rootpre, r_par[r]);
      const int y = r_y[r];
      const uint32_t s0 = r_s[r], e0 = (uint32_t)run_end(s_F[y], (int)s0), len = e0 - s0 + 1;
      atomicAdd(&szx[c], (len << 18) + (s0 + e0) * len / 2);
      atomicAdd(&ssy[c], (uint32_t)y * len);
    }
    __syncthreads();
    DM_PH(dm_phase_acc_frontier, 6);
    const long long base = sbase;
    const long long sh0 = (long long)(blockIdx.x % kShards) * g.slot_per;
    for (int r = tid; r < nruns; r += kFT) {
      if (r_par[r] != r) continue;
      const int c = root_rank(s_root, s_rootpre, r);
      if (base + c >= g.slot_per) { atomicOr(&cnt[CNT_OVERFLOW], kOvSlots); continue; }
      const long long slot = sh0 + base + c;
      const long long gy = (long long)g.row0 + ty0 + r_y[r];
      const long long gx = (long long)tx0 + r_s[r];
      const uint32_t zx = szx[c];
      const long long sz = zx >> 18;
      slot_label[slot] = gy * g.W + gx;  // (slot_parent[slot] == slot since k_frontier_bits)
      const long long sx = sz * tx0 + (zx & 0x3FFFFu);
      const long long sy = sz * ((long long)g.row0 + ty0) + ssy[c];
      slot_own[3 * slot + 0] = sz; slot_own[3 * slot + 1] = sx; slot_own[3 * slot + 2] = sy;
      slot_acc[3 * slot + 0] = sz; slot_acc[3 * slot + 1] = sx; slot_acc[3 * slot + 2] = sy;
    }
    // ---- 5. unions across the tile's edges -------------------------------------
    // Wave w owns edge w ([0] first row, [1] last row, [2] first col, [3]
    // last col; lane = position along it) and the slot of its lane's cell.
    // For each neighbour relation (the edge, and for waves 0/1 the two
    // corners of the row) the tile arrives at the pair's hand-off word
    // (rel: stamp << 2 | arrived sides, one 64-bit atomic max per arrival);
    // the tile that arrives second finds the other's side bit and performs
    // the pair's unions, reading the first tile's published edge.  A tile
    // arrives only at relations whose cells on its side hold frontier cells,
    // so a pair without frontier cells on both sides is never united, and a
    // pair is united by exactly one of its tiles (memory-side atomics
    // serialise the two arrivals).  Publication (MI355X_MICROARCH.md,
    // inter-workgroup visibility, hand-off row 1): the edge's slot ids are
    // written with sc1 stores by the wave that then arrives, after its own
    // s_waitcnt vmcnt(0); the second tile reads them with sc1 loads after its
    // arrival returned.  Unions are keyed by slot index (dm_uf_unite_idx);
    // k_frontier_resolve folds each set's min label into its root.
    {
      const int side = tid >> 6, pos = lane;
      const int y = side == 0 ? 0 : side == 1 ? 63 : pos;
      const int x = side == 0 || side == 1 ? pos : side == 2 ? 0 : 63;
      int32_t sl = -1;
      if ((s_F[y] >> x) & 1ull) {
        const long long v = base + root_rank(s_root, s_rootpre, r_par[run_of(s_rbase, s_F, y, x)]);
        sl = v < g.slot_per ? (int32_t)(sh0 + v) : -1;
      }
      const uint64_t fb = __ballot(sl >= 0);
      if constexpr (EDGE) {
      // publish only: the edge's slot ids and its stamp (k_frontier_edges
      // reads both after this kernel; the kernel boundary orders them)
      if (fb) {
        border[j * 256 + tid] = sl;
        if (lane == 0) rel[4 * g.NT + 4 * j + side] = stamp;
      }
      } else {
      if (fb) {
        __hip_atomic_store(&border[j * 256 + tid], sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int32_t tx = tile % g.TX, ty = tile / g.TX;
        const bool up = ty > 0, down = ty + 1 < g.TY, left = tx > 0, right = tx + 1 < g.TX;
        // this lane's relation: lane 0 the edge, lanes 1 / 2 the row's corners
        // at x = 0 / x = 63; (pair word, my side bit, neighbour tile)
        int64_t e = -1;
        unsigned long long mine = 0;
        int32_t nb = -1;
        const int64_t NT = g.NT;
        if (lane == 0) {
          if (side == 0 && up) { e = NT + tile - g.TX; mine = 2; nb = tile - g.TX; }
          if (side == 1 && down) { e = NT + tile; mine = 1; nb = tile + g.TX; }
          if (side == 2 && left) { e = tile - 1; mine = 2; nb = tile - 1; }
          if (side == 3 && right) { e = tile; mine = 1; nb = tile + 1; }
        } else if (lane == 1 && (fb & 1ull)) {        // corner x = 0
          if (side == 0 && up && left) { e = 2 * NT + tile - g.TX - 1; mine = 2; nb = tile - g.TX - 1; }
          if (side == 1 && down && left) { e = 3 * NT + tile; mine = 1; nb = tile + g.TX - 1; }
        } else if (lane == 2 && (fb >> 63)) {         // corner x = 63
          if (side == 0 && up && right) { e = 3 * NT + tile - g.TX + 1; mine = 2; nb = tile - g.TX + 1; }
          if (side == 1 && down && right) { e = 2 * NT + tile; mine = 1; nb = tile + g.TX + 1; }
        }
        bool second = false;
        if (e >= 0) {
          const unsigned long long old = __hip_atomic_fetch_max(&rel[e], (stamp << 2) | mine, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
          second = (old >> 2) == stamp && (old & (3ull ^ mine)) != 0ull;
        }
        const uint64_t sec = __ballot(second);
        const int32_t nb0 = __shfl(nb, 0);
        // the edge: cell pos against the neighbour's cells pos-1, pos, pos+1
        // on its facing edge (first row <-> last row, first col <-> last col)
        if (sec & 1ull) {
          const int opp = side ^ 1;
          const int32_t v = __hip_atomic_load(&border[(int64_t)nb0 * 256 + opp * 64 + pos], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
          int32_t sb[3];
          sb[0] = __shfl_up(v, 1);
          sb[1] = v;
          sb[2] = __shfl_down(v, 1);
          if (pos == 0) sb[0] = -1;
          if (pos == 63) sb[2] = -1;
          // skip the pairs the previous lane (previous edge cell) issues
          const int32_t psl = __shfl_up(sl, 1);
          int32_t psb[3];
          for (int q = 0; q < 3; ++q) psb[q] = __shfl_up(sb[q], 1);
          for (int q = 0; q < 3; ++q) {
            const int32_t b = sb[q];
            if (sl < 0 || b < 0) continue;
            bool dup = false;
            for (int r = 0; r < q; ++r) dup |= sb[r] == b;
            if (pos > 0 && psl == sl) dup |= (psb[0] == b) | (psb[1] == b) | (psb[2] == b);
            if (!dup) dm_uf_unite_idx(slot_parent, sl, b, &cnt[CNT_OVERFLOW], kOvUnionFind);
          }
        }
        // the corners: lane 1 unites cell x = 0, lane 2 cell x = 63 of the
        // row with the diagonal neighbour's facing corner cell
        {
          const int32_t c0 = __shfl(sl, 0), c63 = __shfl(sl, 63);
          if (second && lane != 0) {
            const int32_t me = lane == 1 ? c0 : c63;
            // the neighbour's corner cell: upper tiles' last row, lower tiles'
            // first row, at the column facing this one
            const int nrow = side == 0 ? 1 : 0;
            const int ncol = lane == 1 ? 63 : 0;
            const int32_t b = __hip_atomic_load(&border[(int64_t)nb * 256 + nrow * 64 + ncol], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            if (me >= 0 && b >= 0) dm_uf_unite_idx(slot_parent, me, b, &cnt[CNT_OVERFLOW], kOvUnionFind);
          }
        }
      }
      }
    }
    // band edge rows (cross-band merging) and optional dense outputs
    const bool dense = g.want_mask || g.want_labels;
    if (dense || ty0 == 0 || ty0 + DM_TS >= g.R) {
      for (int c = tid; c < DM_TS * DM_TS; c += kFT) {
        const int y = c >> 6, x = c & 63;
        const int32_t gy = ty0 + y, gx = tx0 + x;
        if (gx >= g.W || gy >= g.R) continue;
        const bool edge = gy == 0 || gy == g.R - 1;
        if (!dense && !edge) continue;
        const bool f = (s_F[y] >> x) & 1ull;
        long long sl = -1;
        if (f) {
          sl = base + root_rank(s_root, s_rootpre, r_par[run_of(s_rbase, s_F, y, x)]);
          sl = sl < g.slot_per ? sh0 + sl : -1;
        }
        const int64_t gi = (int64_t)gy * g.W + gx;
        if (g.want_mask) mask[gi] = f;
        if (g.want_labels) cell_slot[gi] = (int32_t)sl;
        if (f) {
          if (gy == 0) edge_slot[gx] = (int32_t)sl;
          if (gy == g.R - 1) edge_slot[g.W + gx] = (int32_t)sl;
        }
      }
    }
    __syncthreads();
    DM_PH(dm_phase_acc_frontier, 7);
  }
  }
  DM_PH_FLUSH(dm_phase_acc_frontier);
}

// ---- one wave per tile ------------------------------------------------------
// k_frontier_tile: each 64-lane wave of a workgroup takes its own listed
// tile (no workgroup barrier anywhere: the four waves run independently),
// lane y holding tile row y as two 64-bit words (free, unknown).  A tile
// needs only a small LDS slice (kRunsFast runs: parent + packed sums), so
// DM_FL_OCC workgroups = 4*DM_FL_OCC tiles per CU are in flight: a C3 pass's
// ~3.3k listed tiles all at once, and an explored map's tiles without
// frontier cells (load, 2 ballots, done) stream at the rate of their loads.
// A tile with more runs than that (noise-like frontiers: random states,
// checkerboards) is listed for k_frontier_tile_big, the 256-thread kernel
// with a whole-tile LDS table, launched right after (same tile-edge
// hand-off: it arrives later than every tile here, so it unites with them).
constexpr int kFW = 4;            // tile-waves per workgroup
constexpr int64_t kDenseRuns = 48;  // runs per frontier tile above which a pass is "dense"
constexpr int64_t kDenseMaxTiles = 4096;  // ... if it has at most this many tiles with frontier cells
// 384 runs (18.7 KB of LDS per 4-wave workgroup) lets 7 workgroups share a
// CU (<= 72 VGPRs): at C5's sparse scans the pass is 28 tile-waves per CU of
// latency chains, not bytes, so occupancy is what moves it (r02 A/B,
// profiles/r02_frontier_occupancy_ab.log: C5 48 beams k_frontier_tile 165 ->
// 135 us, 192 beams tile + big 369 -> 350 us; 256 runs sends too many 1 cm
// tiles to k_frontier_tile_big, 512 runs fits only 6 workgroups)
#ifndef DM_FL_RUNS
#define DM_FL_RUNS 384
#endif
constexpr int kRunsFast = DM_FL_RUNS;  // runs a tile-wave keeps in LDS
#ifndef DM_FL_STRIDED
#define DM_FL_STRIDED 0
#endif
#ifndef DM_FL_OCC
#define DM_FL_OCC 7               // workgroups per CU (LDS 18.7 KB each, <= 72 VGPRs)
#endif

// Orders this wave's LDS accesses across lanes (LDS executes one wave's
// instructions in order; this keeps the compiler from moving them).
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Row gy (band-local; -1 / R are the halo rows) as a pointer to its column 0,
// or nullptr where there is no row ("not unknown").
__device__ inline const int8_t* row_base(const FGeom& g, const int8_t* state, const int8_t* halo, int32_t gy) {
  if (gy >= 0 && gy < g.R) return state + (int64_t)gy * g.W;
  if (gy == -1 && g.has_before) return halo;
  if (gy == g.R && g.has_after) return halo + g.W;
  return nullptr;
}

// Bits of the 4 bytes of w that equal zero, at bit positions 0..3.
__device__ inline uint32_t zero_byte_bits(uint32_t w) {
  uint32_t t = (w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  t = ~(t | w | 0x7F7F7F7Fu);                   // 0x80 in each zero byte
  return (((t >> 7) * 0x00204081u) >> 21) & 0xFu;
}

__device__ inline uint64_t dilate_row(uint64_t U, uint32_t uL, uint32_t uR) {
  return U | (U << 1) | (U >> 1) | (uint64_t)uL | ((uint64_t)uR << 63);
}

// 16 cells (16-B chunk k of tile row gy) as unknown bits | free bits << 16.
__device__ inline uint32_t chunk_bits(const FGeom& g, const int8_t* __restrict__ state,
                                      const int8_t* __restrict__ halo, int32_t tx0, int32_t gy, int k) {
  const int8_t* rb = row_base(g, state, halo, gy);
  if (!rb) return 0u;
  const int32_t x0 = tx0 + 16 * k;
  const int8_t* p = rb + x0;
  uint32_t u = 0u, f = 0u;
  if (x0 + 16 <= g.W && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u |= zero_byte_bits(~wd[j]) << (4 * j);
      f |= zero_byte_bits(wd[j]) << (4 * j);
    }
  } else {
    for (int j = 0; j < 16 && x0 + j < g.W; ++j) {
      u |= (uint32_t)(p[j] == -1) << j;
      f |= (uint32_t)(p[j] == 0) << j;
    }
  }
  if (gy < 0 || gy >= g.R) f = 0u;  // halo rows hold no band cells
  return u | (f << 16);
}

// Unknown bit of cell (x, gy) (0 outside the grid / band + halos).
__device__ inline uint32_t unknown_at(const FGeom& g, const int8_t* __restrict__ state,
                                      const int8_t* __restrict__ halo, int32_t x, int32_t gy) {
  if (x < 0 || x >= g.W) return 0u;
  const int8_t* rb = row_base(g, state, halo, gy);
  return rb && rb[x] == -1 ? 1u : 0u;
}

// The tile's rows, one per lane (lane y: U / Fr = unknown / free bits of tile
// row y, uL / uR = unknown bits of its cells at x = -1 / 64), and for lane 0 /
// lane 63 the unknown bits of rows -1 / 64 (Ue, eL, eR).  The interior loads
// are coalesced: load q, lane l reads the 16-B chunk l % 4 of row 16q + l / 4
// (16 rows x 64 B per wave instruction), then each lane gathers its row's four
// chunks with shuffles.
#ifndef DM_SEEN_HALO
#define DM_SEEN_HALO 1  // 0: every halo cell loaded (A/B builds)
#endif
// unseen (wave-uniform): bit 0 left, 1 right, 2 above, 3 below, 4 above-left,
// 5 above-right, 6 below-left, 7 below-right neighbour tile exists in this
// band and is still all unknown (tile_seen 0): its facing cells are unknown
// without a load (columns past the map's edge excepted).
__device__ inline void tile_rows(const FGeom& g, const int8_t* __restrict__ state, const int8_t* __restrict__ halo,
                                 int32_t tx0, int32_t ty0, int lane, uint32_t unseen, uint64_t& U, uint64_t& Fr,
                                 uint32_t& uL, uint32_t& uR, uint64_t& Ue, uint32_t& eL, uint32_t& eR) {
  uint32_t wq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) wq[q] = chunk_bits(g, state, halo, tx0, ty0 + 16 * q + (lane >> 2), lane & 3);
  // rows -1 (lanes 0-3) and 64 (lanes 4-7), unknown bits only
  uint32_t we = 0u;
  if (lane < 8) {
    if ((unseen >> (lane < 4 ? 2 : 3)) & 1u) {
      const int32_t x0 = tx0 + 16 * (lane & 3);  // the in-map columns of the chunk
      we = x0 >= g.W ? 0u : (x0 + 16 <= g.W ? 0xFFFFu : (1u << (g.W - x0)) - 1u);
    } else {
      we = chunk_bits(g, state, halo, tx0, lane < 4 ? ty0 - 1 : ty0 + DM_TS, lane & 3);
    }
  }
  // column halos of this lane's row; lanes 0 / 63 also the corners
  // (rows past the band's end take the halo row / nothing, as loaded)
  const bool in_band = ty0 + lane < g.R;
  uL = ((unseen & 1u) && in_band) ? 1u : unknown_at(g, state, halo, tx0 - 1, ty0 + lane);
  uR = ((unseen & 2u) && in_band) ? 1u : unknown_at(g, state, halo, tx0 + DM_TS, ty0 + lane);
  eL = 0u;
  eR = 0u;
  if (lane == 0 || lane == 63) {
    const int32_t ey = lane == 0 ? ty0 - 1 : ty0 + DM_TS;
    eL = ((unseen >> (lane == 0 ? 4 : 6)) & 1u) ? 1u : unknown_at(g, state, halo, tx0 - 1, ey);
    eR = ((unseen >> (lane == 0 ? 5 : 7)) & 1u) ? 1u : unknown_at(g, state, halo, tx0 + DM_TS, ey);
  }
  U = 0ull;
  Fr = 0ull;
  Ue = 0ull;
  const int src = (lane & 15) << 2, qsel = lane >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = __shfl(wq[q], src + k);
    const uint32_t sel = qsel == 0 ? t[0] : qsel == 1 ? t[1] : qsel == 2 ? t[2] : t[3];
    U |= (uint64_t)(sel & 0xFFFFu) << (16 * k);
    Fr |= (uint64_t)(sel >> 16) << (16 * k);
    const uint32_t te = __shfl(we, (lane == 63 ? 4 : 0) + k);
    Ue |= (uint64_t)(te & 0xFFFFu) << (16 * k);
  }
}

// Unions of the cells of one of this tile's edges with the neighbour tile's
// facing edge (published slot ids, sc1 loads): lane = position along the
// edge, cell pos against the neighbour's cells pos-1, pos, pos+1.  A lane
// skips the pairs the previous lane (previous edge cell) issues.
[[maybe_unused]] __device__ inline void edge_unions(int32_t sl, const int32_t* border, int32_t nb, int opp, int lane,
                                   int32_t* slot_parent, unsigned long long* flag) {
  const int32_t v = __hip_atomic_load(&border[(int64_t)nb * 256 + opp * 64 + lane], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  int32_t sb[3];
  sb[0] = __shfl_up(v, 1);
  sb[1] = v;
  sb[2] = __shfl_down(v, 1);
  if (lane == 0) sb[0] = -1;
  if (lane == 63) sb[2] = -1;
  const int32_t psl = __shfl_up(sl, 1);
  int32_t psb[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) psb[q] = __shfl_up(sb[q], 1);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int32_t b = sb[q];
    if (sl < 0 || b < 0) continue;
    bool dup = false;
    for (int r = 0; r < q; ++r) dup |= sb[r] == b;
    if (lane > 0 && psl == sl) dup |= (psb[0] == b) | (psb[1] == b) | (psb[2] == b);
    if (!dup) dm_uf_unite_idx(slot_parent, sl, b, flag, kOvUnionFind);
  }
}

// The 64 bits of one fmask row (16 nibble bytes) of one kind: shift 0 the
// free nibbles, 4 the unknown nibbles; each 4-byte word folds to 16 bits.
__device__ inline uint64_t nib_row(uint4 v, int shift) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint64_t m = 0ull;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t x = (w[q] >> shift) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    m |= (uint64_t)x << (16 * q);
  }
  return m;
}

// Frontier bit rows of the listed tiles, one wave per tile (lane y = tile
// row y): F = free & 3x3 dilation of unknown (out-of-grid / missing halo
// cells are "not unknown").  The only kernel of a pass that reads the map:
// with dm_set_overlap the next batch's map update may start right after it,
// while the labelling kernels below (which read only these rows) run on the
// pass stream.  The map is read as the per-tile free / unknown bit rows
// (fmask, kept by the integrate apply): the tile's 1 KB record, and one edge
// word (fedge) of each of its 8 neighbours — 1 KB of coalesced loads plus 8
// uniform 8-byte ones instead of the tile's 4 KB of state bytes plus ~130
// scattered halo lines (or the neighbours' whole records for one byte per row).
// Tiles next to a band halo (sharded maps) read the state bytes and the
// halo rows instead.  Also copies the list length into the pass's counters.
__global__ __launch_bounds__(kFW * 64) void k_frontier_bits(
    FGeom g, const int8_t* __restrict__ state, const int8_t* __restrict__ halo, const uint8_t* __restrict__ fmask,
    const uint64_t* __restrict__ fedge, const uint8_t* __restrict__ tile_seen, const int32_t* __restrict__ ftiles,
    const unsigned long long* __restrict__ ftiles_n, unsigned long long* list_n, uint64_t* __restrict__ fbits,
    unsigned long long* cnt, int use_fmask, int32_t* __restrict__ big_flag, unsigned long long* fsh,
    int32_t* __restrict__ edge_slot, int64_t n_edge, int32_t* __restrict__ slot_parent,
    const unsigned long long* __restrict__ halt, unsigned long long* stamp_word) {
  const int w = threadIdx.x >> 6, lane = __lane_id();
  // the persistent tile list's length: appended only by the map updates on
  // this stream, before and after this kernel, so every workgroup reads the
  // same value; the pass's kernels read this snapshot (list_n)
  const int64_t nft = (int64_t)*ftiles_n;
  // the pass's resets (every workgroup a share): counters, slot shards, edge
  // slots, and every slot as its own root a launch ahead of the tile
  // kernels' in-kernel unions (their CASes and possibly stale finds then
  // only ever see a slot as a root or as hooked, dm_uf.h)
  {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // slots, clusters, overflow (kOvPipeline while the handle's sticky
    // hand-off error is set: the map misses a batch, DM_ERR_PIPELINE)
    if (i0 < 3) cnt[CNT_SLOTS + i0] = (i0 == 2 && *halt) ? kOvPipeline : 0ull;
    if (i0 == 3) cnt[CNT_BIG] = 0ull;
    if (i0 == 4) {  // this pass's stamp: every pass's bits run on the handle's stream, one after the other
      const unsigned long long st = *stamp_word + 1;
      *stamp_word = st;
      cnt[CNT_STAMP] = st;
    }
    if (i0 == 5) {
      *list_n = (unsigned long long)nft;
      cnt[CNT_FL0] = (unsigned long long)nft;
    }
    if (i0 < kShards * kShardWords) fsh[i0] = 0ull;
    for (int64_t i = i0; i < n_edge; i += stride) edge_slot[i] = -1;
    for (int64_t i = i0; i < g.slot_cap; i += stride) slot_parent[i] = (int32_t)i;
  }
  // four consecutive listed tiles per workgroup: horizontal neighbours share
  // the 128-byte lines of their rows and halo columns.  (Consecutive chunks
  // on one XCD, for its L2, cut C3's bytes 28 -> 20 MB per launch but made
  // this kernel and the step slower: DESIGN.md §3.2)
  for (int64_t jj = (int64_t)blockIdx.x * kFW + w; jj < nft; jj += (int64_t)gridDim.x * kFW) {
    const int32_t tile = __builtin_amdgcn_readfirstlane(ftiles[jj]);
    const int32_t tx = tile % g.TX, ty = tile / g.TX;
    const int32_t tx0 = tx * DM_TS, ty0 = ty * DM_TS;  // ty0 band-local
    uint64_t U, Fr, Ue;
    uint32_t uL, uR, eL, eR;
    if (!use_fmask || (ty == 0 && g.has_before) || (ty == g.TY - 1 && g.has_after)) {
      // neighbour tiles of this band that are still all unknown (uniform loads);
      // relies on the tile_seen invariant of dm_internal.h (every state writer
      // sets the flag or is followed by k_recount)
      uint32_t unseen = 0u;
      if (DM_SEEN_HALO) {
        const bool l = tx > 0, r = tx + 1 < g.TX, u = ty > 0, d = ty + 1 < g.TY;
        const int64_t t = tile;
        if (l && !tile_seen[t - 1]) unseen |= 1u;
        if (r && !tile_seen[t + 1]) unseen |= 2u;
        if (u && !tile_seen[t - g.TX]) unseen |= 4u;
        if (d && !tile_seen[t + g.TX]) unseen |= 8u;
        if (u && l && !tile_seen[t - g.TX - 1]) unseen |= 16u;
        if (u && r && !tile_seen[t - g.TX + 1]) unseen |= 32u;
        if (d && l && !tile_seen[t + g.TX - 1]) unseen |= 64u;
        if (d && r && !tile_seen[t + g.TX + 1]) unseen |= 128u;
      }
      tile_rows(g, state, halo, tx0, ty0, lane, unseen, U, Fr, uL, uR, Ue, eL, eR);
    } else {
      // fmask: [tile][row][16] nibble bytes (free | unknown << 4)
      const uint8_t* rec = fmask + (int64_t)tile * (DM_TS * 16);
      const uint4 v = *reinterpret_cast<const uint4*>(rec + lane * 16);
      Fr = nib_row(v, 0);
      U = nib_row(v, 4);
      // the neighbours from their edge words (fedge: unknown column 0,
      // column 63, row 0, row 63): column -1 is the left tile's column 63,
      // column 64 the right tile's column 0
      uL = tx > 0 ? (uint32_t)((fedge[(int64_t)(tile - 1) * 4 + 1] >> lane) & 1ull) : 0u;
      uR = tx + 1 < g.TX ? (uint32_t)((fedge[(int64_t)(tile + 1) * 4] >> lane) & 1ull) : 0u;
      // lane 0: row -1 (the tile above, its row 63); lane 63: row 64 (the
      // tile below, its row 0); eL / eR the diagonal neighbours' corner cells
      Ue = 0ull;
      eL = 0u;
      eR = 0u;
      if ((lane == 0 && ty > 0) || (lane == 63 && ty + 1 < g.TY)) {
        const int64_t nt = (int64_t)tile + (lane == 0 ? -(int64_t)g.TX : (int64_t)g.TX);
        const int wr = lane == 0 ? 3 : 2;
        Ue = fedge[nt * 4 + wr];
        if (tx > 0) eL = (uint32_t)(fedge[(nt - 1) * 4 + wr] >> 63);
        if (tx + 1 < g.TX) eR = (uint32_t)(fedge[(nt + 1) * 4 + wr] & 1ull);
      }
    }
    const uint64_t h = dilate_row(U, uL, uR);
    const uint64_t he = dilate_row(Ue, eL, eR);
    uint64_t hu = __shfl_up(h, 1);
    uint64_t hd = __shfl_down(h, 1);
    if (lane == 0) hu = he;
    if (lane == 63) hd = he;
    const uint64_t F = Fr & (h | hu | hd);
    fbits[jj * DM_TS + lane] = F;
    // a tile with more runs than a tile-wave keeps is flagged for
    // k_frontier_tile_big, which runs beside the wave kernel:
    // a plain store per listed tile (an append to one shared list was a
    // same-address atomic per run-rich tile: +90 us at C5's 192 beams)
    if (big_flag) {
      int nr = __popcll(run_starts(F));
      for (int o = 32; o > 0; o >>= 1) nr += __shfl_xor(nr, o);
      if (lane == 0) big_flag[jj] = nr > kRunsFast ? 1 : 0;
    }
  }
}

template <bool EDGE>
__global__ __launch_bounds__(kFW * 64, DM_FL_OCC) void k_frontier_tile(
    FGeom g, const uint64_t* __restrict__ fbits,
    const int32_t* __restrict__ ftiles, const unsigned long long* __restrict__ list_n,
    int32_t* border, unsigned long long* rel,
    long long* __restrict__ slot_label, int32_t* slot_parent,
    long long* __restrict__ slot_own, long long* __restrict__ slot_acc,
    uint8_t* __restrict__ mask, int32_t* __restrict__ cell_slot, int32_t* __restrict__ edge_slot,
    unsigned long long* cnt, unsigned long long* fsh, int32_t* __restrict__ big_list) {
  const unsigned long long stamp = cnt[CNT_STAMP];  // this pass's (k_frontier_bits)
  __shared__ int32_t s_par[kFW][kRunsFast];
  __shared__ unsigned long long s_acc[kFW][kRunsFast];  // size << 40 | sum_x << 20 | sum_y (tile-local)
  __shared__ uint64_t s_rootw[kFW][kRunsFast / 64];     // root-run bits
  __shared__ int32_t s_rootpre[kFW][kRunsFast / 64];    // roots before each word
  const int w = threadIdx.x >> 6, lane = __lane_id();
  int32_t* par = s_par[w];
  unsigned long long* acc = s_acc[w];
  uint64_t* rootw = s_rootw[w];
  int32_t* rootpre = s_rootpre[w];
  const int64_t nft = (int64_t)*list_n;
  // list position of this wave's first tile: the four waves of a workgroup
  // take four consecutive listed tiles (horizontal neighbours share the
  // 128-byte lines of their rows and their halo columns: measured 129 vs
  // 190 us on the explored C3 map against tiles a quarter list apart)
#if DM_FL_STRIDED
  const int64_t wid = (int64_t)w * gridDim.x + blockIdx.x;
#else
  const int64_t wid = (int64_t)blockIdx.x * kFW + w;
#endif
  const int shard = (int)(wid % kShards);
  const long long sh0 = (long long)shard * g.slot_per;
  const bool dense = g.want_mask || g.want_labels;
  DM_PH_INIT();
  for (int64_t jj = wid; jj < nft; jj += (int64_t)gridDim.x * kFW) {
    DM_PH(dm_phase_acc_ftile, 9);
    const int32_t tile = __builtin_amdgcn_readfirstlane(ftiles[jj]);
    // ---- 1-2. frontier bit rows (k_frontier_bits): lane y = tile row y ----------
    const uint64_t F = fbits[jj * DM_TS + lane];
    DM_PH_COUNT(dm_phase_acc_ftile, 16, 1);
    const int32_t tx = tile % g.TX, ty = tile / g.TX;
    const int32_t tx0 = tx * DM_TS, ty0 = ty * DM_TS;  // ty0 band-local
    DM_PH(dm_phase_acc_ftile, 0);
    if (__ballot(F != 0ull) == 0ull) continue;  // no frontier cell: nothing to publish
    // ---- 3. runs of set bits, numbered row-major ---------------------------
    const uint64_t st = run_starts(F);
    const int c = __popcll(st);
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const int rbase = incl - c;
    const int nruns = __shfl(incl, 63);
    if (lane == 0) {  // statistics for the next pass's kernel choice (shard sums)
      atomicAdd(&fsh[shard * kShardWords + SH_RUNS], (unsigned long long)nruns);
      atomicAdd(&fsh[shard * kShardWords + SH_FTF], 1ull);
    }
    if (nruns > kRunsFast) {  // too many for this wave's LDS: flagged for the big kernel by k_frontier_bits
      if (lane == 0) atomicAdd(&fsh[shard * kShardWords + SH_BIG], 1ull);
      continue;
    }
    for (int r = lane; r < nruns; r += 64) {
      par[r] = r;
      acc[r] = 0ull;
    }
    wave_lds_sync();
    DM_PH(dm_phase_acc_ftile, 1);
    DM_PH_COUNT(dm_phase_acc_ftile, 17, 1);
    DM_PH_COUNT(dm_phase_acc_ftile, 18, nruns);
    // ---- 4. union every run with the runs above it (extended by a cell) ------
    const uint64_t Fa = __shfl_up(F, 1);
    const uint64_t sta = __shfl_up(st, 1);
    const int rba = __shfl_up(rbase, 1);
    if (lane > 0 && Fa) {
      uint64_t s_ = st;
      int r = rbase;
      while (s_) {
        const int s0 = __ffsll((unsigned long long)s_) - 1;
        const int e0 = run_end(F, s0);
        const int lo = s0 > 0 ? s0 - 1 : 0, hi = e0 < 63 ? e0 + 1 : 63;
        uint64_t P = Fa & upto_mask(hi) & ~(lo > 0 ? upto_mask(lo - 1) : 0ull);
        while (P) {
          const int q = __ffsll((unsigned long long)P) - 1;
          lds_unite(par, r, rba + __popcll(sta & upto_mask(q)) - 1);
          const uint64_t rest = ~(Fa >> q);
          const int len = rest ? __ffsll((unsigned long long)rest) - 1 : 64 - q;
          P &= ~upto_mask(q + len - 1);
        }
        ++r;
        s_ &= s_ - 1;
      }
    }
    wave_lds_sync();
    DM_PH(dm_phase_acc_ftile, 2);
    // ---- 5. compress; root bits; component id = rank of the root run ---------
    for (int r0 = 0; r0 < nruns; r0 += 64) {
      const int r = r0 + lane;
      int32_t x = r;
      if (r < nruns) {
        int32_t p = ((volatile int32_t*)par)[r];
        while (p != x) {
          x = p;
          p = ((volatile int32_t*)par)[x];
        }
        par[r] = x;
      }
      const uint64_t rb = __ballot(r < nruns && x == r);
      if (lane == 0) rootw[r0 >> 6] = rb;
    }
    wave_lds_sync();
    const int nw = (nruns + 63) >> 6;
    int ncomp;
    {
      const int pc = lane < nw ? __popcll(rootw[lane]) : 0;
      int inc2 = pc;
#pragma unroll
      for (int d = 1; d < 8; d <<= 1) {
        const int v = __shfl_up(inc2, d);
        if (lane >= d) inc2 += v;
      }
      if (lane < nw) rootpre[lane] = inc2 - pc;
      ncomp = __shfl(inc2, 7);
    }
    DM_PH(dm_phase_acc_ftile, 3);
    // ---- 6. per-component sums, in the root run's acc word -------------------
    {
      uint64_t s_ = st;
      int r = rbase;
      while (s_) {
        const int s0 = __ffsll((unsigned long long)s_) - 1;
        const int e0 = run_end(F, s0);
        const unsigned long long len = (unsigned long long)(e0 - s0 + 1);
        atomicAdd(&acc[par[r]], (len << 40) | ((unsigned long long)((s0 + e0) * (e0 - s0 + 1) / 2) << 20) |
                                    (unsigned long long)(lane * (e0 - s0 + 1)));
        ++r;
        s_ &= s_ - 1;
      }
    }
    wave_lds_sync();
    DM_PH(dm_phase_acc_ftile, 4);
    // ---- 7. slots: one per component from this wave's shard region -----------
    unsigned long long sb0 = 0ull;
    if (lane == 0) sb0 = atomicAdd(&fsh[shard * kShardWords + SH_SLOT], (unsigned long long)ncomp);
    const long long base = (long long)__shfl(sb0, 0);
    auto slot_of_run = [&](int r) -> int32_t {
      const int root = par[r];
      const long long v = base + rootpre[root >> 6] + __popcll(rootw[root >> 6] & ((1ull << (root & 63)) - 1ull));
      return v < g.slot_per ? (int32_t)(sh0 + v) : -1;
    };
    {
      uint64_t s_ = st;
      int r = rbase;
      while (s_) {
        const int s0 = __ffsll((unsigned long long)s_) - 1;
        if (par[r] == r) {
          const int32_t slot = slot_of_run(r);
          if (slot < 0) {
            atomicOr(&cnt[CNT_OVERFLOW], kOvSlots);
          } else {
            const unsigned long long a = acc[r];
            const long long sz = (long long)(a >> 40);
            const long long sx = sz * tx0 + (long long)((a >> 20) & 0xFFFFFull);
            const long long sy = sz * ((long long)g.row0 + ty0) + (long long)(a & 0xFFFFFull);
            slot_label[slot] = ((long long)g.row0 + ty0 + lane) * g.W + tx0 + s0;
            slot_own[3 * (int64_t)slot + 0] = sz;
            slot_own[3 * (int64_t)slot + 1] = sx;
            slot_own[3 * (int64_t)slot + 2] = sy;
            slot_acc[3 * (int64_t)slot + 0] = sz;
            slot_acc[3 * (int64_t)slot + 1] = sx;
            slot_acc[3 * (int64_t)slot + 2] = sy;
          }
        }
        ++r;
        s_ &= s_ - 1;
      }
    }
    DM_PH(dm_phase_acc_ftile, 5);
    // ---- 8. edges: publish, arrive, unite -------------------
    // sides [0] first row, [1] last row, [2] first col, [3] last col; lane =
    // position along the side.  The published slot ids are sc1 stores drained
    // by this wave before it arrives at any pair word (MI355X_MICROARCH.md,
    // inter-workgroup visibility, hand-off row 1); the second tile of a pair
    // reads them with sc1 loads after its own arrival returned.
    int32_t sl[4];
    {
      const uint64_t F0 = __shfl(F, 0), F63 = __shfl(F, 63);
      const uint64_t st0 = __shfl(st, 0), st63 = __shfl(st, 63);
      const int rb0 = __shfl(rbase, 0), rb63 = __shfl(rbase, 63);
      sl[0] = ((F0 >> lane) & 1ull) ? slot_of_run(rb0 + __popcll(st0 & upto_mask(lane)) - 1) : -1;
      sl[1] = ((F63 >> lane) & 1ull) ? slot_of_run(rb63 + __popcll(st63 & upto_mask(lane)) - 1) : -1;
      sl[2] = (F & 1ull) ? slot_of_run(rbase) : -1;  // column 0 of row `lane`: its first run
      sl[3] = (F >> 63) ? slot_of_run(rbase + c - 1) : -1;  // column 63: its last run
    }
    uint64_t fb[4];
#pragma unroll
    for (int sd = 0; sd < 4; ++sd) fb[sd] = __ballot(sl[sd] >= 0);
    if constexpr (EDGE) {
    // publish only (k_frontier_edges unites the pairs after this kernel)
#pragma unroll
    for (int sd = 0; sd < 4; ++sd)
      if (fb[sd]) {
        border[(int64_t)tile * 256 + sd * 64 + lane] = sl[sd];
        if (lane == 0) rel[4 * g.NT + 4 * (int64_t)tile + sd] = stamp;
      }
    DM_PH(dm_phase_acc_ftile, 6);
    } else {
#pragma unroll
    for (int sd = 0; sd < 4; ++sd)
      if (fb[sd]) __hip_atomic_store(&border[(int64_t)tile * 256 + sd * 64 + lane], sl[sd], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    if (fb[0] | fb[1] | fb[2] | fb[3]) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      DM_PH(dm_phase_acc_ftile, 6);
      const bool up = ty > 0, down = ty + 1 < g.TY, left = tx > 0, right = tx + 1 < g.TX;
      const int64_t NT = g.NT;
      // lane i arrives at relation i: 0 up, 1 down, 2 left, 3 right edge;
      // 4 up-left, 5 up-right, 6 down-left, 7 down-right corner
      int64_t e = -1;
      unsigned long long mine = 0ull;
      int32_t nb = -1;
      if (lane == 0 && fb[0] && up) { e = NT + tile - g.TX; mine = 2; nb = tile - g.TX; }
      if (lane == 1 && fb[1] && down) { e = NT + tile; mine = 1; nb = tile + g.TX; }
      if (lane == 2 && fb[2] && left) { e = tile - 1; mine = 2; nb = tile - 1; }
      if (lane == 3 && fb[3] && right) { e = tile; mine = 1; nb = tile + 1; }
      if (lane == 4 && (fb[0] & 1ull) && up && left) { e = 2 * NT + tile - g.TX - 1; mine = 2; nb = tile - g.TX - 1; }
      if (lane == 5 && (fb[0] >> 63) && up && right) { e = 3 * NT + tile - g.TX + 1; mine = 2; nb = tile - g.TX + 1; }
      if (lane == 6 && (fb[1] & 1ull) && down && left) { e = 3 * NT + tile; mine = 1; nb = tile + g.TX - 1; }
      if (lane == 7 && (fb[1] >> 63) && down && right) { e = 2 * NT + tile; mine = 1; nb = tile + g.TX + 1; }
      bool second = false;
      if (e >= 0) {
        const unsigned long long old = __hip_atomic_fetch_max(&rel[e], (stamp << 2) | mine, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
        second = (old >> 2) == stamp && (old & (3ull ^ mine)) != 0ull;
      }
      const uint64_t sec = __ballot(second);
      DM_PH(dm_phase_acc_ftile, 7);
      unsigned long long* uflag = &cnt[CNT_OVERFLOW];
#pragma unroll
      for (int sd = 0; sd < 4; ++sd)
        if ((sec >> sd) & 1ull) edge_unions(sl[sd], border, __shfl(nb, sd), sd ^ 1, lane, slot_parent, uflag);
      // corners: the diagonal neighbour's facing corner cell (upper tiles:
      // its last row, lower tiles: its first row)
      const int32_t c00 = __shfl(sl[0], 0), c630 = __shfl(sl[0], 63);
      const int32_t c063 = __shfl(sl[1], 0), c6363 = __shfl(sl[1], 63);
      if (second && lane >= 4) {
        const int32_t me = lane == 4 ? c00 : lane == 5 ? c630 : lane == 6 ? c063 : c6363;
        const int nrow = lane < 6 ? 1 : 0;
        const int ncol = (lane == 4 || lane == 6) ? 63 : 0;
        const int32_t b = __hip_atomic_load(&border[(int64_t)nb * 256 + nrow * 64 + ncol], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        if (b >= 0) dm_uf_unite_idx(slot_parent, me, b, uflag, kOvUnionFind);
      }
      DM_PH(dm_phase_acc_ftile, 8);
    }
    }
    // ---- 9. band edge rows (cross-band merging) and optional dense outputs ---
    const int32_t gy = ty0 + lane;
    if (gy < g.R && (dense || gy == 0 || gy == g.R - 1)) {
      uint64_t s_ = F;
      while (s_) {
        const int x = __ffsll((unsigned long long)s_) - 1;
        s_ &= s_ - 1;
        const int32_t gx = tx0 + x;
        const int32_t sv = slot_of_run(rbase + __popcll(st & upto_mask(x)) - 1);
        const int64_t gi = (int64_t)gy * g.W + gx;
        if (g.want_mask) mask[gi] = 1;
        if (g.want_labels) cell_slot[gi] = sv;
        if (gy == 0) edge_slot[gx] = sv;
        if (gy == g.R - 1) edge_slot[g.W + gx] = sv;
      }
    }
    DM_PH(dm_phase_acc_ftile, 10);
  }
  DM_PHW_FLUSH(dm_phase_acc_ftile);
}

// Unions across tile edges, after the tile kernels of a pass (DM_EDGE_KERNEL).
// One wave per listed tile, which owns the relations to its right, lower,
// lower-left and lower-right neighbours (every adjacent tile pair has exactly
// one owner).  A relation is united only where both tiles published the
// facing edge in THIS pass (rel[4 * tile + side] == stamp: the tile has
// frontier cells on that edge; a stale record of an earlier pass is never
// read).  The right and lower edges: lane = position along the edge, its
// cell against the neighbour's cells pos-1, pos, pos+1 (edge_unions); the
// corners: one lane each.  Unions are keyed by slot index, as in the tile
// kernels (dm_uf_unite_idx); k_frontier_resolve folds the min labels.  In
// the tile kernels the same unions waited behind the border stores' drain,
// a returning hand-off atomic and the neighbour's border loads (C3: 35 % of
// k_frontier_tile_big's workgroup time, profiles/r06_phase_c3.log); here
// they are thousands of short independent waves.
#ifndef DM_EDGE_WAVES
#define DM_EDGE_WAVES 1  // waves per listed tile in k_frontier_edges (2: one per relation, A/B)
#endif
__global__ __launch_bounds__(kFW * 64) void k_frontier_edges(FGeom g, const int32_t* __restrict__ ftiles,
                                                             const unsigned long long* __restrict__ list_n,
                                                             const int32_t* __restrict__ border,
                                                             const unsigned long long* __restrict__ rel,
                                                             int32_t* slot_parent, unsigned long long* cnt) {
  constexpr int kRel = DM_EDGE_WAVES == 2 ? 1 : 2;  // relations per wave
  const unsigned long long stamp = cnt[CNT_STAMP];
  const int w = threadIdx.x >> 6, lane = __lane_id();
  const int64_t nft = (int64_t)*list_n;
  unsigned long long* uflag = &cnt[CNT_OVERFLOW];
  const unsigned long long* est = rel + 4 * g.NT;  // the per-edge stamps (EDGE tile kernels)
  __shared__ int2 s_pairs[kFW][kRel * 4 * 64];  // a wave's pairs (<= 3 per lane + a corner, per relation)
  // relation 0: the tile's right edge (and both lower corners, on lanes 0 /
  // 63); relation 1: its lower edge.  One wave per listed tile takes both
  // (DM_EDGE_WAVES 1), or wave 2j + r relation r of tile j (2)
  const int64_t nv = DM_EDGE_WAVES == 2 ? 2 * nft : nft;
  for (int64_t v = (int64_t)blockIdx.x * kFW + w; v < nv; v += (int64_t)gridDim.x * kFW) {
    const int64_t tile = __builtin_amdgcn_readfirstlane(ftiles[DM_EDGE_WAVES == 2 ? v >> 1 : v]);
    const int32_t tx = (int32_t)(tile % g.TX), ty = (int32_t)(tile / g.TX);
    const bool right = tx + 1 < g.TX, down = ty + 1 < g.TY, left = tx > 0;
    // everything in ONE round of loads after the tile id: the stamps that
    // say which records are this pass's, and the records themselves
    // (speculative: a record of an earlier pass is read but not used)
    unsigned long long m_me[kRel], m_nb[kRel];
    int32_t sl[kRel], v_nb[kRel];
    bool has_nb[kRel];
#pragma unroll
    for (int q = 0; q < kRel; ++q) {
      const int rk = DM_EDGE_WAVES == 2 ? (int)(v & 1) : q;
      const int64_t nb = rk == 0 ? (right ? tile + 1 : tile) : (down ? tile + g.TX : tile);
      const int my_side = rk == 0 ? 3 : 1, nb_side = rk == 0 ? 2 : 0;
      has_nb[q] = rk == 0 ? right : down;
      m_me[q] = est[4 * tile + my_side];
      m_nb[q] = est[4 * nb + nb_side];
      sl[q] = border[tile * 256 + my_side * 64 + lane];
      v_nb[q] = border[nb * 256 + nb_side * 64 + lane];
    }
    // corners (with relation 0, lanes 0 / 63): this tile's (63, 0) / (63, 63)
    // against the lower-left tile's (0, 63) / the lower-right tile's (0, 0)
    const bool rel0 = DM_EDGE_WAVES == 2 ? (v & 1) == 0 : true;
    const bool corner_lane = rel0 && down && ((lane == 0 && left) || (lane == 63 && right));
    const int64_t dn = lane == 0 ? tile + g.TX - 1 : tile + g.TX + 1;
    unsigned long long m_row = 0ull, m_dn = 0ull;
    int32_t c_me = -1, c_dn = -1;
    if (corner_lane) {
      m_row = est[4 * tile + 1];
      m_dn = est[4 * dn + 0];
      c_me = border[tile * 256 + 64 + lane];
      c_dn = border[dn * 256 + (lane == 0 ? 63 : 0)];
    }
    // each lane's distinct pairs (cell pos against the neighbour's pos-1,
    // pos, pos+1, minus those the previous lane issues), compacted into the
    // wave's list, so each lane then runs ONE union at a time instead of up
    // to three (or six) in turn
    int2* lst = s_pairs[w];
    int total = 0;
#pragma unroll
    for (int q = 0; q < kRel; ++q) {
      int32_t sb[3] = {-1, -1, -1};
      bool keep[3] = {false, false, false};
      if (has_nb[q] && m_me[q] == stamp && m_nb[q] == stamp) {  // uniform
        sb[0] = __shfl_up(v_nb[q], 1);
        sb[1] = v_nb[q];
        sb[2] = __shfl_down(v_nb[q], 1);
        if (lane == 0) sb[0] = -1;
        if (lane == 63) sb[2] = -1;
        const int32_t psl = __shfl_up(sl[q], 1);
        int32_t psb[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) psb[k] = __shfl_up(sb[k], 1);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int32_t b = sb[k];
          bool dup = sl[q] < 0 || b < 0;
#pragma unroll
          for (int r = 0; r < k; ++r) dup |= sb[r] == b;
          if (lane > 0 && psl == sl[q]) dup |= (psb[0] == b) | (psb[1] == b) | (psb[2] == b);
          keep[k] = !dup;
        }
      }
      const bool kc = q == 0 && corner_lane && m_row == stamp && m_dn == stamp && c_me >= 0 && c_dn >= 0;
      const int np = (int)keep[0] + (int)keep[1] + (int)keep[2] + (int)kc;
      int incl = np;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
      int at = total + incl - np;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (keep[k]) lst[at++] = make_int2(sl[q], sb[k]);
      if (kc) lst[at] = make_int2(c_me, c_dn);
      total += __shfl(incl, 63);
    }
    if (total == 0) continue;
    wave_lds_sync();
    for (int i = lane; i < total; i += 64) {
      const int2 pr = lst[i];
      EDGE_UNITE(slot_parent, pr.x, pr.y, uflag, kOvUnionFind);
    }
    wave_lds_sync();
  }
}

// Slot s is in use iff its offset inside its shard region is below that
// shard's allocation count.  The slot loops walk only the used part of the
// regions: index v in [0, kShards * span) is offset v % span of shard
// v / span, with span = the fullest shard's count rounded up to a wave (so a
// wave stays in one shard), instead of all slot_cap slots (4 per map tile).
// Returns span (0: no slots in use).
__device__ inline int64_t load_shard_counts(const FGeom& g, const unsigned long long* fsh, int64_t* s_n) {
  __shared__ int64_t s_span;
  if (threadIdx.x < kShards)
    s_n[threadIdx.x] = min((int64_t)fsh[threadIdx.x * kShardWords + SH_SLOT], g.slot_per);
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t m = 0;
    for (int i = 0; i < kShards; ++i) m = max(m, s_n[i]);
    s_span = (m + 63) & ~(int64_t)63;
  }
  __syncthreads();
  return s_span;
}

// Slot of loop index v (see load_shard_counts) and whether it is in use.
__device__ inline int64_t slot_at(const FGeom& g, const int64_t* s_n, int64_t span, int64_t v, bool* used) {
  const int64_t sh = v / span, off = v - sh * span;
  *used = off < s_n[sh];
  return sh * g.slot_per + off;
}

// Roots, and every non-root slot's sums and label folded into its root: the
// set's size / sum_x / sum_y add up, its label is the min over its slots
// (SPEC a9: the tile-edge unions hook by slot index, so the root slot is not
// the min-label one).  A component spread over many tiles (a robot's star of
// long thin rays on a 1 cm map) has thousands of slots: one global atomic
// each would queue them on the same four addresses.  The values are first
// combined per workgroup in an LDS table keyed by root (64-bit LDS atomics),
// then flushed with one global atomic per (workgroup, root, field); a root
// that finds no LDS entry within kRootProbe probes goes straight to global
// memory.  The min label lands in slot_label[root] (only roots' entries are
// written; a non-root's own label is read once, never changed).
constexpr int kRootHash = 512;
constexpr int kRootProbe = 8;

__device__ inline void add_to_root(long long* slot_acc, long long* slot_label, int32_t r, const long long* v,
                                   long long lab) {
  for (int f = 0; f < 3; ++f)
    atomicAdd((unsigned long long*)&slot_acc[3 * (int64_t)r + f], (unsigned long long)v[f]);
  atomicMin(&slot_label[r], lab);
}

__global__ __launch_bounds__(256) void k_frontier_resolve(FGeom g, const int32_t* __restrict__ slot_parent,
                                                          int32_t* __restrict__ slot_root,
                                                          const long long* __restrict__ slot_own,
                                                          long long* slot_acc,
                                                          const unsigned long long* fsh, int fuse,
                                                          long long* slot_label,
                                                          long long* __restrict__ clusters,
                                                          int32_t* __restrict__ slot_k,
                                                          unsigned long long* cnt) {
  __shared__ int64_t s_n[kShards];
  __shared__ int32_t hkey[kRootHash];
  __shared__ unsigned long long hacc[3][kRootHash];
  __shared__ long long hmin[kRootHash];
  for (int e = threadIdx.x; e < kRootHash; e += blockDim.x) {
    hkey[e] = -1;
    hacc[0][e] = hacc[1][e] = hacc[2][e] = 0;
    hmin[e] = 0x7FFFFFFFFFFFFFFFll;
  }
  const int64_t span = load_shard_counts(g, fsh, s_n);  // (its barriers also order the table init)
  const int lane = __lane_id();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // wave-aligned (the fused compaction below allocates per wave)
  for (int64_t v0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); v0 < kShards * span; v0 += stride) {
    bool used;
    const int64_t s = slot_at(g, s_n, span, v0 + lane, &used);
    const int32_t r = used ? dm_uf_root(slot_parent, (int32_t)s, &cnt[CNT_OVERFLOW], kOvUnionFind) : -1;
    if (used) slot_root[s] = r;
    if (fuse) {
      // min_size <= 1: every root is a cluster, so k_frontier_compact's
      // work happens here; its label and sums are not final yet (other
      // workgroups still fold into the root), so the record holds -(slot + 1)
      // and the sort kernel reads them by slot (record_vals)
      const bool root = used && r == (int32_t)s;
      const unsigned long long bal = __ballot(root);
      if (bal) {
        const int lead = __ffsll(bal) - 1;
        unsigned long long k0 = 0;
        if (lane == lead) k0 = atomicAdd(&cnt[CNT_CLUSTERS], (unsigned long long)__popcll(bal));
        k0 = __shfl(k0, lead);
        const unsigned long long k = k0 + __popcll(bal & ((1ull << lane) - 1));
        if (root && (int64_t)k < g.clu_cap) {
          slot_k[s] = (int32_t)k;
          clusters[4 * k + 0] = -1;
          clusters[4 * k + 1] = -(long long)s - 1;
        }
      }
    }
    if (!used || r == (int32_t)s) continue;
    const long long v[3] = {slot_own[3 * s + 0], slot_own[3 * s + 1], slot_own[3 * s + 2]};
    const long long lab = slot_label[s];
    uint32_t h = ((uint32_t)r * 2654435761u) >> 23;  // 9 bits
    bool done = false;
    for (int p = 0; p < kRootProbe && !done; ++p, h = (h + 1) & (kRootHash - 1)) {
      const int32_t k = atomicCAS(&hkey[h], -1, r);
      if (k == -1 || k == r) {
        for (int f = 0; f < 3; ++f) atomicAdd(&hacc[f][h], (unsigned long long)v[f]);
        atomicMin(&hmin[h], lab);
        done = true;
      }
    }
    if (!done) add_to_root(slot_acc, slot_label, r, v, lab);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kRootHash; e += blockDim.x) {
    const int32_t r = hkey[e];
    if (r < 0) continue;
    const long long v[3] = {(long long)hacc[0][e], (long long)hacc[1][e], (long long)hacc[2][e]};
    add_to_root(slot_acc, slot_label, r, v, hmin[e]);
  }
}

// Roots of size >= min_size become cluster records; one counter atomic per
// wave (ballot + popcount) instead of one per cluster.
__global__ __launch_bounds__(256) void k_frontier_compact(FGeom g, const int32_t* __restrict__ slot_root,
                                                          const long long* __restrict__ slot_label,
                                                          const long long* __restrict__ slot_acc,
                                                          long long* __restrict__ clusters,
                                                          int32_t* __restrict__ slot_k,
                                                          unsigned long long* cnt,
                                                          const unsigned long long* fsh) {
  __shared__ int64_t s_n[kShards];
  const int64_t span = load_shard_counts(g, fsh, s_n);
  const int lane = __lane_id();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); v0 < kShards * span; v0 += stride) {
    bool used;
    const int64_t s = slot_at(g, s_n, span, v0 + lane, &used);
    bool keep = used && slot_root[s] == (int32_t)s;
    const long long sz = keep ? slot_acc[3 * s] : 0;
    keep = keep && sz >= g.min_size;
    const unsigned long long bal = __ballot(keep);
    if (!bal) continue;
    unsigned long long k0 = 0;
    if (lane == __ffsll(bal) - 1) k0 = atomicAdd(&cnt[CNT_CLUSTERS], (unsigned long long)__popcll(bal));
    k0 = __shfl(k0, __ffsll(bal) - 1);
    if (!keep) continue;
    const unsigned long long k = k0 + __popcll(bal & ((1ull << lane) - 1));
    if ((int64_t)k >= g.clu_cap) continue;
    slot_k[s] = (int32_t)k;
    clusters[4 * k + 0] = slot_label[s];
    clusters[4 * k + 1] = sz;
    clusters[4 * k + 2] = slot_acc[3 * s + 1];
    clusters[4 * k + 3] = slot_acc[3 * s + 2];
  }
}

// Block 0 of the sort kernel (the pipeline's last kernel: every counter is
// final) sets the sorted flag and writes the readback header: the counters,
// then the fullest slot shard; the host reads it together with the first
// sorted records from the mapped buffer in ONE step.
__device__ inline void write_rb_header(int64_t K, int64_t cap, unsigned long long* sorted,
                                       const unsigned long long* __restrict__ cnt, int ncnt,
                                       int sorted_idx, const unsigned long long* __restrict__ fsh,
                                       dm_raw_record* host_out) {
  const int tid = threadIdx.x;
  if (tid == 0) *sorted = K <= cap ? 1ull : 0ull;
  if (!host_out) return;
  unsigned long long* header = dm_rb_header(host_out);
  if (tid < ncnt) header[tid] = tid == sorted_idx ? (K <= cap ? 1ull : 0ull) : cnt[tid];
  if (tid == ncnt && fsh) {
    unsigned long long most = 0, runs = 0, ftf = 0, big = 0;
    for (int i = 0; i < kShards; ++i) {
      most = max(most, fsh[i * kShardWords + SH_SLOT]);
      runs += fsh[i * kShardWords + SH_RUNS];
      ftf += fsh[i * kShardWords + SH_FTF];
      big += fsh[i * kShardWords + SH_BIG];
    }
    header[ncnt] = most;
    header[ncnt + 1] = runs;
    header[ncnt + 2] = ftf;
    header[ncnt + 3] = big;
  }
}

// A record written by the fused compaction (k_frontier_resolve, min_size
// <= 1) holds -(slot + 1) instead of its size: its label and sums are read
// by slot (final after the resolve kernel).  Records are only read here,
// never rewritten (other workgroups read the keys concurrently); the raw
// records of a pass the device does not sort are completed by
// fix_raw_records.
__device__ inline void record_vals(const long long* clusters, const long long* sums, const long long* labels,
                                   int64_t i, long long* lab, long long* sz, long long* sx, long long* sy) {
  const long long m = clusters[4 * i + 1];
  if (sums && m < 0) {
    const int64_t sl = -m - 1;
    *lab = labels[sl];
    *sz = sums[3 * sl];
    *sx = sums[3 * sl + 1];
    *sy = sums[3 * sl + 2];
  } else {
    *lab = clusters[4 * i];
    *sz = m;
    *sx = clusters[4 * i + 2];
    *sy = clusters[4 * i + 3];
  }
}

// Sort key (label) of record i.
__device__ inline long long record_key(const long long* clusters, const long long* labels, int64_t i) {
  if (labels) {
    const long long m = clusters[4 * i + 1];
    if (m < 0) return labels[-m - 1];
  }
  return clusters[4 * i];
}

// Raw records of a pass the device does not sort (K > cap): values in place
// (the host sorts them).  One writer per record, no concurrent key readers.
__device__ inline void fix_raw_records(long long* clusters, const long long* sums, const long long* labels,
                                       int64_t K) {
  if (!sums) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x) {
    long long lab, sz, sx, sy;
    record_vals(clusters, sums, labels, i, &lab, &sz, &sx, &sy);
    clusters[4 * i + 0] = lab;
    clusters[4 * i + 1] = sz;
    clusters[4 * i + 2] = sx;
    clusters[4 * i + 3] = sy;
  }
}

// Raw record i ([4] int64 label, size, sum_x, sum_y) -> dm_cluster at its
// sorted position, centroid cx_m = ox + ((double)sum_x / (double)size + 0.5)
// * res (SPEC a10: one IEEE division, then add; no FMA contraction).
__device__ inline void put_sorted(double ox, double oy, double res, const long long* clusters,
                                  const long long* sums, const long long* labels,
                                  int64_t i, int64_t rank, dm_cluster* __restrict__ out,
                                  int32_t* __restrict__ rank_of, dm_raw_record* __restrict__ host_out,
                                  int64_t host_cap) {
  dm_cluster c;
  long long lab, sz, sx, sy;
  record_vals(clusters, sums, labels, i, &lab, &sz, &sx, &sy);
  c.label = lab;
  c.size = sz;
  c.sum_x = sx;
  c.sum_y = sy;
  c.cx_m = dm_centroid(ox, c.sum_x, c.size, res);
  c.cy_m = dm_centroid(oy, c.sum_y, c.size, res);
  out[rank] = c;
  // mapped host readback: the 32-byte record (the host adds the centroids)
  if (host_out && rank < host_cap) host_out[rank] = dm_raw_record{lab, sz, sx, sy};
  if (rank_of) rank_of[i] = (int32_t)rank;
}

// Cluster list sorted by label, with centroids (SPEC a10).  Labels are
// unique (one per component), so a record's position is the number of
// records with a smaller label.  One workgroup per 64 records (lane = record),
// its waves split the keys: the labels are staged through LDS in chunks
// (every thread's loads in flight at once) and each wave counts over its
// share of the chunk with wave-uniform LDS broadcasts; the waves' partial
// counts are summed in LDS.  O(K^2) compares spread over
// ceil(K/64) workgroups: no serial single-workgroup network, a few
// microseconds at C3's ~1.6k clusters.  Records become dm_cluster with
// cx_m = ox + ((double)sum_x / (double)size + 0.5) * res (IEEE division in
// double on host and device).  rank_of (may be NULL) receives each input
// record's sorted position.  More than kRankSortCap records: *sorted = 0
// and the host sorts the raw records.
// DM_SORT_THREADS / _CHUNK (A/B): 256 threads with 2048-key chunks measured
// 17.6 vs 11.1 us at C3 (profiles/r03_sort_width_fk_fmask_ab.log): the
// waves' share of the compares, not the placement of a 16-wave workgroup
#ifndef DM_SORT_THREADS
#define DM_SORT_THREADS 1024
#endif
#ifndef DM_SORT_CHUNK
#define DM_SORT_CHUNK 4096
#endif
constexpr int kSortChunk = DM_SORT_CHUNK;
constexpr int kSortThreads = DM_SORT_THREADS;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int64_t kRankSortCap = 1 << 16;

__global__ __launch_bounds__(kSortThreads) void k_rank_sort(double ox, double oy, double res,
                                                            long long* clusters, const long long* sums,
                                                            const long long* labels,
                                                            const unsigned long long* __restrict__ count,
                                                            int64_t cap, dm_cluster* __restrict__ out,
                                                            int32_t* __restrict__ rank_of,
                                                            unsigned long long* sorted,
                                                            const unsigned long long* __restrict__ cnt,
                                                            int ncnt, int sorted_idx,
                                                            const unsigned long long* __restrict__ fsh,
                                                            dm_raw_record* __restrict__ host_out,
                                                            int64_t host_cap) {
  __shared__ long long keys[kSortChunk];
  __shared__ int32_t part[kSortWaves][64];
  const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
  const int64_t K = (int64_t)*count;
  if (blockIdx.x == 0) write_rb_header(K, cap, sorted, cnt, ncnt, sorted_idx, fsh, host_out);
  if (K > cap) {
    fix_raw_records(clusters, sums, labels, K);
    return;
  }
  // grid-stride over groups of 64 records (the grid is sized from the
  // expected count; the loop bound is uniform within a workgroup)
  for (int64_t g0 = (int64_t)blockIdx.x * 64; g0 < K; g0 += (int64_t)gridDim.x * 64) {
    const int64_t i = g0 + lane;
    const long long key = i < K ? record_key(clusters, labels, i) : 0;
    int32_t r = 0;
    for (int64_t c0 = 0; c0 < K; c0 += kSortChunk) {
      const int n = (int)min((int64_t)kSortChunk, K - c0);
      __syncthreads();
      {
        long long v[kSortChunk / kSortThreads];
#pragma unroll
        for (int q = 0; q < kSortChunk / kSortThreads; ++q) {
          const int e = tid + q * kSortThreads;
          v[q] = e < n ? record_key(clusters, labels, c0 + e) : 0;
        }
#pragma unroll
        for (int q = 0; q < kSortChunk / kSortThreads; ++q) {
          const int e = tid + q * kSortThreads;
          if (e < n) keys[e] = v[q];
        }
      }
      __syncthreads();
      const int per = (n + kSortWaves - 1) / kSortWaves;
      const int lo = min(n, w * per), hi = min(n, lo + per);
      int e = lo;
      for (; e + 4 <= hi; e += 4)
        r += (keys[e] < key) + (keys[e + 1] < key) + (keys[e + 2] < key) + (keys[e + 3] < key);
      for (; e < hi; ++e) r += keys[e] < key;
    }
    part[w][lane] = r;
    __syncthreads();  // (the next group's first barrier keeps part until wave 0 read it)
    if (w == 0 && i < K) {
      int32_t rank = 0;
#pragma unroll
      for (int q = 0; q < kSortWaves; ++q) rank += part[q][lane];
      put_sorted(ox, oy, res, clusters, sums, labels, i, rank, out, rank_of, host_out, host_cap);
    }
  }
}

// ---- row-bucket sort for many clusters (the default for K > sort_min) --------------------------
// A label is the row-major index y * W + x of a component's first cell, so
// label order is (row, column) order: one counting pass by row puts every
// record in its row's range, and a record's place inside that range is the
// number of records of the same row with a smaller column.  Four kernels
// whatever the key width:
//   k_rs_count  per record: key = label - base, row = key / W, slot = its
//               arrival in the row (atomic on the row's counter)
//   k_rs_scan   exclusive scan of the row counts -> row offsets (rows + 1
//               of them) by 8192-row workgroups that publish their totals,
//               and the counters back to zero for the next sort (they are
//               zero when allocated)
//   k_rs_place  record -> offset[row] + slot (unordered inside the row)
//   k_rs_rank   position p: rank among its row's keys (a scan of the row's
//               range, O(b) for a row of b records), then the same record
//               write + readback header as k_rank_sort.
// A frontier's components are spread over many rows (C5's 219k clusters of
// 64 robots: a few per row), so b is small; a pathological row of b records
// costs O(b^2) compares but stays exact.
__global__ __launch_bounds__(256) void k_rs_count(const long long* __restrict__ clusters,
                                                  const long long* __restrict__ labels,
                                                  const unsigned long long* __restrict__ count, int64_t cap,
                                                  long long base, int64_t W, int32_t* __restrict__ row_cnt,
                                                  unsigned long long* __restrict__ keys, int32_t* __restrict__ slot,
                                                  unsigned long long* status, int n_status) {
  const int64_t K = (int64_t)*count;
  if (K > cap) return;
  if (blockIdx.x == 0)  // k_rs_scan's published-total words and its failure word, for this sort
    for (int e = threadIdx.x; e <= n_status; e += blockDim.x) status[e] = 0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = (unsigned long long)(record_key(clusters, labels, i) - base);
    const int64_t row = (int64_t)(key / (unsigned long long)W);
    keys[i] = key;
    slot[i] = atomicAdd(&row_cnt[row], 1);
  }
}

// Row offsets by many small workgroups (a 1024-thread workgroup waits for a
// whole CU to drain while the next batch's k_tile_accum fills the chip: the
// single-workgroup scan measured 27-250 us at C5): workgroup b scans rows
// [b * kRsChunk, +kRsChunk) in registers (256 threads x 32 rows), publishes
// its total in status[b] (bit 63 = published; k_rs_count zeroed the words),
// then adds the totals of ALL earlier workgroups (each published right after
// its own reduce, so no serial chain: a workgroup only waits for earlier
// ones, which were dispatched first).
constexpr int kRsPer = 32;
constexpr int64_t kRsChunk = 256 * kRsPer;
__global__ __launch_bounds__(256) void k_rs_scan(const unsigned long long* __restrict__ count, int64_t cap,
                                                 int64_t rows, int32_t* __restrict__ row_cnt,
                                                 int32_t* __restrict__ row_off, unsigned long long* status) {
  const int64_t K = (int64_t)*count;
  if (K > cap) return;
  __shared__ int32_t wsum[4];
  __shared__ unsigned long long s_pre;
  const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
  const int64_t blk = blockIdx.x;
  const int64_t b = blk * kRsChunk + (int64_t)tid * kRsPer;
  int32_t v[kRsPer];
  if (b + kRsPer <= rows) {
#pragma unroll
    for (int q = 0; q < kRsPer / 4; ++q) {
      const int4 t = reinterpret_cast<const int4*>(row_cnt + b)[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int q = 0; q < kRsPer / 4; ++q) reinterpret_cast<int4*>(row_cnt + b)[q] = make_int4(0, 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < kRsPer; ++i) {
      v[i] = b + i < rows ? row_cnt[b + i] : 0;
      if (b + i < rows) row_cnt[b + i] = 0;
    }
  }
  int32_t seg = 0;
#pragma unroll
  for (int i = 0; i < kRsPer; ++i) seg += v[i];
  int32_t incl = seg;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  const int32_t total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  int32_t run = incl - seg;
  for (int q = 0; q < w; ++q) run += wsum[q];
  if (tid == 0)
    __hip_atomic_store(&status[blk], (1ull << 63) | (unsigned long long)(uint32_t)total, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // the earlier workgroups' totals (bounded polls: they were dispatched
  // before this one, so they publish).  A poll that gives up marks the sort
  // failed (status[gridDim.x]): k_rs_rank then reports the records unsorted
  // and the host sorts them, instead of placing them by wrong offsets
  long long pre = 0;
  for (int64_t e = tid; e < blk; e += 256) {
    unsigned long long sv = 0ull;
    for (int it = 0; it < (1 << 22); ++it) {
      sv = __hip_atomic_load(&status[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (sv >> 63) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (!(sv >> 63))
      __hip_atomic_store(&status[gridDim.x], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pre += (long long)(sv & 0xFFFFFFFFull);
  }
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
  if (tid == 0) s_pre = 0;
  __syncthreads();
  if (lane == 0 && pre) atomicAdd(&s_pre, (unsigned long long)pre);
  __syncthreads();
  run += (int32_t)s_pre;
  if (b + kRsPer <= rows) {
#pragma unroll
    for (int q = 0; q < kRsPer / 4; ++q) {
      int4 t;
      t.x = run; run += v[4 * q];
      t.y = run; run += v[4 * q + 1];
      t.z = run; run += v[4 * q + 2];
      t.w = run; run += v[4 * q + 3];
      reinterpret_cast<int4*>(row_off + b)[q] = t;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kRsPer; ++i) {
      if (b + i < rows) row_off[b + i] = run;
      run += v[i];
    }
  }
  if (blk == (int64_t)gridDim.x - 1 && tid == 0) row_off[rows] = (int32_t)s_pre + total;
}

__global__ __launch_bounds__(256) void k_rs_place(const unsigned long long* __restrict__ count, int64_t cap,
                                                  int64_t W, const unsigned long long* __restrict__ keys,
                                                  const int32_t* __restrict__ slot,
                                                  const int32_t* __restrict__ row_off,
                                                  unsigned long long* __restrict__ keys_out,
                                                  int32_t* __restrict__ idx_out) {
  const int64_t K = (int64_t)*count;
  if (K > cap) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = keys[i];
    const int64_t p = (int64_t)row_off[(int64_t)(key / (unsigned long long)W)] + slot[i];
    keys_out[p] = key;
    idx_out[p] = (int32_t)i;
  }
}

__global__ __launch_bounds__(256) void k_rs_rank(double ox, double oy, double res, long long* clusters,
                                                 const long long* sums, const long long* labels,
                                                 const unsigned long long* __restrict__ count, int64_t cap,
                                                 int64_t W, const unsigned long long* __restrict__ keys,
                                                 const int32_t* __restrict__ idx,
                                                 const int32_t* __restrict__ row_off,
                                                 dm_cluster* __restrict__ out, int32_t* __restrict__ rank_of,
                                                 unsigned long long* sorted, const unsigned long long* __restrict__ cnt,
                                                 int ncnt, int sorted_idx, const unsigned long long* __restrict__ fsh,
                                                 dm_raw_record* __restrict__ host_out, int64_t host_cap,
                                                 const unsigned long long* __restrict__ scan_failed) {
  const int64_t K = (int64_t)*count;
  // k_rs_scan gave up on a workgroup total: the offsets are wrong, so the
  // records stay raw and unsorted (the host sorts them), as when K > cap
  if (*scan_failed) cap = -1;
  if (blockIdx.x == 0) write_rb_header(K, cap, sorted, cnt, ncnt, sorted_idx, fsh, host_out);
  if (K > cap) {
    fix_raw_records(clusters, sums, labels, K);
    return;
  }
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < K; p += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = keys[p];
    const int64_t row = (int64_t)(key / (unsigned long long)W);
    const int32_t lo = row_off[row], hi = row_off[row + 1];
    int32_t r = 0;
    int32_t q = lo;
    for (; q + 4 <= hi; q += 4)
      r += (keys[q] < key) + (keys[q + 1] < key) + (keys[q + 2] < key) + (keys[q + 3] < key);
    for (; q < hi; ++q) r += keys[q] < key;
    put_sorted(ox, oy, res, clusters, sums, labels, idx[p], (int64_t)lo + r, out, rank_of, host_out, host_cap);
  }
}

// Cell slot -> final label (the root of a set is its min-label slot).
__global__ __launch_bounds__(256) void k_slot_labels(int64_t n, int64_t slot_cap, const int32_t* __restrict__ cslot,
                                                     const int32_t* __restrict__ slot_root,
                                                     const long long* __restrict__ slot_label,
                                                     long long* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = cslot[i];
    out[i] = (s < 0 || s >= slot_cap) ? -1 : slot_label[slot_root[s]];
  }
}

int grid_for(int64_t n, int threads, int64_t cap) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

static_assert(sizeof(FGeom) == 88, "FGeom has no implicit padding");

static FGeom make_fgeom(const dm_grid* g, bool want_mask, bool want_labels) {
  FGeom fg;
  fg.W = (int32_t)g->W;
  fg.R = (int32_t)g->R;
  fg.row0 = (int32_t)g->row0;
  fg.TX = (int32_t)g->TX;
  fg.TY = (int32_t)g->TY;
  fg.NT = g->NT;
  fg.has_before = g->has_halo[0];
  fg.has_after = g->has_halo[1];
  fg.want_mask = want_mask ? 1 : 0;
  fg.want_labels = want_labels ? 1 : 0;
  fg.H = g->H;
  fg.slot_cap = g->slot_cap;
  fg.slot_per = g->slot_cap / kShards;
  fg.clu_cap = g->slot_cap;
  fg.min_size = g->p.min_frontier_size;
  return fg;
}

DM_PH_READER(frontier)
DM_PH_READER(ftile)

// Band edge-row labels (dm_get_edge_labels; only the host-side band merge
// reads them), from the last frontier call's slots.
int dm_launch_edge_labels(dm_grid* g) {
  DM_LAUNCH(k_slot_labels, dim3(grid_for(2 * g->W, 256, 1024)), dim3(256), 0, g->stream,
                     2 * g->W, g->slot_cap, g->edge_slot, g->slot_root, g->slot_label, g->edge_label);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_rank_sort(hipStream_t stream, long long* clusters, const long long* sums,
                        const long long* labels, const unsigned long long* d_count,
                        int64_t max_records, double ox, double oy, double res, dm_cluster* out,
                        int32_t* rank_of, unsigned long long* d_sorted, const unsigned long long* cnt,
                        int ncnt, int sorted_idx, const unsigned long long* fsh, dm_raw_record* host_out,
                        int64_t host_cap, int64_t expect) {
  const int64_t cap = std::min<int64_t>(max_records, kRankSortCap);
  // one workgroup per 64 expected records (twice the last pass's count, at
  // least 2048): a thousand idle 1024-thread workgroups cost microseconds
  const int64_t want = dm_quantize_up(std::max<int64_t>(2 * expect, 2048));
  DM_LAUNCH(k_rank_sort, dim3(grid_for(std::min(cap, want), 64, 1 << 20)), dim3(kSortThreads), 0, stream,
                     ox, oy, res, clusters, sums, labels, d_count, cap, out, rank_of, d_sorted, cnt, ncnt, sorted_idx,
                     fsh, host_out, host_cap);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_bucket_sort(dm_grid* g, hipStream_t stream, long long* clusters, const long long* sums,
                          const long long* labels, const unsigned long long* d_count,
                          int64_t max_records, int64_t row_base, int64_t rows, dm_cluster* out,
                          int32_t* rank_of, unsigned long long* d_sorted, const unsigned long long* cnt,
                          int ncnt, int sorted_idx, const unsigned long long* fsh, dm_raw_record* host_out,
                          int64_t host_cap) {
  if (max_records > g->bs_cap || rows > g->rs_rows)
    return dm_set_error(DM_ERR_INVALID_ARG, "row sort: %lld records over %lld rows exceed its workspace",
                        (long long)max_records, (long long)rows);
  // key = label - base over [0, rows * W)
  const long long base = row_base * g->W;
  // grids follow the expected count (the kernels stride; blocks past the
  // device-side count return)
  const int64_t expect = std::min<int64_t>(max_records, std::max<int64_t>(2 * g->sort_hint, 4096));
  const int eg = grid_for(expect, 256, 4096);
  const int nsb = (int)((rows + kRsChunk - 1) / kRsChunk);
  DM_LAUNCH(k_rs_count, dim3(eg), dim3(256), 0, stream, clusters, labels, d_count, max_records, base, g->W,
            g->rs_cnt, g->bs_key, g->bs_idx2, g->rs_status, nsb);
  DM_HIP(hipGetLastError());
  DM_LAUNCH(k_rs_scan, dim3(nsb), dim3(256), 0, stream, d_count, max_records, rows, g->rs_cnt, g->rs_off,
            g->rs_status);
  DM_HIP(hipGetLastError());
  DM_LAUNCH(k_rs_place, dim3(eg), dim3(256), 0, stream, d_count, max_records, g->W, g->bs_key, g->bs_idx2,
            g->rs_off, g->bs_key2, g->bs_idx);
  DM_HIP(hipGetLastError());
  DM_LAUNCH(k_rs_rank, dim3(eg), dim3(256), 0, stream, g->p.origin_x, g->p.origin_y, g->p.resolution, clusters,
            sums, labels, d_count, max_records, g->W, g->bs_key2, g->bs_idx, g->rs_off, out, rank_of, d_sorted, cnt,
            ncnt, sorted_idx, fsh, host_out, host_cap, g->rs_status + nsb);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

// Enqueues the band pipeline (no synchronisation): tile list, tile CCL,
// border merge, roots, compaction, sort.  Shared by dm_launch_frontiers and
// the cross-band export (dm_merge.hip).
int dm_enqueue_frontiers(dm_grid* g, bool want_mask, bool want_labels, bool split, hipStream_t* end_stream) {
  const FGeom fg = make_fgeom(g, want_mask, want_labels);
  const int64_t cells = g->R * g->W;
  // the bit rows run on g->stream after everything shared with
  // the pass stream (labelling of earlier passes) -- except for split passes,
  // which keep that order on the pass stream itself
  if (!split) DM_HIP(dm_join_pass_stream(g));
  ++g->rb[g->cur_slot].wepoch;  // this pass rewrites the selected slot's records
  ++g->fr_pass;
  g->fparity ^= 1;
  dm_grid::FrWs& fw = g->fw[g->fparity];
  if (fw.busy_pending) {  // the set's previous pass (two passes ago) may still run
    DM_HIP(hipStreamWaitEvent(g->stream, fw.busy, 0));
    fw.busy_pending = false;
  }
  dm_select_fw(g, g->fparity);
  unsigned long long* list_n = g->fl_n + 16 * (g->fr_pass % 3);  // this pass's list length (k_frontier_bits)
  // every relist_period passes (1, 2, 4, ... 16) the tile list goes back into
  // tile order, into the other list (dm_launch_relist: the passes still
  // labelling keep theirs)
  if (++g->relist_age >= g->relist_period)
    if (int rc = dm_launch_relist(g, true)) return rc;
  KernelTimer t;
  if (want_mask) DM_HIP(hipMemsetAsync(g->mask, 0, (size_t)cells, g->stream));
  if (want_labels) DM_HIP(hipMemsetAsync(g->cell_slot, 0xFF, sizeof(int32_t) * (size_t)cells, g->stream));
  // one wave per listed tile; the grid follows the last collected pass's
  // list length (+25 %, quantised; the kernels grid-stride, so any count is
  // covered)
  const int64_t want_waves = g->ftile_hint > 0 ? dm_quantize_up(g->ftile_hint + g->ftile_hint / 4 + 64) : g->NT;
  const int wave_grid = grid_for(std::min<int64_t>(want_waves, g->NT), kFW, 8192);
  // k_frontier_bits also resets the pass's arrays (slot parents: 4 per map
  // tile): at least 64 workgroups
  const int bits_grid = std::max(wave_grid, 64);
  // fmask while the passes list many tiles (dm_internal.h, fmask_on); a
  // switch on rebuilds the records first unless they still match the state
  const bool want_on = g->fmask_mode == 1 || (g->fmask_mode == 0 && g->ftile_hint >= kFmaskOnTiles);
  const bool want_off = g->fmask_mode == 2 || (g->fmask_mode == 0 && g->ftile_hint < kFmaskOnTiles / 4);
  if (!g->fmask_on && want_on) {
    if (!g->fmask_valid) {
      if (int rc = dm_launch_recount(g)) return rc;
    }
    g->fmask_on = true;
  } else if (g->fmask_on && want_off) {
    g->fmask_on = false;
  }
  // Tile kernel, chosen from the last collected pass (both are exact for any
  // map; they differ in speed): tiles whose frontiers are dense (more than
  // kDenseRuns runs per tile with frontier cells on average, e.g. C3's ray
  // fans, ~100) take the 256-thread kernel, one tile per workgroup; sparse
  // ones (an explored map's few frontier tiles among many listed tiles, a
  // 1 cm map's thin rays) the wave-per-tile kernel, which also screens the
  // listed tiles without frontier cells at the rate of one 8-byte load per
  // lane; tiles with more than kRunsFast runs are listed by k_frontier_bits
  // for the 256-thread kernel, which runs beside it on big_stream.
  // Dense only while the tiles fit about two rounds of the 256-thread
  // kernel's slots: with tens of thousands of tiles (a 1 cm map's rays) the
  // wave kernel's 4x more tiles in flight win even where runs are many.
  const bool dense = g->frontier_kernel == 2 ||
                     (g->frontier_kernel == 0 && g->ftf_hint > 0 && g->runs_hint > kDenseRuns * g->ftf_hint &&
                      g->ftf_hint <= kDenseMaxTiles);
  // Tile-edge unions in the tile kernels or in k_frontier_edges after them
  // (DESIGN.md §3.2): the edge kernel for sparse passes with fewer clusters
  // than listed tiles (C5 12-768 beams: passes 3-10 % shorter, steps up to
  // 11 %), in-kernel for dense passes (C3: the extra launch costs more than
  // the tiles save, 3-4 % per step) and for sparse passes with more
  // clusters than tiles (C5-4096's 4.6 per tile: many distinct pairs per
  // edge, step 2-15 % slower with the edge kernel);
  // profiles/r06_edge_kernel_ab.log.  Both are exact for any map.
  const bool edge = DM_EDGE_KERNEL == 2 ||
                    (DM_EDGE_KERNEL == 1 && !dense && g->sort_hint <= std::max<int64_t>(g->ftile_hint, 1));
  auto* const big_kernel = edge ? k_frontier_tile_big<true> : k_frontier_tile_big<false>;
  auto* const wave_kernel = edge ? k_frontier_tile<true> : k_frontier_tile<false>;
  dm_timer_begin(g, "frontier_bits", &t);
  DM_LAUNCH(k_frontier_bits, dim3(bits_grid), dim3(kFW * 64), 0, g->stream, fg, g->state, g->halo, g->fmask,
            g->fedge, g->tile_seen, g->ftiles, g->ftiles_n, list_n, g->fbits, g->cnt, g->fmask_on ? 1 : 0,
            dense ? nullptr : g->big_tiles, g->fsh, g->edge_slot, 2 * g->W, g->slot_parent, g->fe_flag + kHaltWord,
            g->bits_flag + kStampWord);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  // the map has been read: with split, the rest runs on the pass stream,
  // after the bit rows' hand-off
  hipStream_t ps = g->stream;
  if (split) {
    ps = g->pass_stream;
    hipEvent_t eb = g->ev_bits[g->fparity];
    DM_HIP(hipEventRecord(eb, g->stream));
    // the integrate workspaces are free once the grid stream is past the
    // accumulations.  (Re-recorded two passes later: a front-end waiting on it
    // then waits longer than needed, never too little -- every record follows
    // the accumulations it frees in stream order.)
    DM_HIP(dm_mark_ws_free(g, eb));
    DM_HIP(hipStreamWaitEvent(ps, eb, 0));
  }
  if (end_stream) *end_stream = ps;
  if (!dense) {
    // the run-rich tiles (listed by k_frontier_bits) on big_stream, beside
    // the wave kernel: the round-2 launch order ran them after it (C5 at 192
    // beams: 157 us of big tiles behind 194 us of wave tiles).  The tile-edge
    // hand-off unites tiles whatever kernel and order processed them.
    // the grid follows the last pass's count (the kernel grid-strides)
    const int big_grid =
        grid_for(std::min<int64_t>(g->NT, dm_quantize_up(g->big_hint + g->big_hint / 4 + 64)), 1, 8192);
    DM_HIP(hipEventRecord(g->ev_bigfork, ps));
    DM_HIP(hipStreamWaitEvent(g->big_stream, g->ev_bigfork, 0));
    dm_timer_begin(g, "frontier_big", &t, g->big_stream);
    DM_LAUNCH(big_kernel, dim3(big_grid), dim3(kFT), 0, g->big_stream, fg, g->fbits,
              g->big_tiles,
              g->ftiles, list_n, g->border, g->rel, g->slot_label, g->slot_parent, g->slot_own,
              g->slot_acc, g->mask, g->cell_slot, g->edge_slot, g->cnt, g->fsh, 0);
    dm_timer_end(g, &t);
    DM_HIP(hipGetLastError());
    DM_HIP(hipEventRecord(g->ev_big, g->big_stream));
    dm_timer_begin(g, "frontier_tile", &t, ps);
    DM_LAUNCH(wave_kernel, dim3(wave_grid), dim3(kFW * 64), 0, ps, fg, g->fbits,
                       g->ftiles, list_n, g->border, g->rel,
                       g->slot_label, g->slot_parent, g->slot_own, g->slot_acc, g->mask, g->cell_slot,
                       g->edge_slot, g->cnt, g->fsh, g->big_tiles);
    dm_timer_end(g, &t);
    DM_HIP(hipGetLastError());
    DM_HIP(hipStreamWaitEvent(ps, g->ev_big, 0));
  } else {
    dm_timer_begin(g, "frontier_tile", &t, ps);
    // one workgroup per listed tile of the last collected pass (+25 %; the
    // kernel grid-strides): thousands of empty workgroups would only keep
    // the dispatcher from the other streams' kernels
    // (caps of 256-1024 workgroups, to leave the map update more slots,
    // measured slower: DESIGN.md §3.3.2)
    const int dense_grid = grid_for(std::min<int64_t>(g->NT, g->ftile_hint > 0 ? want_waves : g->NT), 1, 8192);
    DM_LAUNCH(big_kernel, dim3(dense_grid), dim3(kFT), 0, ps, fg, g->fbits, nullptr,
              g->ftiles, list_n,
              g->border, g->rel, g->slot_label, g->slot_parent, g->slot_own, g->slot_acc, g->mask,
              g->cell_slot, g->edge_slot, g->cnt, g->fsh, 1);
    dm_timer_end(g, &t);
    DM_HIP(hipGetLastError());
  }
  if (edge) {
    dm_timer_begin(g, "frontier_edges", &t, ps);
    // DM_EDGE_WAVES waves per listed tile (the kernel grid-strides)
    DM_LAUNCH(k_frontier_edges, dim3(grid_for(DM_EDGE_WAVES * std::min<int64_t>(want_waves, g->NT), kFW, 16384)),
              dim3(kFW * 64), 0, ps, fg, g->ftiles, list_n, g->border, g->rel,
              g->slot_parent, g->cnt);
    dm_timer_end(g, &t);
    DM_HIP(hipGetLastError());
  }
  const int sgrid = grid_for(g->slot_cap, 256, 1024);
  dm_timer_begin(g, "frontier_resolve", &t, ps);
  // min_size <= 1: every root is a cluster, compacted by the resolve itself
  // (no k_frontier_compact); the sort reads the sums by slot
  const int fuse = g->p.min_frontier_size <= 1 ? 1 : 0;
  // one workgroup per CU: fewer workgroups = fewer per-root flushes
  DM_LAUNCH(k_frontier_resolve, dim3(grid_for(g->slot_cap, 256, g->n_cu)), dim3(256), 0, ps, fg,
                     g->slot_parent, g->slot_root, g->slot_own, g->slot_acc, g->fsh, fuse, g->slot_label,
                     g->clusters, g->slot_k, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  if (!fuse) {
    dm_timer_begin(g, "frontier_compact", &t, ps);
    DM_LAUNCH(k_frontier_compact, dim3(sgrid), dim3(256), 0, ps, fg,
                       g->slot_root, g->slot_label, g->slot_acc, g->clusters, g->slot_k, g->cnt, g->fsh);
    dm_timer_end(g, &t);
    DM_HIP(hipGetLastError());
  }
  if (want_labels) {
    DM_LAUNCH(k_slot_labels, dim3(grid_for(cells, 256, 8192)), dim3(256), 0, ps,
                       cells, g->slot_cap, g->cell_slot, g->slot_root, g->slot_label, g->labels);
    DM_HIP(hipGetLastError());
  }
  dm_timer_begin(g, "sort_clusters", &t, ps);
  // the last collected pass predicts this one's cluster count (either sort
  // is exact for any count; only their speed differs)
  const int rc = g->sort_hint > g->sort_min
      ? dm_launch_bucket_sort(g, ps, g->clusters, fuse ? g->slot_acc : nullptr, fuse ? g->slot_label : nullptr,
                              g->cnt + CNT_CLUSTERS, g->slot_cap, g->row0, g->R, g->out_clu,
                              g->rank_of, g->cnt + CNT_SORTED, g->cnt, CNT_N, CNT_SORTED, g->fsh,
                              g->h_out_dev, g->h_out_cap)
      : dm_launch_rank_sort(ps, g->clusters, fuse ? g->slot_acc : nullptr, fuse ? g->slot_label : nullptr,
                            g->cnt + CNT_CLUSTERS, g->slot_cap, g->p.origin_x,
                            g->p.origin_y, g->p.resolution, g->out_clu, g->rank_of, g->cnt + CNT_SORTED,
                            g->cnt, CNT_N, CNT_SORTED, g->fsh, g->h_out_dev, g->h_out_cap, g->sort_hint);
  dm_timer_end(g, &t);
  return rc;
}

// After a frontier pass completed: the counters plus a speculative first
// chunk of the sorted cluster records are in g->h_out (k_rank_sort wrote the
// readback header and the first h_out_cap records straight into the mapped
// host buffer: no copy command).  Returns DM_ERR_CAPACITY (with
// *n_clusters = slots needed) when the slot arrays overflowed.
int dm_frontiers_readback(dm_grid* g, int64_t* n_clusters, int64_t* copied) {
  const unsigned long long* hdr = dm_rb_header(g->h_out);
  memcpy(g->h_cnt, hdr, sizeof(unsigned long long) * CNT_N);
  *copied = std::min<int64_t>(g->h_out_cap, g->slot_cap);
  const unsigned long long most = hdr[CNT_N];
  if (g->h_cnt[CNT_OVERFLOW] & kOvPipeline)
    return dm_set_error(DM_ERR_PIPELINE, "the overlapped pipeline's front-end hand-off timed out: a map "
                                         "update was skipped; dm_reset the handle");
  if ((int64_t)most > g->slot_cap / kShards || (g->h_cnt[CNT_OVERFLOW] & kOvSlots)) {
    *n_clusters = (int64_t)most * kShards;  // slot capacity that fits the fullest shard
    return DM_ERR_CAPACITY;
  }
  if (g->h_cnt[CNT_OVERFLOW] & kOvUnionFind)
    return dm_set_error(DM_ERR_INCOMPLETE, "frontier union-find did not converge within its bound "
                                           "(dm_uf.h): this pass has no result");
  *n_clusters = (int64_t)g->h_cnt[CNT_CLUSTERS];
  g->sort_hint = *n_clusters;
  // this pass's tile-list length (the other parity's counter is 0 or smaller)
  g->ftile_hint = (int64_t)g->h_cnt[CNT_FL0];
  g->runs_hint = (int64_t)hdr[CNT_N + 1];
  g->ftf_hint = (int64_t)hdr[CNT_N + 2];
  g->big_hint = (int64_t)hdr[CNT_N + 3];
  return DM_OK;
}

// Runs the frontier pipeline with ONE synchronisation (dm_frontiers_readback).
int dm_launch_frontiers(dm_grid* g, bool want_mask, bool want_labels, int64_t* n_clusters,
                        int64_t* copied) {
  int rc = dm_enqueue_frontiers(g, want_mask, want_labels);
  if (rc) return rc;
  DM_HIP(hipStreamSynchronize(g->stream));
  return dm_frontiers_readback(g, n_clusters, copied);
}
