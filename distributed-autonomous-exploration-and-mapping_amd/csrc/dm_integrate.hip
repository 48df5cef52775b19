// dm_integrate.hip — LaserScan batch -> log-odds occupancy grid (gfx950).
//
// Replaces the ray-trace + grid update slam_toolbox performs before
// publishing /map (launched at server/thymio_project/launch/
// pc_server.launch.py:12-19; resolution / max range from
// server/thymio_project/config/slam_config.yaml:26-27).  SPEC rows a4-a7 of
// SURVEY.md §8(a), restated in DESIGN.md §2.
//
// Design: the per-call hit/miss counts never touch HBM.  Each
// ray is cut into pieces that lie inside one 64x64 tile; pieces are binned by
// tile; one workgroup per touched tile accumulates its pieces' counts in LDS
// (lanes stride along the ray's major axis, so one wave-instruction covers up
// to 64 cells of one piece with conflict-free LDS atomics), then applies the
// log-odds update to the tile's cells in one coalesced read-modify-write of L
// and state.  Integer counts make the result independent of atomic order.
//
//   k_beam_prep   one thread per beam: endpoint cells (double, no FMA),
//                 Bresenham params, per-tile piece counts (wave-aggregated
//                 atomics), first-touch list of active tiles
//   k_scan_active one workgroup: exclusive scan of piece counts
//   k_scatter     one thread per beam: pieces -> per-tile bins
//   k_tile_apply  one workgroup per active tile (grid-stride): LDS counts +
//                 fused apply, tile summaries, counter reset
#include "dm_internal.h"

namespace {

constexpr int kApplyThreads = 256;
constexpr int kLdsPitch = DM_TS + 1;  // +1 dword: y-major pieces hit distinct banks

struct Geom {
  RayGeom r;
  int32_t act_cap;
  int64_t seg_cap;
  int64_t item_cap;
  int64_t heavy_cap;
  int64_t nb;  // beams in this call
};

__device__ inline int lane_id() { return __lane_id(); }

// Per-block tile histogram in LDS (open addressing).  The 256 beams of a block
// are consecutive beams of one scan, so their pieces fall in a few tens of
// tiles: one global atomic per (block, tile) instead of one per piece, and no
// same-address contention on the tile around each sensor (4096 pieces per
// scan).  A tile that finds no slot within kProbe probes takes the per-piece
// global path; inserts only ever fill slots, so a later lookup of the same
// tile takes the same decision.
constexpr int kHash = 1024;
constexpr int kProbe = 32;

__device__ inline uint32_t tile_hash(int32_t t) { return ((uint32_t)t * 2654435761u) >> 22; }

__device__ inline int hash_insert(int32_t* hkey, int32_t tile) {
  uint32_t h = tile_hash(tile);
  for (int p = 0; p < kProbe; ++p, h = (h + 1) & (kHash - 1)) {
    const int32_t k = atomicCAS(&hkey[h], -1, tile);
    if (k == -1 || k == tile) return (int)h;
  }
  return -1;
}

__device__ inline int hash_find(const int32_t* hkey, int32_t tile) {
  uint32_t h = tile_hash(tile);
  for (int p = 0; p < kProbe; ++p, h = (h + 1) & (kHash - 1)) {
    const int32_t k = hkey[h];
    if (k == tile) return (int)h;
    if (k == -1) return -1;
  }
  return -1;
}

__device__ inline void first_touch(const Geom& g, int32_t tile, int32_t old, int32_t* tile_slot,
                                   int32_t* act_tiles, unsigned long long* cnt) {
  if (old != 0) return;
  const unsigned long long slot = atomicAdd(&cnt[CNT_ACTIVE], 1ull);
  if (slot < (unsigned long long)g.act_cap) {
    act_tiles[slot] = tile;
    tile_slot[tile] = (int32_t)slot;
  } else {
    tile_slot[tile] = -1;
    atomicOr(&cnt[CNT_OVERFLOW], 1ull);
  }
}

__global__ __launch_bounds__(256) void k_beam_prep(RayArgs a, Geom g, const double* __restrict__ pose4,
                                                   const float* __restrict__ ranges,
                                                   const double* __restrict__ trig,
                                                   Beam* __restrict__ beams, int32_t* tile_count,
                                                   int32_t* tile_slot, int32_t* act_tiles,
                                                   unsigned long long* cnt) {
  __shared__ int32_t hkey[kHash];
  __shared__ int32_t hcnt[kHash];
  const int tid = threadIdx.x;
  for (int e = tid; e < kHash; e += 256) { hkey[e] = -1; hcnt[e] = 0; }
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + tid;
  const int64_t nb = (int64_t)a.S * a.N;
  if (b < nb) {
    const int32_t s = (int32_t)(b / a.N), i = (int32_t)(b % a.N);
    const Beam bm = dm_make_beam(a, pose4, ranges, trig, s, i);
    beams[b] = bm;
    if (bm.flags & 1) {
      dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t, int32_t) {
        const int h = hash_insert(hkey, tile);
        if (h >= 0) {
          atomicAdd(&hcnt[h], 1);
        } else {
          const int32_t old = atomicAdd(&tile_count[tile], 1);
          first_touch(g, tile, old, tile_slot, act_tiles, cnt);
        }
      });
    }
  }
  __syncthreads();
  for (int e = tid; e < kHash; e += 256) {
    const int32_t tile = hkey[e];
    if (tile < 0) continue;
    const int32_t old = atomicAdd(&tile_count[tile], hcnt[e]);
    first_touch(g, tile, old, tile_slot, act_tiles, cnt);
  }
}

// Work plan for the apply phase (one block).  Per active tile j with c_j
// pieces: exclusive scans of c_j (bin offsets), of ceil(c_j / kChunk) (work
// items) and of [c_j > kChunk] (heavy-tile ordinals).  A light tile is one
// work item that accumulates AND applies; a heavy tile's pieces are split
// into kChunk-piece items on different CUs that merge their counts in a
// per-tile slab, applied by k_heavy_apply.
constexpr int kChunk = 256;
static_assert(kChunk < 65536, "packed 16-bit LDS counts");

__device__ inline void block_scan3(int64_t v[3], int64_t excl[3], int64_t tot[3], int64_t (*ws)[3]) {
  const int tid = threadIdx.x, lane = __lane_id(), wid = tid >> 6;
  int64_t incl[3] = {v[0], v[1], v[2]};
  for (int d = 1; d < 64; d <<= 1) {
    for (int q = 0; q < 3; ++q) {
      const int64_t t = __shfl_up(incl[q], d);
      if (lane >= d) incl[q] += t;
    }
  }
  if (lane == 63) for (int q = 0; q < 3; ++q) ws[wid][q] = incl[q];
  __syncthreads();
  if (tid == 0) {
    int64_t run[3] = {0, 0, 0};
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
      for (int q = 0; q < 3; ++q) { const int64_t t = ws[w][q]; ws[w][q] = run[q]; run[q] += t; }
    for (int q = 0; q < 3; ++q) ws[16][q] = run[q];
  }
  __syncthreads();
  for (int q = 0; q < 3; ++q) {
    excl[q] = ws[wid][q] + incl[q] - v[q];
    tot[q] = ws[16][q];
  }
}

__global__ __launch_bounds__(1024) void k_plan(Geom g, const int32_t* __restrict__ act_tiles,
                                               const int32_t* __restrict__ tile_count,
                                               int32_t* __restrict__ act_off, int32_t* __restrict__ act_cur,
                                               int32_t* __restrict__ act_heavy,
                                               int32_t* __restrict__ heavy_list,
                                               int2* __restrict__ items, unsigned long long* cnt) {
  __shared__ int64_t ws[17][3];
  const int tid = threadIdx.x;
  const int64_t n = min((int64_t)cnt[CNT_ACTIVE], (int64_t)g.act_cap);
  const int64_t per = (n + 1023) / 1024;
  const int64_t lo = min((int64_t)tid * per, n), hi = min(lo + per, n);
  int64_t v[3] = {0, 0, 0};
  for (int64_t j = lo; j < hi; ++j) {
    const int64_t c = tile_count[act_tiles[j]];
    v[0] += c;
    v[1] += (c + kChunk - 1) / kChunk;
    v[2] += c > kChunk;
  }
  int64_t ex[3], tot[3];
  block_scan3(v, ex, tot, ws);
  if (tid == 0) {
    cnt[CNT_SEGS] = (unsigned long long)tot[0];
    cnt[CNT_ITEMS] = (unsigned long long)min(tot[1], g.item_cap);
    cnt[CNT_HEAVY] = (unsigned long long)min(tot[2], g.heavy_cap);
    if (tot[1] > g.item_cap || tot[2] > g.heavy_cap) atomicOr(&cnt[CNT_OVERFLOW], 8ull);
  }
  for (int64_t j = lo; j < hi; ++j) {
    const int64_t c = tile_count[act_tiles[j]];
    act_off[j] = (int32_t)ex[0];
    act_cur[j] = (int32_t)ex[0];
    const int64_t ni = (c + kChunk - 1) / kChunk;
    const bool heavy = c > kChunk;
    act_heavy[j] = heavy && ex[2] < g.heavy_cap ? (int32_t)ex[2] : -1;
    if (heavy && ex[2] < g.heavy_cap) heavy_list[ex[2]] = (int32_t)j;
    for (int64_t q = 0; q < ni; ++q)
      if (ex[1] + q < g.item_cap) items[ex[1] + q] = make_int2((int32_t)j, (int32_t)q);
    ex[0] += c;
    ex[1] += ni;
    ex[2] += heavy;
  }
}

__device__ inline void put_seg(const Geom& g, Seg* segs, int64_t idx, int64_t b, int32_t k0,
                               int32_t k1, unsigned long long* cnt) {
  if (idx >= 0 && idx < g.seg_cap) {
    Seg sg;
    sg.beam = (uint32_t)b;
    sg.k0 = (uint16_t)k0;
    sg.k1 = (uint16_t)k1;
    segs[idx] = sg;
  } else {
    atomicOr(&cnt[CNT_OVERFLOW], 2ull);
  }
}

// Pieces -> per-tile bins.  Same LDS histogram as k_beam_prep; one global
// cursor bump per (block, tile), then LDS cursors place each piece.
__global__ __launch_bounds__(256) void k_scatter(RayArgs a, Geom g, const Beam* __restrict__ beams,
                                                 const int32_t* __restrict__ tile_slot,
                                                 int32_t* act_cur, Seg* __restrict__ segs,
                                                 unsigned long long* cnt) {
  __shared__ int32_t hkey[kHash];
  __shared__ int32_t hcnt[kHash];
  __shared__ int32_t hbase[kHash];
  const int tid = threadIdx.x;
  for (int e = tid; e < kHash; e += 256) { hkey[e] = -1; hcnt[e] = 0; }
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + tid;
  const int64_t nb = (int64_t)a.S * a.N;
  Beam bm;
  bm.flags = 0;
  if (b < nb) bm = beams[b];
  const bool valid = (b < nb) && (bm.flags & 1);
  if (valid) {
    dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t k0, int32_t k1) {
      const int h = hash_insert(hkey, tile);
      if (h >= 0) {
        atomicAdd(&hcnt[h], 1);
      } else {
        const int32_t slot = tile_slot[tile];
        const int64_t idx = (slot >= 0 && slot < g.act_cap) ? (int64_t)atomicAdd(&act_cur[slot], 1) : -1;
        put_seg(g, segs, idx, b, k0, k1, cnt);
      }
    });
  }
  __syncthreads();
  for (int e = tid; e < kHash; e += 256) {
    const int32_t tile = hkey[e];
    if (tile < 0) continue;
    const int32_t slot = tile_slot[tile];
    hbase[e] = (slot >= 0 && slot < g.act_cap) ? atomicAdd(&act_cur[slot], hcnt[e]) : -1;
    hcnt[e] = 0;
  }
  __syncthreads();
  if (valid) {
    dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t k0, int32_t k1) {
      const int h = hash_find(hkey, tile);
      if (h < 0) return;  // placed by the global path above
      const int32_t base = hbase[h];
      const int64_t idx = base >= 0 ? (int64_t)base + atomicAdd(&hcnt[h], 1) : -1;
      put_seg(g, segs, idx, b, k0, k1, cnt);
    });
  }
}

struct ApplyArgs {
  float l_occ, l_free, l_min, l_max, occ_t, free_t;
};

__device__ inline int8_t state_of(const ApplyArgs& p, float L) {
  if (L == 0.0f) return -1;
  if (L >= p.occ_t) return 100;
  if (L <= p.free_t) return 0;
  return -1;
}

// SPEC a6 in this exact op order (no FMA: -ffp-contract=off).
__device__ inline float apply_one(const ApplyArgs& p, float L, uint32_t h, uint32_t m) {
  const float t = (float)h * p.l_occ;
  const float u = (float)m * p.l_free;
  L = L + t;
  L = L + u;
  if (L < p.l_min) L = p.l_min;
  if (L > p.l_max) L = p.l_max;
  return L;
}

// Log-odds update of one tile from per-cell counts (SPEC a6/a7): thread ->
// 4 consecutive cells of a row (float4 / char4 accesses), 16 threads per row.
// counts(ly, cx, h4, m4) supplies the counts.  Adds to *sh_T / *sh_free.
template <class Counts>
__device__ inline void apply_tile(const Geom& g, const ApplyArgs& p, int32_t tx0, int32_t ty0,
                                  float* __restrict__ L, int8_t* __restrict__ state, int vec_ok,
                                  Counts&& counts, int32_t* sh_T, int32_t* sh_free) {
  constexpr int kRows = DM_TS / 16;
  const int tid = threadIdx.x;
  int32_t dT = 0, dFree = 0;
  const int cx = (tid & 15) * 4;
  uint32_t h4[kRows][4], m4[kRows][4];
  bool any[kRows];
  int64_t base[kRows];
#pragma unroll
  for (int rr = 0; rr < kRows; ++rr) {
    const int ly = (tid >> 4) + 16 * rr;
    counts(ly, cx, h4[rr], m4[rr]);
    any[rr] = (ty0 + ly < g.r.R) &&
              ((h4[rr][0] | m4[rr][0]) | (h4[rr][1] | m4[rr][1]) | (h4[rr][2] | m4[rr][2]) |
               (h4[rr][3] | m4[rr][3])) != 0u;
    base[rr] = (int64_t)(ty0 + ly) * g.r.W + tx0 + cx;
  }
  const bool vec = vec_ok && tx0 + cx + 4 <= g.r.W;
  if (vec) {
    // issue every row's loads before the first use: one memory latency
    float4 l4[kRows];
    char4 s4[kRows];
#pragma unroll
    for (int rr = 0; rr < kRows; ++rr) {
      if (any[rr]) {
        l4[rr] = *reinterpret_cast<const float4*>(L + base[rr]);
        s4[rr] = *reinterpret_cast<const char4*>(state + base[rr]);
      }
    }
#pragma unroll
    for (int rr = 0; rr < kRows; ++rr) {
      if (!any[rr]) continue;
      float lv[4] = {l4[rr].x, l4[rr].y, l4[rr].z, l4[rr].w};
      int8_t sv[4] = {(int8_t)s4[rr].x, (int8_t)s4[rr].y, (int8_t)s4[rr].z, (int8_t)s4[rr].w};
      for (int e = 0; e < 4; ++e) {
        if ((h4[rr][e] | m4[rr][e]) == 0u) continue;
        const int8_t old = sv[e];
        lv[e] = apply_one(p, lv[e], h4[rr][e], m4[rr][e]);
        sv[e] = state_of(p, lv[e]);
        dT += 1;
        dFree += (sv[e] == 0) - (old == 0);
      }
      *reinterpret_cast<float4*>(L + base[rr]) = make_float4(lv[0], lv[1], lv[2], lv[3]);
      *reinterpret_cast<char4*>(state + base[rr]) = make_char4(sv[0], sv[1], sv[2], sv[3]);
    }
  } else {
    for (int rr = 0; rr < kRows; ++rr) {
      if (!any[rr]) continue;
      for (int e = 0; e < 4; ++e) {
        if ((h4[rr][e] | m4[rr][e]) == 0u) continue;
        if (tx0 + cx + e >= g.r.W) continue;
        const int64_t i = base[rr] + e;
        const int8_t old = state[i];
        const float nl = apply_one(p, L[i], h4[rr][e], m4[rr][e]);
        const int8_t ns = state_of(p, nl);
        L[i] = nl;
        state[i] = ns;
        dT += 1;
        dFree += (ns == 0) - (old == 0);
      }
    }
  }
  if (dT) atomicAdd(sh_T, dT);
  if (dFree) atomicAdd(sh_free, dFree);
}

// One work item = up to kChunk pieces of one tile.  Pieces (and their beams)
// are staged in LDS by all 256 lanes at once; each wave then walks pieces with
// its lanes along the piece's major axis (up to 64 cells per wave-instruction,
// distinct cells, LDS atomics).  A light tile (one item) applies its counts
// right away; a heavy tile's item adds its non-zero counts to the tile's slab
// with row-contiguous global atomics (256 B per wave-instruction).
__global__ __launch_bounds__(kApplyThreads) void k_tile_accum(
    Geom g, ApplyArgs p, const int2* __restrict__ items, const int32_t* __restrict__ act_tiles,
    const int32_t* __restrict__ act_off, const int32_t* __restrict__ act_heavy,
    const Seg* __restrict__ segs, const Beam* __restrict__ beams, int32_t* tile_count,
    int32_t* tile_free, uint32_t* __restrict__ slabs, float* __restrict__ L,
    int8_t* __restrict__ state, unsigned long long* cnt, int vec_ok) {
  // per-cell counts of this item, packed: hits << 16 | misses.  An item has
  // at most kChunk = 256 pieces and a piece visits a cell at most once, so
  // neither half can exceed 256: no carry between the halves.
  __shared__ uint32_t cnt16[DM_TS * kLdsPitch];
  __shared__ Seg s_seg[kChunk];
  __shared__ Beam s_beam[kChunk];
  __shared__ int32_t sh_free, sh_T;
  __shared__ uint32_t sh_U;
  const int tid = threadIdx.x, lane = lane_id();
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t n_items = (int64_t)cnt[CNT_ITEMS];
  for (int64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int2 item = items[it];
    const int32_t j = item.x;
    const int32_t tile = act_tiles[j];
    const int32_t count = tile_count[tile];
    const int32_t heavy = act_heavy[j];
    const int32_t c0 = act_off[j] + item.y * kChunk;
    const int32_t nseg = min(kChunk, act_off[j] + count - c0);
    for (int e = tid; e < DM_TS * kLdsPitch; e += kApplyThreads) cnt16[e] = 0u;
    if (tid == 0) { sh_free = 0; sh_T = 0; sh_U = 0u; }
    if (tid < nseg) {
      const Seg sg = segs[c0 + tid];
      s_seg[tid] = sg;
      if ((int64_t)sg.beam < g.nb) {
        s_beam[tid] = beams[sg.beam];
      } else {  // cannot happen; keeps a logic error in-bounds
        Beam z;
        z.flags = 0;
        s_beam[tid] = z;
      }
    }
    __syncthreads();
    const int32_t tx0 = (tile % g.r.TX) * DM_TS;
    const int32_t ty0 = (tile / g.r.TX) * DM_TS;  // band-local
    uint32_t myU = 0;
    for (int si = wid; si < nseg; si += kApplyThreads / 64) {
      const Seg sg = s_seg[si];
      const Beam bm = s_beam[si];
      const int32_t k = (int32_t)sg.k0 + lane;
      if (k <= (int32_t)sg.k1 && (bm.flags & 1)) {
        int32_t x, yl;
        dm_cell(bm, k, g.r.row0, &x, &yl);
        const int32_t lx = x - tx0, ly = yl - ty0;
        if (x >= 0 && x < g.r.W && yl >= 0 && yl < g.r.R && (uint32_t)lx < DM_TS && (uint32_t)ly < DM_TS) {
          const bool is_hit = (k == bm.n) && (bm.flags & 2);
          atomicAdd(&cnt16[ly * kLdsPitch + lx], is_hit ? 0x10000u : 1u);
          ++myU;
        }
      }
    }
    if (myU) atomicAdd(&sh_U, myU);
    __syncthreads();
    if (heavy < 0) {
      apply_tile(g, p, tx0, ty0, L, state, vec_ok,
                 [&](int ly, int cx, uint32_t* h4, uint32_t* m4) {
                   for (int e = 0; e < 4; ++e) {
                     const uint32_t v = cnt16[ly * kLdsPitch + cx + e];
                     h4[e] = v >> 16;
                     m4[e] = v & 0xFFFFu;
                   }
                 },
                 &sh_T, &sh_free);
    } else {
      uint32_t* sh = slabs + (int64_t)heavy * (2 * DM_TS * DM_TS);
      for (int e = tid; e < DM_TS * DM_TS; e += kApplyThreads) {
        const int ly = e >> 6, lx = e & 63;
        const uint32_t v = cnt16[ly * kLdsPitch + lx];
        const uint32_t h = v >> 16, m = v & 0xFFFFu;
        if (h) atomicAdd(&sh[e], h);
        if (m) atomicAdd(&sh[DM_TS * DM_TS + e], m);
      }
    }
    __syncthreads();
    if (tid == 0) {
      if (sh_T) atomicAdd(&cnt[CNT_T], (unsigned long long)sh_T);
      if (sh_U) atomicAdd(&cnt[CNT_U], (unsigned long long)sh_U);
      if (heavy < 0) {
        tile_free[tile] += sh_free;
        tile_count[tile] = 0;  // ready for the next call
      }
    }
    __syncthreads();
  }
}

// Heavy tiles: apply the merged slab counts, then clear the slab and the
// tile's piece count for the next call.
__global__ __launch_bounds__(kApplyThreads) void k_heavy_apply(
    Geom g, ApplyArgs p, const int32_t* __restrict__ heavy_list, const int32_t* __restrict__ act_tiles,
    int32_t* tile_count, int32_t* tile_free, uint32_t* __restrict__ slabs, float* __restrict__ L,
    int8_t* __restrict__ state, unsigned long long* cnt, int vec_ok) {
  __shared__ int32_t sh_free, sh_T;
  const int tid = threadIdx.x;
  const int64_t nh = (int64_t)cnt[CNT_HEAVY];
  for (int64_t h = blockIdx.x; h < nh; h += gridDim.x) {
    const int32_t tile = act_tiles[heavy_list[h]];
    if (tid == 0) { sh_free = 0; sh_T = 0; }
    __syncthreads();
    uint32_t* sh = slabs + h * (2 * DM_TS * DM_TS);
    const int32_t tx0 = (tile % g.r.TX) * DM_TS;
    const int32_t ty0 = (tile / g.r.TX) * DM_TS;
    apply_tile(g, p, tx0, ty0, L, state, vec_ok,
               [&](int ly, int cx, uint32_t* h4, uint32_t* m4) {
                 const uint4 a = *reinterpret_cast<const uint4*>(sh + ly * DM_TS + cx);
                 const uint4 b = *reinterpret_cast<const uint4*>(sh + DM_TS * DM_TS + ly * DM_TS + cx);
                 h4[0] = a.x; h4[1] = a.y; h4[2] = a.z; h4[3] = a.w;
                 m4[0] = b.x; m4[1] = b.y; m4[2] = b.z; m4[3] = b.w;
               },
               &sh_T, &sh_free);
    // clear all 64 rows (apply_tile stops at the band's last row)
    for (int e = tid * 4; e < 2 * DM_TS * DM_TS; e += kApplyThreads * 4)
      *reinterpret_cast<uint4*>(sh + e) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if (tid == 0) {
      if (sh_T) {
        atomicAdd(&cnt[CNT_T], (unsigned long long)sh_T);
        atomicAdd(&cnt[CNT_TH], (unsigned long long)sh_T);
      }
      tile_free[tile] += sh_free;
      tile_count[tile] = 0;
    }
    __syncthreads();
  }
}

// ---- maintenance kernels ----------------------------------------------------

__global__ __launch_bounds__(256) void k_recount(Geom g, const int8_t* __restrict__ state,
                                                 int32_t* __restrict__ tile_free) {
  const int64_t tile = blockIdx.x;
  const int32_t tx0 = (int32_t)(tile % g.r.TX) * DM_TS, ty0 = (int32_t)(tile / g.r.TX) * DM_TS;
  __shared__ int32_t acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  int32_t c = 0;
  for (int e = threadIdx.x; e < DM_TS * DM_TS; e += 256) {
    const int32_t x = tx0 + (e & 63), y = ty0 + (e >> 6);
    if (x < g.r.W && y < g.r.R) c += state[(int64_t)y * g.r.W + x] == 0;
  }
  if (c) atomicAdd(&acc, c);
  __syncthreads();
  if (threadIdx.x == 0) tile_free[tile] = acc;
}

__global__ __launch_bounds__(256) void k_state_from_l(ApplyArgs p, int64_t cells, const float* __restrict__ L,
                                                      int8_t* __restrict__ state) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x)
    state[i] = state_of(p, L[i]);
}

__global__ __launch_bounds__(256) void k_set_state(ApplyArgs p, int64_t cells, const int8_t* __restrict__ in,
                                                   float* __restrict__ L, int8_t* __restrict__ state) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int8_t v = in[i];
    const float l = v == 100 ? p.l_occ : (v == 0 ? p.l_free : 0.0f);
    L[i] = l;
    state[i] = state_of(p, l);
  }
}

// f2: get_map_image's mapping (server/thymio_project/thymio_project/main.py:
// 258-266): 0 -> 255, 100 -> 0, else 127, rows flipped.
__global__ __launch_bounds__(256) void k_map_image(int64_t R, int64_t W, const int8_t* __restrict__ state,
                                                   uint8_t* __restrict__ img) {
  const int64_t cells = R * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t y = i / W, x = i - y * W;
    const int8_t v = state[i];
    img[(R - 1 - y) * W + x] = v == 0 ? 255 : (v == 100 ? 0 : 127);
  }
}

Geom make_geom(const dm_grid* g) {
  Geom ge;
  ge.r.W = (int32_t)g->W;
  ge.r.R = (int32_t)g->R;
  ge.r.row0 = (int32_t)g->row0;
  ge.r.TX = (int32_t)g->TX;
  ge.r.TY = (int32_t)g->TY;
  ge.act_cap = (int32_t)g->act_cap;
  ge.seg_cap = g->segs_cap;
  ge.item_cap = g->item_cap;
  ge.heavy_cap = g->heavy_cap;
  ge.nb = 0;
  return ge;
}

ApplyArgs make_apply(const dm_grid* g) {
  ApplyArgs a;
  a.l_occ = g->p.l_occ;
  a.l_free = g->p.l_free;
  a.l_min = g->p.l_min;
  a.l_max = g->p.l_max;
  a.occ_t = g->p.occ_thresh;
  a.free_t = g->p.free_thresh;
  return a;
}

int grid_for(int64_t n, int threads, int64_t cap = 8192) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

int dm_launch_integrate(dm_grid* g, int32_t S, const double* d_pose4, int32_t N,
                        const float* d_ranges, const double* d_trig) {
  const int64_t nb = (int64_t)S * N;
  DM_HIP(hipMemsetAsync(g->cnt, 0, sizeof(unsigned long long) * CNT_N, g->stream));
  if (nb == 0) return DM_OK;
  RayArgs a;
  a.S = S;
  a.N = N;
  a.ox = g->p.origin_x;
  a.oy = g->p.origin_y;
  a.res = g->p.resolution;
  a.range_min = g->p.range_min;
  a.range_max = g->p.range_max;
  Geom ge = make_geom(g);
  ge.nb = nb;
  const int nblk = (int)((nb + 255) / 256);
  KernelTimer t;
  dm_timer_begin(g, "beam_prep", &t);
  hipLaunchKernelGGL(k_beam_prep, dim3(nblk), dim3(256), 0, g->stream, a, ge, d_pose4, d_ranges,
                     d_trig, g->beams, g->tile_count, g->tile_slot, g->act_tiles, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "plan", &t);
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, g->stream, ge, g->act_tiles, g->tile_count,
                     g->act_off, g->act_cur, g->act_heavy, g->heavy_list, g->items, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "scatter", &t);
  hipLaunchKernelGGL(k_scatter, dim3(nblk), dim3(256), 0, g->stream, a, ge, g->beams,
                     g->tile_slot, g->act_cur, g->segs, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  const int vec_ok = (g->W % 4 == 0) ? 1 : 0;
  dm_timer_begin(g, "tile_accum", &t);
  hipLaunchKernelGGL(k_tile_accum, dim3(grid_for(g->item_cap, 1, 4096)), dim3(kApplyThreads), 0,
                     g->stream, ge, make_apply(g), g->items, g->act_tiles, g->act_off, g->act_heavy,
                     g->segs, g->beams, g->tile_count, g->tile_free, g->slabs, g->L, g->state,
                     g->cnt, vec_ok);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "heavy_apply", &t);
  hipLaunchKernelGGL(k_heavy_apply, dim3(grid_for(g->heavy_cap, 1, 2048)), dim3(kApplyThreads), 0,
                     g->stream, ge, make_apply(g), g->heavy_list, g->act_tiles, g->tile_count,
                     g->tile_free, g->slabs, g->L, g->state, g->cnt, vec_ok);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_recount(dm_grid* g) {
  const Geom ge = make_geom(g);
  hipLaunchKernelGGL(k_recount, dim3((unsigned)g->NT), dim3(256), 0, g->stream, ge, g->state,
                     g->tile_free);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_state_from_logodds(dm_grid* g) {
  const int64_t cells = g->R * g->W;
  hipLaunchKernelGGL(k_state_from_l, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream,
                     make_apply(g), cells, g->L, g->state);
  DM_HIP(hipGetLastError());
  return dm_launch_recount(g);
}

int dm_launch_set_state(dm_grid* g, const int8_t* d_in) {
  const int64_t cells = g->R * g->W;
  hipLaunchKernelGGL(k_set_state, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream,
                     make_apply(g), cells, d_in, g->L, g->state);
  DM_HIP(hipGetLastError());
  return dm_launch_recount(g);
}

int dm_launch_map_image(dm_grid* g, uint8_t* d_img) {
  const int64_t cells = g->R * g->W;
  hipLaunchKernelGGL(k_map_image, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream, g->R,
                     g->W, g->state, d_img);
  DM_HIP(hipGetLastError());
  return DM_OK;
}
