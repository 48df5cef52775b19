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
//   k_beam_prep   one thread per beam (or beam chunk): endpoint cells (double,
//                 no FMA), Bresenham params, per-block LDS histogram of pieces
//                 per tile -> tile_count, first-touch lists of active tiles
//   k_plan        one thread per active tile: its bin and work items by
//                 wave-aggregated bumps
//   k_scatter     one thread per beam: pieces -> per-tile bins (packed)
//   k_tile_accum  one workgroup per work item: LDS counts + fused apply;
//                 heavy tiles merged in slabs, sparse tiles load only the
//                 cells they touch
#include "dm_internal.h"
#include "dm_phase.h"

#include <algorithm>

DM_PH_DECL(integrate)
DM_TL_DECL(accum)

namespace {

constexpr int kLdsPitch = DM_TS + 1;  // +1 dword: y-major pieces hit distinct banks

struct Geom {
  RayGeom r;
  int32_t act_cap;
  int64_t seg_cap;
  int64_t hitem_cap, heavy_cap;  // capacities of hitems / heavy_list (k_plan clamps its writes)
  int64_t nb;  // beams in this call
  int32_t chunks, chunk_len;  // each beam enumerated as `chunks` k-ranges (dm_integrate_chunks)
  int32_t sparse_pieces;  // light tiles with at most this many pieces are sparse items
  int32_t pad;
};

// Thread v of k_beam_prep / k_scatter: beam v % nb, k-range v / nb (chunk-
// major, so a wave's lanes stay on neighbouring beams and the lane-run /
// per-block tile aggregation keeps working).  The last chunk runs to the end.
struct BeamChunk {
  int64_t b;
  int32_t k_lo, k_hi;
};

__device__ inline BeamChunk beam_chunk(const Geom& g, int64_t v) {
  BeamChunk c;
  if (g.chunks == 1) {
    c.b = v; c.k_lo = 0; c.k_hi = 0x7FFFFFFF;
    return c;
  }
  const int32_t q = (int32_t)(v / g.nb);
  c.b = v - (int64_t)q * g.nb;
  c.k_lo = q * g.chunk_len;
  c.k_hi = q + 1 == g.chunks ? 0x7FFFFFFF : c.k_lo + g.chunk_len - 1;
  return c;
}

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

// Loop-free wave aggregation of the pieces emitted by the active lanes right
// now: a run is a maximal group of consecutive active lanes with the same
// tile (lane i+1 holds the next beam of the scan, so most pieces of a wave
// fall in a few runs).  Only the head lane of a run touches the hash table /
// global counters, with the run's length; the others take a rank in the run.
struct LaneRun {
  bool head;
  int head_lane;
  int len;   // valid in the head lane
  int rank;  // active lanes of the run before this lane
};

__device__ inline LaneRun lane_run(int32_t tile) {
  const int lane = lane_id();
  const unsigned long long act = __ballot(1);
  const int32_t prev = __shfl_up(tile, 1);
  const bool prev_act = lane > 0 && ((act >> (lane - 1)) & 1ull);
  const bool head = !(prev_act && prev == tile);
  const unsigned long long heads = __ballot(head);
  const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= lane
  LaneRun r;
  r.head = head;
  r.head_lane = 63 - __clzll(heads & le);
  const unsigned long long after = heads & ~le;
  const unsigned long long before_end = after ? ((1ull << (__ffsll(after) - 1)) - 1ull) : ~0ull;
  const unsigned long long from_head = ~((1ull << r.head_lane) - 1ull);
  r.len = __popcll(act & from_head & before_end);
  r.rank = __popcll(act & from_head & ((1ull << lane) - 1ull));
  return r;
}

// First touch of a tile in this call: append it to this workgroup's shard of
// the active list (k_plan compacts the shards and assigns tile slots).
__device__ inline void first_touch(const Geom& g, int32_t tile, int32_t old, int32_t* act_raw,
                                   unsigned long long* ish, unsigned long long* cnt) {
  if (old != 0) return;
  const int sh = blockIdx.x % kShards;
  const unsigned long long l = atomicAdd(&ish[sh * kShardWords + SH_ACT], 1ull);
  if (l < (unsigned long long)g.act_cap) act_raw[(int64_t)sh * g.act_cap + (int64_t)l] = tile;
  else atomicOr(&cnt[CNT_IOVERFLOW], 1ull);
}

// A piece as k_tile_accum consumes it: tile-local LDS addresses (pitch
// kLdsPitch), packed to 16 bytes (dm_ray.h).
__device__ inline PackedPiece make_piece(const Geom& g, const Beam& bm, int32_t tile, int32_t k0, int32_t k1) {
  const int32_t tx0 = (tile % g.r.TX) * DM_TS;
  const int32_t ty0 = (tile / g.r.TX) * DM_TS;
  return dm_pack_piece(dm_tile_piece(bm, k0, k1, g.r.row0, tx0, ty0, kLdsPitch));
}

__global__ __launch_bounds__(256) void k_beam_prep(RayArgs a, Geom g, const double* __restrict__ pose4,
                                                   const float* __restrict__ ranges,
                                                   const double* __restrict__ trig,
                                                   Beam* __restrict__ beams, int32_t* tile_count,
                                                   int32_t* act_raw, unsigned long long* ish,
                                                   int2* __restrict__ blk_hist, int32_t* __restrict__ blk_n,
                                                   unsigned long long* cnt) {
  __shared__ int32_t hkey[kHash];
  __shared__ int32_t hcnt[kHash];
  __shared__ int32_t s_nh;
  const int tid = threadIdx.x;
  for (int e = tid; e < kHash; e += 256) { hkey[e] = -1; hcnt[e] = 0; }
  if (tid == 0) s_nh = 0;
  __syncthreads();
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + tid;
  if (v < g.nb * g.chunks) {
    const BeamChunk bc = beam_chunk(g, v);
    const int32_t s = (int32_t)(bc.b / a.N), i = (int32_t)(bc.b % a.N);
    const Beam bm = dm_make_beam(a, pose4, ranges, trig, s, i);
    if (bc.k_lo == 0) beams[bc.b] = bm;
    if ((bm.flags & 1) && bc.k_lo <= bm.n) {
      dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t, int32_t) {
        const LaneRun run = lane_run(tile);
        if (run.head) {
          const int h = hash_insert(hkey, tile);
          if (h >= 0) {
            atomicAdd(&hcnt[h], run.len);
          } else {
            const int32_t old = atomicAdd(&tile_count[tile], run.len);
            first_touch(g, tile, old, act_raw, ish, cnt);
          }
        }
      }, bc.k_lo, bc.k_hi);
    }
  }
  __syncthreads();
  // flush the histogram, and keep it (compacted) for k_scatter: its single
  // placement pass then needs no counting pass of its own
  int2* my_hist = blk_hist + (int64_t)blockIdx.x * kHash;
  for (int e = tid; e < kHash; e += 256) {
    const int32_t tile = hkey[e];
    if (tile < 0) continue;
    const int32_t old = atomicAdd(&tile_count[tile], hcnt[e]);
    first_touch(g, tile, old, act_raw, ish, cnt);
    my_hist[atomicAdd(&s_nh, 1)] = make_int2(tile, hcnt[e] | (e << 16));
  }
  __syncthreads();
  if (tid == 0) blk_n[blockIdx.x] = s_nh;
}

// Work plan for the apply phase (one block).  A tile's pieces are cut into
// work items of at most kChunk (= one per thread of a 256-thread workgroup).
// A light tile (<= kChunk pieces) is one item that accumulates AND applies;
// a heavy tile (around a sensor: up to every beam of a scan starts there) is
// split into several items on different CUs that merge their counts in a
// per-tile slab, applied by the tile's last item.  Per active tile j with c_j
// pieces, exclusive scans of: c_j (bin offsets), heavy items, light items,
// heavy ordinals.  Heavy items are listed first (they are the long ones).
// Item = {tile, first piece, pieces, slab code or -1 (light / medium)}.
constexpr int kChunk = kIntegrateChunk;
// Tiles with more pieces than kChunk but at most kMedium (the ring around a
// sensor: rays fan out, so a per-thread walk does not pile onto one cell) are
// one item walked in rounds; only tiles beyond kMedium (the sensor's own)
// are split over workgroups and merged in a slab.
constexpr int kMedium = kIntegrateMedium;
static_assert(kMedium < 65536, "packed 16-bit LDS counts of medium tiles");
constexpr int kTileWords = DM_TS * kLdsPitch;
constexpr int kQuarter = 256;  // threads of an apply workgroup (= kChunk)
static_assert(kChunk < 65536, "packed 16-bit LDS counts");
static_assert(kChunk == kQuarter, "one piece per thread");


constexpr int kPlanThreads = 256;

// Wave-aggregated bump allocation of K counters at once: every active lane
// gets v[k] lane-exclusive units of counter k (out[k]: its first unit), with
// ONE atomic instruction per wave for all K counters.
template <int K>
__device__ inline void wave_alloc_n(unsigned long long* const (&counter)[K], const unsigned long long (&v)[K],
                                    unsigned long long (&out)[K]) {
  const int lane = __lane_id();
  unsigned long long incl[K], total[K], base[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    incl[k] = v[k];
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long t = __shfl_up(incl[k], d);
      if (lane >= d) incl[k] += t;
    }
    total[k] = __shfl(incl[k], 63);
    base[k] = 0ull;
  }
  // lane 63 - k adds counter k's total: K lanes, K different addresses, ONE
  // atomic instruction (a uniform-address atomic per counter would each be
  // expanded by the compiler's atomic optimizer and waited for in turn)
  const int kk = 63 - lane;
  unsigned long long* addr = counter[0];
  unsigned long long mine = 0ull;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (kk == k) { addr = counter[k]; mine = total[k]; }
  unsigned long long got = 0ull;
  if (kk < K) got = atomicAdd(addr, mine);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    base[k] = __shfl(got, 63 - k);
    out[k] = base[k] + incl[k] - v[k];
  }
}

// Work plan for the apply phase, one thread per active tile and no global
// scan: bin order does not matter, so each tile's bin (its pieces' range in
// `pieces`) and its work items are bump-allocated with wave-aggregated
// atomics (wave_alloc_n: one round trip for all five counters; the former
// one-call-per-counter form waited for each in turn, k_plan 9.8 -> 8.4 us at C3).  Writes k_scatter's bin cursor per tile and the
// items; counters: pieces, heavy + medium items, light items, sparse items, heavy tiles.
__global__ __launch_bounds__(kPlanThreads) void k_plan(Geom g, const int32_t* __restrict__ act_raw,
                                                       const unsigned long long* __restrict__ ish,
                                                       int32_t* __restrict__ tile_cur,
                                                       const int32_t* __restrict__ tile_count,
                                                       int4* __restrict__ hitems, int4* __restrict__ litems,
                                                       int32_t* __restrict__ heavy_list,
                                                       unsigned long long* cnt) {
  __shared__ int32_t soff[kShards + 1];
  const int tid = threadIdx.x, lane = __lane_id();
  if (tid < 64) {  // shard offsets of the first-touch lists (every workgroup)
    const int32_t c = tid < kShards ? (int32_t)min((unsigned long long)g.act_cap, ish[tid * kShardWords + SH_ACT]) : 0;
    int32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t t = __shfl_up(incl, d);
      if (lane >= d) incl += t;
    }
    if (tid < kShards) soff[tid] = incl - c;
    if (tid == kShards - 1) soff[kShards] = incl;
  }
  __syncthreads();
  const int64_t n = min((int64_t)soff[kShards], (int64_t)g.act_cap);
  if (blockIdx.x == 0 && tid == 0) cnt[CNT_ACTIVE] = (unsigned long long)n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + (tid & ~63); j0 < n; j0 += stride) {
    const int64_t j = j0 + lane;
    int32_t t = -1, c = 0;
    if (j < n) {
      int a = 0, b = kShards - 1;  // largest shard with soff[shard] <= j
      while (a < b) {
        const int mid = (a + b + 1) >> 1;
        if (soff[mid] <= j) a = mid; else b = mid - 1;
      }
      t = act_raw[(int64_t)a * g.act_cap + (j - soff[a])];
      c = tile_count[t];
    }
    const bool heavy = c > kMedium;
    const bool medium = c > kChunk && !heavy;
    const bool sparse = t >= 0 && c <= g.sparse_pieces;
    const bool light = t >= 0 && c <= kChunk && !sparse;
    const int32_t nh_items = heavy ? (c + kChunk - 1) / kChunk : (medium ? 1 : 0);
    unsigned long long* const ctr[5] = {&cnt[CNT_SEGS], &cnt[CNT_ITEMS], &cnt[CNT_LITEMS], &cnt[CNT_SITEMS],
                                        &cnt[CNT_HEAVY]};
    const unsigned long long want[5] = {(unsigned long long)c, (unsigned long long)nh_items, light ? 1ull : 0ull,
                                        sparse ? 1ull : 0ull, heavy ? 1ull : 0ull};
    unsigned long long got[5];
    wave_alloc_n<5>(ctr, want, got);
    const unsigned long long p0 = got[0], hi = got[1], li = got[2], si = got[3], ho = got[4];
    if (t < 0) continue;
    tile_cur[t] = (int32_t)p0;  // k_scatter's cursor: the tile's bin start
    // the host sizes every list for the worst case (grow_integrate); a write
    // past a capacity anyway is flagged (DM_ERR_CAPACITY) and dropped
    // light items fill litems from the bottom, sparse ones from the top: a
    // tile is one or the other, so the two never meet below act_cap tiles
    const bool fits = (int64_t)(p0 + c) <= g.seg_cap && (int64_t)(hi + nh_items) <= g.hitem_cap &&
                      (int64_t)li < (int64_t)g.act_cap && (int64_t)si < (int64_t)g.act_cap &&
                      (int64_t)ho < g.heavy_cap;
    if (!fits) {
      atomicOr(&cnt[CNT_IOVERFLOW], 4ull);
      continue;
    }
    if (sparse) {
      litems[(int64_t)g.act_cap - 1 - (int64_t)si] = make_int4(t, (int32_t)p0, c, -1);
    } else if (light) {
      litems[li] = make_int4(t, (int32_t)p0, c, -1);
    } else if (medium) {  // one item, walked in rounds of kChunk, applied directly
      hitems[hi] = make_int4(t, (int32_t)p0, c, -1);
    } else {
      // a cell's count in this call is at most the tile's piece count: below
      // 65536 the slab is packed (hits << 16 | misses, one word per cell)
      const int32_t wide = c >= 65536 ? 1 : 0;
      heavy_list[ho] = t | (wide << 31);
      for (int32_t q = 0; q < nh_items; ++q)
        hitems[hi + q] = make_int4(t, (int32_t)p0 + q * kChunk, min(kChunk, c - q * kChunk),
                                   (int32_t)(2 * ho + wide));
    }
  }
}

__device__ inline void put_piece(const Geom& g, PackedPiece* pieces, int64_t idx, const Beam& bm,
                                 int32_t tile, int32_t k0, int32_t k1, unsigned long long* cnt) {
  if (idx >= 0 && idx < g.seg_cap) {
    pieces[idx] = make_piece(g, bm, tile, k0, k1);
  } else {
    atomicOr(&cnt[CNT_IOVERFLOW], 2ull);
  }
}

// Pieces -> per-tile bins, in ONE enumeration pass: the workgroup's
// (tile, count) histogram comes from k_beam_prep (same 256 beams), one
// global cursor bump per histogram entry reserves the workgroup's range of
// each tile's bin, LDS cursors place the pieces.  Runs whose tile is not in
// the histogram (k_beam_prep's LDS table was full: those counted straight
// into tile_count) bump the global cursor themselves.
__global__ __launch_bounds__(256) void k_scatter(RayArgs a, Geom g, const Beam* __restrict__ beams,
                                                 int32_t* tile_cur, const int2* __restrict__ blk_hist,
                                                 const int32_t* __restrict__ blk_n,
                                                 PackedPiece* __restrict__ pieces, unsigned long long* cnt) {
  __shared__ int32_t hkey[kHash];
  __shared__ int32_t hcnt[kHash];
  __shared__ int32_t hbase[kHash];
  const int tid = threadIdx.x;
  for (int e = tid; e < kHash; e += 256) { hkey[e] = -1; hcnt[e] = 0; }
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + tid;
  const bool in = v < g.nb * g.chunks;
  const BeamChunk bc = beam_chunk(g, in ? v : 0);
  Beam bm;
  bm.flags = 0;
  if (in) bm = beams[bc.b];
  const int32_t nh = blk_n[blockIdx.x];
  __syncthreads();
  const int2* my_hist = blk_hist + (int64_t)blockIdx.x * kHash;
  for (int e = tid; e < nh; e += 256) {
    const int2 te = my_hist[e];
    const int h = hash_insert(hkey, te.x);  // the same entries fit: same table size
    if (h >= 0) hbase[h] = atomicAdd(&tile_cur[te.x], te.y & 0xFFFF);
  }
  __syncthreads();
  const bool valid = in && (bm.flags & 1) && bc.k_lo <= bm.n;
  if (valid) {
    dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t k0, int32_t k1) {
      const LaneRun run = lane_run(tile);
      int32_t pos = -1;
      if (run.head) {
        const int h = hash_find(hkey, tile);
        pos = h >= 0 ? hbase[h] + atomicAdd(&hcnt[h], run.len) : atomicAdd(&tile_cur[tile], run.len);
      }
      pos = __shfl(pos, run.head_lane);
      put_piece(g, pieces, (int64_t)pos + run.rank, bm, tile, k0, k1, cnt);
    }, bc.k_lo, bc.k_hi);
  }
}

struct ApplyArgs {
  float l_occ, l_free, l_min, l_max, occ_t, free_t;
};

// SPEC a7 as selects (no branches), lowest priority first: L == 0 -> -1,
// else L >= occ_t -> 100, else L <= free_t -> 0, else -1.
__device__ inline int8_t state_of(const ApplyArgs& p, float L) {
  int32_t r = -1;
  r = L <= p.free_t ? 0 : r;
  r = L >= p.occ_t ? 100 : r;
  r = L == 0.0f ? -1 : r;
  return (int8_t)r;
}

// SPEC a6 in this exact op order (no FMA: -ffp-contract=off).
__device__ inline float apply_one(const ApplyArgs& p, float L, uint32_t h, uint32_t m) {
  const float t = (float)h * p.l_occ;
  const float u = (float)m * p.l_free;
  L = L + t;
  L = L + u;
  // clamp: if (L < l_min) L = l_min; if (L > l_max) L = l_max — one v_med3
  // for finite L and l_min <= l_max (validate_params checks both)
  return __builtin_amdgcn_fmed3f(L, p.l_min, p.l_max);
}

// Mask-free forms for the dense apply (CellRows::apply).  gfx950 wants two
// wait states between a VALU compare that writes a lane mask and the
// v_cndmask reading it, and the compiler turned the per-cell selects into
// exec-masked branches (3 scalar instructions + hazard s_nops per cell):
// the selects below are v_bfi_b32 on masks built by integer arithmetic.
#ifndef DM_APPLY_BFI
#define DM_APPLY_BFI 1  // 0: the compare / select form (A/B builds)
#endif
// x != 0 ? 0xFFFFFFFF : 0
__device__ inline uint32_t nz_mask(uint32_t x) {
  uint32_t r;
  asm("v_min_u32_e32 %0, 1, %1\n\tv_sub_u32_e32 %0, 0, %0" : "=&v"(r) : "v"(x));
  return r;
}
// (m & a) | (~m & b)
__device__ inline uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// SPEC a7 from sign bits of exact differences (L finite, thresholds without
// signed zeros: make_apply): L >= occ_t <=> L - occ_t >= +0 (a difference of
// two different floats is never zero, and rounds to -0 at worst when
// flushed: negative either way), L <= free_t <=> free_t - L >= +0, L == 0
// <=> |bits| == 0.  Returns the state as an int (-1 / 0 / 100).
__device__ inline uint32_t state_bits(const ApplyArgs& p, float L) {
  const int32_t sge = (int32_t)__float_as_uint(L - p.occ_t) >> 31;   // -1: L < occ_t
  const int32_t sle = (int32_t)__float_as_uint(p.free_t - L) >> 31;  // -1: L > free_t
  const int32_t mz = (int32_t)((__float_as_uint(L) & 0x7FFFFFFFu) - 1u) >> 31;  // -1: L == 0
  uint32_t s = bfi((uint32_t)sle, 0xFFFFFFFFu, 0u);   // L > free_t ? -1 : 0
  s = bfi((uint32_t)sge, s, 100u);                    // L >= occ_t ? 100 : s
  return s | (uint32_t)mz;                            // L == 0 ? -1
}

// Bits 0..3: which of the 4 bytes of w are 0 (free); bits 4..7: which are
// 0xFF (unknown) — a state word's fmask byte.
__device__ inline uint8_t state_nibbles(uint32_t w) {
  auto zb = [](uint32_t v) {
    uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    t = ~(t | v | 0x7F7F7F7Fu);                 // 0x80 in each zero byte
    return (((t >> 7) * 0x00204081u) >> 21) & 0xFu;
  };
  return (uint8_t)(zb(w) | (zb(~w) << 4));
}

// The same for the 4 cells from column x0 of row y read one by one (a ragged
// tile column or an unaligned map: cells past the map's edge are neither).
template <class G>
__device__ inline uint8_t state_nibbles_at(const G& g, const int8_t* __restrict__ state, int32_t x0, int32_t y) {
  uint32_t fn = 0u, un = 0u;
  for (int e = 0; e < 4; ++e) {
    if (x0 + e >= g.r.W) break;
    const int8_t b = state[(int64_t)y * g.r.W + x0 + e];
    fn |= (b == 0 ? 1u : 0u) << e;
    un |= (b == -1 ? 1u : 0u) << e;
  }
  return (uint8_t)(fn | (un << 4));
}

// Bits 0, 4, ..., 60 of x packed into bits 0..15.
__device__ inline uint32_t every4th(uint64_t x) {
  x &= 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  return (uint32_t)((x | (x >> 24)) & 0xFFFFull);
}

// A tile's edge words (fedge, dm_internal.h) from the fmask stores of one
// wave: lane l holds the 4 nibble bytes `out` of 16-cell chunk l % 4 of tile
// row 16 q + l / 4 (every lane calls, in step: ballots and shuffles).
struct EdgeAcc {
  uint64_t w[4] = {0ull, 0ull, 0ull, 0ull};  // unknown column 0, column 63, row 0, row 63
};
__device__ inline void edge_acc(EdgeAcc& e, uint32_t out, int q, int lane) {
  const int c = lane & 3;
  const uint64_t b0 = __ballot(c == 0 && ((out >> 4) & 1u));   // cell 0's unknown bit
  const uint64_t b3 = __ballot(c == 3 && ((out >> 31) & 1u));  // cell 63's
  e.w[0] |= (uint64_t)every4th(b0) << (16 * q);
  e.w[1] |= (uint64_t)every4th(b3 >> 3) << (16 * q);
  if (q == 0 || q == 3) {  // rows 0 (lanes 0..3) and 63 (lanes 60..63)
    const uint32_t u16 = ((out >> 4) & 0xFu) | ((out >> 8) & 0xF0u) | ((out >> 12) & 0xF00u) | ((out >> 16) & 0xF000u);
    const int base = q == 0 ? 0 : 60;
    uint64_t r = 0ull;
#pragma unroll
    for (int k = 0; k < 4; ++k) r |= (uint64_t)__shfl(u16, base + k) << (16 * k);
    e.w[q == 0 ? 2 : 3] = r;
  }
}

// Lanes 0..3 store the tile's four edge words; `rows` (uniform) are the tile
// rows this wave rewrote: the others keep their stored bits.
__device__ inline void edge_store(const EdgeAcc& e, uint64_t* __restrict__ fedge, int64_t tile, uint64_t rows,
                                  int lane) {
  if (lane >= 4) return;
  const uint64_t v = lane == 0 ? e.w[0] : lane == 1 ? e.w[1] : lane == 2 ? e.w[2] : e.w[3];
  const uint64_t m = lane < 2 ? rows : ((rows >> (lane == 2 ? 0 : 63)) & 1ull) ? ~0ull : 0ull;
  uint64_t* p = fedge + tile * 4 + lane;
  if (m == ~0ull) *p = v;
  else if (m) *p = (*p & ~m) | (v & m);
}

// Number of zero bytes of x (exact, no false positives).
__device__ inline int32_t zero_bytes(uint32_t x) {
  uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  t = ~(t | x | 0x7F7F7F7Fu);
  return __popc(t);
}

// Cells of one tile owned by one thread: 4 consecutive cells (float4 / char4)
// of ROWS rows ly0, ly0 + dly, ...  Their L / state are loaded BEFORE the
// pieces are accumulated (they do not depend on the counts), so the apply
// step finds them in registers: one memory latency hidden behind the
// accumulation instead of one exposed after it.
template <int ROWS>
struct CellRows {
  float4 l[ROWS];
  char4 s[ROWS];
  bool vec;

  // Unconditional loads (cells outside the map, or a ragged column that the
  // apply reads cell by cell, load the map's first cells instead and are
  // ignored): a fixed number of loads per thread lets the compiler wait for
  // the pieces issued before them with vmcnt(N) instead of vmcnt(0).
  __device__ void prefetch(const Geom& g, int32_t tx0, int32_t ty0, int ly0, int dly, int cx,
                           const float* __restrict__ L, const int8_t* __restrict__ state, int vec_ok) {
    vec = vec_ok && tx0 + cx + 4 <= g.r.W;
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) {
      const int32_t y = ty0 + ly0 + rr * dly;
      const int64_t base = (vec && y < g.r.R) ? (int64_t)y * g.r.W + tx0 + cx : 0;
      l[rr] = *reinterpret_cast<const float4*>(L + base);
      s[rr] = *reinterpret_cast<const char4*>(state + base);
    }
  }

  // Sparse items: after the walk, load only the 4-cell groups that have a
  // count (touched(ly) for this thread's group of row ly); the apply skips
  // the others, so a tile crossed by a ray or two does not read its 20 KB of
  // L and state.
  template <class Touched>
  __device__ void load_touched(const Geom& g, int32_t tx0, int32_t ty0, int ly0, int dly, int cx,
                               const float* __restrict__ L, const int8_t* __restrict__ state, int vec_ok,
                               Touched&& touched) {
    vec = vec_ok && tx0 + cx + 4 <= g.r.W;
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) {
      const int32_t y = ty0 + ly0 + rr * dly;
      l[rr] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      s[rr] = make_char4(0, 0, 0, 0);
      if (vec && y < g.r.R && touched(ly0 + rr * dly)) {
        const int64_t base = (int64_t)y * g.r.W + tx0 + cx;
        l[rr] = *reinterpret_cast<const float4*>(L + base);
        s[rr] = *reinterpret_cast<const char4*>(state + base);
      }
    }
  }

  // counts(ly, h4, m4) supplies the counts of this thread's 4 cells of row ly.
  // Adds the touched cells to *sh_T and the change in free cells to
  // *sh_free; the updates U of the applied cells to *sh_U only if sh_U is
  // given (a tile inside the map counts them in the walk instead: every cell
  // step is one update; an edge tile's pieces also step over cells past the
  // map's edge, which are not updates).
  template <class Counts>
  __device__ void apply(const Geom& g, const ApplyArgs& p, int32_t tx0, int32_t ty0, int ly0, int dly,
                        int cx, float* __restrict__ L, int8_t* __restrict__ state, Counts&& counts,
                        int32_t* sh_T, int32_t* sh_free, uint32_t* sh_U) {
    int32_t dT = 0, dFree = 0;
    uint32_t dU = 0;
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) {
      const int ly = ly0 + rr * dly;
      const int32_t y = ty0 + ly;
      if (y >= g.r.R) continue;
      uint32_t h4[4], m4[4];
      counts(ly, h4, m4);
      if (((h4[0] | m4[0]) | (h4[1] | m4[1]) | (h4[2] | m4[2]) | (h4[3] | m4[3])) == 0u) continue;
      const int64_t base = (int64_t)y * g.r.W + tx0 + cx;
      if (sh_U) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dU += tx0 + cx + e < g.r.W ? h4[e] + m4[e] : 0u;
      }
      if (vec && DM_APPLY_BFI) {
        // branch- and compare-free per cell: untouched cells keep their values
        const float lv[4] = {l[rr].x, l[rr].y, l[rr].z, l[rr].w};
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(&s[rr]);
        uint32_t nlb[4], nsw = 0u, msk = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t mh = nz_mask(h4[e] | m4[e]);
          const float nl = apply_one(p, lv[e], h4[e], m4[e]);
          nlb[e] = bfi(mh, __float_as_uint(nl), __float_as_uint(lv[e]));
          nsw |= (state_bits(p, nl) & 0xFFu) << (8 * e);
          msk |= (mh & 0xFFu) << (8 * e);
          dT += (int32_t)(mh & 1u);
        }
        const uint32_t ns = bfi(msk, nsw, sw);
        dFree += zero_bytes(ns) - zero_bytes(sw);
        *reinterpret_cast<float4*>(L + base) =
            make_float4(__uint_as_float(nlb[0]), __uint_as_float(nlb[1]), __uint_as_float(nlb[2]),
                        __uint_as_float(nlb[3]));
        *reinterpret_cast<uint32_t*>(state + base) = ns;
      } else if (vec) {
        // branch-free per cell: untouched cells keep their values
        float lv[4] = {l[rr].x, l[rr].y, l[rr].z, l[rr].w};
        int8_t sv[4] = {(int8_t)s[rr].x, (int8_t)s[rr].y, (int8_t)s[rr].z, (int8_t)s[rr].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool hit = (h4[e] | m4[e]) != 0u;
          const float nl = apply_one(p, lv[e], h4[e], m4[e]);
          const int8_t ns = state_of(p, nl);
          lv[e] = hit ? nl : lv[e];
          sv[e] = hit ? ns : sv[e];
          dT += hit ? 1 : 0;
        }
        const char4 ns4 = make_char4(sv[0], sv[1], sv[2], sv[3]);
        dFree += zero_bytes(*reinterpret_cast<const uint32_t*>(&ns4)) -
                 zero_bytes(*reinterpret_cast<const uint32_t*>(&s[rr]));
        *reinterpret_cast<float4*>(L + base) = make_float4(lv[0], lv[1], lv[2], lv[3]);
        *reinterpret_cast<char4*>(state + base) = ns4;
      } else {
        for (int e = 0; e < 4; ++e) {
          if ((h4[e] | m4[e]) == 0u || tx0 + cx + e >= g.r.W) continue;
          const int64_t i = base + e;
          const int8_t old = state[i];
          const float nl = apply_one(p, L[i], h4[e], m4[e]);
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
    if (dU) atomicAdd(sh_U, dU);
  }
};

// One piece per thread, walked cell by cell into the packed LDS count tile
// (PieceCursor: no division per cell; +1 per cell, then +0xFFFF at the hit
// cell turns that miss into a hit).  The walk starts at a staggered step
// (lane mod length) and wraps around: pieces that share their first cells
// (every ray of a scan starts at the sensor's cell) then sit on different
// cells at every step instead of piling a wave's atomics onto one LDS word.
// The wave's trip count is its longest piece.
__device__ inline int32_t walk_tp(uint32_t* tl, const TilePiece& tp, int32_t len, int lane) {
  int32_t wl = len;
  for (int o = 32; o > 0; o >>= 1) wl = max(wl, __shfl_xor(wl, o));
  const int32_t s0 = len > 0 ? lane % len : 0;
  PieceCursor cur;
  cur.init(tp);
  if (s0 > 0) {  // jump to step s0: the closed form once (dm_piece_addr)
    const int32_t num = tp.rem0 + s0 * tp.two_adb;
    const int32_t dq = dm_udiv_small(num, tp.two_n, __builtin_amdgcn_rcpf((float)tp.two_n));
    cur.addr = tp.addr0 + s0 * tp.da + dq * tp.db;
    cur.rem = num - dq * tp.two_n;
  }
  int32_t k = s0;
  for (int32_t st = 0; st < wl; ++st) {
    if (st < len) {
      atomicAdd(&tl[cur.addr], 1u);
      cur.step(tp);
      if (++k == len) cur.init(tp);  // wrap to the piece's first cell
    }
  }
  if (len > 0 && tp.addr_end >= 0) atomicAdd(&tl[tp.addr_end], 0xFFFFu);
  return len;
}

__device__ inline int32_t walk_piece(uint32_t* tl, const PackedPiece& mine, bool valid, int lane) {
  const TilePiece tp = dm_unpack_piece(mine.x, mine.y, mine.z, mine.w);
  return walk_tp(tl, tp, valid ? tp.len : 0, lane);
}

#ifndef DM_SPLIT_WALK
#define DM_SPLIT_WALK 1  // 0: one lane per piece (the round-4 walk, for A/B builds)
#endif

// Light tiles: their pieces cross the tile from different directions and
// rarely share cells, so each lane walks from its first cell, with no
// stagger and no wrap.  A lane whose part has ended adds into its own spare
// word past the tile (tl[kTileWords + lane], never read) instead of masking
// the step: no exec-mask branch per step, no pile-up on one word.
// With fewer pieces than lanes: each piece is split over
// f = lanes / c lanes (dm_split_part), lane `part` of them walking cells
// [j0, j0 + n) from the closed-form cell j0 (PieceCursor::init_at).  The
// wave's trip count is its longest part instead of its longest piece: C3's
// light items (95 pieces on average) 45 -> 31 steps on the critical path.
// The part that ends the piece adds the hit (SPEC a6).
__device__ inline int32_t walk_tp_split(uint32_t* tl, const TilePiece& tp, int32_t len, int32_t f, int32_t part,
                                        float rf, int lane) {
  const SplitPart sp = dm_split_part(len, f, part, rf);
  int32_t wl = sp.n;
  for (int o = 32; o > 0; o >>= 1) wl = max(wl, __shfl_xor(wl, o));
  const int32_t spare = kTileWords + lane;
  PieceCursor cur;
  if (f == 1) cur.init(tp);
  else cur.init_at(tp, sp.j0, __builtin_amdgcn_rcpf((float)tp.two_n));
  for (int32_t st = 0; st < wl; ++st) {
    atomicAdd(&tl[st < sp.n ? cur.addr : spare], 1u);
    cur.step(tp);
  }
  if (sp.n > 0 && sp.j0 + sp.n == len && tp.addr_end >= 0) atomicAdd(&tl[tp.addr_end], 0xFFFFu);
  return sp.n;
}

// Sparse items: the same walk into a byte-packed count tile (pitch 64, one
// byte per cell: hits << 4 | misses, +1 per cell and +0x0F at the hit cell,
// which turns that miss into a hit).  A cell of a tile with at most 15
// pieces is visited at most 15 times, so the final byte 16·hits + misses is
// at most 255 and no partial sum carries into the next cell.
constexpr int kSparseMax = 15;
#ifndef DM_SPARSE_LIST
#define DM_SPARSE_LIST 256  // touched 4-cell groups a wave lists (more: four row passes; 0 = always the passes, A/B)
#endif
constexpr int kSparseList = DM_SPARSE_LIST > 0 ? DM_SPARSE_LIST : 1;

__device__ inline int32_t to_pitch64(int32_t a) {  // pitch-65 address or step -> pitch 64
  return a >= 0 ? a - a / kLdsPitch : -((-a) - (-a) / kLdsPitch);
}

// Split as walk_tp_split: a sparse tile's c <= 15 pieces over the wave's 64
// lanes, f = 64 / c >= 4 lanes per piece (lane `part` of them).
__device__ inline int32_t walk_piece_bytes(uint32_t* tq, const PackedPiece& mine, bool valid, int32_t f,
                                           int32_t part, float rf) {
  TilePiece tp = dm_unpack_piece(mine.x, mine.y, mine.z, mine.w);
  const int32_t len = valid ? tp.len : 0;
  const SplitPart sp = dm_split_part(len, f, part, rf);
  int32_t wl = sp.n;
  for (int o = 32; o > 0; o >>= 1) wl = max(wl, __shfl_xor(wl, o));
  tp.addr0 = to_pitch64(tp.addr0);
  tp.da = to_pitch64(tp.da);
  tp.db = to_pitch64(tp.db);
  PieceCursor cur;
  if (f == 1) cur.init(tp);
  else cur.init_at(tp, sp.j0, __builtin_amdgcn_rcpf((float)tp.two_n));
  for (int32_t st = 0; st < wl; ++st) {
    if (st < sp.n) atomicAdd(&tq[cur.addr >> 2], 1u << (8 * (cur.addr & 3)));
    cur.step(tp);
  }
  if (sp.n > 0 && sp.j0 + sp.n == len && tp.addr_end >= 0) {
    const int32_t e = to_pitch64(tp.addr_end);
    atomicAdd(&tq[e >> 2], 0x0Fu << (8 * (e & 3)));
  }
  return sp.n;
}

__device__ inline PackedPiece no_piece() {
  PackedPiece q;
  q.x = 0u; q.y = 0u; q.z = 0u; q.w = 1u;
  return q;
}

// A tile's new tile_free word after a net change of dfree free cells from
// `old` (the item applying the tile is its only writer in the call): a tile
// whose free count rises from 0 while kTileListed is clear is appended to the
// persistent frontier tile list (dm_internal.h, ftiles) and flagged.  Tiles
// that were listed stay listed (the pass skips tiles without frontier bits).
__device__ inline int32_t free_update(int32_t old, int32_t dfree, int32_t tile, int32_t* tlist,
                                      unsigned long long* tlist_n) {
  int32_t v = old + dfree;
  if (dfree > 0 && !(old & kTileListed)) {
    v |= kTileListed;
    tlist[atomicAdd(tlist_n, 1ull)] = tile;
  }
  return v;
}

// The heavy finisher's counters; old_free is the tile's tile_free word as
// loaded before its apply (no other item of the call writes it).
__device__ inline void finish_tile(const Geom& g, int32_t tile, int32_t T, int32_t dfree, uint32_t U,
                                   bool heavy, int32_t* tile_count, int32_t* tile_free, int32_t old_free,
                                   int32_t* tlist, unsigned long long* tlist_n, unsigned long long* ish) {
  unsigned long long* sh = ish + (blockIdx.x % kShards) * kShardWords;
  if (T) {
    atomicAdd(&sh[SH_T], (unsigned long long)T);
    if (heavy) atomicAdd(&sh[SH_TH], (unsigned long long)T);
  }
  if (U) atomicAdd(&sh[SH_U], (unsigned long long)U);
  if (dfree) tile_free[tile] = free_update(old_free, dfree, tile, tlist, tlist_n);
  tile_count[tile] = 0;  // ready for the next call
}

// One 16-row quarter q of heavy tile h (ordinal in heavy_list): apply the
// merged slab counts to the quarter's cells and clear the slab words.
// Thread tid takes cell (row 4k + tid / 64, column tid % 64) of the quarter:
// each wave instruction touches 256 contiguous slab bytes, the full-rate
// shape for the memory-side atomics.  The read-and-clear is an exchange:
// the slab was only ever written by the items' device-scope atomics, which
// execute at the memory side, so the exchange reads the merged counts there
// and leaves no stale L2 line.  Totals go to the workgroup's LDS counters.
__device__ inline void heavy_quarter(const Geom& g, const ApplyArgs& p, int64_t h, int q, int32_t tile,
                                     bool wide, uint32_t* __restrict__ slabs, float* __restrict__ L,
                                     int8_t* __restrict__ state, int32_t* s_T, int32_t* s_free,
                                     uint32_t* s_U) {
  constexpr int kQ = DM_TS * DM_TS / 4;  // cells per quarter
  const int tid = threadIdx.x;
  const int32_t x = (tile % g.r.TX) * DM_TS + (tid & 63);
  const int32_t yq = (tile / g.r.TX) * DM_TS + q * (DM_TS / 4) + (tid >> 6);
  uint32_t* sh = slabs + h * (2 * DM_TS * DM_TS) + q * kQ + tid;
  uint32_t hc[4], mc[4];
  float lv[4];
  int8_t sv[4];
  // L / state first: their latency then overlaps the exchanges'
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t y = yq + 4 * k;
    lv[k] = 0.0f;
    sv[k] = 0;
    if (y < g.r.R && x < g.r.W) {
      lv[k] = L[(int64_t)y * g.r.W + x];
      sv[k] = state[(int64_t)y * g.r.W + x];
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hc[k] = atomicExch(sh + k * kQuarter, 0u);
    mc[k] = wide ? atomicExch(sh + DM_TS * DM_TS + k * kQuarter, 0u) : 0u;
  }
  int32_t dT = 0, dFree = 0;
  uint32_t dU = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t hk = hc[k], mk;
    if (wide) {
      mk = mc[k];
    } else {  // packed: split the word
      mk = hk & 0xFFFFu;
      hk >>= 16;
    }
    const int32_t y = yq + 4 * k;
    if ((hk | mk) == 0u || y >= g.r.R || x >= g.r.W) continue;
    const int64_t i = (int64_t)y * g.r.W + x;
    const float nl = apply_one(p, lv[k], hk, mk);
    const int8_t ns = state_of(p, nl);
    L[i] = nl;
    state[i] = ns;
    dU += hk + mk;
    dT += 1;
    dFree += (ns == 0) - (sv[k] == 0);
  }
  if (dT) atomicAdd(s_T, dT);
  if (dFree) atomicAdd(s_free, dFree);
  if (dU) atomicAdd(s_U, dU);
}

// Per-cell hit/miss counts never touch HBM: a 256-thread workgroup takes one
// work item (<= kChunk pieces of one tile, one piece per thread), gathers
// them in a packed LDS count tile (hits << 16 | misses) with walk_piece,
// and then
//  * light / medium item (the whole tile): applies the log-odds update to the
//    tile's cells right away, from L / state loaded before the accumulation;
//  * heavy item: adds its counts to the tile's slab (row-contiguous global
//    atomics); the tile's last item to finish (a ticket) applies the merged
//    slab.
// The next item's pieces are loaded right after this item's apply, its
// cells (unconditional loads: a fixed count, so the walk waits for the pieces
// alone with vmcnt(N)) at the top of its iteration, in flight during its
// walk.  7 workgroups per CU (72 VGPRs, no spills): C3's ~3.8k items in ~2
// rounds of the chip's slots (41 us vs 43.5 us at 6).  The per-item statistics stay in thread 0's registers (one flush per
// workgroup) and a light tile's free count is a plain read-modify-write (one
// workgroup owns the tile), so no memory-side atomic sits in front of the
// next item's loads in the wave's in-order vmcnt queue.
#ifndef DM_ACCUM_OCC
#define DM_ACCUM_OCC 7
#endif
#ifndef DM_EARLY_PIECES
#define DM_EARLY_PIECES 1
#endif
constexpr int kAccumPerCu = DM_ACCUM_OCC;  // resident k_tile_accum workgroups per CU (4 waves each)
__global__ __launch_bounds__(kQuarter, kAccumPerCu) void k_tile_accum(
    Geom g, ApplyArgs p, const int4* __restrict__ list_a, int cnt_a, const int4* __restrict__ list_b,
    int cnt_b, int cnt_c, const PackedPiece* __restrict__ pieces, int32_t* tile_count, int32_t* tile_free,
    uint32_t* __restrict__ slabs, float* __restrict__ L, int8_t* __restrict__ state,
    const unsigned long long* __restrict__ cnt, unsigned long long* ish, int vec_ok,
    const int32_t* __restrict__ heavy_list, int32_t* heavy_done, int32_t* tlist, unsigned long long* tlist_n,
    unsigned long long* hint, const unsigned long long* __restrict__ halt, uint8_t* __restrict__ tile_seen) {
  __shared__ uint32_t tl[kTileWords + 64];  // + one spare word per lane (walk_tp_split)
  __shared__ int32_t s_T, s_free, s_last;
  __shared__ uint32_t s_U;
  const int tid = threadIdx.x, lane = lane_id();
  DM_TL_BEGIN();
  // The halt word and the item counts in one round of loads (a workgroup
  // runs about one item at C3, so its first item's dependent loads -- counts,
  // descriptor, pieces -- are on every item's path; the halt check used to
  // be a round of its own in front of them).
  const unsigned long long hv = *halt;
  const unsigned long long ca = cnt[cnt_a];
  const unsigned long long cb = cnt[cnt_b];  // (the one launch passes all three counters)
  const unsigned long long cc = cnt[cnt_c];
  // (clamped to the list capacities: k_plan flags and drops what does not fit)
  const int64_t HI = min((int64_t)ca, g.hitem_cap);
  const int64_t LI = min((int64_t)cb, (int64_t)g.act_cap);
  const int64_t n_items = HI + LI;
  // sparse items (litems from the top, cnt_c of them): a second loop
  const int64_t SI = min((int64_t)cc, (int64_t)g.act_cap);
  const int64_t G = gridDim.x;
  // Sparse items go to the workgroups after the dense ones (rank 0 = the
  // workgroup right after the last dense item, wrapping around the grid), so
  // they run beside the dense items instead of behind the first (longest)
  // ones: a small call (one 360-beam scan) is one round of items, and its
  // sparse tiles used to queue behind its heavy and medium tiles.
  const int64_t sp_rank = ((int64_t)blockIdx.x - n_items % G + G) % G;
  if (blockIdx.x == 0 && tid == 0) {  // the work of this call, for the next call's grid (mapped host memory)
    volatile unsigned long long* h = hint;
    h[0] = (unsigned long long)(n_items + (SI + 3) / 4);
    h[1] = (unsigned long long)(n_items + SI);
  }
  const unsigned long long idle =
      ((int64_t)blockIdx.x >= n_items && sp_rank * (kQuarter / 64) >= SI) ? 1ull : 0ull;
  // a timed-out front-end hand-off (kHaltWord): this call's workspace was
  // never written, so nothing is applied (the host reports DM_ERR_PIPELINE).
  // One exit test on all four loads, so they go out together.
  if ((hv | idle) != 0ull) {
    DM_TL_END(accum, 0);
    return;
  }
  auto item_of = [&](int64_t it) {
    int4 d = it < n_items ? (it < HI ? list_a[it] : list_b[it - HI]) : make_int4(0, 0, 0, -1);
    // an item never reads past the piece array (k_plan keeps p0 + c <= seg_cap)
    d.z = (int64_t)d.y + d.z <= g.seg_cap ? d.z : 0;
    return d;
  };
  const int cx = (tid & 15) * 4;
  __shared__ unsigned long long s_accT, s_accU;  // this workgroup's light-tile totals
  // the first item's loads
  int4 info = item_of(blockIdx.x);
  int4 next = item_of(blockIdx.x + G);
  PackedPiece mine;
  CellRows<4> cells;
  int32_t tfree;
  // a light item's split factor (walk_tp_split; 1 for heavy / medium items)
  auto split_of = [&](const int4& d) -> int32_t {
    const int32_t c = __builtin_amdgcn_readfirstlane(d.z);
    const int32_t heavy = __builtin_amdgcn_readfirstlane(d.w);
    return DM_SPLIT_WALK && heavy < 0 ? dm_split_factor(c, kQuarter) : 1;
  };
  // this thread's piece of item d (piece tid / f of a split light item)
  auto piece_of = [&](int32_t f) -> int32_t {
    return f == 1 ? tid : dm_udiv_small(tid, f, __builtin_amdgcn_rcpf((float)f));
  };
  auto load_pieces = [&](const int4& d) -> PackedPiece {
    const int32_t c0 = __builtin_amdgcn_readfirstlane(d.y);
    const int32_t c = __builtin_amdgcn_readfirstlane(d.z);
    // lanes past the item's pieces re-read its last one (past the list's end:
    // piece 0); unconditional, so the loop carries no phi of the old pieces
    return pieces[c0 + min(piece_of(split_of(d)), max(c - 1, 0))];
  };
  mine = load_pieces(info);
  // DM_EARLY_PIECES: the next item's pieces are issued right after this
  // item's walk, BEFORE its apply stores.  Loads and stores share the wave's
  // in-order vmcnt counter, so pieces issued after the stores (the other
  // form) make the next walk's wait for them also a wait for the previous
  // item's stores to drain.
  PackedPiece mine_n = mine;
  for (int e = tid; e < kTileWords; e += kQuarter) tl[e] = 0u;
  if (tid == 0) { s_T = 0; s_free = 0; s_U = 0u; s_accT = 0ull; s_accU = 0ull; }
  __syncthreads();
  DM_PH_INIT();
  [[maybe_unused]] unsigned long long tl_word = 0;  // timeline (phase build): dense items | sparse << 16 | finisher ticks << 32
  for (int64_t it = blockIdx.x; it < n_items; it += G) {
    tl_word += 1;
    // the descriptor is workgroup-uniform: scalar registers, scalar branches
    const int32_t tile = __builtin_amdgcn_readfirstlane(info.x);
    const int32_t c0 = __builtin_amdgcn_readfirstlane(info.y);
    const int32_t c = __builtin_amdgcn_readfirstlane(info.z);
    const int32_t heavy = __builtin_amdgcn_readfirstlane(info.w);
    const int32_t tx0 = (tile % g.r.TX) * DM_TS, ty0 = (tile / g.r.TX) * DM_TS;
    DM_PH(dm_phase_acc_integrate, 0);
    if (heavy >= 0) {
      // heavy (a sensor's tile): the pieces all start at the sensor's cell;
      // walk_piece's staggered start keeps a wave's lanes on different cells
      walk_piece(tl, mine, tid < c, lane);
      if (DM_EARLY_PIECES) mine_n = load_pieces(next);
      __syncthreads();
      DM_PH(dm_phase_acc_integrate, 1);
      DM_PH_COUNT(dm_phase_acc_integrate, 17, 1);
      DM_PH_COUNT(dm_phase_acc_integrate, 19, c);
      uint32_t* sh = slabs + (int64_t)(heavy >> 1) * (2 * DM_TS * DM_TS);
      if (heavy & 1) {  // wide slab: separate 32-bit hit and miss counts
        for (int e = tid; e < DM_TS * DM_TS; e += kQuarter) {
          const uint32_t v = tl[(e >> 6) * kLdsPitch + (e & 63)];
          const uint32_t h = v >> 16, m = v & 0xFFFFu;
          if (h) atomicAdd(&sh[e], h);
          if (m) atomicAdd(&sh[DM_TS * DM_TS + e], m);
        }
      } else {  // packed slab: the LDS word as is (no carry: counts < 65536)
        for (int e = tid; e < DM_TS * DM_TS; e += kQuarter) {
          const uint32_t v = tl[(e >> 6) * kLdsPitch + (e & 63)];
          if (v) atomicAdd(&sh[e], v);
        }
      }
      DM_PH(dm_phase_acc_integrate, 2);
      // The tile's last item to finish applies the merged slab.  Why no
      // release / acquire fence is needed: every access to a slab word in a
      // call is an agent-scope atomic RMW (the items' adds, the finisher's
      // exchanges), and on gfx950 such an RMW is performed at the memory
      // side, past the XCD's L2 (MI355X_MICROARCH.md §Global float atomics;
      // atomics drop the L2 line, §Workgroup dispatch table), so there is no
      // cached copy a release would have to write back or an acquire to
      // invalidate.  What remains is ordering: a wave's non-returning RMW is
      // counted in vmcnt until the memory side acknowledges it as performed,
      // so after every wave's s_waitcnt vmcnt(0) and the barrier, all of this
      // item's adds are performed before the ticket RMW is issued (the wait
      // is what an agent-scope release does after its L2 write-back: LLVM
      // AMDGPUUsage, GFX942 memory model, release = buffer_wbl2 sc1 +
      // s_waitcnt vmcnt(0)).  The ticket RMWs are totally ordered on their
      // address, so the item whose ticket returns n_it - 1 comes after every
      // other item's adds, and its exchanges read their sums.  A release
      // fence here (the L2 write-back of the items' other, plain stores)
      // measured 42 -> 172 us per call with __threadfence (round 1), and the
      // release / acquire pair on the ticket 67 vs 45 us (round 3).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int32_t n_it = (tile_count[tile] + kChunk - 1) / kChunk;  // k_plan's item count
        s_last = atomicAdd(&heavy_done[heavy >> 1], 1) == n_it - 1;
      }
      __syncthreads();
      if (s_last) {
#ifdef DM_PHASE_TIMING
        const long long tf0 = wall_clock64();
#endif
        const int64_t h = heavy >> 1;
        const bool wide = heavy_list[h] < 0;
        const int32_t old_free = tid == 0 ? tile_free[tile] : 0;  // in flight during the apply
        for (int q = 0; q < 4; ++q)
          heavy_quarter(g, p, h, q, tile, wide, slabs, L, state, &s_T, &s_free, &s_U);
        __syncthreads();
        if (tid == 0) {
          finish_tile(g, tile, s_T, s_free, s_U, true, tile_count, tile_free, old_free, tlist, tlist_n, ish);
          heavy_done[h] = 0;  // ready for the next call
          tile_seen[tile] = 1;
        }
#ifdef DM_PHASE_TIMING
        tl_word += (unsigned long long)(wall_clock64() - tf0) << 32;
#endif
      }
    } else {
      // light / medium: one piece per thread per round (medium tiles walk
      // their later rounds with in-loop loads); the cells' loads fly during
      // the walk
      tfree = tile_free[tile];
      cells.prefetch(g, tx0, ty0, tid >> 4, 16, cx, L, state, vec_ok);
      int32_t u;  // this thread's cell updates (one per step)
      if (c <= kChunk) {
        const int32_t f = split_of(info);
        const int32_t pi = piece_of(f);
        const TilePiece tp = dm_unpack_piece(mine.x, mine.y, mine.z, mine.w);
        u = walk_tp_split(tl, tp, pi < c ? tp.len : 0, f, tid - pi * f, __builtin_amdgcn_rcpf((float)f), lane);
      } else {  // medium: near a sensor, the staggered walk
        u = walk_piece(tl, mine, tid < c, lane);
        for (int32_t r0 = kChunk; r0 < c; r0 += kChunk) {
          const PackedPiece more = r0 + tid < c ? pieces[c0 + r0 + tid] : no_piece();
          u += walk_piece(tl, more, r0 + tid < c, lane);
        }
      }
      const bool inside = tx0 + DM_TS <= g.r.W && ty0 + DM_TS <= g.r.R;  // workgroup-uniform
      if (inside) {
        for (int o = 32; o > 0; o >>= 1) u += __shfl_xor(u, o);
        if (lane == 0) atomicAdd(&s_U, (uint32_t)u);
      }
      if (DM_EARLY_PIECES) mine_n = load_pieces(next);
      __syncthreads();
      DM_PH(dm_phase_acc_integrate, 3);
      DM_PH_COUNT(dm_phase_acc_integrate, 16, 1);
      DM_PH_COUNT(dm_phase_acc_integrate, 18, c);
      cells.apply(g, p, tx0, ty0, tid >> 4, 16, cx, L, state,
                  [&](int ly, uint32_t* h4, uint32_t* m4) {
                    for (int e = 0; e < 4; ++e) {
                      const uint32_t v = tl[ly * kLdsPitch + cx + e];
                      h4[e] = v >> 16;
                      m4[e] = v & 0xFFFFu;
                    }
                  },
                  &s_T, &s_free, inside ? nullptr : &s_U);
      DM_PH(dm_phase_acc_integrate, 4);
    }
    __syncthreads();
    if (tid == 0 && heavy < 0) {
      s_accT += (unsigned long long)s_T;
      s_accU += (unsigned long long)s_U;
      if (s_free) tile_free[tile] = free_update(tfree, s_free, tile, tlist, tlist_n);
      tile_count[tile] = 0;  // ready for the next call
      tile_seen[tile] = 1;
    }
    // the next item: its pieces go out now (or went out after the walk),
    // ahead of its walk
    info = next;
    next = item_of(it + 2 * G);
    mine = DM_EARLY_PIECES ? mine_n : load_pieces(info);
    for (int e = tid; e < kTileWords; e += kQuarter) tl[e] = 0u;
    if (tid == 0) { s_T = 0; s_free = 0; s_U = 0u; }
    __syncthreads();
  }
  // Sparse items (a few pieces: C5's sparse scans on a 1 cm map): walk first,
  // then load and apply only the touched 4-cell groups.  A loop of its own
  // (after the dense items), so none of its registers are live across the
  // dense walk.  The LDS tile is zero here: every dense item clears it.
  // One sparse item per WAVE (round 3; round 2 had one per 128-thread half,
  // whose second wave idled through the walk): with at most kSparseMax
  // pieces a cell is visited at most 15 times, so its counts fit one byte
  // (hits << 4 | misses: walk_piece_bytes), a tile's counts 4 KiB, and the
  // four waves' tiles share the LDS of one dense count tile.  A wave walks,
  // applies and clears its own tile with no workgroup barrier (LDS operations
  // of one wave complete in order; the wavefront fences keep the compiler
  // from moving them), so a CU keeps 4 x 7 = 28 sparse tiles in flight.
  __shared__ int32_t s_wT[kQuarter / 64], s_wfree[kQuarter / 64];
  __shared__ uint32_t s_wU[kQuarter / 64];
  __shared__ uint16_t s_list[kQuarter / 64][kSparseList];  // touched 4-cell groups of each wave's tile
  const int wv = tid >> 6;
  uint32_t* tq = tl + wv * (DM_TS * DM_TS / 4);
  const int hcx = (lane & 15) * 4;
  if (lane == 0) { s_wT[wv] = 0; s_wfree[wv] = 0; s_wU[wv] = 0u; }
  const int nw = kQuarter / 64;
  for (int64_t it = sp_rank * nw + wv; it < SI; it += (int64_t)G * nw) {
    int4 d = list_b[(int64_t)g.act_cap - 1 - it];
    d.z = (int64_t)d.y + d.z <= g.seg_cap ? d.z : 0;  // never past the piece array
    const int32_t tile = d.x, c0 = d.y, c = d.z;
    if (lane == 0 && wv == 0) tl_word += 1ull << 16;
    const int32_t tx0 = (tile % g.r.TX) * DM_TS, ty0 = (tile / g.r.TX) * DM_TS;
    // f = 64 / c lanes per piece (walk_piece_bytes' split)
    const int32_t fs = DM_SPLIT_WALK ? dm_split_factor(c, 64) : 1;
    const float rfs = __builtin_amdgcn_rcpf((float)fs);
    const int32_t spi = fs == 1 ? lane : dm_udiv_small(lane, fs, rfs);
    const PackedPiece sp = spi < c ? pieces[c0 + spi] : no_piece();
    const int32_t sfree = tile_free[tile];
    int32_t u = walk_piece_bytes(tq, sp, spi < c, fs, lane - spi * fs, rfs);
    const bool inside = tx0 + DM_TS <= g.r.W && ty0 + DM_TS <= g.r.R;  // uniform in the wave
    uint32_t wU = 0u;
    if (inside) {
      for (int o = 32; o > 0; o >>= 1) u += __shfl_xor(u, o);
      wU = (uint32_t)u;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    DM_PH(dm_phase_acc_integrate, 6);
    auto counts = [&](int wi, uint32_t* h4, uint32_t* m4) {
      const uint32_t w = tq[wi];
      for (int e = 0; e < 4; ++e) {
        const uint32_t v = (w >> (8 * e)) & 0xFFu;
        h4[e] = v >> 4;
        m4[e] = v & 0xFu;
      }
    };
    // the touched 4-cell groups (non-zero count words, word wi = row * 16 +
    // group) listed in the wave's LDS list, so each lane loads the L / state
    // of one or two of them in ONE load round (a ray or two cross a sparse
    // tile: ~35-70 of its 1024 groups); a tile with more than kSparseList
    // touched groups takes four 16-row passes instead
    uint16_t* lst = s_list[wv];
    int nt = 0;
    {
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int wi = k * 64 + lane;
        const bool nz = tq[wi] != 0u;
        const unsigned long long m = __ballot(nz);
        const int at = nt + __popcll(m & lt);
        if (nz && at < kSparseList) lst[at] = (uint16_t)wi;
        nt += __popcll(m);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (DM_SPARSE_LIST > 0 && nt <= kSparseList) {
      for (int e0 = 0; e0 < nt; e0 += 128) {
        const int ea = e0 + lane, eb = e0 + 64 + lane;
        const int wa = ea < nt ? lst[ea] : 0, wb = eb < nt ? lst[eb] : 0;
        CellRows<1> ca, cb;
        ca.load_touched(g, tx0, ty0, wa >> 4, 0, (wa & 15) * 4, L, state, vec_ok, [&](int) { return ea < nt; });
        cb.load_touched(g, tx0, ty0, wb >> 4, 0, (wb & 15) * 4, L, state, vec_ok, [&](int) { return eb < nt; });
        if (ea < nt)
          ca.apply(g, p, tx0, ty0, wa >> 4, 0, (wa & 15) * 4, L, state,
                   [&](int, uint32_t* h4, uint32_t* m4) { counts(wa, h4, m4); }, &s_wT[wv], &s_wfree[wv],
                   inside ? nullptr : &s_wU[wv]);
        if (eb < nt)
          cb.apply(g, p, tx0, ty0, wb >> 4, 0, (wb & 15) * 4, L, state,
                   [&](int, uint32_t* h4, uint32_t* m4) { counts(wb, h4, m4); }, &s_wT[wv], &s_wfree[wv],
                   inside ? nullptr : &s_wU[wv]);
      }
    } else {
      // the wave covers the tile in four passes of 16 rows (a lane: one
      // 4-cell group of rows ly0, ly0 + 4, ly0 + 8, ly0 + 12)
      for (int pass = 0; pass < 4; ++pass) {
        const int ly0 = (lane >> 4) + 16 * pass;
        CellRows<4> sc;
        sc.load_touched(g, tx0, ty0, ly0, 4, hcx, L, state, vec_ok,
                        [&](int ly) { return tq[ly * 16 + (hcx >> 2)] != 0u; });
        sc.apply(g, p, tx0, ty0, ly0, 4, hcx, L, state,
                 [&](int ly, uint32_t* h4, uint32_t* m4) { counts(ly * 16 + (hcx >> 2), h4, m4); },
                 &s_wT[wv], &s_wfree[wv], inside ? nullptr : &s_wU[wv]);
      }
    }
    DM_PH(dm_phase_acc_integrate, 7);
    DM_PH_COUNT(dm_phase_acc_integrate, 21, 1);
    DM_PH_COUNT(dm_phase_acc_integrate, 22, c);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      const int32_t T = s_wT[wv], df = s_wfree[wv];
      const uint32_t U = s_wU[wv] + wU;
      atomicAdd(&s_accT, (unsigned long long)T);
      atomicAdd(&s_accU, (unsigned long long)U);
      if (df) tile_free[tile] = free_update(sfree, df, tile, tlist, tlist_n);
      tile_count[tile] = 0;  // ready for the next call
      tile_seen[tile] = 1;
      s_wT[wv] = 0;
      s_wfree[wv] = 0;
      s_wU[wv] = 0u;
    }
    for (int e = lane; e < DM_TS * DM_TS / 4; e += 64) tq[e] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long* sh = ish + (blockIdx.x % kShards) * kShardWords;
    if (s_accT) atomicAdd(&sh[SH_T], s_accT);
    if (s_accU) atomicAdd(&sh[SH_U], s_accU);
  }
  DM_PH_FLUSH(dm_phase_acc_integrate);
  DM_TL_END(accum, tl_word);
}

// ---- maintenance kernels ----------------------------------------------------

// Per-call reset of the device counters and integrate shards in one launch.
__global__ __launch_bounds__(256) void k_integrate_reset(unsigned long long* cnt, unsigned long long* ish) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int nI = (int)(sizeof(kIntegrateCounters) / sizeof(kIntegrateCounters[0]));
  if (i < nI) cnt[kIntegrateCounters[i]] = 0ull;
  if (i < kShards * kShardWords) ish[i] = 0ull;
}

// Hand-off between two streams without a cross-queue event wait, which
// holds the waiting stream ~10 us even when its producer finished long
// before.  k_seq_signal runs on the producing stream after the producer
// kernels (the kernel boundary has written their outputs back) and stores a
// sequence number; k_seq_gate, one lane on the consuming stream, polls that
// word and exits, and the consumer kernels' own kernel-boundary acquire then
// sees the outputs.  Uses: the integrate front-end -> k_tile_accum (flag
// fe_flag), a frontier pass's bit rows -> its labelling half on pass_stream
// (bits_flag).  No deadlock: the gate holds one workgroup slot, and all the
// producer waits for is ahead of the gate on the consuming stream.  Bounded:
// after kGateTicks of the 100 MHz wall clock the gate sets err_bit in *err
// (the consumer's result is then reported as an error) and exits.  Under a
// tool that runs one dispatch at a time across all queues (rocprofv3 --pmc)
// a gate can be dispatched before the kernels it waits for and then times
// out: PMC passes run the steps without overlap (tools/pmc_passes.sh).
constexpr unsigned long long kGateTicks = 500000000ull;  // 5 s

__global__ __launch_bounds__(64) void k_seq_signal(unsigned long long* flag) {
  if (threadIdx.x != 0) return;
  // only this stream's signals write the word, one after the other
  const unsigned long long v = __hip_atomic_load(flag + kSigWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(flag + kSigWord, v + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void k_seq_gate(unsigned long long* flag, unsigned long long* err,
                                                 unsigned long long err_bit, unsigned long long ticks,
                                                 unsigned long long fault) {
  if (threadIdx.x != 0) return;
  const unsigned long long seq = flag[kGateWord] + 1;  // this gate's turn (only gates write the word)
  flag[kGateWord] = seq;
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(flag + kSigWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < seq + fault) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > ticks) {
      atomicOr(err, err_bit);
      return;
    }
  }
}

// fmask bytes of a row of cells: byte j = free bits of cells 4j..4j+3 (low
// nibble) | their unknown bits (high nibble), from the row's ballots.
__device__ inline uint8_t fmask_byte(uint64_t fm, uint64_t um, int j) {
  return (uint8_t)(((fm >> (4 * j)) & 0xFull) | (((um >> (4 * j)) & 0xFull) << 4));
}

// Per-tile free counts and fmask records from the state bytes, after a bulk
// state write (reset, dm_set_state, dm_set_logodds).  Element e of the loop
// is cell (e & 63, e >> 6): a wave is one row.
__global__ __launch_bounds__(256) void k_recount(Geom g, const int8_t* __restrict__ state,
                                                 int32_t* __restrict__ tile_free, uint8_t* __restrict__ fmask,
                                                 uint64_t* __restrict__ fedge, uint8_t* __restrict__ tile_seen) {
  const int64_t tile = blockIdx.x;
  const int32_t tx0 = (int32_t)(tile % g.r.TX) * DM_TS, ty0 = (int32_t)(tile / g.r.TX) * DM_TS;
  __shared__ int32_t acc, seen;
  __shared__ uint64_t s_edge[4][4];  // per wave: unknown column 0, column 63, row 0, row 63
  if (threadIdx.x == 0) { acc = 0; seen = 0; }
  __syncthreads();
  int32_t c = 0, known = 0;
  uint64_t ew[4] = {0ull, 0ull, 0ull, 0ull};
  uint8_t* tm = fmask + tile * (DM_TS * 16);
  for (int e = threadIdx.x; e < DM_TS * DM_TS; e += 256) {
    const int32_t x = tx0 + (e & 63), y = ty0 + (e >> 6);
    const int8_t b = (x < g.r.W && y < g.r.R) ? state[(int64_t)y * g.r.W + x] : (int8_t)1;
    c += b == 0;
    known |= (x < g.r.W && y < g.r.R && b != -1) ? 1 : 0;
    const uint64_t fm = __ballot(b == 0);
    const uint64_t um = __ballot(b == -1);
    const int l = e & 63, r = e >> 6;  // a wave is one row
    if (l < 16) tm[r * 16 + l] = fmask_byte(fm, um, l);
    ew[0] |= (um & 1ull) << r;
    ew[1] |= (um >> 63) << r;
    if (r == 0) ew[2] = um;
    if (r == DM_TS - 1) ew[3] = um;
  }
  if (c) atomicAdd(&acc, c);
  if (known) seen = 1;
  const int l4 = __lane_id();
  if (l4 < 4) s_edge[threadIdx.x >> 6][l4] = l4 == 0 ? ew[0] : l4 == 1 ? ew[1] : l4 == 2 ? ew[2] : ew[3];
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_free[tile] = acc;
    tile_seen[tile] = (uint8_t)seen;
  }
  if (threadIdx.x < 4)
    fedge[tile * 4 + threadIdx.x] = s_edge[0][threadIdx.x] | s_edge[1][threadIdx.x] | s_edge[2][threadIdx.x] |
                                    s_edge[3][threadIdx.x];
}

// The persistent frontier tile list from scratch, every tile with a free
// cell in tile order, each tile's kTileListed flag set or cleared to match:
// after bulk state writes (k_recount), and every kRelistPasses passes, which
// puts the tiles appended since in tile order again (the bit-row and tile
// kernels read neighbouring listed tiles together: appended tiles arrive in
// exploration order, and at C3 a list in that order doubled k_frontier_bits'
// fetched bytes).  Ballot compaction over chunks of `iters` x 256 tiles per
// workgroup and round, one list atomic per chunk (the loop bounds are
// uniform within the workgroup: its barriers are safe).
constexpr int kListIters = 16;
__global__ __launch_bounds__(256) void k_list_tiles(int64_t NT, int32_t* __restrict__ tile_free,
                                                    int32_t* __restrict__ ftiles, unsigned long long* list_n,
                                                    int iters) {
  const int lane = __lane_id();
  __shared__ int32_t s_wn[kListIters][4];
  __shared__ unsigned long long s_base;
  const int w = threadIdx.x >> 6;
  const int64_t chunk = (int64_t)iters * blockDim.x;
  for (int64_t c0 = (int64_t)blockIdx.x * chunk; c0 < NT; c0 += (int64_t)gridDim.x * chunk) {
    uint32_t mine = 0u;
    for (int i = 0; i < iters; ++i) {
      const int64_t t = c0 + (int64_t)i * blockDim.x + threadIdx.x;
      if (t >= NT) continue;
      const int32_t v = tile_free[t];
      const bool f = (v & kTileFreeMask) > 0;
      mine |= (f ? 1u : 0u) << i;
      if (f != ((v & kTileListed) != 0)) tile_free[t] = f ? (v | kTileListed) : (v & kTileFreeMask);
    }
    for (int i = 0; i < iters; ++i) {
      const unsigned long long bal = __ballot((mine >> i) & 1u);
      if (lane == 0) s_wn[i][w] = __popcll(bal);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int total = 0;
      for (int i = 0; i < iters; ++i) total += s_wn[i][0] + s_wn[i][1] + s_wn[i][2] + s_wn[i][3];
      s_base = total ? atomicAdd(list_n, (unsigned long long)total) : 0ull;
    }
    __syncthreads();
    int64_t pre = (int64_t)s_base;
    for (int i = 0; i < iters; ++i) {
      const bool f = (mine >> i) & 1u;
      const unsigned long long bal = __ballot(f);
      int before = 0;
      for (int q = 0; q < w; ++q) before += s_wn[i][q];
      if (f) {
        const int64_t t = c0 + (int64_t)i * blockDim.x + threadIdx.x;
        ftiles[pre + before + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)t;
      }
      pre += s_wn[i][0] + s_wn[i][1] + s_wn[i][2] + s_wn[i][3];
    }
    __syncthreads();  // s_wn / s_base are rewritten next round
  }
}

__device__ inline uint64_t upto_rows(int p) {  // bits 0..p inclusive
  return p >= 63 ? ~0ull : ((2ull << p) - 1ull);
}

// fmask records of the tiles this call's map update touched (its work items:
// heavy chunks and medium tiles, then light tiles; a heavy tile appears once
// per chunk and is rewritten with the same bytes), one wave per item, after
// k_tile_accum on the grid stream.  Lane l reads the 16-byte chunk l % 4 of
// tile rows l / 4, 16 + l / 4, ... (coalesced 64-byte row segments) and
// stores its 4 nibble bytes per row.  Kept out of k_tile_accum, whose
// registers are full at 7 workgroups per CU (inside it, every variant
// measured 6-14 us slower per call).
__global__ __launch_bounds__(256) void k_fmask_items(Geom g, const int4* __restrict__ list_a, int cnt_a,
                                                     const int4* __restrict__ list_b, int cnt_b, int cnt_c,
                                                     const PackedPiece* __restrict__ pieces,
                                                     const unsigned long long* __restrict__ cnt,
                                                     const int8_t* __restrict__ state, uint8_t* __restrict__ fmask,
                                                     uint64_t* __restrict__ fedge,
                                                     const unsigned long long* __restrict__ halt) {
  if (*halt) return;  // as k_tile_accum
  const int64_t HI = min((int64_t)cnt[cnt_a], g.hitem_cap);
  const int64_t LI = min((int64_t)cnt[cnt_b], (int64_t)g.act_cap);
  const int64_t SI = min((int64_t)cnt[cnt_c], (int64_t)g.act_cap);  // sparse: list_b from the top
  const int lane = __lane_id();
  for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < HI + LI + SI;
       it += (int64_t)gridDim.x * 4) {
    const int4 d = it < HI ? list_a[it]
                           : (it < HI + LI ? list_b[it - HI] : list_b[(int64_t)g.act_cap - 1 - (it - HI - LI)]);
    const int32_t tile = __builtin_amdgcn_readfirstlane(d.x);
    // a sparse item (<= kSparseMax pieces) rewrites only the rows its pieces
    // cross: a piece is a monotone line inside the tile, so it visits every
    // row between its first and last cell's and no other (the others' state
    // did not change); every other item its whole record
    uint64_t rows = ~0ull;
    if (it >= HI + LI) {
      const int32_t c0 = __builtin_amdgcn_readfirstlane(d.y);
      const int32_t c = __builtin_amdgcn_readfirstlane(d.z);
      uint64_t mine = 0ull;
      if (lane < c && (int64_t)c0 + c <= g.seg_cap) {
        const PackedPiece q = pieces[c0 + lane];
        const TilePiece tp = dm_unpack_piece(q.x, q.y, q.z, q.w);
        if (tp.len > 0) {
          const int32_t ya = tp.addr0 / kLdsPitch;
          const int32_t yb = dm_piece_addr(tp, tp.len - 1, __builtin_amdgcn_rcpf((float)tp.two_n)) / kLdsPitch;
          const int lo = min(ya, yb), hi = max(ya, yb);
          mine = upto_rows(hi) & ~(lo > 0 ? upto_rows(lo - 1) : 0ull);
        }
      }
      for (int o = 32; o > 0; o >>= 1) mine |= __shfl_xor(mine, o);
      rows = mine;
    }
    const int32_t tx0 = (tile % g.r.TX) * DM_TS, ty0 = (tile / g.r.TX) * DM_TS;
    const int32_t x0 = tx0 + (lane & 3) * 16;
    uint8_t* tm = fmask + (int64_t)tile * (DM_TS * 16);
    EdgeAcc ea;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ly = 16 * q + (lane >> 2);
      const bool mine = (rows >> ly) & 1ull;
      const int32_t y = ty0 + ly;
      uint32_t out = 0u;
      if (mine && y < g.r.R) {
        const int64_t off = (int64_t)y * g.r.W + x0;
        if (x0 + 16 <= g.r.W && (off & 15) == 0) {
          const uint4 v = *reinterpret_cast<const uint4*>(state + off);
          const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) out |= (uint32_t)state_nibbles(wd[k]) << (8 * k);
        } else {
          for (int k = 0; k < 4; ++k) out |= (uint32_t)state_nibbles_at(g, state, x0 + 4 * k, y) << (8 * k);
        }
      }
      if (mine) *reinterpret_cast<uint32_t*>(tm + ly * 16 + (lane & 3) * 4) = out;
      edge_acc(ea, out, q, lane);  // every lane: ballots (rows not rewritten are masked in edge_store)
    }
    edge_store(ea, fedge, tile, rows, lane);
  }
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

static_assert(sizeof(Geom) == 72 && sizeof(RayArgs) == 40 && sizeof(ApplyArgs) == 24,
              "kernel argument structs have no implicit padding");

Geom make_geom(const dm_grid* g) {
  Geom ge;
  ge.r.W = (int32_t)g->W;
  ge.r.R = (int32_t)g->R;
  ge.r.row0 = (int32_t)g->row0;
  ge.r.TX = (int32_t)g->TX;
  ge.r.TY = (int32_t)g->TY;
  ge.act_cap = (int32_t)g->act_cap;
  ge.seg_cap = g->segs_cap;
  ge.hitem_cap = g->hitem_cap;
  ge.heavy_cap = g->heavy_cap;
  ge.nb = 0;
  ge.chunks = 1;
  ge.chunk_len = 0;
  ge.sparse_pieces = std::min(g->sparse_pieces, kSparseMax);  // byte-packed counts (walk_piece_bytes)
  ge.pad = 0;
  return ge;
}

ApplyArgs make_apply(const dm_grid* g) {
  ApplyArgs a;
  a.l_occ = g->p.l_occ;
  a.l_free = g->p.l_free;
  // signed zeros normalised to +0: the SPEC's compare-based clamp gives the
  // same result for a bound of -0 or +0 (L is never -0), v_med3 only for +0
  a.l_min = g->p.l_min == 0.0f ? 0.0f : g->p.l_min;
  a.l_max = g->p.l_max == 0.0f ? 0.0f : g->p.l_max;
  // thresholds without signed zeros either (state_bits: sign-bit compares)
  a.occ_t = g->p.occ_thresh == 0.0f ? 0.0f : g->p.occ_thresh;
  a.free_t = g->p.free_thresh == 0.0f ? 0.0f : g->p.free_thresh;
  return a;
}

int grid_for(int64_t n, int threads, int64_t cap = 8192) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

DM_PH_READER(integrate)
DM_TL_READER(accum)

int dm_launch_integrate(dm_grid* g, int32_t S, const double* d_pose4, int32_t N,
                        const float* d_ranges, const double* d_trig) {
  const int64_t nb = (int64_t)S * N;
  // calls alternate between the two workspace sets
  g->iw_cur = (g->iw_cur + 1) % dm_grid::kIntSets;
  dm_grid::IntWs& w = g->iw[g->iw_cur];
  // front-end stream: with overlap, its own stream, after the accumulation
  // that last used this set (ev_free), so it runs beside the previous call's
  // accumulation and a frontier pass still in flight on g->stream
  hipStream_t fs = g->stream;
  if (g->overlap) {
    fs = dm_fe_stream_of(g, g->iw_cur);
    DM_HIP(dm_mark_ws_free(g));  // still owed when no frontier pass came in between
    DM_HIP(hipStreamWaitEvent(fs, w.free_wait ? w.free_wait : w.ev_free, 0));
  }
  DM_LAUNCH(k_integrate_reset, dim3(2), dim3(256), 0, fs, w.cnt, w.sh);
  DM_HIP(hipGetLastError());
  if (nb == 0) {
    if (g->overlap) {  // keep the stream order of the calls
      DM_HIP(hipEventRecord(g->ev_fe, fs));
      DM_HIP(hipStreamWaitEvent(g->stream, g->ev_fe, 0));
      w.free_owed = true;
    }
    return DM_OK;
  }
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
  ge.chunks = dm_integrate_chunks(g, nb);
  ge.chunk_len = (int32_t)((g->nmax + ge.chunks) / ge.chunks);  // ceil((nmax + 1) / chunks)
  const int nblk = (int)((nb * ge.chunks + 255) / 256);
  KernelTimer t;
  dm_timer_begin(g, "beam_prep", &t, fs);
  DM_LAUNCH(k_beam_prep, dim3(nblk), dim3(256), 0, fs, a, ge, d_pose4, d_ranges,
            d_trig, w.beams, w.tile_count, w.act_raw, w.sh, w.blk_hist, w.blk_n, w.cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "plan", &t, fs);
  DM_LAUNCH(k_plan, dim3(grid_for(g->act_cap, kPlanThreads, 256)), dim3(kPlanThreads), 0, fs,
                     ge, w.act_raw, w.sh, w.tile_cur, w.tile_count, w.hitems, w.litems,
                     w.heavy_list, w.cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "scatter", &t, fs);
  DM_LAUNCH(k_scatter, dim3(nblk), dim3(256), 0, fs, a, ge, w.beams,
            w.tile_cur, w.blk_hist, w.blk_n, w.pieces, w.cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  if (g->overlap) {
    // front-end -> map update by a device-side seq gate (an event wait
    // measured 211-213 vs 215-218 x 10^9 updates/s, profiles/r02_fe_gate_ab.log)
    DM_HIP(hipEventRecord(g->ev_fe_end[g->iw_cur % 2], fs));
    unsigned long long* flag = dm_fe_flag_of(g, g->iw_cur);
    if (int rc = dm_launch_signal(fs, flag)) return rc;
    // a timeout sets the sticky halt word (not this call's counters: the
    // front-end's own reset, still queued, would clear them)
    if (int rc = dm_launch_gate(g->stream, flag, g->fe_flag + kHaltWord, 1ull, g->fault_gate ? 1000ull : 0ull,
                                g->fault_gate ? (1ull << 40) : 0ull))
      return rc;
  }
#ifdef DM_FE_DUMMY
  // Diagnostic build only (never the product): one more k_beam_prep of this
  // batch into scratch buffers on the front-end stream AFTER the front-end's
  // hand-off signal (so it delays no accumulation), i.e. extra work beside
  // the map chain; how much the pipelined step grows tells whether the step
  // is bound by the chip's occupancy (workgroup-us) or by latency chains.
  if (g->overlap) {
    struct Dummy {
      Beam* beams = nullptr; int32_t* tc = nullptr; int32_t* act = nullptr; int2* hist = nullptr;
      int32_t* hn = nullptr; unsigned long long* sh = nullptr; unsigned long long* cnt = nullptr;
      int64_t nb = 0, nt = 0, blocks = 0, act_cap = 0;
    };
    static Dummy d;
    if (d.nb < nb || d.nt < g->NT || d.blocks < nblk || d.act_cap < g->act_cap) {
      (void)hipDeviceSynchronize();
      for (void* q : {(void*)d.beams, (void*)d.tc, (void*)d.act, (void*)d.hist, (void*)d.hn, (void*)d.sh,
                      (void*)d.cnt})
        if (q) (void)hipFree(q);
      d.nb = nb; d.nt = g->NT; d.blocks = nblk; d.act_cap = g->act_cap;
      DM_HIP(hipMalloc((void**)&d.beams, sizeof(Beam) * nb));
      DM_HIP(hipMalloc((void**)&d.tc, sizeof(int32_t) * g->NT));
      DM_HIP(hipMalloc((void**)&d.act, sizeof(int32_t) * g->act_cap * kShards));
      DM_HIP(hipMalloc((void**)&d.hist, sizeof(int2) * 1024 * nblk));
      DM_HIP(hipMalloc((void**)&d.hn, sizeof(int32_t) * nblk));
      DM_HIP(hipMalloc((void**)&d.sh, sizeof(unsigned long long) * kShards * kShardWords));
      DM_HIP(hipMalloc((void**)&d.cnt, sizeof(unsigned long long) * CNT_N));
    }
    DM_HIP(hipMemsetAsync(d.tc, 0, sizeof(int32_t) * g->NT, fs));
    DM_LAUNCH(k_integrate_reset, dim3(2), dim3(256), 0, fs, d.cnt, d.sh);
    DM_LAUNCH(k_beam_prep, dim3(nblk), dim3(256), 0, fs, a, ge, d_pose4, d_ranges, d_trig, d.beams, d.tc,
              d.act, d.sh, d.hist, d.hn, d.cnt);
    DM_HIP(hipGetLastError());
  }
#endif
  const int vec_ok = (g->W % 4 == 0) ? 1 : 0;
  // heavy chunks and medium tiles first (the long items), then the light
  // tiles; the last item of each heavy tile applies its merged slab
  dm_timer_begin(g, "tile_accum", &t);
  // one workgroup per item (the kernel grid-strides, so any grid is exact):
  // a grid sized to the capacity (16384 at C3) ran ~3.6 k item workgroups
  // and ~12.8 k that exit at once, whose dispatch held the kernel's end and
  // the front-end streams' first workgroups ~6 us longer in the pipelined
  // step (profiles/r04_accum_timeline.log); the last finished call's count
  // (+1/16 + 64: calls of one workload differ by a few percent; a grid one
  // short of the items only gives a few workgroups a second item) sizes it
  // instead (+25 % + 256 measured 1-3 % slower, profiles/r04_accum_grid_slack_ab.log)
  const volatile unsigned long long* hint = g->h_hint;
  const int64_t cap = g->hitem_cap + g->act_cap;
#ifndef DM_ACCUM_HINT
#define DM_ACCUM_HINT 1  // 0: capacity grids (the round-3 launch, for A/B builds)
#endif
  const int64_t hw = DM_ACCUM_HINT ? (int64_t)hint[0] : 0, hi = DM_ACCUM_HINT ? (int64_t)hint[1] : 0;
  const int64_t accum_wgs = hw > 0 ? std::min(cap, dm_quantize_up(hw + hw / 16 + 64)) : cap;
  DM_LAUNCH(k_tile_accum, dim3(grid_for(accum_wgs, 1, dm_grid::kAccumGrid)),
                     dim3(kQuarter), 0,
                     g->stream, ge, make_apply(g), w.hitems, (int)CNT_ITEMS, w.litems, (int)CNT_LITEMS,
                     (int)CNT_SITEMS, w.pieces, w.tile_count, g->tile_free, w.slabs, g->L, g->state, w.cnt, w.sh, vec_ok,
                     w.heavy_list, w.heavy_done, g->ftiles, g->ftiles_n, g->d_hint, g->fe_flag + kHaltWord,
                     g->tile_seen);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  if (g->overlap) w.free_owed = true;
  // the touched tiles' fmask records (one wave per work item), while the
  // frontier passes read them
  if (!g->fmask_on) {
    g->fmask_valid = false;
    return DM_OK;
  }
  dm_timer_begin(g, "fmask", &t);
  const int64_t fmask_items = hi > 0 ? std::min(cap, dm_quantize_up(hi + hi / 16 + 64)) : cap;
  DM_LAUNCH(k_fmask_items, dim3(grid_for(fmask_items, 4, 8192)), dim3(256), 0, g->stream,
                     ge, w.hitems, (int)CNT_ITEMS, w.litems, (int)CNT_LITEMS, (int)CNT_SITEMS, w.pieces, w.cnt,
                     g->state, g->fmask, g->fedge,
                     g->fe_flag + kHaltWord);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_signal(hipStream_t s, unsigned long long* flag) {
  DM_LAUNCH(k_seq_signal, dim3(1), dim3(64), 0, s, flag);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

int dm_launch_gate(hipStream_t s, unsigned long long* flag, unsigned long long* err, unsigned long long err_bit,
                   unsigned long long ticks, unsigned long long fault) {
  DM_LAUNCH(k_seq_gate, dim3(1), dim3(64), 0, s, flag, err, err_bit, ticks ? ticks : kGateTicks, fault);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

// The persistent frontier tile list rebuilt in tile order from tile_free
// (~256 chunks).  swap: into the other list, after the passes that read it
// (the pass stream's position when it was left: 16 passes ago, done unless
// passes are enqueued faster than they run), then switch; the passes in
// flight keep the current list, which nothing appends to any more.
int dm_launch_relist(dm_grid* g, bool swap) {
  if (swap) {
    const int x = 1 - g->flist_cur;
    if (g->flist_ev_set[x] && hipEventQuery(g->flist_ev[x]) != hipSuccess)
      DM_HIP(hipStreamWaitEvent(g->stream, g->flist_ev[x], 0));
    if (g->pass_stream) {  // passes reading the list being left run there (or on `stream`: ordered)
      DM_HIP(hipEventRecord(g->flist_ev[g->flist_cur], g->pass_stream));
      g->flist_ev_set[g->flist_cur] = true;
    }
    g->flist_cur = x;
    g->ftiles = g->flist[x];
    g->ftiles_n = g->flist_n[x];
  }
  DM_HIP(hipMemsetAsync(g->ftiles_n, 0, sizeof(unsigned long long), g->stream));
  const int iters = (int)std::min<int64_t>(kListIters, std::max<int64_t>(1, (g->NT + 65535) / 65536));
  DM_LAUNCH(k_list_tiles, dim3(grid_for((g->NT + iters - 1) / iters, 256, 1024)), dim3(256), 0, g->stream,
            g->NT, g->tile_free, g->ftiles, g->ftiles_n, iters);
  DM_HIP(hipGetLastError());
  g->relist_age = 0;
  // from a fresh list (bulk writes) the period doubles up to kRelistPasses
  g->relist_period = swap ? std::min(2 * g->relist_period, kRelistPasses) : 1;
  return DM_OK;
}

int dm_launch_recount(dm_grid* g) {
  const Geom ge = make_geom(g);
  // the tile list is rebuilt from position 0: passes still labelling on the
  // pass stream read it (bulk calls have already joined every stream; an
  // fmask switch-on inside dm_enqueue_frontiers may not have)
  DM_HIP(dm_join_pass_stream(g));
  DM_LAUNCH(k_recount, dim3((unsigned)g->NT), dim3(256), 0, g->stream, ge, g->state,
                     g->tile_free, g->fmask, g->fedge, g->tile_seen);
  DM_HIP(hipGetLastError());
  if (int rc = dm_launch_relist(g, false)) return rc;
  g->fmask_valid = true;
  return DM_OK;
}

int dm_launch_state_from_logodds(dm_grid* g) {
  const int64_t cells = g->R * g->W;
  DM_LAUNCH(k_state_from_l, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream,
                     make_apply(g), cells, g->L, g->state);
  DM_HIP(hipGetLastError());
  return dm_launch_recount(g);
}

int dm_launch_set_state(dm_grid* g, const int8_t* d_in) {
  const int64_t cells = g->R * g->W;
  DM_LAUNCH(k_set_state, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream,
                     make_apply(g), cells, d_in, g->L, g->state);
  DM_HIP(hipGetLastError());
  return dm_launch_recount(g);
}

int dm_launch_map_image(dm_grid* g, uint8_t* d_img) {
  const int64_t cells = g->R * g->W;
  DM_LAUNCH(k_map_image, dim3(grid_for(cells, 256)), dim3(256), 0, g->stream, g->R,
                     g->W, g->state, d_img);
  DM_HIP(hipGetLastError());
  return DM_OK;
}
