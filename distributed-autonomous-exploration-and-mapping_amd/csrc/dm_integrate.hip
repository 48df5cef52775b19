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
  int32_t W, R, row0, TX, TY;
  int32_t act_cap;
  int64_t seg_cap;
};

struct PrepArgs {
  int32_t S, N;
  double ox, oy, res;
  float range_min, range_max;
};

__device__ inline int lane_id() { return __lane_id(); }

// Enumerate the pieces of a beam's line that fall in in-band tiles, in order
// of k.  emit(tile, k0, k1).  Closed form: the major coordinate moves one cell
// per k, the minor one is monotone, so the k at which each coordinate leaves
// its tile is computed exactly.
template <class Emit>
__device__ inline void for_each_piece(const Beam& b, const Geom& g, Emit&& emit) {
  const int32_t n = b.n;
  const int32_t off_a = b.xmajor ? 0 : g.row0;
  const int32_t off_b = b.xmajor ? g.row0 : 0;
  const int32_t lim_a = b.xmajor ? g.TX : g.TY;
  const int32_t lim_b = b.xmajor ? g.TY : g.TX;
  int32_t k = 0;
  // iteration cap: every pass advances k by >= 1 and crosses a tile edge or
  // ends the line, so (n/64 + 2) + (adb/64 + 2) passes suffice
  const int32_t max_iter = 2 * (n / DM_TS) + 8;
  for (int32_t it = 0; k <= n && it < max_iter; ++it) {
    const int32_t q = n > 0 ? dm_udiv(2 * k * b.adb + n, 2 * n, b.rden) : 0;
    const int32_t ma = b.sa + k * b.ia - off_a;
    const int32_t mb = b.sb + b.ib * q - off_b;
    const int32_t ta = (int32_t)dm_floordiv(ma, DM_TS);
    const int32_t tb = (int32_t)dm_floordiv(mb, DM_TS);
    int64_t ka;
    if (b.ia > 0) ka = (int64_t)k + (DM_TS * (ta + 1) - ma);
    else if (b.ia < 0) ka = (int64_t)k + (ma - DM_TS * ta) + 1;
    else ka = (int64_t)n + 1;
    int64_t kb;
    if (b.ib == 0) {
      kb = (int64_t)n + 1;
    } else {
      const int64_t Q = (int64_t)q + (b.ib > 0 ? (DM_TS * (tb + 1) - mb) : (mb - DM_TS * tb) + 1);
      const int64_t num = (int64_t)n * (2 * Q - 1);
      const int64_t den = 2 * (int64_t)b.adb;
      kb = (num + den - 1) / den;
    }
    int64_t ke = ka < kb ? ka : kb;
    if (ke > (int64_t)n + 1) ke = (int64_t)n + 1;
    ke -= 1;
    if (ta >= 0 && ta < lim_a && tb >= 0 && tb < lim_b) {
      const int32_t tx = b.xmajor ? ta : tb;
      const int32_t ty = b.xmajor ? tb : ta;
      emit(ty * g.TX + tx, k, (int32_t)ke);
    }
    k = (int32_t)ke + 1;
  }
}

// SPEC a4: endpoint cells of beam (s, i).  Double precision, every product
// rounded separately (compiled with -ffp-contract=off), glibc cos/sin of the
// beam angle table and of the scan yaw come from the host.
__device__ inline Beam make_beam(const PrepArgs& a, const double* pose4, const float* ranges,
                                 const double* trig, int32_t s, int32_t i) {
  Beam bm;
  bm.sa = bm.sb = bm.n = bm.adb = 0;
  bm.ia = bm.ib = 0;
  bm.xmajor = 1;
  bm.flags = 0;
  bm.pad = 0;
  bm.rden = 0.0;
  const double x = pose4[4 * s + 0], y = pose4[4 * s + 1];
  const double cyaw = pose4[4 * s + 2], syaw = pose4[4 * s + 3];
  const float r = ranges[(int64_t)s * a.N + i];
  if (!(isfinite(x) && isfinite(y) && isfinite(cyaw) && isfinite(syaw))) return bm;
  if (!(r >= a.range_min)) return bm;
  const bool hit = r <= a.range_max;
  const double rr = hit ? (double)r : (double)a.range_max;
  const double cphi = trig[2 * i], sphi = trig[2 * i + 1];
  const double a1 = cyaw * cphi;
  const double a2 = syaw * sphi;
  const double dcx = a1 - a2;
  const double b1 = syaw * cphi;
  const double b2 = cyaw * sphi;
  const double dcy = b1 + b2;
  const double t1 = rr * dcx;
  const double ex = x + t1;
  const double t2 = rr * dcy;
  const double ey = y + t2;
  const double fsx = floor((x - a.ox) / a.res);
  const double fsy = floor((y - a.oy) / a.res);
  const double fex = floor((ex - a.ox) / a.res);
  const double fey = floor((ey - a.oy) / a.res);
  const double lim = 1073741824.0;
  if (!(fabs(fsx) < lim && fabs(fsy) < lim && fabs(fex) < lim && fabs(fey) < lim)) return bm;
  const int32_t sx = (int32_t)fsx, sy = (int32_t)fsy, ex_c = (int32_t)fex, ey_c = (int32_t)fey;
  const int32_t dx = ex_c - sx, dy = ey_c - sy;
  const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
  const int8_t ix = dx > 0 ? 1 : (dx < 0 ? -1 : 0);
  const int8_t iy = dy > 0 ? 1 : (dy < 0 ? -1 : 0);
  if (adx >= ady) {
    bm.xmajor = 1; bm.sa = sx; bm.sb = sy; bm.n = adx; bm.adb = ady; bm.ia = ix; bm.ib = iy;
  } else {
    bm.xmajor = 0; bm.sa = sy; bm.sb = sx; bm.n = ady; bm.adb = adx; bm.ia = iy; bm.ib = ix;
  }
  bm.rden = bm.n > 0 ? 1.0 / (double)(2 * bm.n) : 0.0;
  bm.flags = (uint8_t)(1u | (hit ? 2u : 0u));
  return bm;
}

__global__ __launch_bounds__(256) void k_beam_prep(PrepArgs a, Geom g, const double* __restrict__ pose4,
                                                   const float* __restrict__ ranges,
                                                   const double* __restrict__ trig,
                                                   Beam* __restrict__ beams, int32_t* tile_count,
                                                   int32_t* tile_slot, int32_t* act_tiles,
                                                   unsigned long long* cnt) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)a.S * a.N;
  if (b >= nb) return;
  const int32_t s = (int32_t)(b / a.N), i = (int32_t)(b % a.N);
  const Beam bm = make_beam(a, pose4, ranges, trig, s, i);
  beams[b] = bm;
  if (!(bm.flags & 1)) return;
  const int lane = lane_id();
  for_each_piece(bm, g, [&](int32_t tile, int32_t, int32_t) {
    // wave-aggregated increment: one atomic per distinct tile among the
    // lanes emitting now (neighbouring beams share tiles)
    while (true) {
      const unsigned long long act = __ballot(1);
      const int leader = __ffsll(act) - 1;
      const int32_t lt = __shfl(tile, leader);
      if (tile == lt) {
        const unsigned long long m = __ballot(1);
        if (lane == leader) {
          const int32_t old = atomicAdd(&tile_count[lt], (int32_t)__popcll(m));
          if (old == 0) {
            const unsigned long long slot = atomicAdd(&cnt[CNT_ACTIVE], 1ull);
            if (slot < (unsigned long long)g.act_cap) {
              act_tiles[slot] = lt;
              tile_slot[lt] = (int32_t)slot;
            } else {
              atomicOr(&cnt[CNT_OVERFLOW], 1ull);
            }
          }
        }
        break;
      }
    }
  });
}

// Exclusive scan of per-tile piece counts over the active list (one block).
__global__ __launch_bounds__(1024) void k_scan_active(Geom g, const int32_t* __restrict__ act_tiles,
                                                      const int32_t* __restrict__ tile_count,
                                                      int32_t* __restrict__ act_off,
                                                      int32_t* __restrict__ act_cur,
                                                      unsigned long long* cnt) {
  __shared__ int64_t wsum[16];
  const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const int64_t n = min((int64_t)cnt[CNT_ACTIVE], (int64_t)g.act_cap);
  const int64_t per = (n + 1023) / 1024;
  const int64_t lo = min((int64_t)tid * per, n), hi = min(lo + per, n);
  int64_t mine = 0;
  for (int64_t j = lo; j < hi; ++j) mine += tile_count[act_tiles[j]];
  // block exclusive scan of `mine`
  int64_t incl = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    int64_t run = 0;
    for (int w = 0; w < 16; ++w) { const int64_t t = wsum[w]; wsum[w] = run; run += t; }
    cnt[CNT_SEGS] = (unsigned long long)run;
  }
  __syncthreads();
  int64_t off = wsum[wid] + incl - mine;
  for (int64_t j = lo; j < hi; ++j) {
    act_off[j] = (int32_t)off;
    act_cur[j] = (int32_t)off;
    off += tile_count[act_tiles[j]];
  }
}

__global__ __launch_bounds__(256) void k_scatter(PrepArgs a, Geom g, const Beam* __restrict__ beams,
                                                 const int32_t* __restrict__ tile_slot,
                                                 int32_t* act_cur, Seg* __restrict__ segs,
                                                 unsigned long long* cnt) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)a.S * a.N;
  if (b >= nb) return;
  const Beam bm = beams[b];
  if (!(bm.flags & 1)) return;
  const int lane = lane_id();
  for_each_piece(bm, g, [&](int32_t tile, int32_t k0, int32_t k1) {
    while (true) {
      const unsigned long long act = __ballot(1);
      const int leader = __ffsll(act) - 1;
      const int32_t lt = __shfl(tile, leader);
      if (tile == lt) {
        const unsigned long long m = __ballot(1);
        int32_t base = 0;
        if (lane == leader) {
          const int32_t slot = tile_slot[lt];
          base = atomicAdd(&act_cur[slot], (int32_t)__popcll(m));
        }
        base = __shfl(base, leader);
        const int32_t rank = (int32_t)__popcll(m & ((1ull << lane) - 1ull));
        const int64_t idx = (int64_t)base + rank;
        if (idx < g.seg_cap) {
          Seg sg;
          sg.beam = (uint32_t)b;
          sg.k0 = (uint16_t)k0;
          sg.k1 = (uint16_t)k1;
          segs[idx] = sg;
        } else {
          atomicOr(&cnt[CNT_OVERFLOW], 2ull);
        }
        break;
      }
    }
  });
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

__global__ __launch_bounds__(kApplyThreads) void k_tile_apply(
    Geom g, ApplyArgs p, const int32_t* __restrict__ act_tiles, const int32_t* __restrict__ act_off,
    const Seg* __restrict__ segs, const Beam* __restrict__ beams, int32_t* tile_count,
    int32_t* tile_free, float* __restrict__ L, int8_t* __restrict__ state, unsigned long long* cnt,
    int vec_ok) {
  __shared__ uint32_t hit[DM_TS * kLdsPitch];
  __shared__ uint32_t miss[DM_TS * kLdsPitch];
  __shared__ int32_t sh_free, sh_T;
  __shared__ uint32_t sh_U;
  const int tid = threadIdx.x, lane = lane_id();
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t n_active = min((int64_t)cnt[CNT_ACTIVE], (int64_t)g.act_cap);
  for (int64_t j = blockIdx.x; j < n_active; j += gridDim.x) {
    const int32_t tile = act_tiles[j];
    const int32_t off = act_off[j];
    const int32_t count = tile_count[tile];
    for (int e = tid; e < DM_TS * kLdsPitch; e += kApplyThreads) { hit[e] = 0u; miss[e] = 0u; }
    if (tid == 0) { sh_free = 0; sh_T = 0; sh_U = 0u; }
    __syncthreads();
    const int32_t tx0 = (tile % g.TX) * DM_TS;
    const int32_t ty0 = (tile / g.TX) * DM_TS;  // band-local
    uint32_t myU = 0;
    for (int32_t sidx = off + wid; sidx < off + count; sidx += kApplyThreads / 64) {
      const Seg sg = segs[sidx];
      const Beam bm = beams[sg.beam];
      const int32_t k = (int32_t)sg.k0 + lane;
      if (k <= (int32_t)sg.k1) {
        const int32_t q = bm.n > 0 ? dm_udiv(2 * k * bm.adb + bm.n, 2 * bm.n, bm.rden) : 0;
        const int32_t ma = bm.sa + k * bm.ia;
        const int32_t mb = bm.sb + bm.ib * q;
        const int32_t x = bm.xmajor ? ma : mb;
        const int32_t yl = (bm.xmajor ? mb : ma) - g.row0;
        const int32_t lx = x - tx0, ly = yl - ty0;
        if (x >= 0 && x < g.W && yl >= 0 && yl < g.R && (uint32_t)lx < DM_TS && (uint32_t)ly < DM_TS) {
          const bool is_hit = (k == bm.n) && (bm.flags & 2);
          atomicAdd(is_hit ? &hit[ly * kLdsPitch + lx] : &miss[ly * kLdsPitch + lx], 1u);
          ++myU;
        }
      }
    }
    __syncthreads();
    // fused apply: thread -> 4 consecutive cells of a row, 16 threads per row
    int32_t dT = 0, dFree = 0;
    const int cx = (tid & 15) * 4;
    for (int rr = 0; rr < DM_TS / 16; ++rr) {
      const int ly = (tid >> 4) + 16 * rr;
      const int64_t gy = ty0 + ly;
      if (gy >= g.R) break;
      uint32_t h4[4], m4[4];
      bool any = false;
      for (int e = 0; e < 4; ++e) {
        h4[e] = hit[ly * kLdsPitch + cx + e];
        m4[e] = miss[ly * kLdsPitch + cx + e];
        any |= (h4[e] | m4[e]) != 0u;
      }
      if (!any) continue;
      const int64_t base = gy * (int64_t)g.W + tx0 + cx;
      if (vec_ok && tx0 + cx + 4 <= g.W) {
        float4 l4 = *reinterpret_cast<const float4*>(L + base);
        char4 s4 = *reinterpret_cast<const char4*>(state + base);
        float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        int8_t sv[4] = {(int8_t)s4.x, (int8_t)s4.y, (int8_t)s4.z, (int8_t)s4.w};
        for (int e = 0; e < 4; ++e) {
          if ((h4[e] | m4[e]) == 0u) continue;
          const int8_t old = sv[e];
          lv[e] = apply_one(p, lv[e], h4[e], m4[e]);
          sv[e] = state_of(p, lv[e]);
          dT += 1;
          dFree += (sv[e] == 0) - (old == 0);
        }
        *reinterpret_cast<float4*>(L + base) = make_float4(lv[0], lv[1], lv[2], lv[3]);
        *reinterpret_cast<char4*>(state + base) = make_char4(sv[0], sv[1], sv[2], sv[3]);
      } else {
        for (int e = 0; e < 4; ++e) {
          if ((h4[e] | m4[e]) == 0u) continue;
          if (tx0 + cx + e >= g.W) continue;
          const int8_t old = state[base + e];
          const float nl = apply_one(p, L[base + e], h4[e], m4[e]);
          const int8_t ns = state_of(p, nl);
          L[base + e] = nl;
          state[base + e] = ns;
          dT += 1;
          dFree += (ns == 0) - (old == 0);
        }
      }
    }
    if (dT) atomicAdd(&sh_T, dT);
    if (dFree) atomicAdd(&sh_free, dFree);
    if (myU) atomicAdd(&sh_U, myU);
    __syncthreads();
    if (tid == 0) {
      if (sh_T) atomicAdd(&cnt[CNT_T], (unsigned long long)sh_T);
      if (sh_U) atomicAdd(&cnt[CNT_U], (unsigned long long)sh_U);
      tile_free[tile] += sh_free;
      tile_count[tile] = 0;  // ready for the next call
    }
    __syncthreads();
  }
}

// ---- maintenance kernels ----------------------------------------------------

__global__ __launch_bounds__(256) void k_recount(Geom g, const int8_t* __restrict__ state,
                                                 int32_t* __restrict__ tile_free) {
  const int64_t tile = blockIdx.x;
  const int32_t tx0 = (int32_t)(tile % g.TX) * DM_TS, ty0 = (int32_t)(tile / g.TX) * DM_TS;
  __shared__ int32_t acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  int32_t c = 0;
  for (int e = threadIdx.x; e < DM_TS * DM_TS; e += 256) {
    const int32_t x = tx0 + (e & 63), y = ty0 + (e >> 6);
    if (x < g.W && y < g.R) c += state[(int64_t)y * g.W + x] == 0;
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
  ge.W = (int32_t)g->W;
  ge.R = (int32_t)g->R;
  ge.row0 = (int32_t)g->row0;
  ge.TX = (int32_t)g->TX;
  ge.TY = (int32_t)g->TY;
  ge.act_cap = (int32_t)g->act_cap;
  ge.seg_cap = g->segs_cap;
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
  PrepArgs a;
  a.S = S;
  a.N = N;
  a.ox = g->p.origin_x;
  a.oy = g->p.origin_y;
  a.res = g->p.resolution;
  a.range_min = g->p.range_min;
  a.range_max = g->p.range_max;
  const Geom ge = make_geom(g);
  const int nblk = (int)((nb + 255) / 256);
  KernelTimer t;
  dm_timer_begin(g, "beam_prep", &t);
  hipLaunchKernelGGL(k_beam_prep, dim3(nblk), dim3(256), 0, g->stream, a, ge, d_pose4, d_ranges,
                     d_trig, g->beams, g->tile_count, g->tile_slot, g->act_tiles, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "scan_active", &t);
  hipLaunchKernelGGL(k_scan_active, dim3(1), dim3(1024), 0, g->stream, ge, g->act_tiles,
                     g->tile_count, g->act_off, g->act_cur, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  dm_timer_begin(g, "scatter", &t);
  hipLaunchKernelGGL(k_scatter, dim3(nblk), dim3(256), 0, g->stream, a, ge, g->beams,
                     g->tile_slot, g->act_cur, g->segs, g->cnt);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  const int vec_ok = (g->W % 4 == 0) ? 1 : 0;
  const int napply = grid_for(g->act_cap, 1, 4096);
  dm_timer_begin(g, "tile_apply", &t);
  hipLaunchKernelGGL(k_tile_apply, dim3(napply), dim3(kApplyThreads), 0, g->stream, ge,
                     make_apply(g), g->act_tiles, g->act_off, g->segs, g->beams, g->tile_count,
                     g->tile_free, g->L, g->state, g->cnt, vec_ok);
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
