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
  int64_t nb;  // beams in this call
};

__device__ inline int lane_id() { return __lane_id(); }

__global__ __launch_bounds__(256) void k_beam_prep(RayArgs a, Geom g, const double* __restrict__ pose4,
                                                   const float* __restrict__ ranges,
                                                   const double* __restrict__ trig,
                                                   Beam* __restrict__ beams, int32_t* tile_count,
                                                   int32_t* tile_slot, int32_t* act_tiles,
                                                   unsigned long long* cnt) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)a.S * a.N;
  if (b >= nb) return;
  const int32_t s = (int32_t)(b / a.N), i = (int32_t)(b % a.N);
  const Beam bm = dm_make_beam(a, pose4, ranges, trig, s, i);
  beams[b] = bm;
  if (!(bm.flags & 1)) return;
  dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t, int32_t) {
    const int32_t old = atomicAdd(&tile_count[tile], 1);
    if (old == 0) {
      const unsigned long long slot = atomicAdd(&cnt[CNT_ACTIVE], 1ull);
      if (slot < (unsigned long long)g.act_cap) {
        act_tiles[slot] = tile;
        tile_slot[tile] = (int32_t)slot;
      } else {
        tile_slot[tile] = -1;
        atomicOr(&cnt[CNT_OVERFLOW], 1ull);
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

__global__ __launch_bounds__(256) void k_scatter(RayArgs a, Geom g, const Beam* __restrict__ beams,
                                                 const int32_t* __restrict__ tile_slot,
                                                 int32_t* act_cur, Seg* __restrict__ segs,
                                                 unsigned long long* cnt) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)a.S * a.N;
  if (b >= nb) return;
  const Beam bm = beams[b];
  if (!(bm.flags & 1)) return;
  dm_for_each_piece(bm, g.r, [&](int32_t tile, int32_t k0, int32_t k1) {
    const int32_t slot = tile_slot[tile];
    const int64_t idx = (slot >= 0 && slot < g.act_cap) ? (int64_t)atomicAdd(&act_cur[slot], 1) : -1;
    if (idx >= 0 && idx < g.seg_cap) {
      Seg sg;
      sg.beam = (uint32_t)b;
      sg.k0 = (uint16_t)k0;
      sg.k1 = (uint16_t)k1;
      segs[idx] = sg;
    } else {
      atomicOr(&cnt[CNT_OVERFLOW], 2ull);
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
    const int32_t tx0 = (tile % g.r.TX) * DM_TS;
    const int32_t ty0 = (tile / g.r.TX) * DM_TS;  // band-local
    uint32_t myU = 0;
    for (int32_t sidx = off + wid; sidx < off + count; sidx += kApplyThreads / 64) {
      const Seg sg = segs[sidx];
      if ((int64_t)sg.beam >= g.nb) continue;  // cannot happen; keeps a logic error in-bounds
      const Beam bm = beams[sg.beam];
      const int32_t k = (int32_t)sg.k0 + lane;
      if (k <= (int32_t)sg.k1) {
        int32_t x, yl;
        dm_cell(bm, k, g.r.row0, &x, &yl);
        const int32_t lx = x - tx0, ly = yl - ty0;
        if (x >= 0 && x < g.r.W && yl >= 0 && yl < g.r.R && (uint32_t)lx < DM_TS && (uint32_t)ly < DM_TS) {
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
      if (gy >= g.r.R) break;
      uint32_t h4[4], m4[4];
      bool any = false;
      for (int e = 0; e < 4; ++e) {
        h4[e] = hit[ly * kLdsPitch + cx + e];
        m4[e] = miss[ly * kLdsPitch + cx + e];
        any |= (h4[e] | m4[e]) != 0u;
      }
      if (!any) continue;
      const int64_t base = gy * (int64_t)g.r.W + tx0 + cx;
      if (vec_ok && tx0 + cx + 4 <= g.r.W) {
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
          if (tx0 + cx + e >= g.r.W) continue;
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
