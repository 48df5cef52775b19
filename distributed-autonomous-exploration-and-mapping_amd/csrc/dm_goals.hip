// dm_goals.hip — frontier goal selection on the device.
//
// Policy (the host restatement is dm/goals.py, the test reference): robot r
// at (rx, ry) scores cluster c with
//   dx = cx_m - rx; dy = cy_m - ry; dist = sqrt(dx*dx + dy*dy)
//   util = size / (1 + w * dist)            (IEEE double, no FMA)
// over the clusters with size >= min_size and dist >= min_distance, takes the
// best util, ties to the smaller label.  Robots choose in order, each taking
// the best cluster no earlier robot took (greedy assignment; the reference
// explores reactively, main.py:123-188, so there is no reference policy).
//
// Robot r's choice is among its R best clusters (at most R - 1 are taken
// before its turn), so the device computes every robot's top R — one
// bitonic sort per (robot, 4096-record chunk) in LDS, then merges of the
// chunk lists — and the host runs the O(R^2) greedy over those lists.  The
// records are the label-sorted list of the last collected frontier result, so
// "smaller label" is "smaller record index".
#include <algorithm>

#include "dm_internal.h"

namespace {

constexpr int kGoalN = 4096;       // keys per sort (one workgroup)
constexpr int kGoalThreads = 256;

// Key of a candidate: the util's IEEE bits (util > 0, so larger util = larger
// unsigned bits); 0 = not eligible.  Order: larger key first, then smaller
// index.
__device__ inline bool goal_better(unsigned long long ka, uint32_t ia, unsigned long long kb, uint32_t ib) {
  return ka > kb || (ka == kb && ia < ib);
}

// Sort s_k / s_i (kGoalN entries) best-first.
__device__ inline void goal_sort(unsigned long long* s_k, uint32_t* s_i) {
  for (int k = 2; k <= kGoalN; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < kGoalN; i += kGoalThreads) {
        const int l = i ^ j;
        if (l <= i) continue;
        const unsigned long long ka = s_k[i], kb = s_k[l];
        const uint32_t ia = s_i[i], ib = s_i[l];
        // blocks with (i & k) == 0 put the better one first, the others last
        const bool swap = ((i & k) == 0) ? goal_better(kb, ib, ka, ia) : goal_better(ka, ia, kb, ib);
        if (swap) {
          s_k[i] = kb; s_k[l] = ka;
          s_i[i] = ib; s_i[l] = ia;
        }
      }
      __syncthreads();
    }
  }
}

// Workgroup (chunk, robot): the chunk's best T records for the robot.
__global__ __launch_bounds__(kGoalThreads) void k_goal_topk(const dm_cluster* __restrict__ recs, int64_t K,
                                                            const double* __restrict__ robots, int32_t T,
                                                            int64_t min_size, double w, double min_dist,
                                                            unsigned long long* __restrict__ out_k,
                                                            uint32_t* __restrict__ out_i) {
  __shared__ unsigned long long s_k[kGoalN];
  __shared__ uint32_t s_i[kGoalN];
  const int64_t chunk = blockIdx.x, r = blockIdx.y, nch = gridDim.x;
  const double rx = robots[2 * r], ry = robots[2 * r + 1];
  for (int e = threadIdx.x; e < kGoalN; e += kGoalThreads) {
    const int64_t c = chunk * kGoalN + e;
    unsigned long long key = 0ull;
    if (c < K) {
      const dm_cluster q = recs[c];
      const double dx = q.cx_m - rx, dy = q.cy_m - ry;
      const double dist = __dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)));
      if (q.size >= min_size && dist >= min_dist) {
        const double util = __ddiv_rn((double)q.size, __dadd_rn(1.0, __dmul_rn(w, dist)));
        key = (unsigned long long)__double_as_longlong(util);
      }
    }
    s_k[e] = key;
    s_i[e] = c < K ? (uint32_t)c : 0xFFFFFFFFu;
  }
  __syncthreads();
  goal_sort(s_k, s_i);
  for (int t = threadIdx.x; t < T; t += kGoalThreads) {
    const int64_t o = (r * nch + chunk) * T + t;
    out_k[o] = s_k[t];
    out_i[o] = s_i[t];
  }
}

// Workgroup (group, robot): merge `per` consecutive T-lists of the robot's
// nlists into one (the best T of their union).
__global__ __launch_bounds__(kGoalThreads) void k_goal_merge(const unsigned long long* __restrict__ in_k,
                                                             const uint32_t* __restrict__ in_i, int64_t nlists,
                                                             int32_t T, int32_t per,
                                                             unsigned long long* __restrict__ out_k,
                                                             uint32_t* __restrict__ out_i) {
  __shared__ unsigned long long s_k[kGoalN];
  __shared__ uint32_t s_i[kGoalN];
  const int64_t grp = blockIdx.x, r = blockIdx.y, ngrp = gridDim.x;
  const int64_t l0 = grp * per;
  const int64_t n = min((int64_t)per, nlists - l0) * T;
  for (int e = threadIdx.x; e < kGoalN; e += kGoalThreads) {
    const bool in = e < n;
    const int64_t src = (r * nlists + l0) * T + e;
    s_k[e] = in ? in_k[src] : 0ull;
    s_i[e] = in ? in_i[src] : 0xFFFFFFFFu;
  }
  __syncthreads();
  goal_sort(s_k, s_i);
  for (int t = threadIdx.x; t < T; t += kGoalThreads) {
    const int64_t o = (r * ngrp + grp) * T + t;
    out_k[o] = s_k[t];
    out_i[o] = s_i[t];
  }
}

// Centroids of the chosen records (idx < 0: none -> NaN).
__global__ void k_goal_gather(const dm_cluster* __restrict__ recs, const int64_t* __restrict__ idx, int32_t R,
                              double* __restrict__ xy) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int64_t c = idx[r];
  xy[2 * r] = c >= 0 ? recs[c].cx_m : __builtin_nan("");
  xy[2 * r + 1] = c >= 0 ? recs[c].cy_m : __builtin_nan("");
}

}  // namespace

int dm_launch_goal_gather(dm_grid* g, const dm_cluster* d_recs, const int64_t* d_idx, int32_t R, double* d_xy) {
  hipLaunchKernelGGL(k_goal_gather, dim3((R + 63) / 64), dim3(64), 0, g->stream, d_recs, d_idx, R, d_xy);
  DM_HIP(hipGetLastError());
  return DM_OK;
}

// Top-T lists of R robots over K label-sorted records; on return *d_k / *d_i
// point at the final [R][T] lists (in g->goal_* workspace).  T <= 256.
int dm_launch_goal_topk(dm_grid* g, const dm_cluster* d_recs, int64_t K, const double* d_robots, int32_t R,
                        int32_t T, int64_t min_size, double w, double min_dist,
                        const unsigned long long** d_k, const uint32_t** d_i) {
  const int64_t nch = (K + kGoalN - 1) / kGoalN;
  const int64_t need = (int64_t)R * std::max<int64_t>(nch, 1) * T;
  if (need > g->goal_cap) {
    for (int b = 0; b < 2; ++b) {
      if (g->goal_k[b]) (void)hipFree(g->goal_k[b]);
      if (g->goal_i[b]) (void)hipFree(g->goal_i[b]);
      g->goal_k[b] = nullptr;
      g->goal_i[b] = nullptr;
    }
    g->goal_cap = 0;
    for (int b = 0; b < 2; ++b) {
      DM_HIP(hipMalloc((void**)&g->goal_k[b], sizeof(unsigned long long) * (size_t)need));
      DM_HIP(hipMalloc((void**)&g->goal_i[b], sizeof(uint32_t) * (size_t)need));
    }
    g->goal_cap = need;
  }
  int cur = 0;
  KernelTimer t;
  dm_timer_begin(g, "goal_topk", &t);
  hipLaunchKernelGGL(k_goal_topk, dim3((unsigned)std::max<int64_t>(nch, 1), (unsigned)R), dim3(kGoalThreads), 0,
                     g->stream, d_recs, K, d_robots, T, min_size, w, min_dist, g->goal_k[0], g->goal_i[0]);
  DM_HIP(hipGetLastError());
  int64_t nl = std::max<int64_t>(nch, 1);
  const int32_t per = kGoalN / T;  // lists one merge workgroup takes (>= 16)
  while (nl > 1) {
    const int64_t ng = (nl + per - 1) / per;
    hipLaunchKernelGGL(k_goal_merge, dim3((unsigned)ng, (unsigned)R), dim3(kGoalThreads), 0, g->stream,
                       g->goal_k[cur], g->goal_i[cur], nl, T, per, g->goal_k[cur ^ 1], g->goal_i[cur ^ 1]);
    DM_HIP(hipGetLastError());
    cur ^= 1;
    nl = ng;
  }
  dm_timer_end(g, &t);
  *d_k = g->goal_k[cur];
  *d_i = g->goal_i[cur];
  return DM_OK;
}
