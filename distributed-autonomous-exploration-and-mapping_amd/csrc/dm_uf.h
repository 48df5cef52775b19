// dm_uf.h — global-memory union-find shared by the frontier merge
// (k_frontier_merge, dm_frontier.hip) and the cross-band merge
// (k_merge_pairs, dm_merge.hip).
//
// Labels are the SPEC's min row-major index: the root of a
// set is always the element with the smallest label, so the final labels do
// not depend on the order in which unions land.  Every access to parent[] is
// an atomic RMW, performed at the device-coherent point (per-XCD L2s are not
// coherent; MI355X_MICROARCH.md §Workgroup dispatch).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ inline int32_t dm_uf_load(int32_t* p) { return atomicOr(p, 0); }

__device__ inline int32_t dm_uf_find(int32_t* par, int32_t x) {
  for (int it = 0; it < (1 << 22); ++it) {
    const int32_t p = dm_uf_load(par + x);
    if (p == x) return x;
    x = p;
  }
  return x;
}

// Lock-free union: hook the root with the larger label under the other.
__device__ inline void dm_uf_unite(int32_t* par, const long long* label, int32_t a, int32_t b) {
  for (int it = 0; it < (1 << 20); ++it) {
    a = dm_uf_find(par, a);
    b = dm_uf_find(par, b);
    if (a == b) return;
    if (label[a] < label[b]) { const int32_t t = a; a = b; b = t; }
    if (atomicCAS(&par[a], a, b) == a) return;
  }
}

// Plain (non-atomic) find for kernels that run after every union landed.
__device__ inline int32_t dm_uf_root(const int32_t* par, int32_t x) {
  for (int it = 0; it < (1 << 22); ++it) {
    const int32_t p = par[x];
    if (p == x) break;
    x = p;
  }
  return x;
}
