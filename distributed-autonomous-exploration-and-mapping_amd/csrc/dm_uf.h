// dm_uf.h — global-memory union-find shared by the frontier merge
// (k_frontier_merge, dm_frontier.hip) and the cross-band merge
// (k_merge_pairs, dm_merge.hip).
//
// Labels are the SPEC's min row-major index: the root of a
// set is always the element with the smallest label, so the final labels do
// not depend on the order in which unions land.  Hooks are CAS at the
// device-coherent point (per-XCD L2s are not coherent; MI355X_MICROARCH.md
// §Workgroup dispatch); reads are relaxed agent-scope loads (below).
//
// Every loop is bounded.  A loop that runs out of iterations (a chain longer
// than the bound, or a corrupted parent array) does not return a silently
// wrong node: it sets `bit` in *flag (a counter word the readback checks:
// CNT_OVERFLOW / M_FLAGS), and the host turns that into DM_ERR_INCOMPLETE.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kUfFindBound = 1 << 22;
constexpr int kUfUniteBound = 1 << 20;

// Reads of parent[] are relaxed agent-scope loads (global_load sc1: past
// the CU's L1, served by the XCD's L2), not atomic RMWs: a find costs one
// L2 round trip per step instead of one memory-side atomic.  Such a read may
// be stale, but only in one way: a node is hooked exactly once, while it is
// a root, and parents never change otherwise, so a stale read can only show
// a hooked node as still being a root.  dm_uf_unite repairs that with the
// value its failed CAS returns (the node's real parent, read at the
// coherence point), so every retry climbs at least one real edge.
__device__ inline int32_t dm_uf_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline void dm_uf_flag(unsigned long long* flag, unsigned long long bit) {
  if (flag) atomicOr(flag, bit);
}

__device__ inline int32_t dm_uf_find(const int32_t* par, int32_t x, unsigned long long* flag,
                                     unsigned long long bit) {
  for (int it = 0; it < kUfFindBound; ++it) {
    const int32_t p = dm_uf_load(par + x);
    if (p == x) return x;
    x = p;
  }
  dm_uf_flag(flag, bit);
  return x;
}

// Lock-free union: hook the root with the larger label under the other.
// Two nodes found in the same set stay in it (sets only merge), so a == b
// is final even from stale reads.
__device__ inline void dm_uf_unite(int32_t* par, const long long* label, int32_t a, int32_t b,
                                   unsigned long long* flag, unsigned long long bit) {
  for (int it = 0; it < kUfUniteBound; ++it) {
    a = dm_uf_find(par, a, flag, bit);
    b = dm_uf_find(par, b, flag, bit);
    if (a == b) return;
    if (label[a] < label[b]) { const int32_t t = a; a = b; b = t; }
    const int32_t old = atomicCAS(&par[a], a, b);
    if (old == a) return;
    // a was hooked meanwhile (or read stale): continue from its real parent
    a = old;
    b = dm_uf_find(par, b, flag, bit);
    if (a == b) return;
  }
  dm_uf_flag(flag, bit);
}

// Plain (non-atomic) find for kernels that run after every union landed.
__device__ inline int32_t dm_uf_root(const int32_t* par, int32_t x, unsigned long long* flag,
                                     unsigned long long bit) {
  for (int it = 0; it < kUfFindBound; ++it) {
    const int32_t p = par[x];
    if (p == x) return x;
    x = p;
  }
  dm_uf_flag(flag, bit);
  return x;
}

// Find with path halving: every other node on the way is re-pointed to its
// grandparent (a relaxed agent-scope store).  Only a non-root is ever
// re-pointed, and only to an ancestor, so a CAS hooking a root is never
// undone and the forest stays acyclic (parents only point to smaller
// indices); a racing halving store just writes another ancestor.
__device__ inline int32_t dm_uf_find_halve(int32_t* par, int32_t x, unsigned long long* flag,
                                           unsigned long long bit) {
  for (int it = 0; it < kUfFindBound; ++it) {
    const int32_t p = dm_uf_load(par + x);
    if (p == x) return x;
    const int32_t gp = dm_uf_load(par + p);
    if (gp == p) return p;
    __hip_atomic_store(par + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = gp;
  }
  dm_uf_flag(flag, bit);
  return x;
}

// dm_uf_unite_idx with halving finds (many concurrent unions over one
// forest: k_frontier_edges)
__device__ inline void dm_uf_unite_idx_halve(int32_t* par, int32_t a, int32_t b, unsigned long long* flag,
                                             unsigned long long bit) {
  for (int it = 0; it < kUfUniteBound; ++it) {
    a = dm_uf_find_halve(par, a, flag, bit);
    b = dm_uf_find_halve(par, b, flag, bit);
    if (a == b) return;
    if (a < b) { const int32_t t = a; a = b; b = t; }
    const int32_t old = atomicCAS(&par[a], a, b);
    if (old == a) return;
    a = old;
  }
  dm_uf_flag(flag, bit);
}

// dm_uf_unite_idx with both finds walked in step (their loads issued
// together: one round trip per level of the deeper chain instead of one per
// level of each).
__device__ inline void dm_uf_unite_idx2(int32_t* par, int32_t a, int32_t b, unsigned long long* flag,
                                        unsigned long long bit) {
  for (int it = 0; it < kUfUniteBound; ++it) {
    for (int f = 0;; ++f) {
      if (f == kUfFindBound) {
        dm_uf_flag(flag, bit);
        return;
      }
      const int32_t pa = dm_uf_load(par + a), pb = dm_uf_load(par + b);
      if (pa == a && pb == b) break;
      a = pa;
      b = pb;
    }
    if (a == b) return;
    if (a < b) { const int32_t t = a; a = b; b = t; }
    const int32_t old = atomicCAS(&par[a], a, b);
    if (old == a) return;
    a = old;  // hooked meanwhile: climb from its real parent
  }
  dm_uf_flag(flag, bit);
}

// Union keyed by node index instead of label: hook the root with the larger
// index under the other.  Used where the labels are not known yet when the
// unions run (the in-kernel tile-edge unions of k_frontier_tile: a
// neighbour's slot labels are still being written); the set's label (its
// min) is folded into the root afterwards (k_frontier_resolve).  Same
// stale-read argument as dm_uf_unite: parents only ever point to a smaller
// index, so the forest stays acyclic whatever order the CASes land in.
__device__ inline void dm_uf_unite_idx(int32_t* par, int32_t a, int32_t b, unsigned long long* flag,
                                       unsigned long long bit) {
  for (int it = 0; it < kUfUniteBound; ++it) {
    a = dm_uf_find(par, a, flag, bit);
    b = dm_uf_find(par, b, flag, bit);
    if (a == b) return;
    if (a < b) { const int32_t t = a; a = b; b = t; }
    const int32_t old = atomicCAS(&par[a], a, b);
    if (old == a) return;
    a = old;  // hooked meanwhile: climb from its real parent
  }
  dm_uf_flag(flag, bit);
}
