// dm_batch.h — launch batching: the kernels of a hot call are recorded per
// stream and replayed as one single-stream HIP graph launch per stream.
//
// Why: a pipelined C3 step enqueues ~14 kernels on three streams, and each
// hipLaunchKernel costs the host ~2.3-2.6 us, so the host, not the GPU, set
// the step time (tools/pipeline_probe.py, profiles/r02_launch_cost.log).  A
// launch of an instantiated chain graph costs ~2 us whatever its length
// (tools/native/launch_cost.hip: 7 kernels 16 us direct vs 1.7-2.8 us as a
// graph).  Multi-stream graphs are not used: on this runtime their branches
// ran one after the other and their launch cost as much as the kernels'.
//
// How: inside a DmBatchScope (dm_launch_integrate, dm_enqueue_frontiers),
// dm_launch() packs the kernel's arguments, converted to its parameter types,
// into the stream's chain and appends them to the chain's key (kernel, grid,
// block, LDS bytes, argument bytes).  A flush looks the key up in the
// handle's cache of instantiated graphs (LRU), builds and instantiates one on
// a miss, and launches it on the stream.  Everything that changes from call
// to call either lives in device memory (sequence counters, pass stamps) or
// takes few values (workspace parity, readback slot, quantised grid sizes),
// so the steady state hits the cache.  Ordering rules:
//   * a direct stream operation (event record / wait, memset, memcpy) inside
//     a scope first flushes every chain (dm_batch_flush_all), so it keeps its
//     place in stream order;
//   * a kernel that waits on another stream's device-side signal (k_seq_gate)
//     first flushes the other chains (dm_batch_flush_others): the signal is
//     submitted before the gate, as with direct launches, so even streams that
//     share a hardware queue cannot deadlock;
//   * the scope's end flushes what is left.
// Outside a scope (and with profiling on, whose timers put events around each
// kernel, or DM_GRAPHS=0) dm_launch launches directly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <list>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

struct DmRecLaunch {
  const void* func;
  dim3 grid, block;
  unsigned shmem;
  size_t first_arg;  // index into DmChain::offs
  size_t n_args;
};

struct DmChain {
  hipStream_t stream = nullptr;
  std::vector<DmRecLaunch> launches;
  std::vector<unsigned char> args;  // packed arguments of every launch
  std::vector<size_t> offs;         // offset of each argument in args
  std::string key;
  uint64_t flushes = 0;  // graph flushes of this chain: the instance index (DmBatch::kInstances)
};

struct DmBatch {
  static constexpr int kChains = 4;
  // Consecutive flushes of a chain use different instances of the same
  // graph (kInstances in rotation), so an instantiated graph is never
  // relaunched while its previous launch may still be queued.  (With the
  // rotation, some graph launches still blocked the host for 60-115 us per
  // step in the C3 pipeline: DESIGN.md §3.3.)
  static constexpr unsigned kInstances = 4;
  DmChain chains[kChains];
  int n_chains = 0;
  struct Entry {
    hipGraphExec_t exec;
    std::list<std::string>::iterator lru;
  };
  std::unordered_map<std::string, Entry> cache;
  std::list<std::string> order;  // most recently used first
  size_t cap = 512;
  uint64_t hits = 0, misses = 0, graph_launches = 0, direct_launches = 0;
  bool enabled = true;  // DM_GRAPHS=0: never batch (A/B)
};

extern thread_local DmBatch* t_dm_batch;

hipError_t dm_batch_flush(DmBatch* b, DmChain& c);
hipError_t dm_batch_flush_all_of(DmBatch* b);
void dm_batch_release(DmBatch* b);  // destroys the cached graphs

// Flush every chain of the active scope (before a direct stream operation).
inline hipError_t dm_batch_flush_all() { return t_dm_batch ? dm_batch_flush_all_of(t_dm_batch) : hipSuccess; }

// Flush every chain of the active scope except the one of stream s (before a
// kernel on s that waits for another stream's device-side signal).
inline hipError_t dm_batch_flush_others(hipStream_t s) {
  DmBatch* b = t_dm_batch;
  if (!b) return hipSuccess;
  for (int i = 0; i < b->n_chains; ++i) {
    if (b->chains[i].stream == s) continue;
    const hipError_t e = dm_batch_flush(b, b->chains[i]);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Active between construction and finish() / destruction when `on`; nested
// scopes leave the outer one in charge.
class DmBatchScope {
 public:
  DmBatchScope(DmBatch* b, bool on) : prev_(t_dm_batch) {
    if (on && b->enabled && !prev_) {
      t_dm_batch = b;
      mine_ = b;
    }
  }
  // flush what is left and deactivate; returns the flush status
  hipError_t finish() {
    if (!mine_) return hipSuccess;
    const hipError_t e = dm_batch_flush_all_of(mine_);
    t_dm_batch = prev_;
    mine_ = nullptr;
    return e;
  }
  ~DmBatchScope() { (void)finish(); }
  DmBatchScope(const DmBatchScope&) = delete;
  DmBatchScope& operator=(const DmBatchScope&) = delete;

 private:
  DmBatch* prev_;
  DmBatch* mine_ = nullptr;
};

namespace dm_batch_detail {

template <typename T>
inline size_t align_up(size_t off) {
  return (off + alignof(T) - 1) & ~(size_t)(alignof(T) - 1);
}

// Stores argument a as kernel parameter type P at the end of buf.  A value of
// exactly that type is copied byte for byte (argument structs have no
// implicit padding, so equal arguments give equal bytes: the cache key).
template <typename P, typename A>
inline void put(std::vector<unsigned char>& buf, std::vector<size_t>& offs, A&& a) {
  using T = std::decay_t<P>;
  static_assert(std::is_trivially_copyable<T>::value, "kernel parameters must be trivially copyable");
  const size_t off = align_up<T>(buf.size());
  buf.resize(off + sizeof(T));
  if constexpr (std::is_same<std::decay_t<A>, T>::value) {
    memcpy(buf.data() + off, &a, sizeof(T));
  } else {
    const T t = static_cast<T>(a);
    memcpy(buf.data() + off, &t, sizeof(T));
  }
  offs.push_back(off);
}

inline DmChain& chain_for(DmBatch* b, hipStream_t s) {
  for (int i = 0; i < b->n_chains; ++i)
    if (b->chains[i].stream == s) return b->chains[i];
  if (b->n_chains == DmBatch::kChains) {  // cannot happen: a handle has three streams
    (void)dm_batch_flush(b, b->chains[0]);
    b->chains[0].stream = s;
    return b->chains[0];
  }
  DmChain& c = b->chains[b->n_chains++];
  c.stream = s;
  return c;
}

}  // namespace dm_batch_detail

// hipLaunchKernelGGL replacement for every kernel that may run inside a
// DmBatchScope.  Returns the launch status (recording always succeeds).
template <typename... P, typename... A>
hipError_t dm_launch(void (*k)(P...), dim3 grid, dim3 block, unsigned shmem, hipStream_t s, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  DmBatch* b = t_dm_batch;
  if (!b) {
    std::vector<unsigned char> buf;
    std::vector<size_t> offs;
    buf.reserve(512);
    (dm_batch_detail::put<P>(buf, offs, std::forward<A>(a)), ...);
    void* ptrs[sizeof...(P) + 1];
    for (size_t i = 0; i < offs.size(); ++i) ptrs[i] = buf.data() + offs[i];
    return hipLaunchKernel((const void*)k, grid, block, ptrs, shmem, s);
  }
  DmChain& c = dm_batch_detail::chain_for(b, s);
  DmRecLaunch r{(const void*)k, grid, block, shmem, c.offs.size(), sizeof...(P)};
  const size_t a0 = c.args.size();
  (dm_batch_detail::put<P>(c.args, c.offs, std::forward<A>(a)), ...);
  const unsigned hdr[7] = {grid.x, grid.y, grid.z, block.x, block.y, block.z, shmem};
  c.key.append(reinterpret_cast<const char*>(&r.func), sizeof r.func);
  c.key.append(reinterpret_cast<const char*>(hdr), sizeof hdr);
  c.key.append(reinterpret_cast<const char*>(c.args.data() + a0), c.args.size() - a0);
  c.launches.push_back(r);
  return hipSuccess;
}

// Round n up to a quarter-octave step (1, 1.25, 1.5, 1.75 x 2^k; exact below
// 8): grid sizes derived from the last pass's statistics then take few
// values, so the graphs that carry them are reused.
inline int64_t dm_quantize_up(int64_t n) {
  if (n <= 8) return n;
  int sh = 0;
  while ((n >> sh) >= 8) ++sh;
  const int64_t step = (int64_t)1 << sh;  // n in [4, 8) x 2^sh: steps of a quarter octave
  return ((n + step - 1) / step) * step;
}
