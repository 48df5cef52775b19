// dm_batch.cpp — graph cache and flush of the launch batching (dm_batch.h).
#include "dm_batch.h"

thread_local DmBatch* t_dm_batch = nullptr;

namespace {

hipError_t launch_direct(DmChain& c, const DmRecLaunch& r) {
  void* ptrs[64];
  for (size_t i = 0; i < r.n_args && i < 64; ++i) ptrs[i] = c.args.data() + c.offs[r.first_arg + i];
  return hipLaunchKernel(r.func, r.grid, r.block, ptrs, r.shmem, c.stream);
}

hipError_t build(DmChain& c, hipGraphExec_t* exec) {
  hipGraph_t gr = nullptr;
  hipError_t e = hipGraphCreate(&gr, 0);
  if (e != hipSuccess) return e;
  hipGraphNode_t prev = nullptr;
  std::vector<void*> ptrs;
  for (const DmRecLaunch& r : c.launches) {
    ptrs.resize(r.n_args);
    for (size_t i = 0; i < r.n_args; ++i) ptrs[i] = c.args.data() + c.offs[r.first_arg + i];
    hipKernelNodeParams p;
    memset(&p, 0, sizeof p);
    p.func = const_cast<void*>(r.func);
    p.gridDim = r.grid;
    p.blockDim = r.block;
    p.sharedMemBytes = r.shmem;
    p.kernelParams = ptrs.data();
    p.extra = nullptr;
    hipGraphNode_t node = nullptr;
    e = hipGraphAddKernelNode(&node, gr, prev ? &prev : nullptr, prev ? 1 : 0, &p);
    if (e != hipSuccess) break;
    prev = node;
  }
  if (e == hipSuccess) e = hipGraphInstantiate(exec, gr, nullptr, nullptr, 0);
  (void)hipGraphDestroy(gr);
  return e;
}

void reset(DmChain& c) {
  c.launches.clear();
  c.args.clear();
  c.offs.clear();
  c.key.clear();
}

}  // namespace

hipError_t dm_batch_flush(DmBatch* b, DmChain& c) {
  if (c.launches.empty()) return hipSuccess;
  hipError_t e = hipSuccess;
  if (c.launches.size() == 1) {  // a one-node graph saves nothing
    e = launch_direct(c, c.launches[0]);
    ++b->direct_launches;
    reset(c);
    return e;
  }
  const unsigned inst = (unsigned)(c.flushes++ % DmBatch::kInstances);
  c.key.append(reinterpret_cast<const char*>(&inst), sizeof inst);
  auto it = b->cache.find(c.key);
  if (it != b->cache.end()) {
    ++b->hits;
    b->order.splice(b->order.begin(), b->order, it->second.lru);
  } else {
    ++b->misses;
    hipGraphExec_t exec = nullptr;
    e = build(c, &exec);
    if (e != hipSuccess) {
      // fall back to direct launches in order
      (void)hipGetLastError();
      for (const DmRecLaunch& r : c.launches) {
        const hipError_t e2 = launch_direct(c, r);
        if (e2 != hipSuccess) {
          reset(c);
          return e2;
        }
      }
      b->direct_launches += c.launches.size();
      reset(c);
      return hipSuccess;
    }
    if (b->cache.size() >= b->cap) {  // evict the least recently used graph
      auto victim = b->cache.find(b->order.back());
      (void)hipGraphExecDestroy(victim->second.exec);
      b->cache.erase(victim);
      b->order.pop_back();
    }
    b->order.push_front(c.key);
    it = b->cache.emplace(c.key, DmBatch::Entry{exec, b->order.begin()}).first;
  }
  e = hipGraphLaunch(it->second.exec, c.stream);
  ++b->graph_launches;
  reset(c);
  return e;
}

hipError_t dm_batch_flush_all_of(DmBatch* b) {
  hipError_t first = hipSuccess;
  for (int i = 0; i < b->n_chains; ++i) {
    const hipError_t e = dm_batch_flush(b, b->chains[i]);
    if (e != hipSuccess && first == hipSuccess) first = e;
  }
  return first;
}

void dm_batch_release(DmBatch* b) {
  for (auto& kv : b->cache) (void)hipGraphExecDestroy(kv.second.exec);
  b->cache.clear();
  b->order.clear();
  for (auto& c : b->chains) reset(c);
  b->n_chains = 0;
}
