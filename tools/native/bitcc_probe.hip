// bitcc_probe.hip -- measurement probe, not part of libdm.
// Built by tools/native/Makefile into libbitcc_probe.so and called by
// tools/bitcc_probe.py with the dm_grid* of a libdm handle in the same
// process (the struct layout comes from the same dm_internal.h).
//
// Bit-parallel tile-local labelling timed against libdm's union-find kernels
// on the last synchronous pass's tiles.  One wave per listed tile, lane y =
// tile row y.  Components are taken one at a time: the first remaining
// frontier cell in row-major order is the seed (and the component's min
// index, i.e. its label); the mask grows by m = fill(F & dilate8(m)) until no
// lane changes, where fill() widens every touched bit to its whole run of F
// (carry propagation up, and the same on bit-reversed rows down).  Totals
// (components, sum of labels, sizes, sum of x, sum of y) are checked against
// the pass's own slots.
#include <algorithm>

#include "../../distributed-autonomous-exploration-and-mapping_amd/csrc/dm_internal.h"

#define PROBE_HIP(x)                        \
  do {                                      \
    const hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return (int)e_;   \
  } while (0)

namespace {

__device__ inline uint64_t run_fill(uint64_t x, uint64_t F, uint64_t RF) {
  const uint64_t up = (((F + x) ^ F) & F) | x;
  const uint64_t rx = __builtin_bitreverse64(x);
  const uint64_t dn = (((RF + rx) ^ RF) & RF) | rx;
  return up | __builtin_bitreverse64(dn);
}

__global__ __launch_bounds__(256) void k_probe_bitcc(int64_t W, int32_t TX, int64_t row0, const uint64_t* __restrict__ fbits,
                                                     const int32_t* __restrict__ ftiles, int64_t nft,
                                                     unsigned long long* tot) {
  const int w = threadIdx.x >> 6, lane = __lane_id();
  for (int64_t jj = (int64_t)blockIdx.x * 4 + w; jj < nft; jj += (int64_t)gridDim.x * 4) {
    const int32_t tile = __builtin_amdgcn_readfirstlane(ftiles[jj]);
    const uint64_t F = fbits[jj * DM_TS + lane];
    if (__ballot(F != 0ull) == 0ull) continue;
    const uint64_t RF = __builtin_bitreverse64(F);
    const long long tx0 = (long long)(tile % TX) * DM_TS;
    const long long gy = (long long)row0 + (long long)(tile / TX) * DM_TS + lane;
    uint64_t rem = F;
    unsigned long long ncomp = 0ull, slab = 0ull;
    while (true) {
      const uint64_t rows = __ballot(rem != 0ull);
      if (rows == 0ull) break;
      const int y0 = __ffsll((unsigned long long)rows) - 1;
      const uint64_t r0 = __shfl(rem, y0);
      const uint64_t seed = r0 & (~r0 + 1ull);
      uint64_t m = lane == y0 ? run_fill(seed, F, RF) : 0ull;
      for (int it = 0; it < 4096; ++it) {
        uint64_t up = __shfl_up(m, 1), dn = __shfl_down(m, 1);
        if (lane == 0) up = 0ull;
        if (lane == 63) dn = 0ull;
        uint64_t d = m | up | dn;
        d |= (d << 1) | (d >> 1);
        const uint64_t x = run_fill(F & d, F, RF);
        if (__ballot(x != m) == 0ull) break;
        m = x;
      }
      ++ncomp;
      slab += (unsigned long long)(((long long)row0 + (long long)(tile / TX) * DM_TS + y0) * W + tx0 +
                                   (__ffsll((unsigned long long)seed) - 1));
      rem &= ~m;
    }
    // size, sum of x, sum of y of all the tile's components = of F
    const unsigned long long c = (unsigned long long)__popcll(F);
    unsigned long long sx = c * (unsigned long long)tx0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const uint64_t plane = b == 0 ? 0xAAAAAAAAAAAAAAAAull : b == 1 ? 0xCCCCCCCCCCCCCCCCull
                           : b == 2 ? 0xF0F0F0F0F0F0F0F0ull : b == 3 ? 0xFF00FF00FF00FF00ull
                           : b == 4 ? 0xFFFF0000FFFF0000ull : 0xFFFFFFFF00000000ull;
      sx += (unsigned long long)__popcll(F & plane) << b;
    }
    unsigned long long sy = c * (unsigned long long)gy, sc = c;
    for (int o = 32; o > 0; o >>= 1) {
      sc += __shfl_xor(sc, o);
      sx += __shfl_xor(sx, o);
      sy += __shfl_xor(sy, o);
    }
    if (lane == 0) {
      atomicAdd(&tot[0], ncomp);
      atomicAdd(&tot[1], slab);
      atomicAdd(&tot[2], sc);
      atomicAdd(&tot[3], sx);
      atomicAdd(&tot[4], sy);
    }
  }
}

// The same totals over the pass's slots (one per tile-local component).
__global__ __launch_bounds__(256) void k_probe_slot_sums(const unsigned long long* __restrict__ fsh, int64_t slot_per,
                                                         const long long* __restrict__ slot_label,
                                                         const long long* __restrict__ slot_own,
                                                         unsigned long long* tot) {
  for (int s = 0; s < kShards; ++s) {
    const int64_t n = std::min<int64_t>((int64_t)fsh[s * kShardWords + SH_SLOT], slot_per);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
      const int64_t sl = (int64_t)s * slot_per + i;
      atomicAdd(&tot[0], 1ull);
      atomicAdd(&tot[1], (unsigned long long)slot_label[sl]);
      atomicAdd(&tot[2], (unsigned long long)slot_own[3 * sl]);
      atomicAdd(&tot[3], (unsigned long long)slot_own[3 * sl + 1]);
      atomicAdd(&tot[4], (unsigned long long)slot_own[3 * sl + 2]);
    }
  }
}

}  // namespace

// After a synchronous dm_frontiers: out[0..4] the probe's totals, out[5..9]
// the pass's slot totals, *ms the probe kernel's mean time over `reps`.
extern "C" int dm_probe_bitcc(dm_grid* g, int reps, double* ms, unsigned long long* out) {
  PROBE_HIP(hipDeviceSynchronize());
  const int64_t slot_per = g->slot_cap / kShards;
  const int64_t nft = (int64_t)g->h_cnt[CNT_FL0];
  unsigned long long* tot = nullptr;
  PROBE_HIP(hipMalloc(&tot, 32 * sizeof(unsigned long long)));
  PROBE_HIP(hipMemset(tot, 0, 32 * sizeof(unsigned long long)));
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nft + 3) / 4, 65536));
  hipEvent_t e0, e1;
  PROBE_HIP(hipEventCreate(&e0));
  PROBE_HIP(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_probe_slot_sums, dim3(256), dim3(256), 0, g->stream, g->fsh, slot_per, g->slot_label,
                     g->slot_own, tot + 8);
  hipLaunchKernelGGL(k_probe_bitcc, dim3(grid), dim3(256), 0, g->stream, (int64_t)g->W, (int32_t)g->TX, (int64_t)g->row0, g->fbits, g->ftiles, nft, tot);
  PROBE_HIP(hipStreamSynchronize(g->stream));
  PROBE_HIP(hipEventRecord(e0, g->stream));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k_probe_bitcc, dim3(grid), dim3(256), 0, g->stream, (int64_t)g->W, (int32_t)g->TX, (int64_t)g->row0, g->fbits, g->ftiles, nft,
                       tot + 16);
  PROBE_HIP(hipEventRecord(e1, g->stream));
  PROBE_HIP(hipEventSynchronize(e1));
  float t = 0.f;
  PROBE_HIP(hipEventElapsedTime(&t, e0, e1));
  *ms = reps > 0 ? (double)t / reps : 0.0;
  unsigned long long h[16];
  PROBE_HIP(hipMemcpy(h, tot, sizeof(h), hipMemcpyDeviceToHost));
  for (int i = 0; i < 5; ++i) {
    out[i] = h[i];
    out[5 + i] = h[8 + i];
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(tot);
  return DM_OK;
}
