// dm_phase.h — opt-in per-phase timing of the big kernels (build with
// -DDM_PHASE_TIMING: `make phase`, a separate libdm_phase.so; the product
// library compiles these macros to nothing).  Thread 0 of each workgroup
// accumulates the wall-clock ticks (100 MHz) between its marks in registers
// and adds them once, at kernel exit, to one of 64 shards of a per-TU device
// accumulator (no same-address atomics inside the timed region); read the
// shard sums with dm_debug_phases_<tu>().
#pragma once

#define DM_PH_SLOTS 24
#define DM_PH_SHARDS 64

#ifdef DM_PHASE_TIMING
#define DM_PH_DECL(tu) __device__ unsigned long long dm_phase_acc_##tu[DM_PH_SHARDS * DM_PH_SLOTS];
#define DM_PH_INIT()                                                           \
  unsigned long long _dm_acc[DM_PH_SLOTS];                                     \
  for (int _k = 0; _k < DM_PH_SLOTS; ++_k) _dm_acc[_k] = 0;                    \
  long long _dm_pt = wall_clock64()
#define DM_PH(acc, k)                                                          \
  do {                                                                         \
    const long long _n = wall_clock64();                                       \
    _dm_acc[k] += (unsigned long long)(_n - _dm_pt);                           \
    _dm_pt = _n;                                                               \
  } while (0)
#define DM_PH_COUNT(acc, k, v) do { _dm_acc[k] += (unsigned long long)(v); } while (0)
#define DM_PH_FLUSH(acc)                                                       \
  do {                                                                         \
    if (threadIdx.x == 0)                                                      \
      for (int _k = 0; _k < DM_PH_SLOTS; ++_k)                                 \
        if (_dm_acc[_k])                                                       \
          atomicAdd(&acc[(blockIdx.x % DM_PH_SHARDS) * DM_PH_SLOTS + _k], _dm_acc[_k]); \
  } while (0)
// wave-level variant (kernels whose waves run independently): lane 0 of
// every wave flushes its own accumulators
#define DM_PHW_FLUSH(acc)                                                      \
  do {                                                                         \
    if (__lane_id() == 0)                                                      \
      for (int _k = 0; _k < DM_PH_SLOTS; ++_k)                                 \
        if (_dm_acc[_k])                                                       \
          atomicAdd(&acc[((blockIdx.x * 4 + (threadIdx.x >> 6)) % DM_PH_SHARDS) * DM_PH_SLOTS + _k], _dm_acc[_k]); \
  } while (0)
#define DM_PH_READER(tu)                                                       \
  extern "C" int dm_debug_phases_##tu(unsigned long long* out, int n, int reset) { \
    static unsigned long long h[DM_PH_SHARDS * DM_PH_SLOTS];                   \
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(dm_phase_acc_##tu), sizeof h) != hipSuccess) return -3; \
    for (int k = 0; k < n && k < DM_PH_SLOTS; ++k) {                           \
      out[k] = 0;                                                              \
      for (int s = 0; s < DM_PH_SHARDS; ++s) out[k] += h[s * DM_PH_SLOTS + k]; \
    }                                                                          \
    if (reset) {                                                               \
      for (auto& v : h) v = 0;                                                 \
      if (hipMemcpyToSymbol(HIP_SYMBOL(dm_phase_acc_##tu), h, sizeof h) != hipSuccess) return -3; \
    }                                                                          \
    return 0;                                                                  \
  }
// Per-workgroup timeline of the last launch of a kernel (DM_TL_*): thread 0
// of workgroup b < DM_TL_MAX stores {start tick, end tick, XCC id << 32 |
// HW_ID, user word} (wall clock, 100 MHz); read with dm_debug_timeline_<tu>().
#define DM_TL_MAX 65536
#define DM_TL_DECL(tu) __device__ unsigned long long dm_tl_##tu[DM_TL_MAX * 4];
#define DM_TL_BEGIN() const long long _dm_tl0 = wall_clock64()
#define DM_TL_END(tu, word)                                                    \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < DM_TL_MAX) {                          \
      const unsigned long long _hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)); \
      const unsigned long long _xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xFu; \
      unsigned long long* _r = dm_tl_##tu + 4 * (unsigned long long)blockIdx.x; \
      _r[0] = (unsigned long long)_dm_tl0;                                     \
      _r[1] = (unsigned long long)wall_clock64();                              \
      _r[2] = (_xcc << 32) | _hw;                                              \
      _r[3] = (unsigned long long)(word);                                      \
    }                                                                          \
  } while (0)
#define DM_TL_READER(tu)                                                       \
  extern "C" int dm_debug_timeline_##tu(unsigned long long* out, int n_wg) {   \
    if (n_wg > DM_TL_MAX) n_wg = DM_TL_MAX;                                    \
    if (hipDeviceSynchronize() != hipSuccess) return -3;                       \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dm_tl_##tu), sizeof(unsigned long long) * 4 * (size_t)n_wg) != hipSuccess) \
      return -3;                                                               \
    return 0;                                                                  \
  }
#else
#define DM_TL_DECL(tu)
#define DM_TL_BEGIN() do {} while (0)
#define DM_TL_END(tu, word) do {} while (0)
#define DM_TL_READER(tu)
#define DM_PH_DECL(tu)
#define DM_PH_INIT() do {} while (0)
#define DM_PH(acc, k) do {} while (0)
#define DM_PH_COUNT(acc, k, v) do {} while (0)
#define DM_PH_FLUSH(acc) do {} while (0)
#define DM_PHW_FLUSH(acc) do {} while (0)
#define DM_PH_READER(tu)
#endif
