// dm_probe.hip — in-harness atomic-throughput peaks.
//
// The north star asks for the raycast's atomic throughput against MI355X
// peak; no vendor figure exists for integer atomics, so the peak is measured
// here, on the device the bench runs on, with the two atomic forms the hot
// path issues:
//   k_peak_lds     ds_add_u32, every lane its own bank (uncontended, no
//                  return) — k_tile_accum's per-cell count adds
//   k_peak_global  global_atomic_add_u32, no return, 256 contiguous bytes per
//                  wave instruction (the full-rate shape, MI355X_MICROARCH.md
//                  §Global float atomics), rows spread over a 256 MiB buffer —
//                  the heavy tiles' slab adds
// Each kernel runs long enough (milliseconds) that the launch overhead is
// noise; rates are operations per second over the whole chip.
#include "dm_internal.h"

namespace {

constexpr int kProbeThreads = 256;
constexpr int kLdsIters = 4096;   // x16 adds per thread
constexpr int kGlobIters = 256;   // x4 wave instructions per wave

__global__ __launch_bounds__(kProbeThreads) void k_peak_lds(uint32_t* __restrict__ out, uint32_t seed) {
  __shared__ uint32_t s[16 * kProbeThreads];
  const int tid = threadIdx.x;
  for (int e = tid; e < 16 * kProbeThreads; e += kProbeThreads) s[e] = 0u;
  __syncthreads();
  // lane l of a wave adds to word (k * 256 + tid): consecutive words, one
  // per bank, so no two lanes of a wave-instruction's group share a bank
  const uint32_t v = seed | 1u;
  for (int it = 0; it < kLdsIters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) __hip_atomic_fetch_add(&s[k * kProbeThreads + tid], v, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  uint32_t acc = 0u;
  for (int k = 0; k < 16; ++k) acc += s[k * kProbeThreads + tid];
  out[(int64_t)blockIdx.x * kProbeThreads + tid] = acc;  // keeps the adds live
}

__global__ __launch_bounds__(kProbeThreads) void k_peak_global(uint32_t* __restrict__ buf, int64_t rows,
                                                                uint32_t seed) {
  // row = 64 words (256 B); each wave instruction adds to one whole row
  const int lane = __lane_id();
  const int64_t wave = (int64_t)blockIdx.x * (kProbeThreads / 64) + (threadIdx.x >> 6);
  uint64_t h = (uint64_t)(wave + 1) * 0x9E3779B97F4A7C15ull ^ seed;
  for (int it = 0; it < kGlobIters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h = h * 6364136223846793005ull + 1442695040888963407ull;
      const int64_t row = (int64_t)((h >> 24) % (uint64_t)rows);
      atomicAdd(&buf[row * 64 + lane], 1u);
    }
  }
}

}  // namespace

extern "C" int dm_atomic_peak(int device, double* out, int32_t cap, int32_t* n_out) {
  if (cap > 0 && !out) return dm_set_error(DM_ERR_INVALID_ARG, "out is NULL");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return dm_set_error(DM_ERR_INVALID_ARG, "device %d not available", device);
  DM_HIP(hipSetDevice(device));
  int ncu = 256;
  DM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
  const int64_t blocks = 8 * (int64_t)ncu;  // 8 resident 256-thread workgroups per CU
  const int64_t rows = (256ll << 20) / 256;  // 256 MiB of 256-B rows
  uint32_t* lds_out = nullptr;
  uint32_t* buf = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double v[2] = {0.0, 0.0};
  auto cleanup = [&]() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (lds_out) (void)hipFree(lds_out);
    if (buf) (void)hipFree(buf);
  };
  hipError_t e = hipMalloc((void**)&lds_out, sizeof(uint32_t) * (size_t)(blocks * kProbeThreads));
  if (e == hipSuccess) e = hipMalloc((void**)&buf, sizeof(uint32_t) * (size_t)(rows * 64));
  if (e == hipSuccess) e = hipMemset(buf, 0, sizeof(uint32_t) * (size_t)(rows * 64));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  for (int pass = 0; pass < 2 && e == hipSuccess; ++pass) {  // pass 0 warms up
    float ms = 0.0f;
    hipLaunchKernelGGL(k_peak_lds, dim3((unsigned)blocks), dim3(kProbeThreads), 0, st, lds_out, 7u + pass);
    e = hipEventRecord(e0, st);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_peak_lds, dim3((unsigned)blocks), dim3(kProbeThreads), 0, st, lds_out, 11u + pass);
      e = hipEventRecord(e1, st);
    }
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && ms > 0.0f)
      v[0] = (double)blocks * kProbeThreads * kLdsIters * 16.0 / (ms * 1e-3);
    hipLaunchKernelGGL(k_peak_global, dim3((unsigned)blocks), dim3(kProbeThreads), 0, st, buf, rows, 3u + pass);
    if (e == hipSuccess) e = hipEventRecord(e0, st);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_peak_global, dim3((unsigned)blocks), dim3(kProbeThreads), 0, st, buf, rows,
                         5u + pass);
      e = hipEventRecord(e1, st);
    }
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && ms > 0.0f)
      v[1] = (double)blocks * kProbeThreads * kGlobIters * 4.0 / (ms * 1e-3);
  }
  if (e == hipSuccess) e = hipGetLastError();
  cleanup();
  if (e != hipSuccess) return dm_hip_check(e, "dm_atomic_peak");
  for (int32_t i = 0; i < cap && i < 2; ++i) out[i] = v[i];
  if (n_out) *n_out = 2;
  return DM_OK;
}
