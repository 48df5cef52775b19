// fetch_probe.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access shapes libdm's kernels use (MI355X_MICROARCH.md
// §HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
// streaming read (16 B/lane) ... Other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//
// Each kernel moves a KNOWN number of bytes over 1 GiB buffers (4x the 256
// MiB Infinity Cache, so nothing is served on-die between passes) in one
// shape; run it under rocprofv3 --pmc FETCH_SIZE and, separately, WRITE_SIZE
// (tools/fetch_calib.sh), then tools/fetch_calib.py divides the known bytes
// by the counters: the per-shape factors bench.py applies per kernel.
// The known bytes of every kernel are printed as one JSON line.
//
//   probe_ld16     coalesced float4 loads (16 B/lane)                 read N
//   probe_ld8      coalesced u64 loads (8 B/lane)                     read N
//   probe_ld4      coalesced u32 loads (4 B/lane)                     read N
//   probe_bits     k_frontier_bits' shape: one wave per listed 64x64
//                  tile, lane y loads the tile's free and unknown rows
//                  (two u64 per lane = 1 KiB per tile), every 3rd tile  read tiles * 1 KiB
//   probe_accum    k_tile_accum's apply shape: per 64x64 tile, 64 rows of
//                  f32 L (float4 per lane) and int8 state (char4 per
//                  lane) loaded, then stored                            read = write = tiles * 20 KiB
//   probe_atomic   global no-return atomicAdd u32, 256 contiguous bytes
//                  per wave instruction (k_tile_accum's heavy-slab adds)  RMW N
//   probe_st16     coalesced float4 stores                             write N
//   probe_st4      coalesced u32 stores                                write N
//   probe_line16   one 16-B load per 128-B line (scattered pieces)      lines * 128 B touched
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

constexpr size_t kBytes = 1ull << 30;  // per buffer

__global__ void probe_ld16(const float4* __restrict__ a, size_t n, float* __restrict__ sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) sink[0] = s;
}

__global__ void probe_ld8(const uint64_t* __restrict__ a, size_t n, uint64_t* __restrict__ sink) {
  uint64_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s ^= a[i];
  if (s == 0x1234567ull) sink[0] = s;
}

__global__ void probe_ld4(const uint32_t* __restrict__ a, size_t n, uint32_t* __restrict__ sink) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s ^= a[i];
  if (s == 0x1234567u) sink[0] = s;
}

// one wave per listed tile; a tile's 1 KiB record = 64 free words, then 64
// unknown words (the fmask layout, dm_internal.h); tiles listed: every 3rd
__global__ void probe_bits(const uint64_t* __restrict__ rec, int64_t ntiles, uint64_t* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  uint64_t s = 0;
  for (int64_t t = wave; t * 3 < ntiles; t += waves) {
    const uint64_t* r = rec + (t * 3) * 128;
    s ^= r[lane] & ~r[64 + lane];
  }
  if (s == 0x1234567ull) sink[0] = s;
}

// 256 threads per tile: thread t owns row t / 4 ... as k_tile_accum's apply:
// 16 lanes span a 256-B row of L (float4 each) and its 64-B row of state
// (char4 each); 4 row groups of 16 rows per 256-thread pass
__global__ void probe_accum(float* __restrict__ L, char4* __restrict__ st, int64_t ntiles, int64_t W) {
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16
  const int64_t TX = W / 64;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t x0 = (t % TX) * 64, y0 = (t / TX) * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int64_t y = y0 + g * 16 + ty;
      float4* lp = reinterpret_cast<float4*>(L + y * W + x0) + tx;
      char4* sp = st + (y * W + x0) / 4 + tx;
      float4 v = *lp;
      char4 c = *sp;
      v.x += 1.f; v.y += 1.f; v.z += 1.f; v.w += 1.f;
      c.x ^= 1; c.y ^= 1; c.z ^= 1; c.w ^= 1;
      *lp = v;
      *sp = c;
    }
  }
}

__global__ void probe_atomic(uint32_t* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __hip_atomic_fetch_add(a + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void probe_st16(float4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

__global__ void probe_st4(uint32_t* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

__global__ void probe_line16(const float4* __restrict__ a, size_t lines, float* __restrict__ sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i * 8];  // 128-B stride
    s += v.x;
  }
  if (s == 12345.f) sink[0] = s;
}

int main() {
  void *a = nullptr, *b = nullptr, *sink = nullptr;
  CHECK(hipMalloc(&a, kBytes));
  CHECK(hipMalloc(&b, kBytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(a, 1, kBytes));
  CHECK(hipMemset(b, 0, kBytes));
  CHECK(hipDeviceSynchronize());
  const dim3 grid(8192), blk(256);
  // the accumulate shape: a 16384-wide f32 map of kBytes (16384 rows) and its
  // int8 state (in b), every tile of the first 4096 rows
  const int64_t W = 16384, rows = 4096, ntiles = (W / 64) * (rows / 64);
  const int64_t bits_tiles = (int64_t)(kBytes / 1024);
  hipLaunchKernelGGL(probe_ld16, grid, blk, 0, 0, (const float4*)a, kBytes / 16, (float*)sink);
  hipLaunchKernelGGL(probe_ld8, grid, blk, 0, 0, (const uint64_t*)a, kBytes / 8, (uint64_t*)sink);
  hipLaunchKernelGGL(probe_ld4, grid, blk, 0, 0, (const uint32_t*)a, kBytes / 4, (uint32_t*)sink);
  hipLaunchKernelGGL(probe_bits, grid, blk, 0, 0, (const uint64_t*)a, bits_tiles, (uint64_t*)sink);
  hipLaunchKernelGGL(probe_accum, grid, blk, 0, 0, (float*)a, (char4*)b, ntiles, W);
  hipLaunchKernelGGL(probe_atomic, grid, blk, 0, 0, (uint32_t*)b, kBytes / 4);
  hipLaunchKernelGGL(probe_st16, grid, blk, 0, 0, (float4*)b, kBytes / 16);
  hipLaunchKernelGGL(probe_st4, grid, blk, 0, 0, (uint32_t*)a, kBytes / 4);
  hipLaunchKernelGGL(probe_line16, grid, blk, 0, 0, (const float4*)b, kBytes / 128, (float*)sink);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  const double G = (double)kBytes;
  const double accum = (double)ntiles * (64.0 * 256.0 + 64.0 * 64.0);
  printf("{\"probe_ld16\": {\"read\": %.0f, \"write\": 0}, \"probe_ld8\": {\"read\": %.0f, \"write\": 0}, "
         "\"probe_ld4\": {\"read\": %.0f, \"write\": 0}, \"probe_bits\": {\"read\": %.0f, \"write\": 0}, "
         "\"probe_accum\": {\"read\": %.0f, \"write\": %.0f}, \"probe_atomic\": {\"read\": %.0f, \"write\": %.0f}, "
         "\"probe_st16\": {\"read\": 0, \"write\": %.0f}, \"probe_st4\": {\"read\": 0, \"write\": %.0f}, "
         "\"probe_line16\": {\"read\": %.0f, \"write\": 0}}\n",
         G, G, G, (double)((bits_tiles + 2) / 3) * 1024.0, accum, accum, G, G, G, G, G);
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(sink));
  return 0;
}
