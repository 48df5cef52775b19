// dm_ld06.hip — LD06 PointData -> LaserScan ranges on the GPU (SURVEY.md §8
// row a1, "next" item f3: device-side scan packing for many robots).
//
// Restates the LD06 driver's ToLaserscanMessagePublish (prebuilt
// ldlidar_stl_ros2_node @0x7f853 in the reference; semantics read from its
// disassembly, never executed):
//   range     = (float)distance_mm / 1000.0f            (rodata 0xbc84c)
//   distance == 0 && intensity == 0 -> range = intensity = NaN
//   angle_rad = (float)((double)deg * 3141.59 / 180000.0) (rodata 0xbc850/8)
//   idx       = (int)ceilf((angle_rad - angle_min) / angle_increment),
//               angle_min = 0.0f, angle_increment = 6.2831855f / (float)(N - 1)
//   idx >= N or < 0 -> dropped; laser_scan_dir -> idx = N - idx - 1
//   slot NaN -> range, else slot > range -> range   (keep the nearest return)
//   intensities[idx] = intensity of the LAST point that reached the slot
// Slots start NaN.  Keep-min over non-NaN returns is order-independent, so
// one workgroup per scan reduces with LDS atomicMin on the (non-negative)
// float bits; the intensity "last writer" is the max point index (atomicMax).
#include "dm_internal.h"

namespace {

constexpr uint32_t kEmpty = 0x7F800000u;  // +inf bits: no finite return yet

__global__ __launch_bounds__(256) void k_ld06_scans(const dm_ld06_point* __restrict__ pts,
                                                    const int64_t* __restrict__ offsets, int32_t N,
                                                    int dir, float* __restrict__ ranges,
                                                    float* __restrict__ intensities) {
  extern __shared__ uint32_t lds[];
  uint32_t* minbits = lds;                          // [N]
  int32_t* last = reinterpret_cast<int32_t*>(lds + N);  // [N]
  const int s = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < N; i += blockDim.x) { minbits[i] = kEmpty; last[i] = -1; }
  __syncthreads();
  const int64_t p0 = offsets[s], p1 = offsets[s + 1];
  const float inc = (6.2831855f - 0.0f) / (float)(N - 1);
  for (int64_t k = p0 + tid; k < p1; k += blockDim.x) {
    const dm_ld06_point pt = pts[k];
    float range = (float)pt.distance_mm / 1000.0f;
    const bool none = pt.distance_mm == 0 && pt.intensity == 0;
    const float angle_rad = (float)((double)pt.angle_deg * 3141.59 / 180000.0);
    const float q = (angle_rad - 0.0f) / inc;
    const float c = ceilf(q);
    // (int)ceilf: out-of-int-range or NaN angles are dropped like idx >= N
    if (!(c >= 0.0f) || !(c < (float)N)) continue;
    const int idx0 = (int)c;
    const int idx = dir ? N - idx0 - 1 : idx0;
    if (!none) atomicMin(&minbits[idx], __float_as_uint(range));
    atomicMax(&last[idx], (int32_t)(k - p0));
  }
  __syncthreads();
  for (int i = tid; i < N; i += blockDim.x) {
    const uint32_t b = minbits[i];
    ranges[(int64_t)s * N + i] = b == kEmpty ? __builtin_nanf("") : __uint_as_float(b);
    if (intensities) {
      const int32_t l = last[i];
      float v = __builtin_nanf("");
      if (l >= 0) {
        const dm_ld06_point pt = pts[p0 + l];
        if (!(pt.distance_mm == 0 && pt.intensity == 0)) v = (float)pt.intensity;
      }
      intensities[(int64_t)s * N + i] = v;
    }
  }
}

}  // namespace

int dm_launch_ld06(dm_grid* g, int32_t S, const dm_ld06_point* d_pts, const int64_t* d_offsets,
                   int32_t N, int dir, float* d_ranges, float* d_intensities) {
  if (S <= 0) return DM_OK;
  const size_t lds = (size_t)N * 8;
  KernelTimer t;
  dm_timer_begin(g, "ld06_scans", &t);
  hipLaunchKernelGGL(k_ld06_scans, dim3(S), dim3(256), lds, g->stream, d_pts, d_offsets, N, dir,
                     d_ranges, d_intensities);
  dm_timer_end(g, &t);
  DM_HIP(hipGetLastError());
  return DM_OK;
}
