// Host cost of kernel launches vs a HIP graph of the same launches (MI355X
// diagnostic for the pipelined step).  Each kernel is one
// workgroup spinning `us` microseconds on the 100 MHz wall clock.
//  (a) 14 launches per step round-robin over 3 streams (no dependencies)
//  (b) one captured graph per step: two branches of 7 kernels each (fork /
//      join by events during capture) -> does the GPU run the branches
//      side by side (step time ~ 7 x us) or one after the other (14 x us)?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_spin(unsigned long long ticks) {
  if (threadIdx.x) return;
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

struct G64 { int a[16]; };
struct R40 { int s, n; double x, y, z; float lo, hi; };
__global__ void k_many(G64 g, R40 r, const double* p0, const float* p1, const double* p2, void* p3, int* p4,
                       int* p5, unsigned long long* p6, int* p7, unsigned long long* p8, void* p9, int* p10,
                       unsigned long long* p11, int i0, int i1) {
  if (threadIdx.x == 0 && g.a[0] == 12345) *p4 = r.s + i0 + i1;
}
struct AllArgs { G64 g; R40 r; void* p[12]; int i0, i1; };
__global__ void k_one(AllArgs a) {
  if (threadIdx.x == 0 && a.g.a[0] == 12345) *(int*)a.p[4] = a.r.s + a.i0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s[3];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  const int steps = 400;
  for (unsigned long long us : {0ull, 5ull}) {
    const unsigned long long ticks = us * 100;
    // (a) plain launches
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      double t0 = now_us(), host = 0;
      for (int i = 0; i < steps; ++i) {
        double a = now_us();
        for (int k = 0; k < 14; ++k) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[k % 3], ticks);
        host += now_us() - a;
      }
      CK(hipDeviceSynchronize());
      printf("spin %llu us: 14 launches/step: host %.1f us/step, wall %.1f us/step\n", us, host / steps,
             (now_us() - t0) / steps);
    }
    // (b) graph: fork into two branches of 7 kernels, join
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, s[0]));
    CK(hipStreamWaitEvent(s[1], fork, 0));
    for (int k = 0; k < 7; ++k) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], ticks);
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[1], ticks);
    }
    CK(hipEventRecord(join, s[1]));
    CK(hipStreamWaitEvent(s[0], join, 0));
    hipGraph_t g;
    CK(hipStreamEndCapture(s[0], &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    size_t n = 0;
    CK(hipGraphGetNodes(g, nullptr, &n));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      double t0 = now_us(), host = 0;
      for (int i = 0; i < steps; ++i) {
        double a = now_us();
        CK(hipGraphLaunch(ge, s[0]));
        host += now_us() - a;
      }
      CK(hipDeviceSynchronize());
      printf("spin %llu us: graph (%zu nodes, 2 x 7 kernels): host %.1f us/launch, wall %.1f us/step\n", us, n,
             host / steps, (now_us() - t0) / steps);
    }
    // (c) the same graph, but only the single-stream chain (7 kernels)
    CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 7; ++k) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], ticks);
    hipGraph_t g2;
    CK(hipStreamEndCapture(s[0], &g2));
    hipGraphExec_t ge2;
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    CK(hipDeviceSynchronize());
    double t0 = now_us(), host = 0;
    for (int i = 0; i < steps; ++i) {
      double a = now_us();
      CK(hipGraphLaunch(ge2, s[0]));
      host += now_us() - a;
    }
    CK(hipDeviceSynchronize());
    printf("spin %llu us: chain graph (7 kernels): host %.1f us/launch, wall %.1f us/step\n", us, host / steps,
           (now_us() - t0) / steps);
    // (d) 7 plain launches on one stream
    CK(hipDeviceSynchronize());
    t0 = now_us(); host = 0;
    for (int i = 0; i < steps; ++i) {
      double a = now_us();
      for (int k = 0; k < 7; ++k) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], ticks);
      host += now_us() - a;
    }
    CK(hipDeviceSynchronize());
    printf("spin %llu us: 7 launches one stream: host %.1f us/step, wall %.1f us/step\n", us, host / steps,
           (now_us() - t0) / steps);
  }
  // argument count: 16 arguments (two structs + 12 pointers + 2 ints) vs the
  // same bytes in one struct argument
  {
    G64 g{}; R40 r{}; AllArgs aa{};
    int* d = nullptr;
    CK(hipMalloc(&d, 64));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      double host = 0;
      for (int i = 0; i < steps; ++i) {
        double a = now_us();
        for (int k = 0; k < 14; ++k)
          hipLaunchKernelGGL(k_many, dim3(64), dim3(256), 0, s[k % 3], g, r, (const double*)d, (const float*)d,
                             (const double*)d, (void*)d, d, d, (unsigned long long*)d, d, (unsigned long long*)d,
                             (void*)d, d, (unsigned long long*)d, 1, 2);
        host += now_us() - a;
      }
      CK(hipDeviceSynchronize());
      printf("16 args: host %.2f us/launch\n", host / steps / 14);
      host = 0;
      for (int i = 0; i < steps; ++i) {
        double a = now_us();
        for (int k = 0; k < 14; ++k) hipLaunchKernelGGL(k_one, dim3(64), dim3(256), 0, s[k % 3], aa);
        host += now_us() - a;
      }
      CK(hipDeviceSynchronize());
      printf("1 struct arg (same bytes): host %.2f us/launch\n", host / steps / 14);
      host = 0;
      for (int i = 0; i < steps; ++i) {
        double a = now_us();
        for (int k = 0; k < 14; ++k) hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s[k % 3], 0ull);
        host += now_us() - a;
      }
      CK(hipDeviceSynchronize());
      printf("1 scalar arg: host %.2f us/launch\n", host / steps / 14);
    }
  }
  return 0;
}
