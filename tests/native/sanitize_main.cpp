// TEST INFRASTRUCTURE: the CPU builds of the hot path's host-side code under
// AddressSanitizer + UndefinedBehaviorSanitizer (ASan/UBSan on
// the CPU build).  Runs the kernel emulation (emulate.cpp, built from the
// kernels' own geometry header csrc/dm_ray.h) against the C oracle
// (oracle/dm_oracle.c) on seeded scan batches — ragged maps, a row band,
// chunked beams, sensors outside the map, NaN / zero / infinite ranges — plus
// a frontier pass of the oracle with halos, and exits non-zero on any
// mismatch; the sanitizers abort on any memory or UB error.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/dm.h"

extern "C" int emu_integrate(int32_t W, int32_t R, int32_t row0, double ox, double oy, double res,
                             float range_min, float range_max, float l_occ, float l_free,
                             float l_min, float l_max, float occ_t, float free_t, float* L,
                             int8_t* state, int32_t S, const double* pose4, int32_t N,
                             const float* ranges, const double* trig, uint64_t* out_U,
                             uint64_t* out_T, uint64_t* out_segs, int32_t chunk_len);
extern "C" int or_integrate(const dm_params* p, float* L, int8_t* state, int32_t S, const double* poses,
                            int32_t N, const float* ranges, float angle_min, float angle_increment,
                            uint64_t* out_U, uint64_t* out_T);
extern "C" int or_frontiers(const dm_params* p, const int8_t* state, const int8_t* halo_before,
                            const int8_t* halo_after, uint8_t* mask, int64_t* labels, dm_cluster* out,
                            int64_t cap, int64_t* n_out);

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
double urand() {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (double)(g_rng >> 11) * (1.0 / 9007199254740992.0);
}

dm_params make(int64_t W, int64_t H, double res, int64_t r0, int64_t rows) {
  dm_params p;
  memset(&p, 0, sizeof p);
  p.width = W; p.height = H; p.resolution = res;
  p.origin_x = -0.5 * W * res; p.origin_y = -0.5 * H * res;
  p.range_min = 0.02f; p.range_max = 12.0f;
  p.l_occ = 0.85f; p.l_free = -0.4f; p.l_min = -2.0f; p.l_max = 3.5f;
  p.min_frontier_size = 1; p.band_row0 = r0; p.band_rows = rows;
  return p;
}

int run_case(int64_t W, int64_t H, double res, int64_t r0, int64_t rows, int S, int N, int chunk_len) {
  const dm_params p = make(W, H, res, r0, rows);
  const int64_t R = rows > 0 ? rows : H - r0;
  std::vector<float> Le((size_t)(R * W), 0.0f), Lo((size_t)(R * W), 0.0f);
  std::vector<int8_t> se((size_t)(R * W), -1), so((size_t)(R * W), -1);
  const float inc = (float)(2.0 * M_PI / (N - 1));
  std::vector<double> trig(2 * (size_t)N);
  for (int i = 0; i < N; ++i) {
    const double phi = 0.0 + (double)i * (double)inc;
    trig[2 * i] = cos(phi);
    trig[2 * i + 1] = sin(phi);
  }
  for (int batch = 0; batch < 2; ++batch) {
    std::vector<double> poses(3 * (size_t)S), pose4(4 * (size_t)S);
    std::vector<float> ranges((size_t)S * N);
    for (int s = 0; s < S; ++s) {
      poses[3 * s] = p.origin_x + (urand() * 1.4 - 0.2) * W * res;
      poses[3 * s + 1] = p.origin_y + (urand() * 1.4 - 0.2) * H * res;
      poses[3 * s + 2] = (urand() * 2 - 1) * M_PI;
      pose4[4 * s] = poses[3 * s];
      pose4[4 * s + 1] = poses[3 * s + 1];
      pose4[4 * s + 2] = cos(poses[3 * s + 2]);
      pose4[4 * s + 3] = sin(poses[3 * s + 2]);
      for (int i = 0; i < N; ++i) {
        const double u = urand();
        float r = (float)(round(urand() * 15.6 * 1000.0) / 1000.0);
        if (u < 0.03) r = NAN;
        else if (u < 0.04) r = 0.0f;
        else if (u < 0.05) r = INFINITY;
        ranges[(size_t)s * N + i] = r;
      }
    }
    uint64_t Ue = 0, Te = 0, G = 0, Uo = 0, To = 0;
    if (emu_integrate((int32_t)W, (int32_t)R, (int32_t)r0, p.origin_x, p.origin_y, p.resolution, p.range_min,
                      p.range_max, p.l_occ, p.l_free, p.l_min, p.l_max, p.occ_thresh, p.free_thresh, Le.data(),
                      se.data(), S, pose4.data(), N, ranges.data(), trig.data(), &Ue, &Te, &G, chunk_len) != 0)
      return 1;
    if (or_integrate(&p, Lo.data(), so.data(), S, poses.data(), N, ranges.data(), 0.0f, inc, &Uo, &To) != 0)
      return 2;
    if (Ue != Uo || Te != To) {
      fprintf(stderr, "counts differ: %llu/%llu vs %llu/%llu\n", (unsigned long long)Ue, (unsigned long long)Te,
              (unsigned long long)Uo, (unsigned long long)To);
      return 3;
    }
  }
  if (memcmp(Le.data(), Lo.data(), Le.size() * sizeof(float)) != 0 || memcmp(se.data(), so.data(), se.size()) != 0)
    return 4;
  // frontiers with halos (rows just outside the band: unknown / free stripes)
  std::vector<int8_t> hb((size_t)W), ha((size_t)W);
  for (int64_t x = 0; x < W; ++x) {
    hb[x] = (x / 7) % 2 ? -1 : 0;
    ha[x] = (x / 5) % 3 ? 0 : -1;
  }
  std::vector<uint8_t> mask((size_t)(R * W));
  std::vector<int64_t> labels((size_t)(R * W));
  std::vector<dm_cluster> out(1 << 16);
  int64_t n = 0;
  if (or_frontiers(&p, so.data(), r0 > 0 ? hb.data() : nullptr, r0 + R < H ? ha.data() : nullptr, mask.data(),
                   labels.data(), out.data(), (int64_t)out.size(), &n) != 0)
    return 5;
  printf("case %lldx%lld res %.2f band %lld+%lld S %d N %d chunk %d: ok, %lld clusters\n", (long long)W,
         (long long)H, res, (long long)r0, (long long)R, S, N, chunk_len, (long long)n);
  return 0;
}

}  // namespace

int main() {
  int rc = 0;
  rc |= run_case(257, 513, 0.05, 0, 0, 6, 700, 0);
  rc |= run_case(130, 70, 0.05, 0, 0, 5, 500, 64);
  rc |= run_case(300, 700, 0.05, 320, 192, 8, 600, 97);
  rc |= run_case(500, 500, 0.01, 128, 0, 3, 3000, 0);
  rc |= run_case(96, 96, 0.1, 0, 0, 12, 256, 0);
  return rc;
}
