/* TEST INFRASTRUCTURE: drives libdm's C-ABI (include/dm.h) from a plain C
 * program linked against a libdm whose HOST code is built with ASan + UBSan
 * (hipcc -Xarch_host -fsanitize=...; the device code is the product's).
 * Without a GPU it walks the argument-validation and error paths; with one
 * (tests/test_gpu_sanitized_host.py) it also runs the product calls:
 * integrate (host and async inputs), frontiers (sync, pipelined, dense
 * outputs), halos, band export + merge, checkpoint, LD06 conversion.  Exit 0
 * = every call returned what it should; the sanitizers abort on any host
 * memory / UB error. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dm.h"

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#define CHECK(call, want)                                                              \
  do {                                                                                 \
    int _rc = (call);                                                                  \
    if (_rc != (want)) {                                                               \
      fprintf(stderr, "%s:%d %s -> %d (want %d): %s\n", __FILE__, __LINE__, #call, _rc, \
              (want), dm_last_error());                                                \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

static uint64_t rng = 88172645463325252ull;
static double urand(void) {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (double)(rng >> 11) * (1.0 / 9007199254740992.0);
}

static int errors_only(void) {
  dm_params p;
  dm_grid* g = NULL;
  CHECK(dm_default_params(NULL, 10, 10), DM_ERR_INVALID_ARG);
  CHECK(dm_default_params(&p, 400, 300), DM_OK);
  CHECK(dm_create(NULL, &p, 0), DM_ERR_INVALID_ARG);
  CHECK(dm_create(&g, NULL, 0), DM_ERR_INVALID_ARG);
  p.band_row0 = 10;
  CHECK(dm_create(&g, &p, 0), DM_ERR_INVALID_ARG);
  p.band_row0 = 0;
  p.resolution = -1.0;
  CHECK(dm_create(&g, &p, 0), DM_ERR_INVALID_ARG);
  CHECK(dm_integrate(NULL, 1, NULL, 1, NULL, 0.0f, 0.1f, NULL, NULL), DM_ERR_INVALID_ARG);
  CHECK(dm_frontiers(NULL, NULL, NULL, NULL, 0, NULL), DM_ERR_INVALID_ARG);
  CHECK(dm_destroy(NULL), DM_OK);
  if (!dm_version() || !dm_last_error()) return 1;
  return 0;
}

static int product(void) {
  const int W = 400, H = 320, S = 4, N = 720;
  dm_params p;
  dm_grid* g = NULL;
  CHECK(dm_default_params(&p, W, H), DM_OK);
  CHECK(dm_create(&g, &p, 0), DM_OK);
  double poses[3 * S];
  float* ranges = (float*)malloc(sizeof(float) * S * N);
  const float inc = (float)(2.0 * M_PI / (N - 1));
  for (int batch = 0; batch < 3; ++batch) {
    for (int s = 0; s < S; ++s) {
      poses[3 * s] = (urand() - 0.5) * W * p.resolution;
      poses[3 * s + 1] = (urand() - 0.5) * H * p.resolution;
      poses[3 * s + 2] = (urand() * 2 - 1) * M_PI;
      for (int i = 0; i < N; ++i) ranges[s * N + i] = urand() < 0.05 ? NAN : (float)(urand() * 14.0);
    }
    uint64_t U = 0, T = 0;
    CHECK(dm_integrate(g, S, poses, N, ranges, 0.0f, inc, &U, &T), DM_OK);
    if (U == 0) return 2;
    CHECK(dm_integrate_async(g, S, poses, N, ranges, 0.0f, inc), DM_OK);
    CHECK(dm_synchronize(g), DM_OK);
  }
  uint8_t* mask = (uint8_t*)malloc((size_t)W * H);
  int64_t* labels = (int64_t*)malloc(sizeof(int64_t) * W * H);
  dm_cluster clu[4096];
  int64_t n = 0;
  CHECK(dm_frontiers(g, mask, labels, clu, 4096, &n), DM_OK);
  CHECK(dm_frontiers(g, NULL, NULL, NULL, 0, &n), n > 0 ? DM_ERR_CAPACITY : DM_OK);
  CHECK(dm_frontiers_begin(g), DM_OK);
  CHECK(dm_integrate_async(g, S, poses, N, ranges, 0.0f, inc), DM_OK);
  CHECK(dm_frontiers_end(g, clu, 4096, &n), DM_OK);
  int8_t* st = (int8_t*)malloc((size_t)W * H);
  float* L = (float*)malloc(sizeof(float) * W * H);
  uint8_t* img = (uint8_t*)malloc((size_t)W * H);
  CHECK(dm_get_state(g, st), DM_OK);
  CHECK(dm_get_logodds(g, L), DM_OK);
  CHECK(dm_map_image(g, img), DM_OK);
  CHECK(dm_save(g, "/tmp/dm_api_san.dmap"), DM_OK);
  CHECK(dm_load(g, "/tmp/dm_api_san.dmap"), DM_OK);
  CHECK(dm_load(g, "/nonexistent/x.dmap"), DM_ERR_IO);
  uint64_t stats[16];
  int32_t ns = 0;
  CHECK(dm_last_stats(g, stats, 16, &ns), DM_OK);
  dm_kernel_stat ks[32];
  CHECK(dm_profile_enable(g, 1), DM_OK);
  CHECK(dm_frontiers(g, NULL, NULL, clu, 4096, &n), DM_OK);
  CHECK(dm_profile_read(g, ks, 32, &ns), DM_OK);
  /* two row bands: halos, exports, merge */
  dm_params pb = p;
  pb.band_row0 = 0; pb.band_rows = 192;
  dm_grid* b0 = NULL;
  dm_grid* b1 = NULL;
  CHECK(dm_create(&b0, &pb, 0), DM_OK);
  pb.band_row0 = 192; pb.band_rows = 0;
  CHECK(dm_create(&b1, &pb, 0), DM_OK);
  CHECK(dm_set_state(b0, st), DM_OK);
  CHECK(dm_set_state(b1, st + (size_t)192 * W), DM_OK);
  int8_t *f0 = (int8_t*)malloc(W), *l0 = (int8_t*)malloc(W), *f1 = (int8_t*)malloc(W), *l1 = (int8_t*)malloc(W);
  CHECK(dm_get_edge_rows(b0, f0, l0), DM_OK);
  CHECK(dm_get_edge_rows(b1, f1, l1), DM_OK);
  CHECK(dm_set_halo(b0, NULL, f1), DM_OK);
  CHECK(dm_set_halo(b1, l0, NULL), DM_OK);
  int64_t nb = 0, ng = 0, nm = 0;
  CHECK(dm_export_bytes(b0, 4096, &nb), DM_OK);
  unsigned char* d_exp = NULL;
  if (hipMalloc((void**)&d_exp, (size_t)(2 * nb)) != hipSuccess) return 3;
  CHECK(dm_frontiers_export_device(b0, d_exp, 4096), DM_OK);
  CHECK(dm_frontiers_export_device(b1, d_exp + nb, 4096), DM_OK);
  CHECK(dm_synchronize(b0), DM_OK);
  CHECK(dm_synchronize(b1), DM_OK);
  CHECK(dm_merge_bands(b0, d_exp, 2, 4096, 1, clu, 4096, &nm), DM_OK);
  CHECK(dm_merge_bands_begin(b1, d_exp, 2, 4096, 1), DM_OK);
  CHECK(dm_merge_bands_end(b1, clu, 4096, &nm), DM_OK);
  CHECK(dm_frontiers(g, NULL, NULL, clu, 4096, &ng), DM_OK);
  if (nm != ng) {
    fprintf(stderr, "merged %lld clusters, single map %lld\n", (long long)nm, (long long)ng);
    return 4;
  }
  (void)hipFree(d_exp);
  int64_t n0 = 0, n1 = 0;
  CHECK(dm_frontiers(b0, NULL, NULL, clu, 4096, &n0), DM_OK);
  CHECK(dm_frontiers(b1, NULL, NULL, clu, 4096, &n1), DM_OK);
  int64_t *e0 = (int64_t*)malloc(sizeof(int64_t) * W), *e1 = (int64_t*)malloc(sizeof(int64_t) * W);
  CHECK(dm_get_edge_labels(b0, e0, e1), DM_OK);
  /* LD06 conversion */
  dm_ld06_point pts[450];
  int64_t off[2] = {0, 450};
  for (int i = 0; i < 450; ++i) {
    pts[i].angle_deg = (float)(i * 0.8);
    pts[i].distance_mm = (uint16_t)(urand() * 8000);
    pts[i].intensity = (uint8_t)(urand() * 255);
    pts[i].pad = 0;
  }
  float r450[450], i450[450];
  CHECK(dm_ld06_to_scans(g, 1, pts, off, 450, 1, r450, i450), DM_OK);
  double pk[2];
  CHECK(dm_atomic_peak(0, pk, 2, &ns), DM_OK);
  CHECK(dm_destroy(b0), DM_OK);
  CHECK(dm_destroy(b1), DM_OK);
  CHECK(dm_destroy(g), DM_OK);
  free(ranges); free(mask); free(labels); free(st); free(L); free(img);
  free(f0); free(l0); free(f1); free(l1); free(e0); free(e1);
  printf("api_san: product calls ok (%lld clusters)\n", (long long)n);
  return 0;
}

int main(int argc, char** argv) {
  int rc = errors_only();
  if (rc) return rc;
  if (argc > 1 && !strcmp(argv[1], "--gpu")) {
    rc = product();
    if (!rc) printf("api_san: ok\n");
    fflush(stdout);
    fflush(stderr);
    /* Every handle is destroyed and checked above.  Skip the HIP runtime's
     * own teardown: with cached graph executables (libdm's launch batching)
     * it frees device memory after ASan's device allocator was unloaded and
     * trips its CHECK (sanitizer_allocator_device.h) -- runtime code, not
     * libdm's. */
    _exit(rc);
  }
  if (!rc) printf("api_san: ok\n");
  return rc;
}
