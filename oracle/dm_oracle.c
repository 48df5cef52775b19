/*
 * dm_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the hot-path
 * SPEC used as the parity checker by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in the
 * product (libdm.so, the dm Python package) links, loads or calls this.
 *
 * PARITY STATUS: the reference contains no implementation of this path
 * (the grid is built by the un-vendored third-party slam_toolbox,
 * frontiers exist nowhere).  This restatement follows, from the reference:
 *   - the LaserScan encoding of the LD06 driver (ToLaserscanMessagePublish,
 *     ldlidar_stl_ros2_node @0x7f853: angle_i = angle_min + i*angle_increment,
 *     NaN = no return, range_min 0.02f at rodata 0xbc840);
 *   - resolution 0.05 / max_laser_range 12.0 (slam_config.yaml:26-27);
 *   - the OccupancyGrid int8 row-major -1/0/100 encoding with origin at the
 *     bottom-left cell (server/thymio_project/thymio_project/main.py:251-266).
 * The grid arithmetic itself is "parity unpinned" against the reference and
 * pinned by this build's SPEC plus a second, independent
 * NumPy/scipy restatement (oracle/np_oracle.py) that must agree bit for bit.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; glibc cos/sin).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dm.h"

/* ------------------------------------------------------------------ a4 --- */
/* Endpoint cells of every beam.  out_cells: [S*N][4] int64 (sx, sy, ex, ey);
 * out_flags: [S*N] bit0 = valid, bit1 = hit.  SPEC a4. */
int or_endpoints(const dm_params* p, int32_t S, const double* poses, int32_t N,
                 const float* ranges, float angle_min, float angle_increment,
                 int64_t* out_cells, uint8_t* out_flags) {
  double* cphi = (double*)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
  double* sphi = (double*)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
  if (!cphi || !sphi) { free(cphi); free(sphi); return -4; }
  for (int32_t i = 0; i < N; ++i) {
    /* phi_i = (double)angle_min + (double)i * (double)angle_increment */
    double phi = (double)angle_min + (double)i * (double)angle_increment;
    cphi[i] = cos(phi);
    sphi[i] = sin(phi);
  }
  for (int32_t s = 0; s < S; ++s) {
    double x = poses[3 * s + 0], y = poses[3 * s + 1], yaw = poses[3 * s + 2];
    double cy = cos(yaw), sy = sin(yaw);
    int pose_ok = isfinite(x) && isfinite(y) && isfinite(yaw);
    for (int32_t i = 0; i < N; ++i) {
      size_t b = (size_t)s * (size_t)N + (size_t)i;
      int64_t* c = out_cells + 4 * b;
      c[0] = c[1] = c[2] = c[3] = 0;
      out_flags[b] = 0;
      float r = ranges[b];
      if (!pose_ok) continue;
      if (!(r >= p->range_min)) continue; /* NaN or too short: skipped */
      int hit = (r <= p->range_max);
      double rr = hit ? (double)r : (double)p->range_max;
      /* rotate the beam direction by the scan yaw: two products then a sum,
       * each rounded (no FMA) */
      double a1 = cy * cphi[i];
      double a2 = sy * sphi[i];
      double dcx = a1 - a2;
      double b1 = sy * cphi[i];
      double b2 = cy * sphi[i];
      double dcy = b1 + b2;
      double t1 = rr * dcx;
      double ex = x + t1;
      double t2 = rr * dcy;
      double ey = y + t2;
      double fsx = floor((x - p->origin_x) / p->resolution);
      double fsy = floor((y - p->origin_y) / p->resolution);
      double fex = floor((ex - p->origin_x) / p->resolution);
      double fey = floor((ey - p->origin_y) / p->resolution);
      const double lim = 1073741824.0; /* 2^30: beyond that the beam is dropped */
      if (!(fabs(fsx) < lim && fabs(fsy) < lim && fabs(fex) < lim && fabs(fey) < lim))
        continue;
      c[0] = (int64_t)fsx; c[1] = (int64_t)fsy; c[2] = (int64_t)fex; c[3] = (int64_t)fey;
      out_flags[b] = (uint8_t)(1u | (hit ? 2u : 0u));
    }
  }
  free(cphi);
  free(sphi);
  return 0;
}

/* ------------------------------------------------------------------ a5 --- */
/* Cell k (0..n) of the closed-form Bresenham line from (sx,sy) to (ex,ey). */
static void or_line_cell(int64_t sx, int64_t sy, int64_t ex, int64_t ey, int64_t k,
                         int64_t* cx, int64_t* cy) {
  int64_t dx = ex - sx, dy = ey - sy;
  int64_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
  int64_t ix = dx > 0 ? 1 : (dx < 0 ? -1 : 0);
  int64_t iy = dy > 0 ? 1 : (dy < 0 ? -1 : 0);
  if (adx == 0 && ady == 0) { *cx = sx; *cy = sy; return; }
  if (adx >= ady) {
    *cx = sx + k * ix;
    *cy = sy + iy * ((2 * k * ady + adx) / (2 * adx));
  } else {
    *cy = sy + k * iy;
    *cx = sx + ix * ((2 * k * adx + ady) / (2 * ady));
  }
}

int64_t or_line_length(int64_t sx, int64_t sy, int64_t ex, int64_t ey) {
  int64_t adx = ex > sx ? ex - sx : sx - ex;
  int64_t ady = ey > sy ? ey - sy : sy - ey;
  return adx > ady ? adx : ady; /* n; the line has n+1 cells */
}

/* Cells of one line into out (capacity n+1): returns n+1. */
int64_t or_line_cells(int64_t sx, int64_t sy, int64_t ex, int64_t ey, int64_t* out_xy) {
  int64_t n = or_line_length(sx, sy, ex, ey);
  for (int64_t k = 0; k <= n; ++k) or_line_cell(sx, sy, ex, ey, k, out_xy + 2 * k, out_xy + 2 * k + 1);
  return n + 1;
}

/* ----------------------------------------------------------- a6 / a7 --- */
static int8_t or_state_of(const dm_params* p, float L) {
  if (L == 0.0f) return -1;
  if (L >= p->occ_thresh) return 100;
  if (L <= p->free_thresh) return 0;
  return -1;
}

static int64_t band_rows_of(const dm_params* p) {
  return p->band_rows > 0 ? p->band_rows : p->height - p->band_row0;
}

/* Integrate one call.  L and state are the band arrays [band_rows][width].
 * h/m counts are per call (uint32), applied once, then dropped.  Returns 0. */
int or_integrate(const dm_params* p, float* L, int8_t* state, int32_t S,
                 const double* poses, int32_t N, const float* ranges,
                 float angle_min, float angle_increment, uint64_t* out_U,
                 uint64_t* out_T) {
  int64_t W = p->width, H = p->height;
  int64_t r0 = p->band_row0, R = band_rows_of(p);
  size_t cells = (size_t)(W * R);
  size_t nb = (size_t)S * (size_t)N;
  int64_t* ep = (int64_t*)malloc(sizeof(int64_t) * 4 * (nb ? nb : 1));
  uint8_t* fl = (uint8_t*)malloc(nb ? nb : 1);
  uint32_t* h = (uint32_t*)calloc(cells, sizeof(uint32_t));
  uint32_t* m = (uint32_t*)calloc(cells, sizeof(uint32_t));
  size_t tcap = 1 << 16, tn = 0;
  int64_t* touched = (int64_t*)malloc(sizeof(int64_t) * tcap);
  if (!ep || !fl || !h || !m || !touched) {
    free(ep); free(fl); free(h); free(m); free(touched);
    return -4;
  }
  or_endpoints(p, S, poses, N, ranges, angle_min, angle_increment, ep, fl);
  uint64_t U = 0;
  for (size_t b = 0; b < nb; ++b) {
    if (!(fl[b] & 1)) continue;
    int hit = (fl[b] & 2) != 0;
    int64_t sx = ep[4 * b], sy = ep[4 * b + 1], ex = ep[4 * b + 2], ey = ep[4 * b + 3];
    int64_t n = or_line_length(sx, sy, ex, ey);
    for (int64_t k = 0; k <= n; ++k) {
      int64_t cx, cy;
      or_line_cell(sx, sy, ex, ey, k, &cx, &cy);
      if (cx < 0 || cx >= W || cy < 0 || cy >= H) continue;
      if (cy < r0 || cy >= r0 + R) continue;
      size_t idx = (size_t)((cy - r0) * W + cx);
      if (h[idx] == 0 && m[idx] == 0) {
        if (tn == tcap) {
          tcap *= 2;
          int64_t* nt = (int64_t*)realloc(touched, sizeof(int64_t) * tcap);
          if (!nt) { free(ep); free(fl); free(h); free(m); free(touched); return -4; }
          touched = nt;
        }
        touched[tn++] = (int64_t)idx;
      }
      if (k == n && hit) h[idx] += 1; else m[idx] += 1;
      ++U;
    }
  }
  for (size_t t = 0; t < tn; ++t) {
    size_t idx = (size_t)touched[t];
    /* SPEC a6: float32, this op order, no FMA */
    float tt = (float)h[idx] * p->l_occ;
    float uu = (float)m[idx] * p->l_free;
    float l = L[idx];
    l = l + tt;
    l = l + uu;
    if (l < p->l_min) l = p->l_min;
    if (l > p->l_max) l = p->l_max;
    L[idx] = l;
    state[idx] = or_state_of(p, l);
  }
  if (out_U) *out_U = U;
  if (out_T) *out_T = (uint64_t)tn;
  free(ep); free(fl); free(h); free(m); free(touched);
  (void)H;
  return 0;
}

/* Recompute state from L for every cell (used after loading L). */
void or_state_from_logodds(const dm_params* p, const float* L, int8_t* state, int64_t cells) {
  for (int64_t i = 0; i < cells; ++i) state[i] = or_state_of(p, L[i]);
}

/* ---------------------------------------------------------- a8 - a10 --- */
static int64_t uf_find(int64_t* par, int64_t a) {
  while (par[a] != a) {
    par[a] = par[par[a]];
    a = par[a];
  }
  return a;
}

static void uf_union(int64_t* par, int64_t a, int64_t b) {
  a = uf_find(par, a);
  b = uf_find(par, b);
  if (a == b) return;
  if (a < b) par[b] = a; else par[a] = b; /* root = min index */
}

/* Frontier mask, 8-CCL min-index labels and clusters for the band.  halo rows
 * (W bytes, may be NULL) are the global rows just outside the band.  mask and
 * labels may be NULL.  Clusters are sorted by label; clusters with
 * size < min_frontier_size are dropped.  Returns 0, or -5 if more than cap
 * clusters (n_out gets the full count). */
int or_frontiers(const dm_params* p, const int8_t* state, const int8_t* halo_before,
                 const int8_t* halo_after, uint8_t* mask, int64_t* labels,
                 dm_cluster* out, int64_t cap, int64_t* n_out) {
  int64_t W = p->width, H = p->height, r0 = p->band_row0, R = band_rows_of(p);
  size_t cells = (size_t)(W * R);
  uint8_t* F = (uint8_t*)calloc(cells ? cells : 1, 1);
  int64_t* par = (int64_t*)malloc(sizeof(int64_t) * (cells ? cells : 1));
  if (!F || !par) { free(F); free(par); return -4; }
  for (int64_t y = 0; y < R; ++y) {
    int64_t gy = r0 + y;
    for (int64_t x = 0; x < W; ++x) {
      size_t i = (size_t)(y * W + x);
      par[i] = -1;
      if (state[i] != 0) continue;
      int f = 0;
      for (int dy = -1; dy <= 1 && !f; ++dy) {
        int64_t ny = gy + dy;
        if (ny < 0 || ny >= H) continue; /* out-of-grid neighbours do not count */
        for (int dx = -1; dx <= 1; ++dx) {
          if (dx == 0 && dy == 0) continue;
          int64_t nx = x + dx;
          if (nx < 0 || nx >= W) continue;
          int8_t v;
          if (ny < r0) { if (!halo_before) continue; v = halo_before[nx]; }
          else if (ny >= r0 + R) { if (!halo_after) continue; v = halo_after[nx]; }
          else v = state[(ny - r0) * W + nx];
          if (v == -1) { f = 1; break; }
        }
      }
      F[i] = (uint8_t)f;
    }
  }
  /* raster-order union-find; root of a set = its min linear index */
  for (int64_t y = 0; y < R; ++y) {
    for (int64_t x = 0; x < W; ++x) {
      size_t i = (size_t)(y * W + x);
      if (!F[i]) continue;
      par[i] = (int64_t)i;
      static const int nbr[4][2] = {{-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
      for (int q = 0; q < 4; ++q) {
        int64_t nx = x + nbr[q][0], ny = y + nbr[q][1];
        if (nx < 0 || nx >= W || ny < 0) continue;
        size_t j = (size_t)(ny * W + nx);
        if (F[j]) uf_union(par, (int64_t)i, (int64_t)j);
      }
    }
  }
  int64_t nclu = 0;
  /* first pass: count roots (size filter needs totals) */
  int64_t* size = (int64_t*)calloc(cells ? cells : 1, sizeof(int64_t));
  if (!size) { free(F); free(par); return -4; }
  for (size_t i = 0; i < cells; ++i) if (F[i]) size[uf_find(par, (int64_t)i)] += 1;
  /* clusters in raster order of their root = sorted by label */
  int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * (cells ? cells : 1));
  if (!slot) { free(F); free(par); free(size); return -4; }
  for (size_t i = 0; i < cells; ++i) {
    slot[i] = -1;
    if (F[i] && par[i] == (int64_t)i && size[i] >= p->min_frontier_size) slot[i] = nclu++;
  }
  int64_t nw = nclu < cap ? nclu : cap;
  for (int64_t c = 0; c < nw; ++c) memset(&out[c], 0, sizeof(dm_cluster));
  for (size_t i = 0; i < cells; ++i) {
    int64_t gy = r0 + (int64_t)(i / (size_t)W), gx = (int64_t)(i % (size_t)W);
    if (mask) mask[i] = F[i];
    if (!F[i]) { if (labels) labels[i] = -1; continue; }
    int64_t root = uf_find(par, (int64_t)i);
    int64_t rl = (r0 + root / W) * W + root % W; /* global linear index */
    if (labels) labels[i] = rl;
    int64_t c = slot[root];
    if (c >= 0 && c < nw) {
      out[c].label = rl;
      out[c].size += 1;
      out[c].sum_x += gx;
      out[c].sum_y += gy;
    }
  }
  for (int64_t c = 0; c < nw; ++c) {
    double mx = (double)out[c].sum_x / (double)out[c].size;
    double my = (double)out[c].sum_y / (double)out[c].size;
    out[c].cx_m = p->origin_x + (mx + 0.5) * p->resolution;
    out[c].cy_m = p->origin_y + (my + 0.5) * p->resolution;
  }
  *n_out = nclu;
  free(F); free(par); free(size); free(slot);
  return nclu > cap ? -5 : 0;
}

/* f2: get_map_image's pixel mapping (main.py:258-266): 0->255, 100->0, else
 * 127, then flipud.  state: [R][W] -> img [R][W]. */
void or_map_image(const int8_t* state, int64_t R, int64_t W, uint8_t* img) {
  for (int64_t y = 0; y < R; ++y)
    for (int64_t x = 0; x < W; ++x) {
      int8_t v = state[y * W + x];
      uint8_t px = (v == 0) ? 255 : (v == 100 ? 0 : 127);
      img[(R - 1 - y) * W + x] = px;
    }
}

/* ------------------------------------------------------------------ a1 --- */
/* LD06 PointData -> LaserScan.ranges/intensities, restating the driver's
 * ToLaserscanMessagePublish (ldlidar_stl_ros2_node @0x7f853, x86-64 build in
 * the reference; read from the disassembly, never executed):
 *   range = (float)distance / 1000.0f                         @0x7fc54-0x7fc60
 *   distance == 0 && intensity == 0 -> range = intensity = NaN @0x7fc96-0x7fcc5
 *   angle_rad = (float)((double)deg * 3141.59 / 180000.0)      @0x7fd38-0x7fd58
 *   idx = (int)ceilf((angle_rad - angle_min) / angle_increment) @0x7fd64-0x7fd89
 *   idx >= N (or < 0) -> dropped                                @0x7fd93-0x7fdac
 *   laser_scan_dir -> idx = N - idx - 1                         @0x7fff2-0x8000d
 *   slot NaN -> range; else slot > range -> range (keep-min)    @0x80037-0x800e2
 *   intensities[idx] = intensity (every point, in order)        @0x800e6-0x8011c
 * with angle_min = 0.0f, angle_increment = (6.2831855f - 0.0f) / (float)(N - 1).
 * Slots start NaN. */
typedef struct { float angle_deg; uint16_t distance_mm; uint8_t intensity; uint8_t pad; } or_ld06_point;

void or_ld06_to_scan(const or_ld06_point* pts, int64_t n, int32_t N, int laser_scan_dir,
                     float* ranges, float* intensities) {
  const float angle_min = 0.0f, angle_max = 6.2831855f;
  const float inc = (angle_max - angle_min) / (float)(N - 1);
  for (int32_t i = 0; i < N; ++i) { ranges[i] = NAN; if (intensities) intensities[i] = NAN; }
  for (int64_t k = 0; k < n; ++k) {
    float range = (float)pts[k].distance_mm / 1000.0f;
    float inten = (float)pts[k].intensity;
    if (pts[k].distance_mm == 0 && pts[k].intensity == 0) { range = NAN; inten = NAN; }
    const float angle_rad = (float)((double)pts[k].angle_deg * 3141.59 / 180000.0);
    const float q = (angle_rad - angle_min) / inc;
    const int idx0 = (int)ceilf(q);
    if (idx0 >= N || idx0 < 0) continue;
    const int idx = laser_scan_dir ? N - idx0 - 1 : idx0;
    if (isnan(ranges[idx])) ranges[idx] = range;
    else if (ranges[idx] > range) ranges[idx] = range;
    if (intensities) intensities[idx] = inten;
  }
}
