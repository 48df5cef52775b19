/*
 * dm_oracle_mt.c — TEST / BENCH INFRASTRUCTURE ONLY.  An OpenMP restatement
 * of the same SPEC as dm_oracle.c on every
 * host core: the "strong CPU" line of bench.py's cpu_baseline (SURVEY.md
 * §8(d): "optionally a -O3 -fopenmp restatement on all host cores, clearly
 * labelled as the build's, not the reference's").  It is the build's own
 * code, not the reference's (the reference has no implementation of this
 * path), and nothing in the product links or calls it.
 * tests/test_oracle.py checks it against dm_oracle.c bit for bit.
 *
 * Integrate: beams in parallel; per-cell counts packed in one uint64 (hits in
 * the high half, misses in the low half) and added with relaxed atomics, so
 * the first adder of a cell (previous value 0) lists it as touched; then the
 * touched cells are applied in parallel (the SPEC's float32 op order, no FMA)
 * and their counters cleared.  Counts are integers, so the result does not
 * depend on the interleaving: it equals dm_oracle.c's.
 * Frontiers: mask in parallel over rows; union-find per strip of rows in
 * parallel (root = min linear index), then the strip seams united serially,
 * then every cell's root found read-only in parallel; cluster sums by atomic
 * adds at the root; clusters listed in raster order of their roots = sorted
 * by label.  Band support as dm_oracle.c (halo rows, band_row0).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dm.h"

int or_endpoints(const dm_params* p, int32_t S, const double* poses, int32_t N,
                 const float* ranges, float angle_min, float angle_increment,
                 int64_t* out_cells, uint8_t* out_flags);

typedef struct or_mt_ctx {
  int64_t cells;
  uint64_t* cnt;      /* [cells] hits << 32 | misses, zero between calls */
  int64_t** touched;  /* per thread */
  int64_t* tcap;
  int64_t* tn;
  int nthreads;
} or_mt_ctx;

static int64_t band_rows_of(const dm_params* p) {
  return p->band_rows > 0 ? p->band_rows : p->height - p->band_row0;
}

void* or_mt_create(const dm_params* p, int nthreads) {
  or_mt_ctx* c = (or_mt_ctx*)calloc(1, sizeof *c);
  if (!c) return NULL;
  c->cells = p->width * band_rows_of(p);
  c->nthreads = nthreads > 0 ? nthreads : omp_get_max_threads();
  c->cnt = (uint64_t*)calloc((size_t)c->cells, sizeof(uint64_t));
  c->touched = (int64_t**)calloc((size_t)c->nthreads, sizeof(int64_t*));
  c->tcap = (int64_t*)calloc((size_t)c->nthreads, sizeof(int64_t));
  c->tn = (int64_t*)calloc((size_t)c->nthreads, sizeof(int64_t));
  if (!c->cnt || !c->touched || !c->tcap || !c->tn) {
    free(c->cnt); free(c->touched); free(c->tcap); free(c->tn); free(c);
    return NULL;
  }
  return c;
}

void or_mt_destroy(void* h) {
  or_mt_ctx* c = (or_mt_ctx*)h;
  if (!c) return;
  for (int t = 0; t < c->nthreads; ++t) free(c->touched[t]);
  free(c->touched); free(c->tcap); free(c->tn); free(c->cnt); free(c);
}

int or_mt_threads(void* h) { return ((or_mt_ctx*)h)->nthreads; }

static inline void line_cell(int64_t sx, int64_t sy, int64_t adx, int64_t ady, int64_t ix, int64_t iy,
                             int64_t k, int64_t* cx, int64_t* cy) {
  if (adx == 0 && ady == 0) { *cx = sx; *cy = sy; return; }
  if (adx >= ady) {
    *cx = sx + k * ix;
    *cy = sy + iy * ((2 * k * ady + adx) / (2 * adx));
  } else {
    *cy = sy + k * iy;
    *cx = sx + ix * ((2 * k * adx + ady) / (2 * ady));
  }
}

static int8_t state_of(const dm_params* p, float L) {
  if (L == 0.0f) return -1;
  if (L >= p->occ_thresh) return 100;
  if (L <= p->free_thresh) return 0;
  return -1;
}

int or_mt_integrate(void* h, const dm_params* p, float* L, int8_t* state, int32_t S, const double* poses,
                    int32_t N, const float* ranges, float angle_min, float angle_increment, uint64_t* out_U,
                    uint64_t* out_T) {
  or_mt_ctx* c = (or_mt_ctx*)h;
  const int64_t W = p->width, H = p->height, r0 = p->band_row0, R = band_rows_of(p);
  const size_t nb = (size_t)S * (size_t)N;
  int64_t* ep = (int64_t*)malloc(sizeof(int64_t) * 4 * (nb ? nb : 1));
  uint8_t* fl = (uint8_t*)malloc(nb ? nb : 1);
  if (!ep || !fl) { free(ep); free(fl); return -4; }
  or_endpoints(p, S, poses, N, ranges, angle_min, angle_increment, ep, fl);
  uint64_t U = 0;
  int oom = 0;
  memset(c->tn, 0, sizeof(int64_t) * (size_t)c->nthreads);
#pragma omp parallel num_threads(c->nthreads) reduction(+ : U)
  {
    const int t = omp_get_thread_num();
#pragma omp for schedule(dynamic, 64)
    for (int64_t b = 0; b < (int64_t)nb; ++b) {
      if (!(fl[b] & 1)) continue;
      const int hit = (fl[b] & 2) != 0;
      const int64_t sx = ep[4 * b], sy = ep[4 * b + 1], ex = ep[4 * b + 2], ey = ep[4 * b + 3];
      const int64_t dx = ex - sx, dy = ey - sy;
      const int64_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
      const int64_t ix = dx > 0 ? 1 : (dx < 0 ? -1 : 0), iy = dy > 0 ? 1 : (dy < 0 ? -1 : 0);
      const int64_t n = adx > ady ? adx : ady;
      for (int64_t k = 0; k <= n; ++k) {
        int64_t cx, cy;
        line_cell(sx, sy, adx, ady, ix, iy, k, &cx, &cy);
        if (cx < 0 || cx >= W || cy < 0 || cy >= H || cy < r0 || cy >= r0 + R) continue;
        const int64_t idx = (cy - r0) * W + cx;
        const uint64_t add = (k == n && hit) ? (1ull << 32) : 1ull;
        const uint64_t prev = __atomic_fetch_add(&c->cnt[idx], add, __ATOMIC_RELAXED);
        if (prev == 0) {
          if (c->tn[t] == c->tcap[t]) {
            const int64_t nc = c->tcap[t] ? 2 * c->tcap[t] : 4096;
            int64_t* nt = (int64_t*)realloc(c->touched[t], sizeof(int64_t) * (size_t)nc);
            if (!nt) { oom = 1; continue; }
            c->touched[t] = nt;
            c->tcap[t] = nc;
          }
          c->touched[t][c->tn[t]++] = idx;
        }
        ++U;
      }
    }
  }
  free(ep);
  free(fl);
  if (oom) return -4;
  uint64_t T = 0;
#pragma omp parallel num_threads(c->nthreads) reduction(+ : T)
  {
    for (int t = 0; t < c->nthreads; ++t) {
      const int64_t* lst = c->touched[t];
#pragma omp for schedule(static) nowait
      for (int64_t i = 0; i < c->tn[t]; ++i) {
        const int64_t idx = lst[i];
        const uint64_t v = c->cnt[idx];
        c->cnt[idx] = 0;
        /* SPEC a6: float32, this op order, no FMA (-ffp-contract=off) */
        const float tt = (float)(uint32_t)(v >> 32) * p->l_occ;
        const float uu = (float)(uint32_t)(v & 0xffffffffu) * p->l_free;
        float l = L[idx];
        l = l + tt;
        l = l + uu;
        if (l < p->l_min) l = p->l_min;
        if (l > p->l_max) l = p->l_max;
        L[idx] = l;
        state[idx] = state_of(p, l);
        ++T;
      }
    }
  }
  if (out_U) *out_U = U;
  if (out_T) *out_T = T;
  return 0;
}

/* ---------------------------------------------------------------- frontiers */
static int64_t find_ro(const int64_t* par, int64_t a) {
  while (par[a] != a) a = par[a];
  return a;
}

static int64_t find_halve(int64_t* par, int64_t a) {
  while (par[a] != a) {
    par[a] = par[par[a]];
    a = par[a];
  }
  return a;
}

static void unite(int64_t* par, int64_t a, int64_t b) {
  a = find_halve(par, a);
  b = find_halve(par, b);
  if (a == b) return;
  if (a < b) par[b] = a; else par[a] = b;
}

/* Same contract as or_frontiers (dm_oracle.c): mask / labels may be NULL;
 * clusters sorted by label, size filter; -5 if more than cap. */
int or_mt_frontiers(void* h, const dm_params* p, const int8_t* state, const int8_t* halo_before,
                    const int8_t* halo_after, uint8_t* mask, int64_t* labels, dm_cluster* out, int64_t cap,
                    int64_t* n_out) {
  or_mt_ctx* c = (or_mt_ctx*)h;
  const int nt = c->nthreads;
  const int64_t W = p->width, H = p->height, r0 = p->band_row0, R = band_rows_of(p);
  const int64_t cells = W * R;
  uint8_t* F = (uint8_t*)malloc((size_t)(cells ? cells : 1));
  int64_t* par = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cells ? cells : 1));
  if (!F || !par) { free(F); free(par); return -4; }
#pragma omp parallel for num_threads(nt) schedule(dynamic, 16)
  for (int64_t y = 0; y < R; ++y) {
    const int64_t gy = r0 + y;
    for (int64_t x = 0; x < W; ++x) {
      const int64_t i = y * W + x;
      par[i] = -1;
      int f = 0;
      if (state[i] == 0) {
        for (int dy = -1; dy <= 1 && !f; ++dy) {
          const int64_t ny = gy + dy;
          if (ny < 0 || ny >= H) continue;
          for (int dx = -1; dx <= 1; ++dx) {
            if (dx == 0 && dy == 0) continue;
            const int64_t nx = x + dx;
            if (nx < 0 || nx >= W) continue;
            int8_t v;
            if (ny < r0) { if (!halo_before) continue; v = halo_before[nx]; }
            else if (ny >= r0 + R) { if (!halo_after) continue; v = halo_after[nx]; }
            else v = state[(ny - r0) * W + nx];
            if (v == -1) { f = 1; break; }
          }
        }
      }
      F[i] = (uint8_t)f;
    }
  }
  /* union-find per strip of rows (unions stay inside the strip), then seams */
  const int64_t strips = nt * 4 < R ? nt * 4 : (R > 0 ? R : 1);
  const int64_t per = (R + strips - 1) / strips;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
  for (int64_t s = 0; s < strips; ++s) {
    const int64_t ya = s * per, yb = (s + 1) * per < R ? (s + 1) * per : R;
    for (int64_t y = ya; y < yb; ++y)
      for (int64_t x = 0; x < W; ++x) {
        const int64_t i = y * W + x;
        if (!F[i]) continue;
        par[i] = i;
        static const int nbr[4][2] = {{-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
        for (int q = 0; q < 4; ++q) {
          const int64_t nx = x + nbr[q][0], ny = y + nbr[q][1];
          if (nx < 0 || nx >= W || ny < ya) continue;
          const int64_t j = ny * W + nx;
          if (F[j]) unite(par, i, j);
        }
      }
  }
  for (int64_t s = 1; s < strips; ++s) {
    const int64_t y = s * per;
    if (y >= R) break;
    for (int64_t x = 0; x < W; ++x) {
      const int64_t i = y * W + x;
      if (!F[i]) continue;
      for (int64_t dx = -1; dx <= 1; ++dx) {
        const int64_t nx = x + dx;
        if (nx < 0 || nx >= W) continue;
        const int64_t j = (y - 1) * W + nx;
        if (F[j]) unite(par, i, j);
      }
    }
  }
  /* roots (read-only finds), sizes and sums at the roots */
  int64_t* acc = (int64_t*)calloc((size_t)(cells ? cells : 1) * 3, sizeof(int64_t));
  if (!acc) { free(F); free(par); return -4; }
#pragma omp parallel for num_threads(nt) schedule(dynamic, 16)
  for (int64_t y = 0; y < R; ++y)
    for (int64_t x = 0; x < W; ++x) {
      const int64_t i = y * W + x;
      if (!F[i]) continue;
      const int64_t rt = find_ro(par, i);
      __atomic_fetch_add(&acc[3 * rt], 1, __ATOMIC_RELAXED);
      __atomic_fetch_add(&acc[3 * rt + 1], x, __ATOMIC_RELAXED);
      __atomic_fetch_add(&acc[3 * rt + 2], r0 + y, __ATOMIC_RELAXED);
    }
  /* clusters in raster order of the roots: per-strip counts, then offsets */
  int64_t* cnt = (int64_t*)calloc((size_t)strips + 1, sizeof(int64_t));
  if (!cnt) { free(F); free(par); free(acc); return -4; }
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
  for (int64_t s = 0; s < strips; ++s) {
    const int64_t a = s * per * W, b = ((s + 1) * per < R ? (s + 1) * per : R) * W;
    int64_t k = 0;
    for (int64_t i = a; i < b; ++i)
      if (F[i] && par[i] == i && acc[3 * i] >= p->min_frontier_size) ++k;
    cnt[s + 1] = k;
  }
  for (int64_t s = 0; s < strips; ++s) cnt[s + 1] += cnt[s];
  const int64_t nclu = cnt[strips];
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
  for (int64_t s = 0; s < strips; ++s) {
    const int64_t a = s * per * W, b = ((s + 1) * per < R ? (s + 1) * per : R) * W;
    int64_t k = cnt[s];
    for (int64_t i = a; i < b; ++i) {
      if (!(F[i] && par[i] == i && acc[3 * i] >= p->min_frontier_size)) continue;
      if (k < cap) {
        dm_cluster* o = &out[k];
        o->label = (r0 + i / W) * W + i % W;
        o->size = acc[3 * i];
        o->sum_x = acc[3 * i + 1];
        o->sum_y = acc[3 * i + 2];
        const double mx = (double)o->sum_x / (double)o->size;
        const double my = (double)o->sum_y / (double)o->size;
        o->cx_m = p->origin_x + (mx + 0.5) * p->resolution;
        o->cy_m = p->origin_y + (my + 0.5) * p->resolution;
      }
      ++k;
    }
  }
  if (mask || labels) {
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < cells; ++i) {
      if (mask) mask[i] = F[i];
      if (labels) {
        if (!F[i]) { labels[i] = -1; continue; }
        const int64_t rt = find_ro(par, i);
        labels[i] = (r0 + rt / W) * W + rt % W;
      }
    }
  }
  *n_out = nclu;
  free(F); free(par); free(acc); free(cnt);
  return nclu > cap ? -5 : 0;
}
