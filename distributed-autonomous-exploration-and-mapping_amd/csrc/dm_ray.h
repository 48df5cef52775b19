// dm_ray.h — per-beam geometry shared by the HIP kernels (dm_integrate.hip)
// and the host-side emulation used by the CPU tests (tests/native/).
//
// SPEC a4 (endpoint cells) and a5 (closed-form Bresenham) of SURVEY.md §8(a),
// restated in DESIGN.md §2; compiled with -ffp-contract=off everywhere.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define DM_HD __host__ __device__
#else
#define DM_HD
#endif

#define DM_TS 64  // tile edge; == DM_TILE of include/dm.h

// Bresenham parameters of one beam, in global cell coordinates.  The line is
// parametrised along its major axis: cell k (0..n) has
//   major = sa + k*ia,  minor = sb + ib * floor((2*k*adb + n) / (2*n))
// (n = |d major| > 0), or just (sa, sb) for n == 0.
struct Beam {
  int32_t sa, sb;   // start cell, major / minor axis
  int32_t n, adb;   // |d major|, |d minor|
  int8_t ia, ib;    // unit steps along major / minor
  uint8_t xmajor;   // 1 if major axis is x
  uint8_t flags;    // bit0 valid, bit1 hit
  int32_t pad;
  double rden;      // 1.0 / (2n), 0 for n == 0
};
static_assert(sizeof(Beam) == 32, "Beam layout");

struct RayGeom {
  int32_t W, R, row0, TX, TY;
};

struct RayArgs {
  int32_t S, N;
  double ox, oy, res;
  float range_min, range_max;
};

DM_HD inline int32_t dm_floordiv32(int32_t a, int32_t b) {
  int32_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// floor(num / den) for 0 <= num < 2^31, den > 0, rden = 1.0/den: a double
// estimate, then one exact integer correction.
DM_HD inline int32_t dm_udiv(int32_t num, int32_t den, double rden) {
  int32_t q = (int32_t)((double)num * rden);
  if ((int64_t)(q + 1) * den <= num) ++q;
  else if ((int64_t)q * den > num) --q;
  return q;
}

// minor-axis step count of cell k
DM_HD inline int32_t dm_minor_steps(const Beam& b, int32_t k) {
  return b.n > 0 ? dm_udiv(2 * k * b.adb + b.n, 2 * b.n, b.rden) : 0;
}

// SPEC a4: endpoint cells of beam (s, i).  Double precision, every product
// rounded separately, C-library cos/sin of the beam angle table (trig) and of
// the scan yaw (pose4[2..3]) computed on the host.
DM_HD inline Beam dm_make_beam(const RayArgs& a, const double* pose4, const float* ranges,
                               const double* trig, int32_t s, int32_t i) {
  Beam bm;
  bm.sa = bm.sb = bm.n = bm.adb = 0;
  bm.ia = bm.ib = 0;
  bm.xmajor = 1;
  bm.flags = 0;
  bm.pad = 0;
  bm.rden = 0.0;
  const double x = pose4[4 * s + 0], y = pose4[4 * s + 1];
  const double cyaw = pose4[4 * s + 2], syaw = pose4[4 * s + 3];
  const float r = ranges[(int64_t)s * a.N + i];
  if (!(isfinite(x) && isfinite(y) && isfinite(cyaw) && isfinite(syaw))) return bm;
  if (!(r >= a.range_min)) return bm;
  const bool hit = r <= a.range_max;
  const double rr = hit ? (double)r : (double)a.range_max;
  const double cphi = trig[2 * i], sphi = trig[2 * i + 1];
  const double a1 = cyaw * cphi;
  const double a2 = syaw * sphi;
  const double dcx = a1 - a2;
  const double b1 = syaw * cphi;
  const double b2 = cyaw * sphi;
  const double dcy = b1 + b2;
  const double t1 = rr * dcx;
  const double ex = x + t1;
  const double t2 = rr * dcy;
  const double ey = y + t2;
  const double fsx = floor((x - a.ox) / a.res);
  const double fsy = floor((y - a.oy) / a.res);
  const double fex = floor((ex - a.ox) / a.res);
  const double fey = floor((ey - a.oy) / a.res);
  const double lim = 1073741824.0;
  if (!(fabs(fsx) < lim && fabs(fsy) < lim && fabs(fex) < lim && fabs(fey) < lim)) return bm;
  const int32_t sx = (int32_t)fsx, sy = (int32_t)fsy, ex_c = (int32_t)fex, ey_c = (int32_t)fey;
  const int32_t dx = ex_c - sx, dy = ey_c - sy;
  const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
  const int8_t ix = dx > 0 ? 1 : (dx < 0 ? -1 : 0);
  const int8_t iy = dy > 0 ? 1 : (dy < 0 ? -1 : 0);
  if (adx >= ady) {
    bm.xmajor = 1; bm.sa = sx; bm.sb = sy; bm.n = adx; bm.adb = ady; bm.ia = ix; bm.ib = iy;
  } else {
    bm.xmajor = 0; bm.sa = sy; bm.sb = sx; bm.n = ady; bm.adb = adx; bm.ia = iy; bm.ib = ix;
  }
  bm.rden = bm.n > 0 ? 1.0 / (double)(2 * bm.n) : 0.0;
  bm.flags = (uint8_t)(1u | (hit ? 2u : 0u));
  return bm;
}

// Enumerate the pieces of a beam's line that fall in in-band tiles, in order
// of k: emit(tile, k0, k1).  The major coordinate moves one cell per k and
// the minor one is monotone in k, so the k at which each coordinate leaves
// its tile is exact integer arithmetic.  Every pass advances
// k by >= 1; the pass cap only guards against a logic error.
// With k_lo / k_hi only the steps k in [k_lo, min(n, k_hi)] are enumerated
// (a chunk of the beam: pieces are cut at the chunk's ends too).
template <class Emit>
DM_HD inline void dm_for_each_piece(const Beam& b, const RayGeom& g, Emit&& emit, int32_t k_lo = 0,
                                    int32_t k_hi = 0x7FFFFFFF) {
  const int32_t n = b.n;
  const int32_t kend = n < k_hi ? n : k_hi;
  const int32_t off_a = b.xmajor ? 0 : g.row0;
  const int32_t off_b = b.xmajor ? g.row0 : 0;
  const int32_t lim_a = b.xmajor ? g.TX : g.TY;
  const int32_t lim_b = b.xmajor ? g.TY : g.TX;
  const int32_t max_iter = 2 * ((kend - k_lo) / DM_TS) + 8;
  // k at which the minor coordinate reaches step count Q:
  //   ceil(n*(2Q-1) / (2*adb)); operands < 2^31 (n, adb <= 16386, Q <= adb+1),
  //   so a double reciprocal (once per beam) + one exact correction replaces a
  //   64-bit integer division per piece
  const int32_t den_b = 2 * b.adb;
  const double rden_b = b.adb > 0 ? 1.0 / (double)den_b : 0.0;
  int32_t k = k_lo;
  for (int32_t it = 0; k <= kend && it < max_iter; ++it) {
    const int32_t q = dm_minor_steps(b, k);
    const int32_t ma = b.sa + k * b.ia - off_a;
    const int32_t mb = b.sb + b.ib * q - off_b;
    const int32_t ta = dm_floordiv32(ma, DM_TS);
    const int32_t tb = dm_floordiv32(mb, DM_TS);
    int64_t ka;
    if (b.ia > 0) ka = (int64_t)k + (DM_TS * (ta + 1) - ma);
    else if (b.ia < 0) ka = (int64_t)k + (ma - DM_TS * ta) + 1;
    else ka = (int64_t)n + 1;
    int64_t kb;
    if (b.ib == 0) {
      kb = (int64_t)n + 1;
    } else {
      const int32_t Q = q + (b.ib > 0 ? (DM_TS * (tb + 1) - mb) : (mb - DM_TS * tb) + 1);
      const int32_t num = n * (2 * Q - 1);
      kb = dm_udiv(num + den_b - 1, den_b, rden_b);
    }
    int64_t ke = ka < kb ? ka : kb;
    if (ke > (int64_t)kend + 1) ke = (int64_t)kend + 1;
    ke -= 1;
    if (ke < k) ke = k;  // never step backwards
    if (ta >= 0 && ta < lim_a && tb >= 0 && tb < lim_b) {
      const int32_t tx = b.xmajor ? ta : tb;
      const int32_t ty = b.xmajor ? tb : ta;
      emit(ty * g.TX + tx, k, (int32_t)ke);
    }
    k = (int32_t)ke + 1;
  }
}

// Cell (x, band-local y) of step k.
DM_HD inline void dm_cell(const Beam& b, int32_t k, int32_t row0, int32_t* x, int32_t* yl) {
  const int32_t q = dm_minor_steps(b, k);
  const int32_t ma = b.sa + k * b.ia;
  const int32_t mb = b.sb + b.ib * q;
  *x = b.xmajor ? ma : mb;
  *yl = (b.xmajor ? mb : ma) - row0;
}

// Incremental walk along a piece (used by k_tile_accum and the host
// emulation): the cell of step k0, then one step per k with the exact integer
// carry of the minor coordinate, q(k) = floor((2k*adb + n) / (2n)):
// rem = (2k*adb + n) mod 2n, rem += 2*adb per step, carry when rem >= 2n
// (adb <= n, so at most one carry per step).  Equals dm_cell(b, k) for every k.
struct PieceWalk {
  int32_t x, yl;           // current cell (global x, band-local y)
  int32_t rem, two_n, two_adb;
  int32_t dxa, dya, dxb, dyb;  // per step / per carry

  DM_HD void init(const Beam& b, int32_t k0, int32_t row0) {
    two_n = 1;
    two_adb = 0;
    int32_t q = 0;
    rem = 0;
    if (b.n > 0) {
      two_n = 2 * b.n;
      two_adb = 2 * b.adb;
      const int32_t num = k0 * two_adb + b.n;
      q = dm_udiv(num, two_n, b.rden);
      rem = num - q * two_n;
    }
    const int32_t ma = b.sa + k0 * b.ia, mb = b.sb + b.ib * q;
    x = b.xmajor ? ma : mb;
    yl = (b.xmajor ? mb : ma) - row0;
    dxa = b.xmajor ? b.ia : 0;
    dya = b.xmajor ? 0 : b.ia;
    dxb = b.xmajor ? 0 : b.ib;
    dyb = b.xmajor ? b.ib : 0;
  }

  DM_HD void step() {
    x += dxa;
    yl += dya;
    rem += two_adb;
    if (rem >= two_n) {
      rem -= two_n;
      x += dxb;
      yl += dyb;
    }
  }
};

// floor(num / den) for 0 <= num < 2^22, 0 < den, from an approximate fp32
// reciprocal of den (relative error < 2^-20): the estimate is within 1 of the
// quotient, one integer correction each way makes it exact.
DM_HD inline int32_t dm_udiv_small(int32_t num, int32_t den, float rden) {
  int32_t q = (int32_t)((float)num * rden);
  if ((q + 1) * den <= num) ++q;
  else if (q * den > num) --q;
  return q;
}

// A piece (beam steps k0..k1 inside one tile) in tile-local LDS word
// addresses, row pitch `pitch`: cell k0 + j sits at
//   addr0 + j*da + db * floor((rem0 + j*two_adb) / two_n)
// (the minor carry of PieceWalk in closed form), so a kernel can walk it one
// cell per step (dm_piece_walk below) or put one lane per cell.  addr_end is
// the address of the beam's hit cell when this piece ends the beam with a hit
// (SPEC a6: the endpoint counts as a hit), else -1.  Every cell of a piece is
// inside the tile by construction (dm_for_each_piece), so the addresses are
// in [0, 64*pitch); cells beyond the grid's last column / the band's last row
// (edge tiles) land on LDS words the apply step ignores.
struct TilePiece {
  int32_t addr0, addr_end, len;
  int32_t da, db;
  int32_t rem0, two_adb, two_n;
};

// tx0 / ty0: the tile's first column / band-local first row.
DM_HD inline TilePiece dm_tile_piece(const Beam& b, int32_t k0, int32_t k1, int32_t row0, int32_t tx0,
                                     int32_t ty0, int32_t pitch) {
  TilePiece tp;
  PieceWalk w;
  w.init(b, k0, row0);
  tp.addr0 = (w.yl - ty0) * pitch + (w.x - tx0);
  tp.len = k1 - k0 + 1;
  tp.da = b.xmajor ? (int32_t)b.ia : (int32_t)b.ia * pitch;
  tp.db = b.xmajor ? (int32_t)b.ib * pitch : (int32_t)b.ib;
  tp.rem0 = w.rem;
  tp.two_adb = w.two_adb;
  tp.two_n = w.two_n;
  tp.addr_end = -1;
  if ((b.flags & 2) && k1 == b.n) {
    // q(n) = adb: the endpoint cell
    const int32_t ma = b.sa + b.n * b.ia, mb = b.sb + b.ib * b.adb;
    const int32_t x = b.xmajor ? ma : mb, yl = (b.xmajor ? mb : ma) - row0;
    tp.addr_end = (yl - ty0) * pitch + (x - tx0);
  }
  return tp;
}

// LDS address of cell k0 + j of a piece (one lane per cell; j < 64 keeps
// num < 2^22).
DM_HD inline int32_t dm_piece_addr(const TilePiece& tp, int32_t j, float rtwo_n) {
  const int32_t dq = dm_udiv_small(tp.rem0 + j * tp.two_adb, tp.two_n, rtwo_n);
  return tp.addr0 + j * tp.da + dq * tp.db;
}

// A TilePiece packed into 16 bytes (k_scatter writes them, k_tile_accum
// reads one per lane): every field fits 16 bits because a piece lies in one
// 64x64 tile (addresses < 64*65, len <= 64) and rays are at most 16386
// cells (validate_params: range_max / resolution <= 16384), so
// rem0 < two_n <= 32774 and two_adb <= two_n.  da / db are +-1 or +-pitch
// (pitch 65 fits int8) or 0.
//   x: addr0 | len << 16      y: (addr_end + 1) | (u8)da << 16 | (u8)db << 24
//   z: rem0 | two_adb << 16   w: two_n
struct PackedPiece {
  uint32_t x, y, z, w;
};
static_assert(sizeof(PackedPiece) == 16, "PackedPiece layout");

DM_HD inline PackedPiece dm_pack_piece(const TilePiece& tp) {
  PackedPiece p;
  p.x = (uint32_t)tp.addr0 | ((uint32_t)tp.len << 16);
  p.y = (uint32_t)(tp.addr_end + 1) | ((uint32_t)(uint8_t)(int8_t)tp.da << 16) |
        ((uint32_t)(uint8_t)(int8_t)tp.db << 24);
  p.z = (uint32_t)tp.rem0 | ((uint32_t)tp.two_adb << 16);
  p.w = (uint32_t)tp.two_n;
  return p;
}

DM_HD inline TilePiece dm_unpack_piece(uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
  TilePiece tp;
  tp.addr0 = (int32_t)(x & 0xFFFFu);
  tp.len = (int32_t)(x >> 16);
  tp.addr_end = (int32_t)(y & 0xFFFFu) - 1;
  tp.da = (int32_t)(int8_t)(uint8_t)(y >> 16);
  tp.db = (int32_t)(int8_t)(uint8_t)(y >> 24);
  tp.rem0 = (int32_t)(z & 0xFFFFu);
  tp.two_adb = (int32_t)(z >> 16);
  tp.two_n = (int32_t)w;
  return tp;
}

// Incremental form: the address of the current cell, then one step per k.
struct PieceCursor {
  int32_t addr, rem;
  DM_HD void init(const TilePiece& tp) { addr = tp.addr0; rem = tp.rem0; }
  // at cell j (0 <= j < 64) of the piece: the closed form once (dm_piece_addr)
  DM_HD void init_at(const TilePiece& tp, int32_t j, float rtwo_n) {
    const int32_t num = tp.rem0 + j * tp.two_adb;
    const int32_t dq = dm_udiv_small(num, tp.two_n, rtwo_n);
    addr = tp.addr0 + j * tp.da + dq * tp.db;
    rem = num - dq * tp.two_n;
  }
  DM_HD void step(const TilePiece& tp) {
    addr += tp.da;
    rem += tp.two_adb;
    if (rem >= tp.two_n) { rem -= tp.two_n; addr += tp.db; }
  }
};

// Split walks (k_tile_accum): an item of c pieces on `lanes` lanes gives
// each piece f = lanes / c lanes (f >= 1); lane t takes part t % f of piece
// t / f, cells [j0, j0 + n) with parts of ceil(len / f) cells.  A piece's
// parts cover its cells exactly once, so the counts do not change; the
// walk's trip count (the longest part on the wave) shrinks by up to f.
struct SplitPart {
  int32_t j0, n;
};
DM_HD inline int32_t dm_split_factor(int32_t c, int32_t lanes) { return c > 0 && c <= lanes ? lanes / c : 1; }
DM_HD inline SplitPart dm_split_part(int32_t len, int32_t f, int32_t part, float rf) {
  SplitPart s;
  if (f == 1) {
    s.j0 = 0;
    s.n = len;
    return s;
  }
  const int32_t plen = dm_udiv_small(len + f - 1, f, rf);  // ceil(len / f), len <= 64
  s.j0 = part * plen;
  const int32_t left = len - s.j0;
  s.n = left < 0 ? 0 : (left < plen ? left : plen);
  return s;
}
