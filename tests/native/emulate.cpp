// TEST INFRASTRUCTURE: sequential host emulation of the dm_integrate.hip
// pipeline (k_beam_prep -> k_scan_active -> k_scatter -> k_tile_apply) built
// from the SAME geometry header the kernels use (csrc/dm_ray.h).  Lets the
// CPU test-suite check the kernels' tiling / binning logic against the oracle
// without a GPU.  Not part of the product.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <math.h>
#include <vector>

#include "../../distributed-autonomous-exploration-and-mapping_amd/csrc/dm_ray.h"

extern "C" int emu_integrate(int32_t W, int32_t R, int32_t row0, double ox, double oy, double res,
                             float range_min, float range_max, float l_occ, float l_free,
                             float l_min, float l_max, float occ_t, float free_t, float* L,
                             int8_t* state, int32_t S, const double* pose4, int32_t N,
                             const float* ranges, const double* trig, uint64_t* out_U,
                             uint64_t* out_T, uint64_t* out_segs, int32_t chunk_len) {
  RayGeom g;
  g.W = W; g.R = R; g.row0 = row0;
  g.TX = (W + DM_TS - 1) / DM_TS;
  g.TY = (R + DM_TS - 1) / DM_TS;
  RayArgs a;
  a.S = S; a.N = N; a.ox = ox; a.oy = oy; a.res = res;
  a.range_min = range_min; a.range_max = range_max;
  const int64_t NT = (int64_t)g.TX * g.TY, nb = (int64_t)S * N;
  std::vector<int32_t> count(NT, 0), slot(NT, -1), act;
  std::vector<Beam> beams(nb);
  // k_beam_prep / k_scatter may enumerate a beam as k-ranges of chunk_len
  // steps on different threads (dm_integrate_chunks); 0 = whole beams
  auto for_chunks = [&](const Beam& bm, auto&& f) {
    if (chunk_len <= 0) { f(0, 0x7FFFFFFF); return; }
    for (int32_t k_lo = 0; k_lo <= bm.n; k_lo += chunk_len) f(k_lo, k_lo + chunk_len - 1);
  };
  for (int64_t b = 0; b < nb; ++b) {  // k_beam_prep
    beams[b] = dm_make_beam(a, pose4, ranges, trig, (int32_t)(b / N), (int32_t)(b % N));
    if (!(beams[b].flags & 1)) continue;
    for_chunks(beams[b], [&](int32_t k_lo, int32_t k_hi) {
      dm_for_each_piece(beams[b], g, [&](int32_t t, int32_t, int32_t) {
        if (count[t]++ == 0) { slot[t] = (int32_t)act.size(); act.push_back(t); }
      }, k_lo, k_hi);
    });
  }
  std::vector<int64_t> off(act.size() + 1, 0), cur(act.size());
  for (size_t j = 0; j < act.size(); ++j) off[j + 1] = off[j] + count[act[j]];  // k_scan_active
  for (size_t j = 0; j < act.size(); ++j) cur[j] = off[j];
  struct Seg { int64_t beam; int32_t k0, k1; };
  std::vector<Seg> segs(off[act.size()]);
  for (int64_t b = 0; b < nb; ++b) {  // k_scatter
    if (!(beams[b].flags & 1)) continue;
    for_chunks(beams[b], [&](int32_t k_lo, int32_t k_hi) {
      dm_for_each_piece(beams[b], g, [&](int32_t t, int32_t k0, int32_t k1) {
        segs[cur[slot[t]]++] = Seg{b, k0, k1};
      }, k_lo, k_hi);
    });
  }
  uint64_t U = 0, T = 0;
  constexpr int32_t kPitch = DM_TS + 1;  // k_tile_accum's LDS row pitch
  std::vector<uint32_t> hit(DM_TS * DM_TS), miss(DM_TS * DM_TS);
  for (size_t j = 0; j < act.size(); ++j) {  // k_tile_accum
    const int32_t t = act[j];
    const int32_t tx0 = (t % g.TX) * DM_TS, ty0 = (t / g.TX) * DM_TS;
    std::fill(hit.begin(), hit.end(), 0u);
    std::fill(miss.begin(), miss.end(), 0u);
    for (int64_t s = off[j]; s < off[j + 1]; ++s) {
      const Beam& bm = beams[segs[s].beam];
      const TilePiece tp0 = dm_tile_piece(bm, segs[s].k0, segs[s].k1, row0, tx0, ty0, kPitch);
      // k_scatter stores the piece packed (16 B); k_tile_accum unpacks it
      const PackedPiece pk = dm_pack_piece(tp0);
      const TilePiece tp = dm_unpack_piece(pk.x, pk.y, pk.z, pk.w);
      if (tp.addr0 != tp0.addr0 || tp.addr_end != tp0.addr_end || tp.len != tp0.len || tp.da != tp0.da ||
          tp.db != tp0.db || tp.rem0 != tp0.rem0 || tp.two_adb != tp0.two_adb || tp.two_n != tp0.two_n)
        return -105;
      const float rtwo_n = 1.0f / (float)tp.two_n;
      PieceCursor cur;
      cur.init(tp);
      if (tp.len < 1 || tp.len > DM_TS) return -101;
      // k_tile_accum's split walks (walk_tp_split / walk_piece_bytes): the
      // parts of a piece over f lanes cover its cells once, each part's
      // cursor starting at the closed-form cell j0
      for (int32_t f : {2, 3, 4, 5, 7, 16, 21, 64, 128, 256}) {
        int32_t covered = 0;
        for (int32_t part = 0; part < f; ++part) {
          const SplitPart spp = dm_split_part(tp.len, f, part, 1.0f / (float)f);
          if (spp.n < 0 || (spp.n > 0 && (spp.j0 != covered || spp.j0 + spp.n > tp.len))) return -106;
          covered += spp.n;
          if (spp.n == 0) continue;
          PieceCursor pc;
          pc.init_at(tp, spp.j0, rtwo_n);
          if (pc.addr != dm_piece_addr(tp, spp.j0, rtwo_n)) return -107;
          for (int32_t i = 1; i < spp.n; ++i) {
            pc.step(tp);
            if (pc.addr != dm_piece_addr(tp, spp.j0 + i, rtwo_n)) return -107;
          }
        }
        if (covered != tp.len) return -106;
      }
      for (int st = 0; st < tp.len; ++st, cur.step(tp)) {
        const int32_t k = segs[s].k0 + st;
        int32_t x, yl;
        dm_cell(bm, k, row0, &x, &yl);
        const int32_t lx = x - tx0, ly = yl - ty0;
        // both address forms must name the closed-form cell, inside the tile
        if ((uint32_t)lx >= DM_TS || (uint32_t)ly >= DM_TS) return -102;
        if (cur.addr != ly * kPitch + lx) return -100;
        if (dm_piece_addr(tp, st, rtwo_n) != cur.addr) return -103;
        const bool is_hit = (k == bm.n) && (bm.flags & 2);
        if (is_hit != (tp.addr_end == cur.addr && st == tp.len - 1)) return -104;
        // the kernel adds 1 per cell, then 0xFFFF at addr_end (a miss becomes a hit)
        (is_hit ? hit : miss)[ly * DM_TS + lx] += 1;
      }
    }
    for (int ly = 0; ly < DM_TS; ++ly)  // U: in-grid cells only, as apply_tile counts it
      for (int lx = 0; lx < DM_TS; ++lx)
        if (tx0 + lx < W && ty0 + ly < R) U += hit[ly * DM_TS + lx] + miss[ly * DM_TS + lx];
    for (int ly = 0; ly < DM_TS; ++ly)
      for (int lx = 0; lx < DM_TS; ++lx) {
        const uint32_t h = hit[ly * DM_TS + lx], m = miss[ly * DM_TS + lx];
        if (!(h | m) || tx0 + lx >= W || ty0 + ly >= R) continue;
        const int64_t i = (int64_t)(ty0 + ly) * W + tx0 + lx;
        float l = L[i];
        const float tt = (float)h * l_occ;
        const float uu = (float)m * l_free;
        l = l + tt;
        l = l + uu;
        if (l < l_min) l = l_min;
        if (l > l_max) l = l_max;
        L[i] = l;
        state[i] = l == 0.0f ? -1 : (l >= occ_t ? 100 : (l <= free_t ? 0 : -1));
        ++T;
      }
  }
  *out_U = U;
  *out_T = T;
  *out_segs = (uint64_t)segs.size();
  return 0;
}
