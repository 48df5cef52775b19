// dm_internal.h — internal types of libdm (not part of the C-ABI).
//
// Device data layout in HBM (one handle = one row band of the map):
//   L      float [R][W]  log-odds, row-major (band-local row = gy - row0)
//   state  int8  [R][W]  OccupancyGrid.data encoding (-1/0/100)
//   tile_* int32 [TY][TX] per 64x64 tile summaries (TX = ceil(W/64),
//          TY = ceil(R/64)): per-call segment counts, active slots, and the
//          number of free cells (drives which tiles the frontier pass visits)
// Per-call workspace (grown on demand, reused across calls):
//   beams  Beam[S*N]     endpoint cells + Bresenham parameters per beam
//   pieces PackedPiece[] ray pieces binned by tile, tile-local addresses
//   active tile lists, frontier slots (one per tile-local component), borders.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/dm.h"

#include "dm_ray.h"


// device counters (uint64 each)
enum {
  CNT_ACTIVE = 0,   // active tiles this integrate call
  CNT_U = 1,        // beam-cell updates
  CNT_T = 2,        // touched cells
  CNT_SEGS = 3,     // segments emitted
  CNT_FTILES = 4,   // tiles visited by the frontier pass (tile_free > 0)
  CNT_SLOTS = 5,    // tile-local frontier components
  CNT_CLUSTERS = 6, // output clusters
  CNT_OVERFLOW = 7, // frontier flags: kOvSlots (slot arrays full), kOvUnionFind (bound hit)
  CNT_ITEMS = 8,    // heavy work items (<= 256 pieces of a heavy tile each)
  CNT_HEAVY = 9,    // heavy tiles (> 256 pieces)
  CNT_TH = 10,      // touched cells of heavy tiles
  CNT_SORTED = 11,  // 1: out_clu holds the clusters sorted by label
  CNT_FL0 = 12,     // frontier tile-list length of the pass (copied by k_frontier_bits)
  CNT_STAMP = 13,   // the pass's stamp (k_frontier_bits: ++ the handle's stamp word), tile-edge hand-offs
  CNT_LITEMS = 14,  // light work items (= light tiles)
  CNT_IOVERFLOW = 15,  // integrate capacity overflow flags (1 first-touch list, 2 pieces, 4 work lists)
  CNT_BIG = 16,     // frontier tiles with more runs than a tile-wave holds (big-tile list length)
  CNT_SITEMS = 17,  // sparse light work items (<= sparse_pieces pieces; stored from the top of litems)
  CNT_N = 18
};
// CNT_OVERFLOW bits of a frontier pass
constexpr unsigned long long kOvSlots = 4ull;      // a slot shard region overflowed
constexpr unsigned long long kOvUnionFind = 8ull;  // a union-find loop hit its bound (dm_uf.h)
constexpr unsigned long long kOvPipeline = 32ull;  // the handle's sticky hand-off error was set (kHaltWord)
// fe_flag[kHaltWord]: sticky error word of the overlapped pipeline.  The
// integrate front-end -> map update gate sets bit 1 when it times out; from
// then on k_tile_accum and k_fmask_items return at once (the workspace they
// would read was not written), k_frontier_bits flags every pass kOvPipeline,
// and the host reports DM_ERR_PIPELINE until dm_reset clears it.
constexpr int kHaltWord = 8;
// Hand-off words (fe_flag, bits_flag): k_seq_signal increments [kSigWord],
// k_seq_gate increments [kGateWord] and waits until [kSigWord] reaches it:
// the n-th gate waits for the n-th signal, with no host-side sequence number
// in the kernel arguments.
constexpr int kSigWord = 0;
constexpr int kGateWord = 4;
constexpr int kStampWord = 8;  // bits_flag: the last frontier pass's stamp (k_frontier_bits)
// Integrate counters, zeroed by each integrate call; the others belong to the
// frontier pass, which may still be running when the next call's front-end
// starts (dm_set_overlap), so the integrate reset never touches them.
constexpr int kIntegrateCounters[] = {CNT_ACTIVE, CNT_U, CNT_T, CNT_SEGS, CNT_ITEMS,
                                      CNT_HEAVY, CNT_TH, CNT_LITEMS, CNT_IOVERFLOW, CNT_SITEMS};

// k_plan's work-item classes (dm_integrate.hip): tiles with more pieces than
// kIntegrateChunk are split into items of kIntegrateChunk pieces, tiles with
// more than kIntegrateMedium are heavy (merged in a slab)
constexpr int kIntegrateChunk = 256;
constexpr int kIntegrateMedium = 1024;


// Sharded counters: same-address device atomics serialise at the memory side
// (~12 ns each, MI355X_MICROARCH.md price list "fanin"), so per-workgroup
// totals go to one of kShards counters, each on its own 128-B line
// (shard = blockIdx.x % kShards); readers sum the shards.
constexpr int kShards = 32;
constexpr int kShardWords = 16;  // 128 B per shard
static_assert(kShards * kShardWords == 512, "k_integrate_reset covers 512 shard words");
// integrate shard fields
enum { SH_U = 0, SH_T = 1, SH_TH = 2, SH_ACT = 3 };
// frontier shard fields: slots allocated, runs and tiles with frontier
// cells (the next pass picks its tile kernel from their ratio)
// and tiles too run-rich for a tile-wave (the next pass sizes the big kernel's grid)
enum { SH_SLOT = 0, SH_RUNS = 1, SH_FTF = 2, SH_BIG = 3 };

// dm_last_stats entries (include/dm.h)
constexpr int kNStats = 11;
constexpr bool dm_stat_is_frontier(int i) { return i >= 7 && i <= 9; }  // the others: integrate

// Readback header in front of the sorted cluster records (device out_clu and
// pinned h_out both point kRbRecords records into their allocation): the
// frontier counters [CNT_N] and the fullest slot shard [CNT_N], written by
// k_rank_sort into the mapped host buffer together with the first records.
// header words: [0, CNT_N) counters, [CNT_N] fullest slot shard, [CNT_N + 1]
// runs, [CNT_N + 2] tiles with frontier cells, [CNT_N + 3] run-rich tiles
// (shard sums)
constexpr int kRbRecords = 6;  // 6 * 48 B = 288 B >= (CNT_N + 3) * 8 B
static_assert(kRbRecords * sizeof(dm_cluster) >= (CNT_N + 4) * sizeof(unsigned long long), "readback header");
// The mapped host readback carries 32-byte records (label, size, sum_x,
// sum_y): the host computes the centroids with the SPEC's double formula
// (one division, then add; no FMA), bit-identical to the device's, so a third
// fewer bytes cross PCIe than whole dm_cluster records.
struct dm_raw_record {
  long long label, size, sum_x, sum_y;
};
constexpr int kRbHostRecords = 6;  // 6 * 32 B = 192 B of header in front of the host records
static_assert(kRbHostRecords * sizeof(dm_raw_record) >= (CNT_N + 4) * sizeof(unsigned long long),
              "readback header");
__host__ __device__ inline unsigned long long* dm_rb_header(dm_raw_record* records) {
  return reinterpret_cast<unsigned long long*>(records - kRbHostRecords);
}
__host__ __device__ inline const unsigned long long* dm_rb_header(const dm_raw_record* records) {
  return reinterpret_cast<const unsigned long long*>(records - kRbHostRecords);
}
// SPEC a10 centroid: origin + (sum / size + 0.5) * res,
// one IEEE division, then add (compiled with -ffp-contract=off, host and device)
__host__ __device__ inline double dm_centroid(double origin, long long sum, long long size, double res) {
  const double m = (double)sum / (double)size;
  return origin + (m + 0.5) * res;
}

struct dm_grid;
// async D2H of both shard-counter blocks into g->h_sh (pinned)
hipError_t dm_copy_shards(dm_grid* g);
inline unsigned long long dm_shard_sum(const unsigned long long* sh, int field) {
  unsigned long long s = 0;
  for (int i = 0; i < kShards; ++i) s += sh[i * kShardWords + field];
  return s;
}

struct KernelTimer {
  std::string name;
  hipEvent_t start, stop;
  hipStream_t stream = nullptr;
};

struct dm_shard_set;  // dm_sharded.cpp

struct dm_grid {
  dm_params p;
  // non-null: a sharded parent (dm_create_sharded); every call runs on its
  // band handles (dm_sharded.cpp) and none of the fields below is allocated
  dm_shard_set* sh = nullptr;
  int device = 0;
  int n_cu = 256;  // compute units of the device: sizes the resident (one-pass) grids
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // dm_set_overlap: the integrate front-end (reset, beam_prep, plan, scatter)
  // runs on fe_stream, so it overlaps a frontier pass still running on
  // `stream`; the accumulation waits for it (ev_fe).  The workspace the
  // front-end hands to the accumulation is double-buffered (iw[2], calls
  // alternate): call k+1's front-end only waits for call k-1's accumulation
  // (iw[p].ev_free), which is long done when the steps are pipelined, so no
  // marker sits behind the accumulation of call k.
  bool overlap = false;
  // DM_FE_STREAMS = 2: consecutive calls' front-ends alternate between two
  // streams (call k on fe_streams[set % 2], the set being its workspace
  // set), so call k+1's front-end may start before call k's has finished
  // instead of queueing behind it; each stream has its own hand-off words
  // (dm_fe_flag_of).  1: one front-end stream (fe_streams[0]).
#ifndef DM_FE_STREAMS
#define DM_FE_STREAMS 1
#endif
  static constexpr int kFeStreams = DM_FE_STREAMS;
  static_assert(kFeStreams == 1 || kFeStreams == 2, "one or two front-end streams");
  hipStream_t fe_streams[2] = {nullptr, nullptr};
  hipEvent_t ev_fe = nullptr;
  // the end of the last front-end of each set parity (before its signal):
  // a caller that refills a buffer every front-end reads (the sharded
  // handle's peer copies of the inputs) orders itself after it
  hipEvent_t ev_fe_end[2] = {nullptr, nullptr};
  // front-end completion word (k_fe_signal / k_fe_gate, dm_integrate.hip):
  // the sequence number of the last call whose front-end finished
  unsigned long long* fe_flag = nullptr;  // [kSigWord] / [kGateWord] hand-off counts, [kHaltWord] sticky error
  // DM_FAULT_GATE=1 (read at dm_create; fault-injection tests only): the
  // front-end gate waits for a sequence number that never comes, ~10 us
  bool fault_gate = false;
  // ev_bits[parity]: the end of a split pass's bit rows on `stream` (the pass
  // stream waits for it); it also frees the integrate workspaces whose
  // accumulations are ahead of it (dm_mark_ws_free), so the next front-end
  // using them can start right away instead of after the whole pass
  hipEvent_t ev_bits[2] = {nullptr, nullptr};
  uint64_t integrate_seq = 0;  // map changes so far
  // Asynchronous passes (dm_frontiers_begin / dm_merge_bands_begin) use a
  // ring of kRbSlots readback slots, so a pass can be started before the
  // previous one was collected.  Each slot owns what its _end reads: the
  // mapped readback buffer (header + first records), the device sorted
  // records, the event marking the pass's end.  out_clu / h_out / h_out_dev /
  // h_out_cap / m_out below point at the slot in use (dm_select_slot).
  struct RbSlot {
    dm_cluster* out_clu = nullptr;    // device sorted band records (after kRbRecords header records)
    dm_raw_record* h_out = nullptr;      // mapped host readback (after the header), 32-byte records
    dm_raw_record* h_out_dev = nullptr;  // its device address
    int64_t h_out_cap = 0;
    dm_cluster* m_out = nullptr;      // device sorted merged records
    hipEvent_t ev = nullptr;
    int kind = 0;                     // pending pass: 0 none, 1 band frontiers, 2 band merge
    uint64_t seq = 0;                 // integrate_seq at the pass's start
    uint64_t gen = 0;                 // rb_gen at the pass's start
    uint64_t pass = 0;                // fr_pass / m_pass of the pass
    int64_t merge_n = 0;              // nranks * rec_cap of a merge
    uint64_t wepoch = 0, mepoch = 0;  // passes / merges that wrote out_clu / m_out so far
  };
#ifndef DM_RB_SLOTS
#define DM_RB_SLOTS 2
#endif
  static constexpr int kRbSlots = DM_RB_SLOTS;  // ring slots of asynchronous passes
  static constexpr int kRbSync = kRbSlots;      // the slot of synchronous calls (dm_frontiers, dm_merge_bands)
  RbSlot rb[kRbSlots + 1];
  int rb_head = 0, rb_count = 0;      // oldest pending slot, pending passes
  int cur_slot = 0;                   // the slot dm_select_slot selected
  uint64_t rb_gen = 0;                // bumped when device record buffers are reallocated
  // frontier / merge passes enqueued so far: an unsorted result (more
  // clusters than the sort kernel takes) lives in the shared raw arrays
  // (clusters / m_clu), valid only while no later pass of its kind ran
  uint64_t fr_pass = 0, m_pass = 0;
  int64_t W = 0, H = 0, R = 0, row0 = 0;
  int64_t TX = 0, TY = 0, NT = 0;
  int32_t nmax = 0;  // max ray length (cells) bound

  float* L = nullptr;
  int8_t* state = nullptr;
  // free cells per tile (bits 0..29) | kTileListed: the tile is on the
  // persistent frontier tile list (ftiles / ftiles_n below)
  int32_t* tile_free = nullptr;
  // [NT][64 rows][16] per tile: byte j of row y holds the free bits of cells
  // 4j..4j+3 (low nibble) and their unknown bits (high nibble); out-of-grid
  // cells are neither.  Kept in step with `state` by every kernel that writes
  // it (k_tile_accum's apply: each thread stores its 4 cells' byte;
  // k_recount after bulk writes); the frontier pass reads these 1 KB per tile
  // instead of the state bytes.  Maintained only while passes list many tiles
  // (fmask_on: a pass listing >= kFmaskOnTiles switches it on, one listing
  // fewer than kFmaskOnTiles / 4 off): a few thousand listed tiles (C3) are
  // latency-bound either way and the per-call update would only add a
  // kernel.  fmask_valid: the records match the state (a full rebuild,
  // k_recount, precedes switching on otherwise).
  uint8_t* fmask = nullptr;
  // fedge: per tile 4 words, the unknown bits of its column 0, column 63
  // (bit = row), row 0 and row 63 (bit = column), written with fmask by the
  // same kernels: a pass reads its neighbours' edges from these 32 B instead
  // of from their 1 KB records (one byte of every 16 B row: all 8 lines)
  uint64_t* fedge = nullptr;
  // tile_seen: 0 while every cell of the tile is still unknown (since the
  // last bulk write: k_recount sets it from the state), 1 once an
  // integrate item applied the tile (k_tile_accum).  The frontier bit rows
  // take an unseen neighbour's facing cells as unknown without reading them:
  // the explored region's borders face unseen tiles, whose halo column would
  // otherwise cost a 128-byte line per row.
  // INVARIANT (the frontier pass is wrong without it): every kernel that
  // writes `state` either sets tile_seen[tile] = 1 for the tiles it wrote
  // (k_tile_accum: light / medium items, the heavy finisher, sparse items)
  // or is followed by k_recount over the map (dm_launch_recount: dm_reset,
  // dm_set_state, dm_set_logodds, dm_load).  A new state writer must do one
  // of the two; tests/test_gpu_tile_seen.py fails against a library whose
  // bit rows trust a stale flag (mutation-checked in round 5).
  uint8_t* tile_seen = nullptr;
  bool fmask_on = false, fmask_valid = false;
  int fmask_mode = 0;  // DM_FMASK=auto|on|off (read at dm_create; tests / A/B): 0 auto, 1 on, 2 off
  unsigned long long* cnt = nullptr;    // CNT_N device counters (frontier fields)
  unsigned long long* h_cnt = nullptr;  // pinned mirror: [CNT_N] frontier counters, [CNT_N] integrate counters
  unsigned long long* fsh = nullptr;    // [kShards][kShardWords] frontier shards
  unsigned long long* h_sh = nullptr;   // pinned mirror of the last call's integrate shards, then fsh

  // integrate workspace capacities (the arrays are per set, IntWs)
  int64_t beams_cap = 0;
  int64_t blk_cap = 0;            // workgroups blk_hist / blk_n hold
  int64_t segs_cap = 0;           // pieces per workspace
  int64_t act_cap = 0;
  int64_t hitem_cap = 0;
  int64_t heavy_cap = 0;
  // what the front-end hands to the accumulation, one set per call parity
  struct IntWs {
    // the front-end's own scratch (k_beam_prep -> k_plan / k_scatter): per
    // set, so two calls' front-ends may run at once (DM_FE_STREAMS)
    Beam* beams = nullptr;          // [beams_cap]
    int2* blk_hist = nullptr;       // [beam blocks][1024] k_beam_prep's (tile, pieces | hash slot << 16) histogram
    int32_t* blk_n = nullptr;       // [beam blocks] its entries
    int32_t* act_raw = nullptr;     // [kShards][act_cap] first-touch lists per shard
    PackedPiece* pieces = nullptr;    // [segs_cap] ray pieces binned by tile
    int4* hitems = nullptr;           // heavy work items {tile, first piece, pieces, heavy ordinal}
    int4* litems = nullptr;           // light work items {tile, first piece, pieces, -1} [act_cap]
    int32_t* heavy_list = nullptr;    // heavy ordinal -> tile
    uint32_t* slabs = nullptr;        // [heavy][2][64*64] merged hit / miss counts
    int32_t* heavy_done = nullptr;    // [heavy] items finished this call (the last one applies the slab)
    int32_t* tile_count = nullptr;    // [NT] pieces per tile (zeroed again by the accumulation)
    int32_t* tile_cur = nullptr;      // [NT] k_scatter's bin cursor per active tile (k_plan)
    unsigned long long* cnt = nullptr;  // [CNT_N] the integrate counters (kIntegrateCounters)
    unsigned long long* sh = nullptr;   // [kShards][kShardWords] integrate shards
    // device copies of host inputs (dm_integrate / _async) of the calls using
    // this set, reused only when the set is (free_wait)
    double* pose4 = nullptr;
    float* ranges = nullptr;
    int64_t pose_cap = 0, ranges_cap = 0;
    // the next front-end using this set waits for free_wait: an event on
    // `stream` after the set's last accumulation, recorded lazily (at the next
    // frontier pass or integrate call) -- ev_free, or the readback-slot event
    // of an asynchronous frontier pass enqueued after that accumulation
    // (dm_frontiers_begin records one anyway: no extra marker)
    hipEvent_t ev_free = nullptr;
    hipEvent_t free_wait = nullptr;
    bool free_owed = false;
  };
  // calls alternate between the two sets
  static constexpr int kIntSets = 2;
  IntWs iw[kIntSets];
  int iw_cur = 0;                // set of the last integrate call
  double* trig = nullptr; int32_t trig_n = -1; float trig_amin = 0, trig_inc = 0;
  int64_t trig_cap = 0;
  // pinned, mapped (x, y, cos, sin) staging of host poses: a ring of two, each
  // reusable once the front-end that read it (k_beam_prep, through the device
  // address) is done (ev_pose), so a host-input call never waits for the
  // previous call (dm_integrate_async)
  static constexpr int kPoseRing = 2;
  double* h_pose4[kPoseRing] = {nullptr, nullptr};
  hipEvent_t ev_pose[kPoseRing] = {nullptr, nullptr};
  double* h_pose4_dev[kPoseRing] = {nullptr, nullptr};  // their device addresses (mapped)
#ifndef DM_HOST_POSE
#define DM_HOST_POSE 1  // 0: poses copied to the device like the ranges (A/B builds)
#endif
  int64_t h_pose_cap = 0;
  int pose_head = 0;
  int32_t last_S = 0, last_N = 0;

  // frontier workspace
  // What a pass's bit-row kernel writes on `stream` while the previous
  // pass's labelling may still run on pass_stream is double-buffered by pass
  // parity (fparity): counters, shards, list, frontier bit rows, edge slots,
  // slot parents.  The current set's arrays are also reachable through the
  // plain fields below (dm_select_fw).  A set is reused two passes later; its
  // previous pass must be done by then (busy: the event that pass recorded,
  // waited on by `stream` unless the host already saw it complete).
  struct FrWs {
    unsigned long long* cnt = nullptr;  // [CNT_N]
    unsigned long long* fsh = nullptr;  // [kShards][kShardWords]
    int32_t* big_tiles = nullptr;       // [NT]
    uint64_t* fbits = nullptr;          // [NT][64]
    int32_t* edge_slot = nullptr;       // [2][W]
    int32_t* slot_parent = nullptr;     // [slot_cap]
    hipEvent_t busy = nullptr;          // the last pass's end (an alias of its readback event or ev_split)
    hipEvent_t ev_split = nullptr;      // end of a split export pass on the pass stream (owned)
    bool busy_pending = false;
    uint64_t busy_pass = 0;             // fr_pass of that pass
  };
  FrWs fw[2];
  // the pass's list lengths (snapshots of *ftiles_n taken by k_frontier_bits),
  // a ring of three on separate lines: pass n uses fl_n[16 * (n % 3)]
  unsigned long long* fl_n = nullptr;
  // pass_stream (dm_set_overlap + dm_frontiers_begin): the labelling half of
  // a pass (tile kernels, resolve, sort) runs there, after the bit-row
  // kernel on `stream` (which alone reads the map), so the next
  // batch's map update overlaps it.  bits_flag / bits_seq: the bit rows'
  // hand-off (k_seq_signal on `stream`, k_seq_gate on pass_stream).
  hipStream_t pass_stream = nullptr;
  // big_stream: k_frontier_tile_big over the tiles k_frontier_bits listed as
  // too run-rich for a tile-wave, beside the wave kernel on the pass stream
  // (forked after the bit rows, joined before the resolve)
  hipStream_t big_stream = nullptr;
  hipEvent_t ev_bigfork = nullptr, ev_big = nullptr;
  unsigned long long* bits_flag = nullptr;  // [kSigWord] / [kGateWord] counts, [kStampWord] pass stamp
  hipEvent_t p_tail = nullptr;        // the last pass_stream pass's end (alias)
  bool p_pending = false;             // pass_stream work `stream` has not been ordered after
  uint64_t p_tail_pass = 0;
  // The persistent frontier tile list: every tile that has held a free cell
  // since the last bulk state write, in the order its first free cell
  // appeared (only free cells can be frontier cells).  Appended by the
  // integrate apply (the item that raises a tile's free count above 0 while
  // kTileListed is clear sets it and takes a list position), rebuilt after
  // bulk writes (dm_launch_recount: k_list_tiles).  Append-only between
  // rebuilds, so a pass reads the first *ftiles_n entries (its snapshot, taken
  // on the map stream after its batch) while later batches append behind them.
  int32_t* ftiles = nullptr;               // [NT] the current list (one of flist)
  unsigned long long* ftiles_n = nullptr;  // [16]: [0] its length
  // Two lists: the periodic rebuild in tile order (dm_launch_relist) writes
  // the other one and switches, so passes still labelling go on reading the
  // old one (nothing appends to it after the switch) and the map stream never
  // waits for them; flist_ev[i]: the pass stream's position when list i was
  // left, which a rebuild into list i waits for (long done 16 passes later)
  int32_t* flist[2] = {nullptr, nullptr};
  unsigned long long* flist_n[2] = {nullptr, nullptr};
  hipEvent_t flist_ev[2] = {nullptr, nullptr};
  bool flist_ev_set[2] = {false, false};
  int flist_cur = 0;
  int relist_age = 0;     // passes since the list was last put in tile order
  int relist_period = 1;  // passes between those rebuilds: 1, 2, 4, ... up to kRelistPasses
                          // (a fresh map's list grows fastest in its first passes)
  int32_t* big_tiles = nullptr;  // [NT] per list position: 1 = too many runs for a tile-wave (k_frontier_bits)
  uint64_t* fbits = nullptr;   // [NT][64] frontier bit rows of the listed tiles (k_frontier_bits)
  int32_t* border = nullptr;   // [tile][4][64] slot ids of a tile's edges (published sides only)
  // tile-edge hand-off words of k_frontier_tile, [4][NT]: horizontal (t, t+1),
  // vertical (t, t+TX), diagonal (t, t+TX+1), anti-diagonal (t, t+TX-1) pairs,
  // each (pass stamp << 2 | arrived sides); never reset (stamped)
  unsigned long long* rel = nullptr;
  int32_t fparity = 0;         // workspace set (fw) of the last frontier pass
  int64_t border_cap = 0;      // in tiles
  int64_t slot_cap = 0;
  long long* slot_label = nullptr;
  int32_t* slot_parent = nullptr;
  int32_t* slot_root = nullptr;
  long long* slot_own = nullptr;  // [slot][3] size, sum_x, sum_y
  long long* slot_acc = nullptr;  // [slot][3]
  long long* clusters = nullptr;  // [cap][4] label,size,sum_x,sum_y (unsorted)
  int32_t* slot_k = nullptr;      // [slot_cap] root slot -> compact cluster index
  int32_t* rank_of = nullptr;     // [slot_cap] compact cluster index -> sorted position
  dm_cluster* out_clu = nullptr;  // [slot_cap] sorted cluster records (k_rank_sort)
  dm_raw_record* h_out = nullptr;  // pinned (mapped, coherent) readback: header + sorted 32-byte records
  dm_raw_record* h_out_dev = nullptr;  // its device address
  int64_t h_out_cap = 0;
  int32_t* cell_slot = nullptr;   // dense [R][W] (only when labels requested)
  int32_t* edge_slot = nullptr;   // [2][W] slots of the band's first / last row
  long long* edge_label = nullptr;// [2][W]
  uint8_t* mask = nullptr;        // dense [R][W] (only when mask requested)
  long long* labels = nullptr;    // dense [R][W] int64 (only when requested)
  int8_t* halo = nullptr;         // [2][W]: row before band, row after band
  int has_halo[2] = {0, 0};
  bool frontier_valid = false;

  // large-K cluster sort (row buckets, dm_frontier.hip k_rs_*): used when
  // the last collected pass of its kind had more than sort_min clusters
  unsigned long long* bs_key = nullptr;   // [bs_cap] sort keys (label - base), two buffers
  unsigned long long* bs_key2 = nullptr;
  int32_t* bs_idx = nullptr;      // [bs_cap] their record indices, two buffers
  int32_t* bs_idx2 = nullptr;
  int64_t bs_cap = 0;
  // per-row counters (zero between sorts) and offsets
  int32_t* rs_cnt = nullptr;      // [rs_rows]
  int32_t* rs_off = nullptr;      // [rs_rows + 1]
  unsigned long long* rs_status = nullptr;  // [rs_rows / 8192 + 2] k_rs_scan's workgroup totals + failure word
  int64_t rs_rows = 0;
  int64_t sort_hint = 0, msort_hint = 0;  // clusters of the last band / merge readback
  int64_t ftile_hint = 0;                 // listed tiles of the last collected frontier pass
  int64_t runs_hint = 0, ftf_hint = 0;    // its runs and tiles with frontier cells
  int64_t big_hint = 0;                   // its tiles left to k_frontier_tile_big by k_frontier_tile
  // the cluster count above which the row sort replaces the rank sort
  // (DM_SORT_MIN, read at dm_create: tests run small maps through both)
  int64_t sort_min = 4096;
  // tile kernel choice: 0 from those statistics, 1 always the wave-per-tile
  // kernel, 2 always the 256-thread kernel (DM_FRONTIER_KERNEL=auto|wave|wg,
  // read at dm_create, for A/B measurements; all three are exact)
  int frontier_kernel = 0;
  // k_tile_accum's largest grid (the kernel grid-strides)
  static constexpr int kAccumGrid = 16384;
  // beams are split into k-ranges below this many threads per CU
  // (dm_integrate_chunks)
  static constexpr int kChunkThreadsPerCu = 512;
  // light tiles with at most this many pieces are sparse work items: walked
  // first, then only their touched cells are loaded (DM_SPARSE_PIECES, read
  // at dm_create: 0 sends every light tile through the dense path, tests)
  int sparse_pieces = 15;

  // cross-band merge workspace (dm_merge.hip), sized nranks * rec_cap
  int64_t m_cap = 0;
  int32_t* m_parent = nullptr;
  long long* m_label = nullptr;
  long long* m_acc = nullptr;     // [m_cap][3] size, sum_x, sum_y
  long long* m_clu = nullptr;     // [m_cap][4] merged records (unsorted)
  dm_cluster* m_out = nullptr;    // [m_cap] merged records, sorted
  unsigned long long* m_cnt = nullptr;    // [4] device: K, flags, sorted, max band K
  unsigned long long* h_mcnt = nullptr;   // pinned mirror
  // [0] workgroups the last accumulation needed (dense items + sparse items
  // / 4), [1] its work items: written by k_tile_accum's workgroup 0 into
  // mapped host memory, read without a wait when the next call is enqueued
  // (a finished earlier call's value; 0 until one finished) to size the
  // accumulation and fmask grids to the work instead of to the capacity
  unsigned long long* h_hint = nullptr;
  unsigned long long* d_hint = nullptr;   // its device address

  // goal selection (dm_goals.hip): the last collected sorted result on the
  // device (a readback slot's out_clu / m_out while that slot's epoch is
  // unchanged), top-T workspaces, robot / index / centroid staging
  int goal_slot = -1, goal_kind = 0;  // kind 1: band frontiers (out_clu), 2: merge (m_out)
  uint64_t goal_epoch = 0, goal_gen = 0;
  int64_t goal_n = 0;
  unsigned long long* goal_k[2] = {nullptr, nullptr};
  uint32_t* goal_i[2] = {nullptr, nullptr};
  int64_t goal_cap = 0;
  double* goal_io = nullptr;          // [4 * 256] robots xy, then centroids xy
  int64_t* goal_idx = nullptr;        // [256]

  // profiling
  bool profile = false;
  std::vector<KernelTimer> pending;
  std::vector<dm_kernel_stat> stats;
};

// Point the current-slot views (out_clu, h_out, h_out_dev, h_out_cap, m_out)
// at readback slot `slot`.
inline void dm_select_slot(dm_grid* g, int slot) {
  const dm_grid::RbSlot& r = g->rb[slot];
  g->cur_slot = slot;
  g->out_clu = r.out_clu;
  g->h_out = r.h_out;
  g->h_out_dev = r.h_out_dev;
  g->h_out_cap = r.h_out_cap;
  g->m_out = r.m_out;
}

// The front-end stream of workspace set `set` and its hand-off words
// (k_seq_signal / k_seq_gate: [kSigWord], [kGateWord] of 16 words per
// stream; the sticky halt word fe_flag[kHaltWord] is shared).
inline hipStream_t dm_fe_stream_of(const dm_grid* g, int set) {
  return g->fe_streams[set % dm_grid::kFeStreams];
}
inline unsigned long long* dm_fe_flag_of(const dm_grid* g, int set) {
  return g->fe_flag + 16 * (set % dm_grid::kFeStreams);
}
// the set (and stream) the next integrate call will use
inline int dm_next_set(const dm_grid* g) { return (g->iw_cur + 1) % dm_grid::kIntSets; }

// Settle the free events owed by the integrate workspaces (their last
// accumulation is enqueued on g->stream before this point): `recorded`, an
// event just recorded on g->stream, or each set's own ev_free recorded now.
inline hipError_t dm_mark_ws_free(dm_grid* g, hipEvent_t recorded = nullptr) {
  for (int i = 0; i < dm_grid::kIntSets; ++i) {
    dm_grid::IntWs& w = g->iw[i];
    if (!w.free_owed) continue;
    w.free_owed = false;
    w.free_wait = recorded ? recorded : w.ev_free;
    if (recorded) continue;
    const hipError_t e = hipEventRecord(w.ev_free, g->stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Point the current-set views (cnt, fsh, big_tiles, fbits,
// edge_slot, slot_parent) at frontier workspace set `s`.
inline void dm_select_fw(dm_grid* g, int s) {
  const dm_grid::FrWs& f = g->fw[s];
  g->cnt = f.cnt;
  g->fsh = f.fsh;
  g->big_tiles = f.big_tiles;
  g->fbits = f.fbits;
  g->edge_slot = f.edge_slot;
  g->slot_parent = f.slot_parent;
}

// Host wait for an event the pipelined caller expects within tens of
// microseconds (a readback slot's pass): poll it instead of
// hipEventSynchronize, which after a short active wait sleeps on an
// interrupt and wakes up tens of microseconds late (the bench's step
// cadence showed +20-80 us spikes on ~10 % of the steps).  After kSpinNs of
// polling it blocks as before: 2 ms, like ShardedMapper._poll's window (a
// pipelined C3 pass ends ~70 us after the host starts waiting; longer waits
// should not keep a host core busy, which several ranks' threads would
// compete for).
inline void dm_cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#elif defined(__aarch64__)
  asm volatile("yield" ::: "memory");
#else
  std::atomic_signal_fence(std::memory_order_seq_cst);
#endif
}

inline hipError_t dm_event_wait(hipEvent_t ev) {
  constexpr long long kSpinNs = 2000000;  // 2 ms
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned it = 0;; ++it) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    if ((it & 63u) == 63u &&
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > kSpinNs)
      return hipEventSynchronize(ev);
    dm_cpu_relax();
  }
}

// Order `stream` after the pass_stream work enqueued so far (the frontier
// arrays other than the parity sets are shared by all passes).
inline hipError_t dm_join_pass_stream(dm_grid* g) {
  if (!g->p_pending) return hipSuccess;
  g->p_pending = false;
  return hipStreamWaitEvent(g->stream, g->p_tail, 0);
}

// A call with too few beams to fill the chip enumerates each beam's pieces
// in `chunks` k-ranges on different threads (k_beam_prep / k_scatter): one
// thread per beam would walk up to 2*nmax/64 pieces serially on a mostly
// idle GPU (sparse scans, 1 cm maps).  Chunks stay >= 64 steps long.
inline int32_t dm_integrate_chunks(const dm_grid* g, int64_t nb) {
  const int64_t want = (int64_t)dm_grid::kChunkThreadsPerCu * (int64_t)(g->n_cu > 0 ? g->n_cu : 256);
  if (nb <= 0 || nb >= want) return 1;
  const int64_t by_len = (g->nmax + 1) / 64 > 1 ? (g->nmax + 1) / 64 : 1;
  const int64_t by_fill = (want + nb - 1) / nb;
  return (int32_t)(by_fill < by_len ? by_fill : by_len);
}


// ---- launchers (dm_integrate.hip / dm_frontier.hip) -----------------------
int dm_launch_integrate(dm_grid* g, int32_t S, const double* d_pose4, int32_t N,
                        const float* d_ranges, const double* d_trig);
int dm_launch_recount(dm_grid* g);
// swap: rebuild into the other list and switch (passes may be in flight);
// otherwise into the current one (every stream joined: bulk writes)
int dm_launch_relist(dm_grid* g, bool swap);
// Passes between rebuilds of the tile list in tile order (dm_launch_relist),
// once the doubling period from a fresh list reaches it.
constexpr int kRelistPasses = 16;
int dm_launch_state_from_logodds(dm_grid* g);
int dm_launch_map_image(dm_grid* g, uint8_t* d_img);
int dm_launch_set_state(dm_grid* g, const int8_t* d_state_in);
// split: the labelling half on g->pass_stream (dm_frontiers_begin with
// overlap); *end_stream receives the stream the pass ends on.
int dm_enqueue_frontiers(dm_grid* g, bool want_mask, bool want_labels, bool split = false,
                         hipStream_t* end_stream = nullptr);
// Hand-off between streams (dm_integrate.hip): k_seq_signal counts
// flag[kSigWord] up; k_seq_gate (one lane) counts flag[kGateWord] up and waits
// until flag[kSigWord] reaches it (+ fault: fault-injection tests), or sets
// err_bit in *err after a bounded time (ticks of the 100 MHz clock, 0: 5 s).
int dm_launch_signal(hipStream_t s, unsigned long long* flag);
int dm_launch_gate(hipStream_t s, unsigned long long* flag, unsigned long long* err, unsigned long long err_bit,
                   unsigned long long ticks = 0, unsigned long long fault = 0);
int dm_launch_edge_labels(dm_grid* g);
int dm_frontiers_readback(dm_grid* g, int64_t* n_clusters, int64_t* copied);
int dm_launch_frontiers(dm_grid* g, bool want_mask, bool want_labels, int64_t* n_clusters,
                        int64_t* copied);
// sums / labels: slot sums (slot_acc) and slot labels when the records were
// written by the fused compaction (-(slot + 1) in place of the size), else
// nullptr.
int dm_launch_rank_sort(hipStream_t stream, long long* clusters, const long long* sums,
                        const long long* labels, const unsigned long long* d_count,
                        int64_t max_records, double ox, double oy, double res, dm_cluster* out,
                        int32_t* rank_of, unsigned long long* d_sorted, const unsigned long long* cnt,
                        int ncnt, int sorted_idx, const unsigned long long* fsh, dm_raw_record* host_out,
                        int64_t host_cap, int64_t expect);
// Listed tiles from which a frontier pass reads fmask instead of state bytes.
constexpr int64_t kFmaskOnTiles = 8192;
// tile_free: the listed flag above the free count (<= 4096)
constexpr int32_t kTileListed = 1 << 30;
constexpr int32_t kTileFreeMask = kTileListed - 1;
// Frontier slots (tile-local components) per map tile allocated at dm_create.
constexpr int64_t kSlotsPerTile = 4;
int dm_grow_bucket_sort(dm_grid* g, int64_t n);
// Row-bucket sort of the raw records (labels of rows [row_base, row_base +
// rows)): same outputs, readback header and flags as dm_launch_rank_sort.
int dm_launch_bucket_sort(dm_grid* g, hipStream_t stream, long long* clusters, const long long* sums,
                          const long long* labels, const unsigned long long* d_count,
                          int64_t max_records, int64_t row_base, int64_t rows, dm_cluster* out,
                          int32_t* rank_of, unsigned long long* d_sorted, const unsigned long long* cnt,
                          int ncnt, int sorted_idx, const unsigned long long* fsh, dm_raw_record* host_out,
                          int64_t host_cap);
// cross-band exchange (dm_merge.hip)
int64_t dm_export_nbytes(int64_t W, int64_t rec_cap);
int dm_launch_export(dm_grid* g, hipStream_t s, void* d_export, int64_t rec_cap);
int dm_launch_merge(dm_grid* g, hipStream_t s, const void* d_gathered, int32_t nranks, int64_t rec_cap,
                    int64_t min_size);
// The stream band exports end on and merges run on (dm_exchange_stream).
inline hipStream_t dm_exchange_stream_of(const dm_grid* g) { return g->overlap ? g->pass_stream : g->stream; }
// goal selection (dm_goals.hip)
int dm_launch_goal_topk(dm_grid* g, const dm_cluster* d_recs, int64_t K, const double* d_robots, int32_t R,
                        int32_t T, int64_t min_size, double w, double min_dist,
                        const unsigned long long** d_k, const uint32_t** d_i);
int dm_launch_goal_gather(dm_grid* g, const dm_cluster* d_recs, const int64_t* d_idx, int32_t R, double* d_xy);
int dm_launch_ld06(dm_grid* g, int32_t S, const dm_ld06_point* d_pts, const int64_t* d_offsets,
                   int32_t N, int dir, float* d_ranges, float* d_intensities);

// sharded parents (dm_sharded.cpp): the public calls dispatch here
int dm_sh_destroy(dm_grid* g);
int dm_sh_reset(dm_grid* g);
int dm_sh_integrate(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges, float amin,
                    float inc, uint64_t* U, uint64_t* T);
int dm_sh_integrate_async(dm_grid* g, int32_t S, const double* poses, int32_t N, const float* ranges,
                          float amin, float inc);
int dm_sh_integrate_device(dm_grid* g, int32_t S, const double* d_pose4, int32_t N, const float* d_ranges,
                           float amin, float inc);
int dm_sh_last_counts(dm_grid* g, uint64_t* U, uint64_t* T);
int dm_sh_last_stats(dm_grid* g, uint64_t* out, int32_t cap, int32_t* n_out);
int dm_sh_get_state(dm_grid* g, int8_t* out);
int dm_sh_get_logodds(dm_grid* g, float* out);
int dm_sh_set_logodds(dm_grid* g, const float* in);
int dm_sh_set_state(dm_grid* g, const int8_t* in);
int dm_sh_frontiers(dm_grid* g, uint8_t* mask, int64_t* labels, dm_cluster* out, int64_t cap, int64_t* n_out);
int dm_sh_frontiers_begin(dm_grid* g);
int dm_sh_frontiers_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out);
int dm_sh_frontiers_poll(dm_grid* g, int32_t* ready);
int dm_sh_assign_goals(dm_grid* g, const double* robots_xy, int32_t n_robots, int64_t min_size, double w,
                       double min_distance, int64_t* out_index, double* out_xy);
int dm_sh_set_overlap(dm_grid* g, int32_t on);
int dm_sh_synchronize(dm_grid* g);
int dm_sh_profile_enable(dm_grid* g, int enable);
int dm_sh_profile_read(dm_grid* g, dm_kernel_stat* out, int32_t cap, int32_t* n_out);
int dm_sh_profile_reset(dm_grid* g);
int dm_sh_map_image(dm_grid* g, uint8_t* out);
int dm_sh_ld06_to_scans(dm_grid* g, int32_t S, const dm_ld06_point* points, const int64_t* offsets, int32_t N,
                        int dir, float* ranges, float* intensities);
int dm_sh_ld06_to_scans_device(dm_grid* g, int32_t S, const dm_ld06_point* d_points, const int64_t* d_offsets,
                               int32_t N, int dir, float* d_ranges, float* d_intensities);

// error plumbing (dm_api.cpp)
int dm_set_error(int code, const char* fmt, ...);
int dm_hip_check(hipError_t e, const char* what);
void dm_timer_begin(dm_grid* g, const char* name, KernelTimer* t, hipStream_t s = nullptr);
void dm_timer_end(dm_grid* g, KernelTimer* t);

#define DM_HIP(call)                                         \
  do {                                                       \
    hipError_t _e = (call);                                  \
    if (_e != hipSuccess) return dm_hip_check(_e, #call);    \
  } while (0)

// Kernel launch.
#define DM_LAUNCH(kernel, grid, block, shmem, stream, ...) \
  hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__)

// Round n up to a quarter-octave step (1, 1.25, 1.5, 1.75 x 2^k; exact below
// 8): grid sizes derived from the last pass's statistics take few values.
inline int64_t dm_quantize_up(int64_t n) {
  if (n <= 8) return n;
  int sh = 0;
  while ((n >> sh) >= 8) ++sh;
  const int64_t step = (int64_t)1 << sh;  // n in [4, 8) x 2^sh: steps of a quarter octave
  return ((n + step - 1) / step) * step;
}
