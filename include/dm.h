/*
 * dm.h — C-ABI of libdm.so: MI355X-native occupancy-grid integration and
 * exploration-frontier extraction (the BASELINE.json north-star hot path).
 *
 * WHAT THIS REPLACES
 *   The reference has no FFI for this path: its boundary is ROS 2 topics.
 *   `/scan` (sensor_msgs/LaserScan, produced by the LD06 driver's
 *   ToLaserscanMessagePublish, pi/src/ldlidar_ros2_ws/install/ldlidar_stl_ros2/
 *   lib/ldlidar_stl_ros2/ldlidar_stl_ros2_node @0x7f853) goes into slam_toolbox
 *   (launched at server/thymio_project/launch/pc_server.launch.py:12-19,
 *   configured by server/thymio_project/config/slam_config.yaml:16-28), which
 *   publishes `/map` (nav_msgs/OccupancyGrid, int8 -1/0/100 row-major) consumed
 *   by ThymioBrain.map_cb (server/thymio_project/thymio_project/main.py:46,80-81)
 *   and get_map_image (main.py:241-279).  Frontier extraction exists nowhere in
 *   the reference; its contract is SURVEY.md §8(a) rows a8-a10.
 *   Each entry point below names the step of that pipeline it takes over.  The
 *   ctypes binding a ROS node would add is shown in INTEGRATION.md.
 *
 * CONVENTIONS
 *   - Every function returns int: DM_OK (0) or a negative DM_ERR_* code; on
 *     error dm_last_error() (thread-local) describes it.  Nothing aborts.
 *   - Host pointers are caller-owned, C-contiguous, borrowed for the call only.
 *   - Functions without a `_device` suffix are synchronous: they return after
 *     their outputs are in host memory.  `_device` functions take device
 *     pointers, enqueue on the handle's stream and return immediately.
 *   - A handle is NOT internally thread-safe (the Python wrapper locks).
 *   - Grid layout: row-major, idx = (cy - band_row0) * width + cx, row 0 at the
 *     map origin (bottom-left), exactly the OccupancyGrid.data layout read by
 *     get_map_image (main.py:256, flipud at :266).
 */
#ifndef DM_H
#define DM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DM_OK 0
#define DM_ERR_INVALID_ARG (-1)
#define DM_ERR_SHAPE (-2)
#define DM_ERR_HIP (-3)
#define DM_ERR_OOM (-4)
#define DM_ERR_CAPACITY (-5)
#define DM_ERR_IO (-6)
#define DM_ERR_STATE (-7)
#define DM_ERR_INCOMPLETE (-8) /* a pass has no result: an export record was incomplete, or a
                                  union-find loop hit its iteration bound */
#define DM_ERR_PIPELINE (-9)   /* a cross-stream hand-off of the overlapped pipeline (dm_set_overlap)
                                  timed out: the map update it guarded was skipped, so the map
                                  misses batches; sticky until dm_reset */
#define DM_ERR_COLLECTIVE (-10) /* a cross-device exchange of a sharded map failed or did not finish
                                  within its timeout (a peer copy of a dm_create_sharded handle; the
                                  RCCL collectives of the multi-process layer, dm/sharded.py);
                                  sticky: the sharded map must be recreated */

/* Tile edge (cells) used by the kernels; band_row0 must be a multiple of it. */
#define DM_TILE 64

/* Map parameters.  Defaults (dm_default_params) come from the reference where
 * it has them: resolution 0.05 (slam_config.yaml:26), max range 12.0
 * (slam_config.yaml:27), LD06 range_min 0.02f (driver rodata 0xbc840).  The
 * log-odds constants are this build's SPEC. */
typedef struct dm_params {
  int64_t width;            /* cells along x (columns), global */
  int64_t height;           /* cells along y (rows), global */
  double resolution;        /* metres per cell */
  double origin_x;          /* world x of the lower-left corner of cell (0,0) */
  double origin_y;          /* world y of the lower-left corner of cell (0,0) */
  float range_min;          /* beams with r < range_min (or NaN) are skipped */
  float range_max;          /* r > range_max: ray truncated there, no hit */
  float l_occ;              /* log-odds added per hit */
  float l_free;             /* log-odds added per miss (negative) */
  float l_min;              /* clamp low */
  float l_max;              /* clamp high */
  float occ_thresh;         /* L >= occ_thresh (and L != 0) -> 100 */
  float free_thresh;        /* L <= free_thresh (and L != 0) -> 0 */
  int64_t min_frontier_size;/* clusters smaller than this are dropped */
  int64_t band_row0;        /* first global row owned by this handle */
  int64_t band_rows;        /* rows owned; 0 means height - band_row0 */
} dm_params;

/* One frontier cluster.  label = min global row-major
 * linear index (cy*width+cx) of the component; sums are over global cell
 * coordinates; cx_m = origin_x + ((double)sum_x/(double)size + 0.5)*resolution. */
typedef struct dm_cluster {
  int64_t label;
  int64_t size;
  int64_t sum_x;
  int64_t sum_y;
  double cx_m;
  double cy_m;
} dm_cluster;

/* Per-kernel timing collected with HIP events when profiling is enabled. */
typedef struct dm_kernel_stat {
  char name[32];
  uint64_t launches;
  double total_ms;
} dm_kernel_stat;

typedef struct dm_grid dm_grid;

/* Fill p with defaults for a width x height map centred on the world origin. */
int dm_default_params(dm_params* p, int64_t width, int64_t height);

/* Create a grid on HIP device `device`: L = 0, state = -1 everywhere.
 * Replaces slam_toolbox's map allocation (grid sized from the scan bounding
 * box on every rebuild upstream; here fixed, device-resident). */
int dm_create(dm_grid** out, const dm_params* p, int device);
int dm_destroy(dm_grid* g);
/* Reset to the empty map (L = 0, state = -1). */
int dm_reset(dm_grid* g);
int dm_get_params(const dm_grid* g, dm_params* out);

/* Integrate S scans of N beams.  poses: [S][3] =
 * (x_m, y_m, yaw_rad) of the laser in the map frame (main.py:202-215 TF chain
 * + pi_hardware.launch.py:26-30 static offset); ranges: [S][N] metres as
 * LaserScan.ranges (NaN = no return); beam i angle = angle_min + i*angle_increment
 * (LaserScan.angle_min / angle_increment).  cos/sin are evaluated on the host
 * with the C library.  out_updates (may be NULL) receives the number of
 * in-band beam-cell updates U; out_touched (may be NULL) the touched cells T.
 * Replaces: slam_toolbox's per-scan ray trace + grid update that produces /map. */
int dm_integrate(dm_grid* g, int32_t S, const double* poses, int32_t N,
                 const float* ranges, float angle_min, float angle_increment,
                 uint64_t* out_updates, uint64_t* out_touched);

/* Asynchronous host-input variant of dm_integrate: the same inputs (host
 * pointers), enqueued and not waited for — the H2D copies of poses and
 * ranges run on the library's streams and, when `ranges` is pinned host
 * memory (hipHostMalloc / torch pin_memory), overlap work in flight (with
 * dm_set_overlap: the previous frontier pass).  `ranges` must stay valid and
 * unchanged until the copy is done: until the second dm_integrate_async call
 * after this one returns, or dm_synchronize / dm_last_counts.  `poses` is
 * read before the call returns.  Read U and T with dm_last_counts.  This is
 * the PCIe-inclusive form of the ROS node's per-scan call. */
int dm_integrate_async(dm_grid* g, int32_t S, const double* poses, int32_t N,
                       const float* ranges, float angle_min, float angle_increment);

/* Device-resident variant (asynchronous on the handle's stream).
 * d_pose4: [S][4] = (x, y, cos(yaw), sin(yaw)) doubles in device memory;
 * d_ranges: [S][N] floats in device memory.  Counters for the call are
 * accumulated on the device; read them with dm_last_counts. */
int dm_integrate_device(dm_grid* g, int32_t S, const double* d_pose4,
                        int32_t N, const float* d_ranges, float angle_min,
                        float angle_increment);
/* U and T of the most recent integrate call (synchronises the stream). */
int dm_last_counts(dm_grid* g, uint64_t* updates, uint64_t* touched);

/* Diagnostics of the most recent calls (synchronises the stream):
 * out[0..6] = integrate: U, T, T applied by the heavy-tile pass, pieces (ray
 * pieces binned by tile), active tiles, apply work items, heavy tiles;
 * out[7..9] = frontiers: tiles visited, tile-local components, clusters;
 * out[10] = integrate: sparse work items (light tiles with at most 15
 * pieces, which load only the cells they touch; counted in out[5] too).
 * *n_out = the number of entries the library has (11); a caller's smaller
 * cap gets the first cap of them. */
int dm_last_stats(dm_grid* g, uint64_t* out, int32_t cap, int32_t* n_out);

/* OccupancyGrid.data for the band: int8[band_rows*width] (-1 / 0 / 100). */
int dm_get_state(dm_grid* g, int8_t* out);
/* Log-odds for the band: float[band_rows*width]. */
int dm_get_logodds(dm_grid* g, float* out);
/* Overwrite L (and derived state / tile summaries) from host floats. */
int dm_set_logodds(dm_grid* g, const float* in);
/* Same as dm_set_logodds but from a host int8 state image: L := +l_occ for
 * 100, l_free for 0, 0 for -1 (testing and map import). */
int dm_set_state(dm_grid* g, const int8_t* in);

/* Frontier extraction: mask (uint8[band_rows*width],
 * may be NULL), labels (int64[band_rows*width], -1 off-frontier, may be NULL),
 * clusters sorted by label (capacity cap).  *n_out receives the number of
 * clusters; if it exceeds cap, DM_ERR_CAPACITY is returned and only cap were
 * written.  For a band, labels are band-local (the min index within the band's
 * part of a component); the sharded layer merges them across bands. */
int dm_frontiers(dm_grid* g, uint8_t* mask, int64_t* labels, dm_cluster* out,
                 int64_t cap, int64_t* n_out);

/* Pipelined frontier passes.  dm_frontiers_begin enqueues a clusters-only
 * frontier pass (the same pipeline as dm_frontiers with mask = labels = NULL)
 * on the handle's stream and returns; dm_frontiers_end waits for THAT pass
 * (an event, not the stream: integrate calls made in between keep running)
 * and returns its clusters exactly as dm_frontiers would have on the map as
 * it was at dm_frontiers_begin.  One pass may be in flight per handle; on
 * DM_ERR_CAPACITY (*n_out = clusters) the pass stays pending, so call _end
 * again with cap >= *n_out.  If
 * the pass overflowed the slot arrays they are grown and DM_ERR_INCOMPLETE
 * is returned with *n_out = 0: that pass has no result (run dm_frontiers).
 * The reference (main.py:123-188) has no frontier step; this is the
 * planner-facing form of SURVEY.md §8 a8-a10 used by a ROS node that keeps
 * integrating scans while the last frontier request completes. */
int dm_frontiers_begin(dm_grid* g);
int dm_frontiers_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out);
/* Non-blocking test of the oldest asynchronous pass (dm_frontiers_begin or
 * dm_merge_bands_begin): *ready = 1 when it has completed (its _end call then
 * returns without waiting), else 0.  DM_ERR_INVALID_ARG if no pass is in
 * flight.  Lets a ROS callback thread publish frontiers without ever
 * blocking on the GPU. */
int dm_frontiers_poll(dm_grid* g, int32_t* ready);
/* The number of asynchronous passes (dm_frontiers_begin /
 * dm_merge_bands_begin) a handle holds in flight: the readback ring's size. */
int dm_max_passes_in_flight(void);

/* Overlap mode (default off).  When on, the integrate front-end of
 * dm_integrate / dm_integrate_device (beam preparation, tile planning, piece
 * scatter: everything that reads poses / ranges and not the map) runs on an
 * internal stream that waits only for the previous integrate call's map
 * update, so it overlaps a frontier pass still in flight on the handle's
 * stream; the map update itself stays in the handle's stream order, after
 * every earlier call.  Results are identical with overlap on or off.  With
 * overlap on, the device inputs of dm_integrate_device must be complete when
 * the call is made (e.g. produced by work the host already synchronised).
 * The streams hand off through bounded device-side waits (5 s); one that
 * times out (a tool that runs one dispatch at a time, e.g. rocprofv3 --pmc,
 * can cause it) skips the map update it guarded and every later call that
 * reads results returns DM_ERR_PIPELINE until dm_reset. */
int dm_set_overlap(dm_grid* g, int32_t on);


/* ---- One map sharded over several devices of this process (SURVEY.md §8(b)
 * "sharded variants: dm_create_sharded(..., int nranks, const int* devices)
 * with the same calls"; §8(e) row bands).  Band r (rows from
 * dm_sharded_band_rows: equal multiples of 64, the last ragged) lives on
 * HIP device devices[r]; a device may repeat (tests run {0, 0, ...} on one
 * GPU).  p covers the whole grid (band_row0 = 0, band_rows = 0).  The handle
 * takes the calls of a dm_create handle — dm_integrate(_async / _device),
 * dm_last_counts / _stats, dm_get_state / _logodds, dm_set_state / _logodds,
 * dm_frontiers (mask and labels are whole-map arrays with global min-index
 * labels), dm_frontiers_begin / _end / _poll, dm_assign_goals,
 * dm_map_image, dm_save / dm_load (the same checkpoint format as one
 * full-map handle), dm_reset, dm_set_overlap, dm_synchronize, dm_profile_*,
 * dm_ld06_to_scans(_device), dm_destroy — with results identical to one
 * dm_create handle of the same params.  Integration sends each band the
 * scans whose max-range disk reaches it; frontier extraction exchanges halo
 * rows and band export records between the devices with peer copies (xGMI)
 * and merges on band 0's device (dm_merge_bands).  The multi-process building
 * blocks below (halos, edge rows / labels, exports, merges, dm_set_stream)
 * return DM_ERR_INVALID_ARG on such a handle.  Replaces: slam_toolbox's
 * single map thread for a map too large (or too many robots) for one GPU;
 * the caller is the ROS node wired at pc_server.launch.py:12-19. */
int dm_create_sharded(dm_grid** out, const dm_params* p, int32_t nranks, const int32_t* devices);
/* The rows [*row0, *row0 + *rows) of band `rank` of `nranks` (the partition
 * of dm_create_sharded and of the multi-process layer, dm/sharded.py). */
int dm_sharded_band_rows(int64_t height, int32_t nranks, int32_t rank, int64_t* row0, int64_t* rows);
/* nranks of a handle (1 for dm_create handles) and the export record
 * capacity its exchange uses now (0 for dm_create handles). */
int dm_sharded_info(const dm_grid* g, int32_t* nranks, int64_t* rec_cap);

/* Sharding support (row bands).  Halo rows are the global
 * rows band_row0-1 (top, "above" = lower row index) and band_row0+band_rows
 * (bottom); NULL = no neighbour there.  Host and device variants. */
int dm_set_halo(dm_grid* g, const int8_t* row_before, const int8_t* row_after);
int dm_set_halo_device(dm_grid* g, const int8_t* d_row_before,
                       const int8_t* d_row_after);
/* Copy the band's first and last state rows (W bytes each). */
int dm_get_edge_rows(dm_grid* g, int8_t* first_row, int8_t* last_row);
int dm_get_edge_rows_device(dm_grid* g, int8_t* d_first_row, int8_t* d_last_row);
/* After dm_frontiers: band-local labels of the first/last rows (int64[W]). */
int dm_get_edge_labels(dm_grid* g, int64_t* first_row, int64_t* last_row);

/* ---- Cross-band frontier exchange, device-resident
 * Replaces the host-side label merge of a row-band sharded map: every band
 * writes an export record into a caller-owned device buffer, the caller
 * all-gathers the records with RCCL (rank order = band order, bands
 * contiguous), and dm_merge_bands resolves labels across band edges and
 * merges the clusters on the device.  Export record (little-endian,
 * dm_export_bytes bytes):
 *   int64 hdr[8]  K (band clusters), flags (0 = complete; bit0 slot overflow,
 *                 bit1 K > rec_cap, bit2 too many clusters to sort on the
 *                 device, bit5 union-find iteration bound hit), band_row0,
 *                 band_rows, width, 0, 0, 0
 *   int32 edge[2][width]  component of each cell of the band's first / last
 *                 row as an index into rec[], -1 off-frontier
 *   int64 rec[rec_cap][4] (label, size, sum_x, sum_y), sorted by label;
 *                 band-local min-index labels, global cell coordinates
 * The band handle must have min_frontier_size <= 1 (the size filter applies
 * to merged clusters: dm_merge_bands' min_size). */
int dm_export_bytes(const dm_grid* g, int64_t rec_cap, int64_t* bytes);
/* Band frontier extraction + export record, asynchronous (no host
 * synchronisation).  Halo rows must be set first.  With dm_set_overlap on,
 * the pass is split as in dm_frontiers_begin: the map reads stay on the
 * handle's stream and the labelling, the sort and the export record run on
 * the handle's exchange stream (dm_exchange_stream), so the next integrate
 * call's map update overlaps them; the caller's all-gather of the record and
 * dm_merge_bands(_begin) then belong on that stream. */
int dm_frontiers_export_device(dm_grid* g, void* d_export, int64_t rec_cap);
/* The hipStream_t the export record of dm_frontiers_export_device is
 * complete on and the merges run on: the handle's stream, or with overlap on
 * its pass stream.  Work ordered after it on that stream (an RCCL all-gather
 * of the record, dm_merge_bands) needs no other synchronisation. */
int dm_exchange_stream(dm_grid* g, void** stream);
/* Merge nranks gathered export records (d_gathered = nranks consecutive
 * records of dm_export_bytes(rec_cap) bytes) into global clusters sorted by
 * label, keeping those with size >= min_size.  Synchronous; runs on
 * dm_exchange_stream, so the gathered buffer must be complete in that
 * stream's order (e.g. all-gathered on it).  Returns
 * DM_ERR_INCOMPLETE (*n_out = largest band K) when a record is flagged
 * incomplete, DM_ERR_CAPACITY (*n_out = clusters) when cap is too small. */
int dm_merge_bands(dm_grid* g, const void* d_gathered, int32_t nranks, int64_t rec_cap,
                   int64_t min_size, dm_cluster* out, int64_t cap, int64_t* n_out);
/* dm_merge_bands split like dm_frontiers_begin / _end: _begin enqueues the
 * merge and returns, _end waits for it (event) and returns its result with
 * dm_merge_bands' error behaviour, except that on DM_ERR_CAPACITY the pass
 * stays pending (call _end again with cap >= *n_out).  d_gathered must stay
 * valid until _end. */
int dm_merge_bands_begin(dm_grid* g, const void* d_gathered, int32_t nranks, int64_t rec_cap,
                         int64_t min_size);
int dm_merge_bands_end(dm_grid* g, dm_cluster* out, int64_t cap, int64_t* n_out);
/* The largest band cluster count K of the last collected merge (every rank
 * merges the same gathered records, so every rank reads the same value: a
 * caller can size rec_cap for the next exports from it consistently). */
int dm_merge_max_band_k(const dm_grid* g, int64_t* max_k);

/* LD06 driver point (ldlidar::PointData fields the LaserScan conversion uses). */
typedef struct dm_ld06_point {
  float angle_deg;      /* 0..360 */
  uint16_t distance_mm;
  uint8_t intensity;
  uint8_t pad;
} dm_ld06_point;

/* LD06 PointData -> LaserScan.ranges/intensities for S revolutions, exactly
 * as the driver's ToLaserscanMessagePublish (ldlidar_stl_ros2_node @0x7f853;
 * SURVEY.md §8 a1): scan s holds points[offsets[s] .. offsets[s+1]), N beams,
 * angle_min 0, angle_increment 6.2831855f/(N-1), NaN = no return, keep the
 * nearest return per beam; laser_scan_dir mirrors the index
 * (pi_hardware.launch.py:20).  ranges_out: float[S][N]; intensities_out may
 * be NULL.  N must be in [2, 8192]. */
int dm_ld06_to_scans(dm_grid* g, int32_t S, const dm_ld06_point* points,
                     const int64_t* offsets, int32_t N, int laser_scan_dir,
                     float* ranges_out, float* intensities_out);
int dm_ld06_to_scans_device(dm_grid* g, int32_t S, const dm_ld06_point* d_points,
                            const int64_t* d_offsets, int32_t N, int laser_scan_dir,
                            float* d_ranges_out, float* d_intensities_out);

/* Checkpoint: raw little-endian {magic, params, float L[band]} . */
int dm_save(dm_grid* g, const char* path);
int dm_load(dm_grid* g, const char* path);

/* Streams and profiling. stream is a hipStream_t (NULL = library's own). */
int dm_set_stream(dm_grid* g, void* stream);
int dm_synchronize(dm_grid* g);
int dm_profile_enable(dm_grid* g, int enable);
int dm_profile_read(dm_grid* g, dm_kernel_stat* out, int32_t cap, int32_t* n_out);
int dm_profile_reset(dm_grid* g);

/* PNG-ready grayscale image of the band's state (f2, main.py:256-266):
 * 0 -> 255, 100 -> 0, anything else -> 127, rows flipped (flipud).
 * out: uint8[band_rows*width]. */
int dm_map_image(dm_grid* g, uint8_t* out);

/* Frontier goals for n_robots robots (replaces the
 * reactive IR / LiDAR policy, server/thymio_project/thymio_project/main.py:
 * 123-188, with map-based exploration).  Over the clusters of the last
 * collected result (dm_frontiers, dm_frontiers_end or dm_merge_bands; on the
 * device), robot r at robots_xy[2r], [2r+1] (metres) scores cluster c:
 *   dist = sqrt(dx*dx + dy*dy), dx = cx_m - x, dy = cy_m - y
 *   util = size / (1 + distance_weight * dist)   (double, no FMA)
 * over clusters with size >= min_size and dist >= min_distance, best util
 * first, ties to the smaller label; robots choose in order, each skipping the
 * clusters earlier robots took.  out_index[r] = index into that result's
 * label-sorted list (-1: none), out_xy[2r], [2r+1] = its centroid (NaN if
 * none).  n_robots <= 256; distance_weight >= 0 (DM_ERR_INVALID_ARG otherwise).
 * DM_ERR_INVALID_ARG if no result is on the device
 * (none collected yet, or a later pass reused its readback slot). */
int dm_assign_goals(dm_grid* g, const double* robots_xy, int32_t n_robots, int64_t min_size,
                    double distance_weight, double min_distance, int64_t* out_index, double* out_xy);

/* Measured uncontended atomic throughput of HIP device `device` (the
 * north star's "atomic throughput against MI355X peak": no vendor figure
 * exists for integer atomics, so the peak is measured in-harness,
 * csrc/dm_probe.hip).  out[0] = LDS ds_add_u32 per second (every lane its own
 * bank: the form k_tile_accum's per-cell counts take), out[1] = global
 * no-return atomicAdd u32 per second (256 contiguous bytes per wave
 * instruction, rows over a 256 MiB buffer: the heavy tiles' slab adds).
 * Runs a few milliseconds of probe kernels on a private stream. */
int dm_atomic_peak(int device, double* out, int32_t cap, int32_t* n_out);

const char* dm_last_error(void);
const char* dm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DM_H */
