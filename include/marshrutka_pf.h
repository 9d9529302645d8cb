/*
 * marshrutka_pf.h — C ABI of the MI355X-native grid shortest-path engine.
 *
 * This is the drop-in boundary for marshrutka's pathfinder hot path
 * (SURVEY.md §8b).  In the reference the path is a crate-private Rust API:
 *
 *   pub struct FindPath<'a> { .. }                 src/pathfinder.rs:183-196
 *   pub fn eval(self, from, to) -> Option<TotalCost>  src/pathfinder.rs:199-248
 *   fn MapGrid::parse(&str) -> Result<MapGrid>       src/grid.rs:47-237
 *
 * Every entry point below names the reference item it replaces.  Types are
 * plain C PODs (no torch / HIP types in any signature) so a Rust `extern "C"`
 * block, ctypes or a C++ caller can bind them directly.
 *
 * Conventions
 *  - All functions return an int status (mr_status); they never abort.
 *  - The caller owns every buffer it passes in.
 *  - A grid handle is immutable after creation; concurrent queries on one
 *    grid from several host threads are safe.
 *  - Widths: the reference stores homeland positions / border shifts in u8
 *    and cell coordinates in i8 (src/index.rs:35-46, src/cell.rs:33-34), which
 *    caps the grid at odd S <= 255.  This ABI widens them to u16 so the
 *    BASELINE sizes (S = 1025, 4097) are representable; for S <= 255 every
 *    result is identical to the reference's.
 */
#ifndef MARSHRUTKA_PF_H
#define MARSHRUTKA_PF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MR_ABI_VERSION 7u

/* ---- status codes ------------------------------------------------------ */
typedef enum mr_status {
    MR_OK = 0,
    MR_NOT_FOUND = 1,          /* eval() returned None (src/pathfinder.rs:247) */
    MR_ERR_INVALID_ARG = -1,   /* null pointer, bad enum value, ...            */
    MR_ERR_INVALID_GRID = -2,  /* MapGrid::parse would fail (src/grid.rs:60-133) or
                                  the cell labels are not a consistent 4-grid     */
    MR_ERR_INVALID_INDEX = -3, /* a CellIndex that is not in the grid; the
                                  reference panics here (src/grid.rs:288-290)    */
    MR_ERR_CAPACITY = -4,      /* caller's command buffer too small; n written   */
    MR_ERR_DEVICE = -5,        /* HIP runtime error                              */
    MR_ERR_LIMIT = -6,         /* grid or label exceeds an engine limit           */
    MR_ERR_NO_DEVICE = -7      /* no gfx950 device visible: the engine has no CPU
                                  fallback and fails loudly                       */
} mr_status;

/* ---- vertex naming (src/index.rs:23-46, src/homeland.rs:26-32) ---------- */
enum { MR_CELL_CENTER = 0, MR_CELL_HOMELAND = 1, MR_CELL_BORDER = 2 };
enum { MR_HOMELAND_BLUE = 0, MR_HOMELAND_RED = 1, MR_HOMELAND_GREEN = 2, MR_HOMELAND_YELLOW = 3 };
enum { MR_BORDER_BR = 0, MR_BORDER_RG = 1, MR_BORDER_GY = 2, MR_BORDER_YB = 3 };

/* CellIndex (src/index.rs:41-46).  kind = MR_CELL_*;
 *   CENTER:   sub = x = y = 0
 *   HOMELAND: sub = homeland, x/y = Pos{x,y} (both >= 1 once canonical)
 *   BORDER:   sub = border, x = shift (>= 1), y = 0
 * Field order gives the derived Ord of the reference (variant, then fields). */
typedef struct mr_cell_index {
    uint8_t kind;
    uint8_t sub;
    uint16_t x;
    uint16_t y;
    uint16_t reserved; /* must be 0 */
} mr_cell_index;

/* ---- grid construction (replaces MapGrid::parse's output, src/grid.rs:31-38) */
enum { MR_POI_NONE = 0, MR_POI_CAMPFIRE = 1, MR_POI_FOUNTAIN = 2, MR_POI_FORUM = 3 };

/* One map cell.  Cells are passed row-major exactly as MapGrid::parse scans
 * them (src/grid.rs:64-77): cell i sits at x = i % S - S/2, y = i / S - S/2. */
typedef struct mr_cell {
    mr_cell_index index;
    uint8_t poi;          /* MR_POI_*  (src/cell.rs:192-201) */
    uint8_t reserved[7];
} mr_cell;

typedef struct mr_grid mr_grid; /* opaque, immutable */

/* Builds the grid and its per-cell precompute (nearest campfire per homeland,
 * src/grid.rs:134-230,297-325).  n_cells must be S*S for odd S.
 * Errors: MR_ERR_INVALID_GRID for the reference's parse errors (not square,
 * Center missing / not at (0,0)) and for cell labels whose index adjacency
 * (src/pathfinder.rs:24-138) is not the geometric 4-neighbourhood. */
int mr_grid_create(const mr_cell *cells, uint32_t n_cells, mr_grid **out);
void mr_grid_destroy(mr_grid *grid);

/* MapGrid::parse (src/grid.rs:47-133): the reference's HTML map format
 * (class "map-grid" > "map-cell" children with corner texts and a centre emoji)
 * into row-major cells.  *n_cells receives the cell count; MR_ERR_CAPACITY if cap
 * is smaller (nothing written).  MR_ERR_INVALID_GRID for the reference's parse
 * errors: no map-grid, not square, a bad background-color, an unindexable cell,
 * Center missing or not at (0,0) (mr_parse_error() names it).  Host only. */
int mr_parse_map_html(const char *html, uint64_t len, mr_cell *cells, uint32_t cap, uint32_t *n_cells);
const char *mr_parse_error(void);
/* mr_parse_map_html + mr_grid_create. */
int mr_grid_from_html(const char *html, uint64_t len, mr_grid **out);
/* MapGrid::square_size / homeland_size (src/grid.rs:280-282) */
uint32_t mr_grid_square_size(const mr_grid *grid);
/* The grid's Scroll-of-Escape region table of `homeland` (grid preprocessing, the
 * analogue of MapGrid::parse's nearest-campfire pass, src/grid.rs:134-230,297-325):
 * the regions are the homeland's campfires in CellIndex order, a cell belongs to the
 * region of its nearest campfire (the Center to none), and for every row-major cell v
 * and region r the table holds {distance, rank} of the nearest cell of r: walk distance
 * on the 4-grid without the Center, ties by the cell's CellIndex rank; {0xFFFFFFFF,
 * 0xFFFFFFFF} for the Center.  Built on the current device on first use (by this call or
 * by a hub plan's creation) and shared by the grid's plans.  *nreg = regions; *build_ms =
 * the build's wall time in ms (upload of the cells' regions and the device passes).
 * With out != NULL copies the V x nreg x 2 words (cap_words must hold them, else
 * MR_ERR_CAPACITY).  MR_ERR_NO_DEVICE without a gfx950 device; no reference counterpart. */
int mr_grid_region_table(mr_grid *grid, uint32_t homeland, uint32_t *out, uint64_t cap_words, uint32_t *nreg,
                         double *build_ms);

/* ---- query parameters: every FindPath field (src/pathfinder.rs:183-196) -- */
enum { MR_SORT_LEGS = 0, MR_SORT_TIME = 1, MR_SORT_MONEY = 2 }; /* CostComparator, src/cost.rs:76-81 */

typedef struct mr_params {
    uint32_t scroll_of_escape_cost;        /* SoE money  */
    uint32_t scroll_of_escape_hq_cost;     /* SHQ money  */
    uint32_t scroll_of_escape_forum_cost;  /* SFm money  */
    uint8_t use_soe;
    uint8_t use_sfm;
    uint8_t use_caravans;
    uint8_t has_hq;                        /* hq_position: Option<CellIndex> */
    mr_cell_index hq_position;
    uint32_t route_guru;                   /* RouteGuru(u32); >5 behaves as 0 (src/skill.rs:21-30) */
    uint32_t fleetfoot;                    /* Fleetfoot(u32); >3 behaves as 0 */
    uint8_t sort_by[2];                    /* (CostComparator, CostComparator) */
    uint8_t homeland;                      /* MR_HOMELAND_* */
    uint8_t reserved;
} mr_params;

/* The app's defaults (src/app.rs:782-811, update_path :704-731):
 * sort (Legs, Money); SoE 50, SHQ 75, SFm 100; use_soe, use_caravans; no HQ;
 * skills 0; homeland Blue. */
void mr_params_default(mr_params *p);

/* ---- results (TotalCost / Command, src/cost.rs:83-206) ------------------ */
enum {
    MR_CMD_NO_MOVE = 0, MR_CMD_CENTRAL = 1, MR_CMD_STANDARD = 2, MR_CMD_CARAVAN = 3,
    MR_CMD_SOE = 4, MR_CMD_SHQ = 5, MR_CMD_SFM = 6
}; /* AggregatedCost variants in declaration (= Ord) order, src/cost.rs:90-110 */

/* Command { aggregated_cost, from, to }.  Only the fields of the variant are
 * meaningful, the rest are 0:  CENTRAL{time}; STANDARD{time(raw, before the
 * Fleetfoot ceil), legs, fleetfoot}; CARAVAN{time, money}; SOE/SHQ/SFM{money}. */
typedef struct mr_command {
    uint8_t kind;
    uint8_t reserved[3];
    uint32_t legs;
    uint32_t money;
    uint32_t fleetfoot;
    int64_t time_s;
    mr_cell_index from;
    mr_cell_index to;
} mr_command;

/* TotalCost { legs, money, time, commands }.  status is the per-query
 * mr_status (MR_OK, MR_NOT_FOUND, MR_ERR_INVALID_INDEX, MR_ERR_CAPACITY). */
typedef struct mr_result {
    uint32_t legs;
    uint32_t money;
    int64_t time_s;
    uint32_t n_commands;
    uint32_t command_offset; /* into the batch's command pool */
    int32_t status;
    uint32_t reserved;
} mr_result;

typedef struct mr_query {
    mr_cell_index from;
    mr_cell_index to;
} mr_query;

/* ---- single query: FindPath { params.., grid }.eval(from, to) ------------
 * Replaces src/pathfinder.rs:199-248.  Writes the label into *out and up to
 * cap commands into cmds.  Returns MR_OK, MR_NOT_FOUND (None), or an error;
 * MR_ERR_CAPACITY means out->n_commands > cap (nothing truncated silently). */
int mr_find_path(const mr_grid *grid, const mr_params *params, mr_cell_index from,
                 mr_cell_index to, mr_result *out, mr_command *cmds, uint32_t cap);

/* ---- batched queries (the GPU hot path) ---------------------------------
 * Answers n independent (from,to) queries.  Queries sharing a source share one
 * single-source solve on the device.  results[i].command_offset indexes pool;
 * the call returns MR_ERR_CAPACITY if pool_cap is smaller than the total number
 * of commands (results[] are still filled so the caller can size the pool). */
int mr_find_path_batch(const mr_grid *grid, const mr_params *params, const mr_query *queries,
                       uint32_t n, mr_result *results, mr_command *pool, uint64_t pool_cap);

/* ---- device-resident plans (bench / multi-GPU) -------------------------- */
typedef struct mr_plan mr_plan;

/* Uploads the grid and the query batch to the current HIP device and groups
 * queries by source.  Inputs stay resident in HBM across mr_plan_run calls. */
int mr_plan_create(const mr_grid *grid, const mr_params *params, const mr_query *queries,
                   uint32_t n, mr_plan **out);
/* The same with `max_cmds` (1..4096) command slots per query in the compact
 * device output (mr_plan_create: 16).  A label with more commands goes to the
 * plan's overflow pool (8 commands per query) and mr_plan_fetch returns it in
 * full; only when that pool is exhausted does it report MR_ERR_CAPACITY. */
int mr_plan_create_ex(const mr_grid *grid, const mr_params *params, const mr_query *queries,
                      uint32_t n, uint32_t max_cmds, mr_plan **out);
/* Enqueues one full pass of the hot path on `stream` (a hipStream_t, or NULL
 * for the plan's own stream).  Asynchronous.  The passes of one plan execute in
 * the order they were enqueued even when they are given different streams (a pass
 * on a new stream first waits for the previous pass to end). */
int mr_plan_run(mr_plan *plan, void *stream);
/* Ordering for consumers of the device outputs: makes `stream` wait (without
 * blocking the host) until every pass enqueued so far has finished; with stream
 * NULL the calling thread waits instead. */
int mr_plan_wait(mr_plan *plan, void *stream);
/* Waits for the plan's work and copies results/commands to host buffers. */
int mr_plan_fetch(mr_plan *plan, mr_result *results, mr_command *pool, uint64_t pool_cap);
/* Device pointers of the compact per-query output records (for an RCCL
 * gather): n * 16 B result records and n * max_cmds * 16 B command slots.
 * Records are in grouped order (queries grouped by source, so each source's
 * records are contiguous); mr_plan_record_queries maps record k to its query.
 * A label longer than max_cmds keeps {0xFFFFFFFF, offset, count} in its first
 * slot and its commands in the plan's own overflow pool.  The call waits for the
 * passes enqueued so far, so the words behind the pointers are whole when it
 * returns; a later mr_plan_run rewrites them (order a reader on another stream with
 * mr_plan_wait). */
int mr_plan_device_outputs(mr_plan *plan, void **d_results, uint64_t *results_bytes,
                           void **d_commands, uint64_t *commands_bytes);
/* Makes subsequent mr_plan_run calls write their compact outputs into caller
 * device buffers (e.g. torch tensors that an RCCL collective then gathers)
 * instead of the plan's own.  Sizes as reported by mr_plan_device_outputs;
 * the caller keeps the buffers alive while the plan uses them. */
int mr_plan_bind_outputs(mr_plan *plan, void *d_results, void *d_commands);
/* The same, and the overflow pool too: a label longer than max_cmds then keeps
 * its commands at d_overflow (overflow_cap commands of 16 B), so that one
 * collective over one caller buffer moves every record of a pass with all its
 * commands.  overflow_cap 0 keeps the plan's own pool (d_overflow is then ignored);
 * a non-zero overflow_cap needs a d_overflow. */
int mr_plan_bind_outputs_ex(mr_plan *plan, void *d_results, void *d_commands, void *d_overflow,
                            uint32_t overflow_cap);
/* Host-side decoding of compact records as mr_plan_device_outputs lays them out
 * (e.g. gathered from another rank's plan over the same grid and params): record
 * k -> out[k] and its commands at pool[out[k].command_offset ..].  `overflow`
 * holds the overflow pool the records' tags point into (overflow_n commands).
 * MR_OK; a per-record status in out[k].status; MR_ERR_CAPACITY if pool_cap is too
 * small; MR_ERR_DEVICE for a record that is not well formed.  Needs no device. */
int mr_decode_records(const mr_grid *grid, const mr_params *params, const void *results, const void *commands,
                      uint32_t n, uint32_t max_cmds, const void *overflow, uint64_t overflow_n,
                      mr_result *out, mr_command *pool, uint64_t pool_cap);
/* Wire records: the plan's last pass re-encoded on the device for a gather, in record
 * order, mr_wire_row_bytes(max_cmds) = 4 + 8 * max_cmds bytes per query (36 B at
 * max_cmds 4, against 80 B of mr_plan_device_outputs): the first command's `from` cell and
 * the command count (or the status) in one word, then {kind|payload, `to` cell} per command.
 * The metrics and the other `from` cells are left out: mr_decode_wire recomputes them from
 * the commands exactly (TotalCost::add_assign, src/cost.rs:299-313; a command starts where
 * the previous one ended, src/pathfinder.rs:223-234).  A label longer than max_cmds has its
 * commands at d_pool (8 B each, pool_cap commands); one that does not fit reads
 * MR_ERR_CAPACITY.  Enqueued on `stream` (null: the plan's) after the plan's last pass;
 * rows and pool are rewritten by the next call.  Needs a grid of at most 2^25 cells.
 * No reference counterpart (the reference returns labels in process). */
uint32_t mr_wire_row_bytes(uint32_t max_cmds);
int mr_plan_wire_records(mr_plan *plan, void *d_rows, void *d_pool, uint32_t pool_cap, void *stream);
/* Host decoding of n wire rows (and their pool of pool_n commands) over the same grid
 * and params: out[k] and its commands at cmds[out[k].command_offset ..], exactly what
 * mr_decode_records gives for the same records.  MR_ERR_CAPACITY if cmd_cap is too small;
 * MR_ERR_DEVICE for a row that is not well formed.  Needs no device. */
int mr_decode_wire(const mr_grid *grid, const mr_params *params, const void *rows, uint32_t n, uint32_t max_cmds,
                   const void *pool, uint64_t pool_n, mr_result *out, mr_command *cmds, uint64_t cmd_cap);
/* query_of_record[k] = the input query whose output is record k of
 * mr_plan_device_outputs (0xFFFFFFFF past the valid queries), k < n. */
int mr_plan_record_queries(const mr_plan *plan, uint32_t *query_of_record, uint32_t n);
/* Number of unique sources (= single-source solves per pass). */
uint32_t mr_plan_num_sources(const mr_plan *plan);
/* The sources the last pass solved with the SSSP kernel (closed form not certain and
 * not certified from a certificate slot; each costs one full single-source search), in
 * source order: up to cap source cells into out, their count in *n.  Sources the
 * certificate answered are left out (they cost no search; mr_plan_stats counts them).
 * Waits for the plan's passes.  A cost signal for balancing sources over ranks
 * (marshrutka_amd/shard.py SourceCosts); no reference counterpart. */
int mr_plan_fallback_sources(mr_plan *plan, mr_cell_index *out, uint32_t cap, uint32_t *n);
/* Every source the hub handed over in the last pass (its closed form not certain), in
 * source order, whichever path then answered it: certified[k] = 1 for one the
 * fixed-point certificate answered from its slot, 0 for one the SSSP kernel solved.  Up
 * to cap entries into out / certified (either may be NULL), their count in *n.  Waits for
 * the plan's passes (tests, diagnostics). */
int mr_plan_handed_over_sources(mr_plan *plan, mr_cell_index *out, uint8_t *certified, uint32_t cap, uint32_t *n);

/* Which solver a plan runs and how the last pass went (diagnostics, bench). */
enum {
    MR_SOLVER_BUCKETED = 0, /* SSSP kernel, bucketed settling (any comparator) */
    MR_SOLVER_LEVELS = 1,   /* SSSP kernel, level-synchronous (Legs-first comparator) */
    MR_SOLVER_HUB = 2,      /* closed-form hub solver (linear run time) + SSSP fallback */
    MR_SOLVER_HUB_WIDE = 3  /* the same for 64..511 specials or no vertex x region table */
};
typedef struct mr_plan_stats {
    uint32_t solver;            /* MR_SOLVER_* */
    uint32_t grid_state_in_lds; /* SSSP kernel: 1 grid state in LDS, 0 in HBM slots */
    uint32_t num_sources;       /* unique sources per pass */
    uint32_t fallback_sources;  /* hub solver: sources re-solved by the SSSP kernel in the last pass */
    uint32_t num_specials;      /* Center, border-1 cells, campfires, HQ */
    uint32_t num_regions;       /* hub solver: Scroll-of-Escape regions of the homeland */
    uint32_t hub_workgroups;    /* hub launch size (4 waves each) */
    uint32_t sssp_workgroups;   /* SSSP launch size */
    uint32_t specials_per_lane; /* hub solver: table entries each lane owns (1 = one per lane) */
    uint32_t region_boundary_cells; /* MR_SOLVER_HUB_WIDE: cells scanned for each source's region row */
    uint32_t fill_launch;       /* all-destinations hub plans: MR_FILL_* (how the fill is launched) */
    uint32_t lane_sources;      /* hub solver: sources solved one per lane (hub_lane_kernel); the rest
                                   (more than 32 queries each) a lane per query (ABI 5).  With
                                   Fleetfoot 1..3 a source the lane or group kernel cannot certify
                                   goes to hub_kernel in the same pass, and counts in
                                   fallback_sources only if hub_kernel cannot certify it either */
    uint32_t certified_sources; /* of fallback_sources, those answered by the fixed-point certificate
                                   in the last pass (the rest ran the SSSP kernel; ABI 6) */
    uint32_t lanes_per_source;  /* hub solver: lanes that share one source's Dijkstra over the
                                   specials: 1 hub_lane_kernel, 8, 16 or 32 hub_group_kernel (by
                                   plan size, or MR_HUB_GROUP), 0 hub_kernel
                                   and the others (ABI 7) */
} mr_plan_stats;
enum {
    MR_FILL_NONE = 0,    /* not an all-destinations hub plan */
    MR_FILL_SERIAL = 1,  /* specials' solve, then the fill, on `stream` */
    MR_FILL_STREAMS = 2, /* the specials' solve on a stream of the plan's own, beside the previous fill */
    MR_FILL_FUSED = 3    /* one launch per pass: the fill + the next pass's specials' solve */
};
/* Fills *out; waits for the plan's stream.  MR_OK or MR_ERR_INVALID_ARG. */
int mr_plan_get_stats(mr_plan *plan, mr_plan_stats *out);
/* Average device time (ms) of the main solve kernel over the last
 * mr_plan_run calls since the previous call to this function, measured with
 * HIP events on the stream the kernel is launched on. */
double mr_plan_kernel_ms(mr_plan *plan, uint32_t *n_launches);
/* Frees the device blocks the engine keeps for reuse by later plans (plan buffers go
 * back to a per-device cache of up to 16 GiB when a plan is destroyed, so creating the
 * next plan needs no hipMalloc).  Blocks of live plans are untouched; safe at any time.
 * mr_grid_destroy trims too, and a failing device allocation trims and retries once.
 * It also releases the host arrays kept for the next plans' grouping (at most 256 MiB
 * per element type) and every calling thread's grouping scratch (about 20 B per query of
 * that thread's largest batch; a plan being created keeps its own until it returns). */
void mr_cache_trim(void);
/* Page-locks [p, p + bytes) of caller memory (hipHostRegister) that mr_plan_fetch then
 * fills by direct DMA instead of through the engine's pinned stage and a host copy: for
 * a caller that reuses its fetch buffers batch after batch.  mr_host_unregister(p)
 * before the memory is freed.  MR_ERR_INVALID_ARG on a null or empty range,
 * MR_ERR_DEVICE when the runtime refuses. */
int mr_host_register(void *p, uint64_t bytes);
int mr_host_unregister(void *p);
/* Waits for the plan's passes and frees it.  Device pointers the plan handed out
 * (mr_plan_device_outputs, mr_sssp_device_records / _tables) are invalid afterwards:
 * their memory may back the next plan's buffers, so a reader on another stream must
 * have finished before this call (mr_plan_wait orders it). */
void mr_plan_destroy(mr_plan *plan);

/* ---- all destinations (single source -> every cell) ------- */
/* One record per (source, cell): the label's metrics and how to rebuild it
 * (mr_sssp_records expands them on the host from the device's cell words). */
typedef struct mr_label_record {
    uint32_t legs, money, time_s;
    uint32_t via; /* boundary table entry of the final walk; 0x80000000 | t = special t's own
                     label; 0xFFFFFFFF = the source */
} mr_label_record;
/* A plan answering every destination of each source: mr_plan_run computes
 * n_sources x V cell words on the device; mr_plan_kernel_ms / mr_plan_get_stats /
 * mr_plan_destroy apply.  Sources may repeat (they share a solve).  Each pass's
 * specials' solve runs inside the previous pass's fill launch, into one of two
 * internal table slots (the first pass solves its own first; MR_FILL_FUSED=0: on a
 * stream of the plan's own beside the previous fill; MR_FILL_OVERLAP=0: one slot,
 * all on `stream`); the records themselves are only written by work on `stream`, so
 * a pass's records are complete once `stream` has reached the end of its run. */
int mr_sssp_plan_create(const mr_grid *grid, const mr_params *params, const mr_cell_index *sources,
                        uint32_t n_sources, mr_plan **out);
/* All-destinations plans: the fill launch's average time (ms) over the window the
 * last mr_plan_kernel_ms call closed (HIP events on the plan's stream). */
double mr_plan_fill_ms(const mr_plan *plan);
/* The V records of the caller's source i, in row-major cell order (waits for the plan). */
int mr_sssp_records(mr_plan *plan, uint32_t i, mr_label_record *out);
/* Device pointer to all cell words and their size: [plan source][row y][pitch], 4 B
 * each, cell (x, y) of a source's grid at word y * pitch + x, rows padded to
 * mr_sssp_record_pitch cells (a multiple of 32: the fill stores whole aligned
 * 128 B lines; pad words are unspecified).  A cell word carries the whole
 * label over its source's table:
 *   b << 20 | k     the walk of k legs from boundary table entry b (0 = the source):
 *                   metrics = entry b's + (k, 0, Fleetfoot-ceil(180 k)), commands =
 *                   entry b's chain ++ [StandardMove{k} b -> cell]
 *   0x80000000 | t  special t's own table label;  0xFFFFFFFF  the source
 * Plan sources are the caller's distinct sources in row-major cell order.  Waits for
 * the passes enqueued so far (the words are whole when it returns); the next
 * mr_plan_run rewrites them (mr_plan_wait orders a reader on another stream). */
int mr_sssp_device_records(mr_plan *plan, void **d_records, uint64_t *bytes);
/* Cell words per row of the device records (S rounded up to a multiple of 32). */
int mr_sssp_record_pitch(mr_plan *plan, uint32_t *cells_per_row);
/* Device pointer to the label tables ([plan source][NS + 1 entries], 28 B each:
 * u32 legs, money, time; u32 meta = length (16 b) | parent entry (10 b) << 16 |
 * state (2 b) << 26 | (tail count - 1) << 31; u32 kp0; u32 from0; u32 u) and their
 * size.  An entry's label is its parent's commands, then {kp0, from0, u} and,
 * with two tail commands, {Scroll of Escape, cell u, the entry's own cell} (from0 =
 * the parent's cell); kp0 =
 * kind << 29 | payload (Standard: legs; Central: moves; Caravan: distance << 1 |
 * coefficient 5), cells by rank in CellIndex order.  Waits for the passes enqueued so
 * far.  The pointer names the latest pass's table slot: it is valid until the next
 * mr_plan_run (passes rotate through slots, and a pass solves the next pass's tables
 * into another slot), so call this again after every run. */
int mr_sssp_device_tables(mr_plan *plan, void **d_tables, uint64_t *bytes);
/* The full label (FindPath::eval(sources[i], dst)) rebuilt from its record:
 * MR_OK, MR_ERR_CAPACITY (out->n_commands > cap) or an error. */
int mr_sssp_label(mr_plan *plan, uint32_t i, mr_cell_index dst, mr_result *out, mr_command *cmds, uint32_t cap);
/* Every destination's full label from the caller's source i (mr_sssp_label for all V
 * cells at once, the all-destinations analogue of mr_plan_fetch): results[v] for
 * row-major cell v, commands at pool[results[v].command_offset ..].  Waits for the
 * plan.  MR_OK, MR_ERR_CAPACITY if pool_cap is too small (results[] are still filled,
 * so the caller can size the pool), or an error. */
int mr_sssp_labels(mr_plan *plan, uint32_t i, mr_result *results, mr_command *pool, uint64_t pool_cap);

/* ---- misc ---------------------------------------------------------------- */
uint32_t mr_abi_version(void);
/* Human-readable description of the last error on this thread. */
const char *mr_last_error(void);
/* 1 if a gfx950 device is visible to this process. */
int mr_device_available(void);

/* ---- the app's command table for a path (src/app.rs:481-561) ----------- */
/* AggregatedCost::time of one command (src/cost.rs:118-150): a StandardMove's
 * raw run time with Fleetfoot's ceil applied for levels 1..3. */
int64_t mr_command_time(const mr_command *cmd);
/* time 0.3 Duration Display ("1h3m10s", "0s"; src/pathfinder.rs:279-285). */
int mr_duration_display(int64_t seconds, char *buf, uint64_t cap);
/* One line per command (NoMove skipped), tab-separated:
 *   "<bot command>\t<duration>\t<running total>\t<start hh:mm:ss>\n"
 * e.g. "/go_direct_b_2_2", "/car_0_0", "/use_soe".  The total adds pause_s per
 * command; starts are back-scheduled from arrive_at_s (seconds after midnight,
 * < 86400), wrapping at midnight.  *len = text length; MR_ERR_CAPACITY if
 * cap <= *len (then nothing is written). */
int mr_render_schedule(const mr_command *cmds, uint32_t n, uint32_t arrive_at_s, uint32_t pause_s, char *buf,
                       uint64_t cap, uint64_t *len);

#ifdef __cplusplus
}
#endif
#endif /* MARSHRUTKA_PF_H */
