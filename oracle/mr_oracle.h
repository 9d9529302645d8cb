/*
 * mr_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference pathfinder (maratik123/marshrutka,
 * src/pathfinder.rs, src/cost.rs, src/index.rs, src/homeland.rs, src/skill.rs,
 * src/grid.rs, src/cell.rs).  It is the parity checker for the HIP engine and
 * the bench's CPU-baseline leg ("kind": "port").  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it; the product path
 * (libmarshrutka_pf.so) never links or calls it.
 *
 * Parity pinning: the reference is Rust and cannot be built in this image
 * (no rustc/cargo, no vendored crates).  Its own tests pin no
 * path result.  This oracle is pinned by (a) the hand-derived known-answer
 * tests of SURVEY.md §8c (tests/test_oracle_kat.py), (b) an independent
 * pure-Python restatement (oracle/py_ref.py) on small grids, whose outputs are
 * committed as golden vectors under tests/golden/, and (c) the one
 * reference-held fixture on this boundary: Duration Display "1h3m10s"
 * (src/pathfinder.rs:279-285).
 *
 * Same POD types and status codes as include/marshrutka_pf.h; functions carry
 * an `mro_` prefix so both libraries can be loaded in one process.
 */
#ifndef MR_ORACLE_H
#define MR_ORACLE_H
#include "../include/marshrutka_pf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mro_grid mro_grid;

int mro_grid_create(const mr_cell *cells, uint32_t n_cells, mro_grid **out);
void mro_grid_destroy(mro_grid *grid);
/* nearest campfire of `homeland` for row-major cell i (src/grid.rs:134-230);
 * returns 1 and writes *out if present, 0 if None. */
int mro_grid_nearest_campfire(const mro_grid *grid, uint32_t i, uint32_t homeland,
                              mr_cell_index *out);
/* the same by direct Manhattan argmin (key of src/grid.rs:319-323) — used by
 * tests to check that the reference's projection shortcut equals argmin. */
int mro_grid_nearest_campfire_direct(const mro_grid *grid, uint32_t i, uint32_t homeland,
                                     mr_cell_index *out);

int mro_find_path(const mro_grid *grid, const mr_params *params, mr_cell_index from,
                  mr_cell_index to, mr_result *out, mr_command *cmds, uint32_t cap);

/* n queries on `threads` host threads (0 = all hardware threads); each query
 * is an independent FindPath::eval as in the reference.  Commands are written
 * to pool at results[i].command_offset (assigned in query order). */
int mro_find_path_batch(const mro_grid *grid, const mr_params *params, const mr_query *queries,
                        uint32_t n, mr_result *results, mr_command *pool, uint64_t pool_cap,
                        uint32_t threads);

/* time::Duration Display, e.g. 3790 -> "1h3m10s" (pinned by
 * src/pathfinder.rs:279-285).  Returns the length written (< cap). */
int mro_duration_display(int64_t seconds, char *buf, uint32_t cap);

/* The hub solver's SoE region table by one BFS per region over the grid minus the
 * Center (the checker of mr_grid_region_table): region[v] = region index of row-major
 * cell v (0xFFFFFFFF: none), rank[v] = its CellIndex rank; out = S*S x nreg x
 * {distance, rank of the nearest region cell}. */
int mro_region_table_bfs(uint32_t S, const uint32_t *rank, const uint32_t *region, uint32_t nreg, uint32_t *out,
                         uint32_t threads);

#ifdef __cplusplus
}
#endif
#endif
