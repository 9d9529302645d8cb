//! Raw bindings of `include/marshrutka_pf.h` (MR_ABI_VERSION 7) for the reference
//! crate (maratik123/marshrutka).  Every `#[repr(C)]` struct here has the header's
//! field order, sizes and offsets; `tests/test_rust_shim.py` checks that against the
//! header compiled by a C compiler (this image has no Rust toolchain, so this file is
//! not compiled here).
//!
//! Which reference item each entry point replaces is noted at the header's
//! declaration; the one the app needs is `mr_find_path`, the body of
//! `FindPath::eval` (src/pathfinder.rs:199-248, called from src/app.rs:704-731).
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

pub const MR_ABI_VERSION: u32 = 7;

// mr_status
pub const MR_OK: c_int = 0;
pub const MR_NOT_FOUND: c_int = 1;
pub const MR_ERR_INVALID_ARG: c_int = -1;
pub const MR_ERR_INVALID_GRID: c_int = -2;
pub const MR_ERR_INVALID_INDEX: c_int = -3;
pub const MR_ERR_CAPACITY: c_int = -4;
pub const MR_ERR_DEVICE: c_int = -5;
pub const MR_ERR_LIMIT: c_int = -6;
pub const MR_ERR_NO_DEVICE: c_int = -7;

// CellIndex variants (src/index.rs:41-46), Homeland (src/homeland.rs:26-32), Border (src/index.rs:23-28)
pub const MR_CELL_CENTER: u8 = 0;
pub const MR_CELL_HOMELAND: u8 = 1;
pub const MR_CELL_BORDER: u8 = 2;

// PoI (src/grid.rs:24-29)
pub const MR_POI_NONE: u8 = 0;
pub const MR_POI_CAMPFIRE: u8 = 1;
pub const MR_POI_FOUNTAIN: u8 = 2;
pub const MR_POI_FORUM: u8 = 3;

// CostComparator (src/cost.rs:76-81)
pub const MR_SORT_LEGS: u8 = 0;
pub const MR_SORT_TIME: u8 = 1;
pub const MR_SORT_MONEY: u8 = 2;

// AggregatedCost variants in declaration (= Ord) order (src/cost.rs:90-110)
pub const MR_CMD_NO_MOVE: u8 = 0;
pub const MR_CMD_CENTRAL: u8 = 1;
pub const MR_CMD_STANDARD: u8 = 2;
pub const MR_CMD_CARAVAN: u8 = 3;
pub const MR_CMD_SOE: u8 = 4;
pub const MR_CMD_SHQ: u8 = 5;
pub const MR_CMD_SFM: u8 = 6;

#[repr(C)]
#[derive(Copy, Clone, Default, Debug, PartialEq, Eq)]
pub struct mr_cell_index {
    pub kind: u8,
    pub sub: u8,
    pub x: u16,
    pub y: u16,
    pub reserved: u16,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_cell {
    pub index: mr_cell_index,
    pub poi: u8,
    pub reserved: [u8; 7],
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_params {
    pub scroll_of_escape_cost: u32,
    pub scroll_of_escape_hq_cost: u32,
    pub scroll_of_escape_forum_cost: u32,
    pub use_soe: u8,
    pub use_sfm: u8,
    pub use_caravans: u8,
    pub has_hq: u8,
    pub hq_position: mr_cell_index,
    pub route_guru: u32,
    pub fleetfoot: u32,
    pub sort_by: [u8; 2],
    pub homeland: u8,
    pub reserved: u8,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_command {
    pub kind: u8,
    pub reserved: [u8; 3],
    pub legs: u32,
    pub money: u32,
    pub fleetfoot: u32,
    pub time_s: i64,
    pub from: mr_cell_index,
    pub to: mr_cell_index,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_result {
    pub legs: u32,
    pub money: u32,
    pub time_s: i64,
    pub n_commands: u32,
    pub command_offset: u32,
    pub status: i32,
    pub reserved: u32,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_query {
    pub from: mr_cell_index,
    pub to: mr_cell_index,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_plan_stats {
    pub solver: u32,
    pub grid_state_in_lds: u32,
    pub num_sources: u32,
    pub fallback_sources: u32,
    pub num_specials: u32,
    pub num_regions: u32,
    pub hub_workgroups: u32,
    pub sssp_workgroups: u32,
    pub specials_per_lane: u32,
    pub region_boundary_cells: u32,
    pub fill_launch: u32,
    pub lane_sources: u32,
    pub certified_sources: u32,
    pub lanes_per_source: u32,
}

#[repr(C)]
#[derive(Copy, Clone, Default, Debug)]
pub struct mr_label_record {
    pub legs: u32,
    pub money: u32,
    pub time_s: u32,
    pub via: u32,
}

/// Opaque handles.
pub enum mr_grid {}
pub enum mr_plan {}

#[link(name = "marshrutka_pf")]
extern "C" {
    // grid: MapGrid::parse's output (src/grid.rs:31-38), nearest campfires (src/grid.rs:134-230)
    pub fn mr_grid_create(cells: *const mr_cell, n_cells: u32, out: *mut *mut mr_grid) -> c_int;
    pub fn mr_grid_destroy(grid: *mut mr_grid);
    pub fn mr_parse_map_html(html: *const c_char, len: u64, cells: *mut mr_cell, cap: u32, n_cells: *mut u32) -> c_int;
    pub fn mr_parse_error() -> *const c_char;
    pub fn mr_grid_from_html(html: *const c_char, len: u64, out: *mut *mut mr_grid) -> c_int;
    pub fn mr_grid_square_size(grid: *const mr_grid) -> u32;
    pub fn mr_grid_region_table(grid: *mut mr_grid, homeland: u32, out: *mut u32, cap_words: u64, nreg: *mut u32,
                                build_ms: *mut f64) -> c_int;
    pub fn mr_params_default(p: *mut mr_params);

    // FindPath::eval (src/pathfinder.rs:199-248), one query and batches
    pub fn mr_find_path(grid: *const mr_grid, params: *const mr_params, from: mr_cell_index, to: mr_cell_index,
                        out: *mut mr_result, cmds: *mut mr_command, cap: u32) -> c_int;
    pub fn mr_find_path_batch(grid: *const mr_grid, params: *const mr_params, queries: *const mr_query, n: u32,
                              results: *mut mr_result, pool: *mut mr_command, pool_cap: u64) -> c_int;

    // device-resident plans
    pub fn mr_plan_create(grid: *const mr_grid, params: *const mr_params, queries: *const mr_query, n: u32,
                          out: *mut *mut mr_plan) -> c_int;
    pub fn mr_plan_create_ex(grid: *const mr_grid, params: *const mr_params, queries: *const mr_query, n: u32,
                             max_cmds: u32, out: *mut *mut mr_plan) -> c_int;
    pub fn mr_plan_run(plan: *mut mr_plan, stream: *mut c_void) -> c_int;
    pub fn mr_plan_wait(plan: *mut mr_plan, stream: *mut c_void) -> c_int;
    pub fn mr_plan_fetch(plan: *mut mr_plan, results: *mut mr_result, pool: *mut mr_command, pool_cap: u64) -> c_int;
    pub fn mr_plan_device_outputs(plan: *mut mr_plan, d_results: *mut *mut c_void, results_bytes: *mut u64,
                                  d_commands: *mut *mut c_void, commands_bytes: *mut u64) -> c_int;
    pub fn mr_plan_bind_outputs(plan: *mut mr_plan, d_results: *mut c_void, d_commands: *mut c_void) -> c_int;
    pub fn mr_plan_bind_outputs_ex(plan: *mut mr_plan, d_results: *mut c_void, d_commands: *mut c_void,
                                   d_overflow: *mut c_void, overflow_cap: u32) -> c_int;
    pub fn mr_decode_records(grid: *const mr_grid, params: *const mr_params, results: *const c_void,
                             commands: *const c_void, n: u32, max_cmds: u32, overflow: *const c_void,
                             overflow_n: u64, out: *mut mr_result, pool: *mut mr_command, pool_cap: u64) -> c_int;
    pub fn mr_wire_row_bytes(max_cmds: u32) -> u32;
    pub fn mr_plan_wire_records(plan: *mut mr_plan, d_rows: *mut c_void, d_pool: *mut c_void, pool_cap: u32,
                                stream: *mut c_void) -> c_int;
    pub fn mr_decode_wire(grid: *const mr_grid, params: *const mr_params, rows: *const c_void, n: u32, max_cmds: u32,
                          pool: *const c_void, pool_n: u64, out: *mut mr_result, cmds: *mut mr_command,
                          cmd_cap: u64) -> c_int;
    pub fn mr_plan_record_queries(plan: *const mr_plan, query_of_record: *mut u32, n: u32) -> c_int;
    pub fn mr_plan_num_sources(plan: *const mr_plan) -> u32;
    pub fn mr_plan_fallback_sources(plan: *mut mr_plan, out: *mut mr_cell_index, cap: u32, n: *mut u32) -> c_int;
    pub fn mr_plan_handed_over_sources(
        plan: *mut mr_plan,
        out: *mut mr_cell_index,
        certified: *mut u8,
        cap: u32,
        n: *mut u32,
    ) -> c_int;
    pub fn mr_plan_get_stats(plan: *mut mr_plan, out: *mut mr_plan_stats) -> c_int;
    pub fn mr_plan_kernel_ms(plan: *mut mr_plan, n_launches: *mut u32) -> f64;
    pub fn mr_plan_destroy(plan: *mut mr_plan);
    pub fn mr_cache_trim();
    pub fn mr_host_register(p: *mut c_void, bytes: u64) -> c_int;
    pub fn mr_host_unregister(p: *mut c_void) -> c_int;

    // all destinations of each source
    pub fn mr_sssp_plan_create(grid: *const mr_grid, params: *const mr_params, sources: *const mr_cell_index,
                               n_sources: u32, out: *mut *mut mr_plan) -> c_int;
    pub fn mr_plan_fill_ms(plan: *const mr_plan) -> f64;
    pub fn mr_sssp_records(plan: *mut mr_plan, i: u32, out: *mut mr_label_record) -> c_int;
    pub fn mr_sssp_device_records(plan: *mut mr_plan, d_records: *mut *mut c_void, bytes: *mut u64) -> c_int;
    pub fn mr_sssp_record_pitch(plan: *mut mr_plan, cells_per_row: *mut u32) -> c_int;
    pub fn mr_sssp_device_tables(plan: *mut mr_plan, d_tables: *mut *mut c_void, bytes: *mut u64) -> c_int;
    pub fn mr_sssp_label(plan: *mut mr_plan, i: u32, dst: mr_cell_index, out: *mut mr_result, cmds: *mut mr_command,
                         cap: u32) -> c_int;
    pub fn mr_sssp_labels(plan: *mut mr_plan, i: u32, results: *mut mr_result, pool: *mut mr_command,
                          pool_cap: u64) -> c_int;

    // misc
    pub fn mr_abi_version() -> u32;
    pub fn mr_last_error() -> *const c_char;
    pub fn mr_device_available() -> c_int;

    // the app's command table (src/app.rs:481-561)
    pub fn mr_command_time(cmd: *const mr_command) -> i64;
    pub fn mr_duration_display(seconds: i64, buf: *mut c_char, cap: u64) -> c_int;
    pub fn mr_render_schedule(cmds: *const mr_command, n: u32, arrive_at_s: u32, pause_s: u32, buf: *mut c_char,
                              cap: u64, len: *mut u64) -> c_int;
}
