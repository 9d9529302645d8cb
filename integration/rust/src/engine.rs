//! The drop-in for the reference's hot path: `FindPath::eval`
//! (src/pathfinder.rs:199-248) answered by libmarshrutka_pf.so on a gfx950 device.
//!
//! Applying it to the reference crate (see ../README.md):
//!   * src/lib.rs: `mod ffi; mod engine;` beside `mod pathfinder;`
//!   * src/grid.rs: `MapGrid` (src/grid.rs:31-38) gains
//!     `pub engine: std::cell::OnceCell<crate::engine::EngineGrid>` (MapGrid derives
//!     Default; OnceCell's default is empty, so MapGrid::parse is unchanged)
//!   * src/pathfinder.rs: the body of `FindPath::eval` becomes
//!     `crate::engine::eval(&self, from, to)`; its signature, `FindPath`'s fields and
//!     the caller `MarshrutkaApp::update_path` (src/app.rs:704-731) are unchanged.
//!
//! Not compiled in this image (no Rust toolchain); tests/test_rust_shim.py checks the
//! ffi layouts and the entry points this file calls against include/marshrutka_pf.h.

use crate::cost::{AggregatedCost, CaravanCost, Command, CostComparator, TotalCost};
use crate::ffi;
use crate::grid::{MapGrid, PoI};
use crate::homeland::Homeland;
use crate::index::{Border, CellIndex, Pos};
use crate::pathfinder::FindPath;
use crate::skill::Fleetfoot;
use smallvec::SmallVec;
use time::Duration;

/// The device-side grid of a `MapGrid`, built once from its row-major cells.
pub struct EngineGrid(*mut ffi::mr_grid);

impl Drop for EngineGrid {
    fn drop(&mut self) {
        unsafe { ffi::mr_grid_destroy(self.0) }
    }
}

impl From<CellIndex> for ffi::mr_cell_index {
    /// The derived `Ord` layout of CellIndex (src/index.rs:41-46): variant, then fields.
    fn from(c: CellIndex) -> Self {
        match c {
            CellIndex::Center => ffi::mr_cell_index::default(),
            CellIndex::Homeland { homeland, pos } => ffi::mr_cell_index {
                kind: ffi::MR_CELL_HOMELAND,
                sub: homeland as u8,
                x: pos.x as u16,
                y: pos.y as u16,
                reserved: 0,
            },
            CellIndex::Border { border, shift } => ffi::mr_cell_index {
                kind: ffi::MR_CELL_BORDER,
                sub: border as u8,
                x: shift as u16,
                y: 0,
                reserved: 0,
            },
        }
    }
}

fn homeland_of(sub: u8) -> Homeland {
    match sub {
        0 => Homeland::Blue,
        1 => Homeland::Red,
        2 => Homeland::Green,
        _ => Homeland::Yellow,
    }
}

fn border_of(sub: u8) -> Border {
    match sub {
        0 => Border::BR,
        1 => Border::RG,
        2 => Border::GY,
        _ => Border::YB,
    }
}

/// Inverse of the `From` above.  The engine only returns cells of the grid, whose
/// positions fit the reference's u8 fields (S <= 255, src/index.rs:35-46).
fn cell_index(c: &ffi::mr_cell_index) -> CellIndex {
    match c.kind {
        ffi::MR_CELL_HOMELAND => CellIndex::Homeland {
            homeland: homeland_of(c.sub),
            pos: Pos { x: c.x as u8, y: c.y as u8 },
        },
        ffi::MR_CELL_BORDER => CellIndex::Border { border: border_of(c.sub), shift: c.x as u8 },
        _ => CellIndex::Center,
    }
}

/// One mr_command back to the reference's Command (src/cost.rs:83-110): the variant
/// tag is the AggregatedCost declaration order, each variant reads its own fields.
fn to_command(c: &ffi::mr_command) -> Command {
    let aggregated_cost = match c.kind {
        ffi::MR_CMD_CENTRAL => AggregatedCost::CentralMove { time: Duration::seconds(c.time_s) },
        ffi::MR_CMD_STANDARD => AggregatedCost::StandardMove {
            time: Duration::seconds(c.time_s),
            legs: c.legs,
            fleetfoot: Fleetfoot(c.fleetfoot),
        },
        ffi::MR_CMD_CARAVAN => AggregatedCost::Caravan(CaravanCost { time: Duration::seconds(c.time_s), money: c.money }),
        ffi::MR_CMD_SOE => AggregatedCost::ScrollOfEscape { money: c.money },
        ffi::MR_CMD_SHQ => AggregatedCost::ScrollOfEscapeHQ { money: c.money },
        ffi::MR_CMD_SFM => AggregatedCost::ScrollOfEscapeForum { money: c.money },
        _ => AggregatedCost::NoMove,
    };
    Command { aggregated_cost, from: cell_index(&c.from), to: cell_index(&c.to) }
}

fn comparator(c: CostComparator) -> u8 {
    match c {
        CostComparator::Legs => ffi::MR_SORT_LEGS,
        CostComparator::Time => ffi::MR_SORT_TIME,
        CostComparator::Money => ffi::MR_SORT_MONEY,
    }
}

impl MapGrid {
    /// The device grid, built on first use from `self.grid` (row-major, as
    /// MapGrid::parse scans it, src/grid.rs:64-77).
    pub fn engine(&self) -> &EngineGrid {
        self.engine.get_or_init(|| {
            let cells: Vec<ffi::mr_cell> = self
                .grid
                .iter()
                .map(|c| ffi::mr_cell {
                    index: c.index.into(),
                    poi: match c.poi {
                        Some(PoI::Campfire) => ffi::MR_POI_CAMPFIRE,
                        Some(PoI::Fountain) => ffi::MR_POI_FOUNTAIN,
                        Some(PoI::Forum) => ffi::MR_POI_FORUM,
                        None => ffi::MR_POI_NONE,
                    },
                    reserved: [0; 7],
                })
                .collect();
            let mut g = std::ptr::null_mut();
            let st = unsafe { ffi::mr_grid_create(cells.as_ptr(), cells.len() as u32, &mut g) };
            // MapGrid::parse already rejected what mr_grid_create rejects (src/grid.rs:60-133);
            // a homeland without a campfire panics in the reference too (src/grid.rs:209)
            assert_eq!(st, ffi::MR_OK, "mr_grid_create");
            EngineGrid(g)
        })
    }
}

fn params(fp: &FindPath) -> ffi::mr_params {
    ffi::mr_params {
        scroll_of_escape_cost: fp.scroll_of_escape_cost,
        scroll_of_escape_hq_cost: fp.scroll_of_escape_hq_cost,
        scroll_of_escape_forum_cost: fp.scroll_of_escape_forum_cost,
        use_soe: fp.use_soe as u8,
        use_sfm: fp.use_sfm as u8,
        use_caravans: fp.use_caravans as u8,
        has_hq: fp.hq_position.is_some() as u8,
        hq_position: fp.hq_position.map(Into::into).unwrap_or_default(),
        route_guru: fp.route_guru.0,
        fleetfoot: fp.fleetfoot.0,
        sort_by: [comparator(fp.sort_by.0), comparator(fp.sort_by.1)],
        homeland: fp.homeland as u8,
        reserved: 0,
    }
}

/// The body of `FindPath::eval(self, from, to) -> Option<TotalCost>`
/// (src/pathfinder.rs:199-248).
pub fn eval(fp: &FindPath, from: CellIndex, to: CellIndex) -> Option<TotalCost> {
    let p = params(fp);
    let grid = fp.grid.engine().0;
    let mut res = ffi::mr_result::default();
    let mut cmds = vec![ffi::mr_command::default(); 64];
    let mut st = unsafe {
        ffi::mr_find_path(grid, &p, from.into(), to.into(), &mut res, cmds.as_mut_ptr(), cmds.len() as u32)
    };
    if st == ffi::MR_ERR_CAPACITY {
        cmds.resize(res.n_commands as usize, Default::default());
        st = unsafe {
            ffi::mr_find_path(grid, &p, from.into(), to.into(), &mut res, cmds.as_mut_ptr(), cmds.len() as u32)
        };
    }
    match st {
        ffi::MR_OK => Some(TotalCost {
            legs: res.legs,
            money: res.money,
            time: Duration::seconds(res.time_s),
            commands: cmds[..res.n_commands as usize].iter().map(to_command).collect::<SmallVec<_>>(),
        }),
        ffi::MR_NOT_FOUND => None,
        // the reference panics on a CellIndex that is not in the grid (src/grid.rs:288-290)
        e => panic!("marshrutka_pf: FindPath::eval failed with status {e}"),
    }
}
