"""ctypes mirror of include/marshrutka_pf.h plus Python-side value types.

The value types mirror the reference's Rust types (CellIndex src/index.rs:41-46,
Command src/cost.rs:83-88, TotalCost src/cost.rs:187-206) closely enough that a
test reads like the reference's own code.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

# ---- status codes (mr_status) ----------------------------------------------
MR_OK = 0
MR_NOT_FOUND = 1
MR_ERR_INVALID_ARG = -1
MR_ERR_INVALID_GRID = -2
MR_ERR_INVALID_INDEX = -3
MR_ERR_CAPACITY = -4
MR_ERR_DEVICE = -5
MR_ERR_LIMIT = -6
MR_ERR_NO_DEVICE = -7

STATUS_NAMES = {
    MR_OK: "MR_OK", MR_NOT_FOUND: "MR_NOT_FOUND", MR_ERR_INVALID_ARG: "MR_ERR_INVALID_ARG",
    MR_ERR_INVALID_GRID: "MR_ERR_INVALID_GRID", MR_ERR_INVALID_INDEX: "MR_ERR_INVALID_INDEX",
    MR_ERR_CAPACITY: "MR_ERR_CAPACITY", MR_ERR_DEVICE: "MR_ERR_DEVICE", MR_ERR_LIMIT: "MR_ERR_LIMIT",
    MR_ERR_NO_DEVICE: "MR_ERR_NO_DEVICE",
}

CELL_CENTER, CELL_HOMELAND, CELL_BORDER = 0, 1, 2
BLUE, RED, GREEN, YELLOW = 0, 1, 2, 3
BR, RG, GY, YB = 0, 1, 2, 3
POI_NONE, POI_CAMPFIRE, POI_FOUNTAIN, POI_FORUM = 0, 1, 2, 3
SORT_LEGS, SORT_TIME, SORT_MONEY = 0, 1, 2
CMD_NO_MOVE, CMD_CENTRAL, CMD_STANDARD, CMD_CARAVAN, CMD_SOE, CMD_SHQ, CMD_SFM = range(7)
CMD_NAMES = ["NoMove", "CentralMove", "StandardMove", "Caravan", "ScrollOfEscape",
             "ScrollOfEscapeHQ", "ScrollOfEscapeForum"]
HOMELAND_ABBREV = "BRGY"
BORDER_NAMES = ["BR", "RG", "GY", "YB"]


class mr_cell_index(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("sub", C.c_uint8), ("x", C.c_uint16), ("y", C.c_uint16),
                ("reserved", C.c_uint16)]


class mr_cell(C.Structure):
    _fields_ = [("index", mr_cell_index), ("poi", C.c_uint8), ("reserved", C.c_uint8 * 7)]


class mr_params(C.Structure):
    _fields_ = [("scroll_of_escape_cost", C.c_uint32), ("scroll_of_escape_hq_cost", C.c_uint32),
                ("scroll_of_escape_forum_cost", C.c_uint32), ("use_soe", C.c_uint8),
                ("use_sfm", C.c_uint8), ("use_caravans", C.c_uint8), ("has_hq", C.c_uint8),
                ("hq_position", mr_cell_index), ("route_guru", C.c_uint32),
                ("fleetfoot", C.c_uint32), ("sort_by", C.c_uint8 * 2), ("homeland", C.c_uint8),
                ("reserved", C.c_uint8)]


class mr_command(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("reserved", C.c_uint8 * 3), ("legs", C.c_uint32),
                ("money", C.c_uint32), ("fleetfoot", C.c_uint32), ("time_s", C.c_int64),
                ("from_", mr_cell_index), ("to", mr_cell_index)]


class mr_result(C.Structure):
    _fields_ = [("legs", C.c_uint32), ("money", C.c_uint32), ("time_s", C.c_int64),
                ("n_commands", C.c_uint32), ("command_offset", C.c_uint32), ("status", C.c_int32),
                ("reserved", C.c_uint32)]


class mr_query(C.Structure):
    _fields_ = [("from_", mr_cell_index), ("to", mr_cell_index)]


class mr_plan_stats(C.Structure):
    _fields_ = [("solver", C.c_uint32), ("grid_state_in_lds", C.c_uint32), ("num_sources", C.c_uint32),
                ("fallback_sources", C.c_uint32), ("num_specials", C.c_uint32), ("num_regions", C.c_uint32),
                ("hub_workgroups", C.c_uint32), ("sssp_workgroups", C.c_uint32),
                ("specials_per_lane", C.c_uint32), ("region_boundary_cells", C.c_uint32),
                ("fill_launch", C.c_uint32), ("lane_sources", C.c_uint32),
                ("certified_sources", C.c_uint32), ("lanes_per_source", C.c_uint32)]


assert C.sizeof(mr_cell_index) == 8
assert C.sizeof(mr_cell) == 16
assert C.sizeof(mr_command) == 40
assert C.sizeof(mr_result) == 32
assert C.sizeof(mr_query) == 16


# ---- value types -------------------------------------------------------------
@dataclass(frozen=True, order=True)
class CellIndex:
    """CellIndex (src/index.rs:41-46); field order = derived Ord."""
    kind: int
    sub: int = 0
    x: int = 0
    y: int = 0

    @staticmethod
    def center() -> "CellIndex":
        return CellIndex(CELL_CENTER)

    @staticmethod
    def homeland(h: int, x: int, y: int) -> "CellIndex":
        """CellIndexBuilder::Homeland{..}.build() (src/index.rs:257-312)."""
        if x == 0 and y == 0:
            return CellIndex.center()
        if x == 0:
            return CellIndex(CELL_BORDER, YB if h in (YELLOW, BLUE) else RG, y, 0)
        if y == 0:
            return CellIndex(CELL_BORDER, BR if h in (BLUE, RED) else GY, x, 0)
        return CellIndex(CELL_HOMELAND, h, x, y)

    @staticmethod
    def border(b: int, shift: int) -> "CellIndex":
        if shift == 0:
            return CellIndex.center()
        return CellIndex(CELL_BORDER, b, shift, 0)

    def to_c(self) -> mr_cell_index:
        return mr_cell_index(self.kind, self.sub, self.x, self.y, 0)

    @staticmethod
    def from_c(c: mr_cell_index) -> "CellIndex":
        return CellIndex(c.kind, c.sub, c.x, c.y)

    def __str__(self) -> str:  # Display (src/index.rs:362-376)
        if self.kind == CELL_CENTER:
            return "0#0"
        if self.kind == CELL_HOMELAND:
            return f"{HOMELAND_ABBREV[self.sub]} {self.x}#{self.y}"
        return f"{BORDER_NAMES[self.sub]} {self.x}"

    @staticmethod
    def parse(s: str) -> "CellIndex":
        """FromStr for CellIndex (src/index.rs:433-446)."""
        if s == "0#0":
            return CellIndex.center()
        left, right = s.split(" ", 1)
        if left in HOMELAND_ABBREV and len(left) == 1:
            x, y = right.split("#")
            return CellIndex.homeland(HOMELAND_ABBREV.index(left), int(x), int(y))
        return CellIndex.border(BORDER_NAMES.index(left), int(right))


@dataclass(frozen=True)
class Command:
    """Command { aggregated_cost, from, to } with AggregatedCost flattened."""
    kind: int
    time_s: int = 0
    legs: int = 0
    money: int = 0
    fleetfoot: int = 0
    from_: CellIndex = CellIndex(CELL_CENTER)
    to: CellIndex = CellIndex(CELL_CENTER)

    def key(self) -> Tuple:
        return (self.kind, self.time_s, self.legs, self.money, self.fleetfoot, self.from_, self.to)

    def as_tuple(self) -> Tuple:
        return (self.kind, self.time_s, self.legs, self.money, self.fleetfoot,
                (self.from_.kind, self.from_.sub, self.from_.x, self.from_.y),
                (self.to.kind, self.to.sub, self.to.x, self.to.y))

    @staticmethod
    def from_c(c: mr_command) -> "Command":
        return Command(c.kind, c.time_s, c.legs, c.money, c.fleetfoot,
                       CellIndex.from_c(c.from_), CellIndex.from_c(c.to))


@dataclass
class TotalCost:
    """TotalCost { legs, money, time, commands } (src/cost.rs:187-206)."""
    legs: int
    money: int
    time_s: int
    commands: List[Command] = field(default_factory=list)

    def as_tuple(self) -> Tuple:
        return (self.legs, self.money, self.time_s, tuple(c.as_tuple() for c in self.commands))


def duration_display(seconds: int) -> str:
    """time 0.3 Duration Display, verbose form (pinned: src/pathfinder.rs:279-285)."""
    if seconds == 0:
        return "0s"
    out = "-" if seconds < 0 else ""
    a = abs(seconds)
    for v, n in ((a // 86400, "d"), (a // 3600 % 24, "h"), (a // 60 % 60, "m"), (a % 60, "s")):
        if v:
            out += f"{v}{n}"
    return out


@dataclass
class Params:
    """Every FindPath field (src/pathfinder.rs:183-196); defaults = the app's
    (src/app.rs:782-811) as wired by update_path (src/app.rs:704-731)."""
    scroll_of_escape_cost: int = 50
    scroll_of_escape_hq_cost: int = 75
    scroll_of_escape_forum_cost: int = 100
    use_soe: bool = True
    use_sfm: bool = False
    use_caravans: bool = True
    hq_position: Optional[CellIndex] = None
    route_guru: int = 0
    fleetfoot: int = 0
    sort_by: Tuple[int, int] = (SORT_LEGS, SORT_MONEY)
    homeland: int = BLUE

    def to_c(self) -> mr_params:
        p = mr_params()
        p.scroll_of_escape_cost = self.scroll_of_escape_cost
        p.scroll_of_escape_hq_cost = self.scroll_of_escape_hq_cost
        p.scroll_of_escape_forum_cost = self.scroll_of_escape_forum_cost
        p.use_soe = int(self.use_soe)
        p.use_sfm = int(self.use_sfm)
        p.use_caravans = int(self.use_caravans)
        p.has_hq = int(self.hq_position is not None)
        if self.hq_position is not None:
            p.hq_position = self.hq_position.to_c()
        p.route_guru = self.route_guru
        p.fleetfoot = self.fleetfoot
        p.sort_by[0], p.sort_by[1] = self.sort_by
        p.homeland = self.homeland
        return p

    def to_json(self) -> dict:
        d = dict(self.__dict__)
        d["hq_position"] = None if self.hq_position is None else list(
            (self.hq_position.kind, self.hq_position.sub, self.hq_position.x, self.hq_position.y))
        d["sort_by"] = list(self.sort_by)
        return d

    @staticmethod
    def from_json(d: dict) -> "Params":
        d = dict(d)
        if d.get("hq_position") is not None:
            d["hq_position"] = CellIndex(*d["hq_position"])
        d["sort_by"] = tuple(d["sort_by"])
        return Params(**d)


def cells_to_c(cells) -> "C.Array":
    """cells: iterable of (CellIndex, poi) in row-major order."""
    cells = list(cells)
    arr = (mr_cell * len(cells))()
    for i, (ci, poi) in enumerate(cells):
        arr[i].index = ci.to_c()
        arr[i].poi = poi
    return arr


def queries_to_c(queries) -> "C.Array":
    queries = list(queries)
    arr = (mr_query * len(queries))()
    for i, (a, b) in enumerate(queries):
        arr[i].from_ = a.to_c()
        arr[i].to = b.to_c()
    return arr


def result_from_c(r: mr_result, pool) -> Optional[TotalCost]:
    if r.status == MR_NOT_FOUND:
        return None
    cmds = [Command.from_c(pool[r.command_offset + j]) for j in range(r.n_commands)]
    return TotalCost(r.legs, r.money, r.time_s, cmds)
