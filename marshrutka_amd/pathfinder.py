"""Host-side mirror of the reference's pathfinder API over the C ABI.

    FindPath { scroll_of_escape_cost, .., sort_by, homeland, grid }.eval(from, to)
        -> Option<TotalCost>                          (src/pathfinder.rs:183-248)

`FindPath(...).eval(a, b)` returns a TotalCost or None exactly like the
reference; `FindPath(...).eval_batch(pairs)` is the batched GPU hot path.  All
compute runs in libmarshrutka_pf.so on a gfx950 device; without one every call
raises EngineError (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from . import abi
from .abi import (MR_ERR_CAPACITY, MR_NOT_FOUND, MR_OK, CellIndex, Params, TotalCost, cells_to_c,
                  mr_cell, mr_cell_index, mr_command, mr_params, mr_plan_stats, mr_query, mr_result, queries_to_c,
                  result_from_c)

LIB_PATH = os.environ.get("MR_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                          "libmarshrutka_pf.so")

EXPORTED_SYMBOLS = [
    "mr_grid_create", "mr_grid_destroy", "mr_grid_square_size", "mr_params_default", "mr_find_path",
    "mr_find_path_batch", "mr_plan_create", "mr_plan_create_ex", "mr_plan_run", "mr_plan_fetch", "mr_plan_device_outputs",
    "mr_plan_num_sources", "mr_plan_record_queries", "mr_plan_fallback_sources", "mr_plan_handed_over_sources", "mr_plan_wait", "mr_plan_get_stats", "mr_plan_kernel_ms", "mr_plan_destroy", "mr_cache_trim", "mr_host_register", "mr_host_unregister", "mr_plan_bind_outputs", "mr_plan_bind_outputs_ex", "mr_decode_records", "mr_wire_row_bytes", "mr_plan_wire_records", "mr_decode_wire", "mr_abi_version", "mr_last_error",
    "mr_device_available", "mr_parse_map_html", "mr_parse_error", "mr_grid_from_html",
    "mr_command_time", "mr_duration_display", "mr_render_schedule", "mr_grid_region_table",
    "mr_sssp_plan_create", "mr_sssp_records", "mr_sssp_device_records", "mr_sssp_record_pitch", "mr_sssp_device_tables", "mr_sssp_label", "mr_sssp_labels", "mr_plan_fill_ms",
]


class EngineError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        super().__init__(f"{abi.STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


_lib = None


def lib():
    """Loads the in-tree HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(abi.MR_ERR_NO_DEVICE, f"{LIB_PATH} missing: run python -m marshrutka_amd.build")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.mr_grid_create.argtypes = [C.POINTER(mr_cell), C.c_uint32, C.POINTER(vp)]
        L.mr_grid_create.restype = C.c_int
        L.mr_grid_destroy.argtypes = [vp]
        L.mr_grid_square_size.argtypes = [vp]
        L.mr_grid_square_size.restype = C.c_uint32
        L.mr_params_default.argtypes = [C.POINTER(mr_params)]
        L.mr_find_path.argtypes = [vp, C.POINTER(mr_params), mr_cell_index, mr_cell_index,
                                   C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint32]
        L.mr_find_path.restype = C.c_int
        L.mr_find_path_batch.argtypes = [vp, C.POINTER(mr_params), C.POINTER(mr_query), C.c_uint32,
                                         C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64]
        L.mr_find_path_batch.restype = C.c_int
        L.mr_plan_create.argtypes = [vp, C.POINTER(mr_params), C.POINTER(mr_query), C.c_uint32, C.POINTER(vp)]
        L.mr_plan_create.restype = C.c_int
        L.mr_plan_run.argtypes = [vp, vp]
        L.mr_plan_run.restype = C.c_int
        L.mr_plan_wait.argtypes = [vp, vp]
        L.mr_plan_wait.restype = C.c_int
        L.mr_plan_fetch.argtypes = [vp, C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64]
        L.mr_plan_fetch.restype = C.c_int
        L.mr_plan_device_outputs.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_uint64), C.POINTER(vp),
                                             C.POINTER(C.c_uint64)]
        L.mr_plan_device_outputs.restype = C.c_int
        L.mr_plan_create_ex.argtypes = [vp, C.POINTER(mr_params), C.POINTER(mr_query), C.c_uint32, C.c_uint32,
                                        C.POINTER(vp)]
        L.mr_plan_create_ex.restype = C.c_int
        L.mr_plan_bind_outputs.argtypes = [vp, vp, vp]
        L.mr_plan_bind_outputs.restype = C.c_int
        L.mr_plan_bind_outputs_ex.argtypes = [vp, vp, vp, vp, C.c_uint32]
        L.mr_plan_bind_outputs_ex.restype = C.c_int
        L.mr_decode_records.argtypes = [vp, C.POINTER(mr_params), vp, vp, C.c_uint32, C.c_uint32, vp, C.c_uint64,
                                        C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64]
        L.mr_decode_records.restype = C.c_int
        L.mr_wire_row_bytes.argtypes = [C.c_uint32]
        L.mr_wire_row_bytes.restype = C.c_uint32
        L.mr_plan_wire_records.argtypes = [vp, vp, vp, C.c_uint32, vp]
        L.mr_plan_wire_records.restype = C.c_int
        L.mr_decode_wire.argtypes = [vp, C.POINTER(mr_params), vp, C.c_uint32, C.c_uint32, vp, C.c_uint64,
                                     C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64]
        L.mr_decode_wire.restype = C.c_int
        L.mr_plan_num_sources.argtypes = [vp]
        L.mr_plan_num_sources.restype = C.c_uint32
        L.mr_plan_record_queries.argtypes = [vp, C.POINTER(C.c_uint32), C.c_uint32]
        L.mr_plan_record_queries.restype = C.c_int
        L.mr_plan_fallback_sources.argtypes = [vp, C.POINTER(mr_cell_index), C.c_uint32, C.POINTER(C.c_uint32)]
        L.mr_plan_fallback_sources.restype = C.c_int
        L.mr_plan_handed_over_sources.argtypes = [vp, C.POINTER(mr_cell_index), C.POINTER(C.c_uint8), C.c_uint32,
                                                  C.POINTER(C.c_uint32)]
        L.mr_plan_handed_over_sources.restype = C.c_int
        L.mr_plan_get_stats.argtypes = [vp, C.POINTER(mr_plan_stats)]
        L.mr_plan_get_stats.restype = C.c_int
        L.mr_plan_kernel_ms.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.mr_plan_kernel_ms.restype = C.c_double
        L.mr_plan_destroy.argtypes = [vp]
        L.mr_cache_trim.argtypes = []
        L.mr_cache_trim.restype = None
        L.mr_host_register.argtypes = [vp, C.c_uint64]
        L.mr_host_register.restype = C.c_int
        L.mr_host_unregister.argtypes = [vp]
        L.mr_host_unregister.restype = C.c_int
        L.mr_abi_version.restype = C.c_uint32
        L.mr_last_error.restype = C.c_char_p
        L.mr_device_available.restype = C.c_int
        L.mr_parse_map_html.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(mr_cell), C.c_uint32, C.POINTER(C.c_uint32)]
        L.mr_parse_map_html.restype = C.c_int
        L.mr_parse_error.restype = C.c_char_p
        L.mr_grid_from_html.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(vp)]
        L.mr_grid_from_html.restype = C.c_int
        L.mr_command_time.argtypes = [C.POINTER(mr_command)]
        L.mr_command_time.restype = C.c_int64
        L.mr_duration_display.argtypes = [C.c_int64, C.c_char_p, C.c_uint64]
        L.mr_duration_display.restype = C.c_int
        L.mr_render_schedule.argtypes = [C.POINTER(mr_command), C.c_uint32, C.c_uint32, C.c_uint32, C.c_char_p,
                                         C.c_uint64, C.POINTER(C.c_uint64)]
        L.mr_render_schedule.restype = C.c_int
        L.mr_sssp_plan_create.argtypes = [vp, C.POINTER(mr_params), C.POINTER(mr_cell_index), C.c_uint32,
                                          C.POINTER(vp)]
        L.mr_sssp_plan_create.restype = C.c_int
        L.mr_sssp_records.argtypes = [vp, C.c_uint32, vp]
        L.mr_sssp_records.restype = C.c_int
        L.mr_sssp_device_records.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_uint64)]
        L.mr_sssp_device_records.restype = C.c_int
        L.mr_sssp_record_pitch.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.mr_sssp_record_pitch.restype = C.c_int
        L.mr_sssp_device_tables.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_uint64)]
        L.mr_sssp_device_tables.restype = C.c_int
        L.mr_sssp_label.argtypes = [vp, C.c_uint32, mr_cell_index, C.POINTER(mr_result), C.POINTER(mr_command),
                                    C.c_uint32]
        L.mr_sssp_label.restype = C.c_int
        L.mr_sssp_labels.argtypes = [vp, C.c_uint32, C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64]
        L.mr_sssp_labels.restype = C.c_int
        L.mr_grid_region_table.argtypes = [vp, C.c_uint32, vp, C.c_uint64, C.POINTER(C.c_uint32),
                                           C.POINTER(C.c_double)]
        L.mr_grid_region_table.restype = C.c_int
        L.mr_plan_fill_ms.argtypes = [vp]
        L.mr_plan_fill_ms.restype = C.c_double
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().mr_last_error() or b"").decode()


def device_available() -> bool:
    return bool(lib().mr_device_available())


def render_schedule(label: TotalCost, arrive_at_s: int, pause_s: int = 0) -> List[Tuple[str, str, str, str]]:
    """The app's command table for a path (src/app.rs:481-561): rows of
    (bot command, duration, running total, back-scheduled start hh:mm:ss)."""
    cmds = (mr_command * max(len(label.commands), 1))()
    for i, c in enumerate(label.commands):
        cmds[i].kind, cmds[i].time_s, cmds[i].legs = c.kind, c.time_s, c.legs
        cmds[i].money, cmds[i].fleetfoot = c.money, c.fleetfoot
        for dst, ci in ((cmds[i].from_, c.from_), (cmds[i].to, c.to)):
            dst.kind, dst.sub, dst.x, dst.y = ci.kind, ci.sub, ci.x, ci.y
    n = C.c_uint64()
    st = lib().mr_render_schedule(cmds, len(label.commands), arrive_at_s, pause_s, None, 0, C.byref(n))
    if st not in (MR_OK, MR_ERR_CAPACITY):
        raise EngineError(st, "render_schedule")
    buf = C.create_string_buffer(n.value + 1)
    st = lib().mr_render_schedule(cmds, len(label.commands), arrive_at_s, pause_s, buf, n.value + 1, C.byref(n))
    if st != MR_OK:
        raise EngineError(st, "render_schedule")
    return [tuple(line.split("\t")) for line in buf.value.decode().splitlines()]


def parse_map_html(html: str) -> List[Tuple[CellIndex, int]]:
    """MapGrid::parse (src/grid.rs:47-133) on the host: the reference's HTML map
    format -> [(CellIndex, poi)] in row-major order.  Raises EngineError
    (MR_ERR_INVALID_GRID) on the reference's parse errors."""
    data = html.encode("utf-8")
    n = C.c_uint32()
    st = lib().mr_parse_map_html(data, len(data), None, 0, C.byref(n))
    if st not in (MR_OK, MR_ERR_CAPACITY):
        raise EngineError(st, (lib().mr_parse_error() or b"").decode())
    cells = (mr_cell * max(n.value, 1))()
    st = lib().mr_parse_map_html(data, len(data), cells, n.value, C.byref(n))
    if st != MR_OK:
        raise EngineError(st, (lib().mr_parse_error() or b"").decode())
    return [(CellIndex(c.index.kind, c.index.sub, c.index.x, c.index.y), c.poi) for c in cells[: n.value]]


class MapGrid:
    """The immutable grid handle (MapGrid, src/grid.rs:31-38)."""

    @classmethod
    def from_html(cls, html: str) -> "MapGrid":
        """MapGrid::parse + the engine's grid (canonical indices, nearest campfires)."""
        return cls(parse_map_html(html))

    @classmethod
    def from_array(cls, arr) -> "MapGrid":
        """From a numpy record array with mr_cell's 16-byte layout (mapgen.cells_array)."""
        g = cls.__new__(cls)
        g._cells = arr
        if arr.dtype.itemsize != C.sizeof(mr_cell) or not arr.flags["C_CONTIGUOUS"]:
            raise EngineError(abi.MR_ERR_INVALID_ARG, "cell array must be contiguous mr_cell records")
        g._create(C.cast(arr.ctypes.data, C.POINTER(mr_cell)), len(arr))
        return g

    def __init__(self, cells: Sequence[Tuple[CellIndex, int]]):
        self._cells = cells_to_c(cells)
        self._create(self._cells, len(cells))

    def _create(self, ptr, n: int) -> None:
        h = C.c_void_p()
        st = lib().mr_grid_create(ptr, n, C.byref(h))
        if st != MR_OK:
            raise EngineError(st, last_error())
        self.handle = h

    @property
    def square_size(self) -> int:
        return lib().mr_grid_square_size(self.handle)

    def homeland_size(self) -> int:  # src/grid.rs:280-282
        return self.square_size // 2

    def region_table(self, homeland: int, fetch: bool = True):
        """mr_grid_region_table: (regions, build_ms, table) — the device-built SoE region
        table of `homeland` as a (V, regions, 2) uint32 array ({distance, rank}), or None
        with fetch=False (build / timing only)."""
        import numpy as np
        nreg, ms = C.c_uint32(), C.c_double()
        st = lib().mr_grid_region_table(self.handle, homeland, None, 0, C.byref(nreg), C.byref(ms))
        if st != MR_OK:
            raise EngineError(st, last_error())
        if not fetch:
            return nreg.value, ms.value, None
        V = self.square_size ** 2
        out = np.empty((V, nreg.value, 2), dtype=np.uint32)
        st = lib().mr_grid_region_table(self.handle, homeland, out.ctypes.data, out.size, C.byref(nreg), C.byref(ms))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return nreg.value, ms.value, out

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.mr_grid_destroy(h)
            self.handle = None


@dataclass
class FindPath:
    """Same fields and defaults as the reference's FindPath (src/pathfinder.rs:183-196)."""
    grid: MapGrid
    scroll_of_escape_cost: int = 50
    scroll_of_escape_hq_cost: int = 75
    scroll_of_escape_forum_cost: int = 100
    use_soe: bool = True
    use_sfm: bool = False
    use_caravans: bool = True
    hq_position: Optional[CellIndex] = None
    route_guru: int = 0
    fleetfoot: int = 0
    sort_by: Tuple[int, int] = (abi.SORT_LEGS, abi.SORT_MONEY)
    homeland: int = abi.BLUE

    def params(self) -> Params:
        return Params(self.scroll_of_escape_cost, self.scroll_of_escape_hq_cost,
                      self.scroll_of_escape_forum_cost, self.use_soe, self.use_sfm, self.use_caravans,
                      self.hq_position, self.route_guru, self.fleetfoot, tuple(self.sort_by), self.homeland)

    @staticmethod
    def with_params(grid: MapGrid, p: Params) -> "FindPath":
        return FindPath(grid, p.scroll_of_escape_cost, p.scroll_of_escape_hq_cost,
                        p.scroll_of_escape_forum_cost, p.use_soe, p.use_sfm, p.use_caravans,
                        p.hq_position, p.route_guru, p.fleetfoot, tuple(p.sort_by), p.homeland)

    def eval(self, from_: CellIndex, to: CellIndex) -> Optional[TotalCost]:
        """FindPath::eval (src/pathfinder.rs:199-248); None when unreachable."""
        p = self.params().to_c()
        res = mr_result()
        cap = 64
        while True:
            cmds = (mr_command * cap)()
            st = lib().mr_find_path(self.grid.handle, C.byref(p), from_.to_c(), to.to_c(), C.byref(res), cmds, cap)
            if st == MR_ERR_CAPACITY:
                cap = res.n_commands
                continue
            break
        if st == MR_NOT_FOUND:
            return None
        if st != MR_OK:
            raise EngineError(st, last_error())
        res.command_offset = 0
        return result_from_c(res, cmds)

    def eval_batch_raw(self, pairs: Sequence[Tuple[CellIndex, CellIndex]]):
        n = len(pairs)
        qs = queries_to_c(pairs)
        p = self.params().to_c()
        res = (mr_result * max(n, 1))()
        cap = max(1, n * 8)
        while True:
            pool = (mr_command * cap)()
            st = lib().mr_find_path_batch(self.grid.handle, C.byref(p), qs, n, res, pool, cap)
            if st == MR_ERR_CAPACITY and any(res[i].status == MR_OK for i in range(n)):
                total = sum(res[i].n_commands for i in range(n) if res[i].status == MR_OK)
                if total > cap:
                    cap = total
                    continue
            break
        if st < 0 and st != abi.MR_ERR_INVALID_INDEX:
            raise EngineError(st, last_error())
        return res, pool

    def eval_batch(self, pairs: Sequence[Tuple[CellIndex, CellIndex]]) -> List[Optional[TotalCost]]:
        res, pool = self.eval_batch_raw(pairs)
        out = []
        for i in range(len(pairs)):
            r = res[i]
            if r.status == MR_OK or r.status == MR_NOT_FOUND:
                out.append(result_from_c(r, pool))
            else:
                raise EngineError(r.status, f"query {i}")
        return out


def _host_array(ctype, n: int):
    """An uninitialised ctypes array of n ctype (numpy-backed; it keeps the buffer alive)."""
    import numpy as np
    buf = np.empty(n * C.sizeof(ctype), dtype=np.uint8)
    return (ctype * n).from_buffer(buf)


def decode_records_raw(grid: MapGrid, params: Params, results, commands, n: int, max_cmds: int, overflow=None):
    """Compact device records (mr_plan_device_outputs layout: 16 B result records,
    max_cmds 16 B command slots each, an overflow pool) as host buffers — e.g. the
    rows another rank gathered — decoded on the host (mr_decode_records): returns the
    (mr_result array, mr_command pool), record k -> entry k."""
    import numpy as np
    res = np.ascontiguousarray(results, dtype=np.uint32)
    cmd = np.ascontiguousarray(commands, dtype=np.uint32)
    ovf = np.ascontiguousarray(overflow if overflow is not None else np.zeros(0), dtype=np.uint32)
    if res.size < 4 * n or cmd.size < 4 * n * max_cmds:
        raise EngineError(abi.MR_ERR_INVALID_ARG, "decode_records: buffers shorter than n records")
    out = (mr_result * max(n, 1))()
    cap = int(n * max_cmds + ovf.size // 4 + 1)
    pool = (mr_command * cap)()
    p = params.to_c()
    st = lib().mr_decode_records(grid.handle, C.byref(p), res.ctypes.data, cmd.ctypes.data, n, max_cmds,
                                 ovf.ctypes.data if ovf.size else None, ovf.size // 4, out, pool, cap)
    if st != MR_OK:
        raise EngineError(st, last_error())
    return out, pool


def wire_row_words(max_cmds: int) -> int:
    """32-bit words of one wire row (mr_wire_row_bytes / 4)."""
    return int(lib().mr_wire_row_bytes(max_cmds)) // 4


def decode_wire_raw(grid: MapGrid, params: Params, rows, n: int, max_cmds: int, pool=None):
    """n wire rows (Plan.wire_records layout) and their pool as host buffers, decoded on the
    host (mr_decode_wire): returns (mr_result array, mr_command pool), row k -> entry k —
    the same as decode_records_raw gives for the plan's compact records."""
    import numpy as np
    w = np.ascontiguousarray(rows, dtype=np.uint32).reshape(-1)
    wp = np.ascontiguousarray(pool if pool is not None else np.zeros(0), dtype=np.uint32).reshape(-1)
    if w.size < n * (1 + 2 * max_cmds):
        raise EngineError(abi.MR_ERR_INVALID_ARG, "decode_wire: buffer shorter than n rows")
    out = (mr_result * max(n, 1))()
    cap = int(n * max_cmds + wp.size // 2 + 1)
    cmds = (mr_command * cap)()
    p = params.to_c()
    st = lib().mr_decode_wire(grid.handle, C.byref(p), w.ctypes.data if w.size else None, n, max_cmds,
                              wp.ctypes.data if wp.size else None, wp.size // 2, out, cmds, cap)
    if st not in (MR_OK, abi.MR_ERR_INVALID_INDEX, abi.MR_ERR_CAPACITY):  # (per-row statuses are in out[k])
        raise EngineError(st, last_error())
    return out, cmds


def decode_records(grid: MapGrid, params: Params, results, commands, n: int, max_cmds: int,
                   overflow=None) -> List[Optional[TotalCost]]:
    """decode_records_raw as labels.  A record whose status is not OK / NOT_FOUND raises."""
    out, pool = decode_records_raw(grid, params, results, commands, n, max_cmds, overflow)
    for k in range(n):
        if out[k].status not in (MR_OK, MR_NOT_FOUND):
            raise EngineError(out[k].status, f"record {k}")
    return [result_from_c(out[k], pool) for k in range(n)]


def labels_digest(results, pool, n: int, order=None) -> str:
    """sha256 over n decoded labels (mr_result array + command pool, as mr_plan_fetch
    or decode_records_raw return them), taken in `order` (entry order[i] first..., or
    entry order by default): metrics, command count, status, then the commands.
    Numpy only, so a rank's million labels hash in well under a second."""
    import hashlib
    import numpy as np
    rdt = np.dtype([("legs", "<u4"), ("money", "<u4"), ("time_s", "<i8"), ("n", "<u4"), ("off", "<u4"),
                    ("status", "<i4"), ("reserved", "<u4")])
    r = np.frombuffer(results, dtype=rdt, count=n)
    if order is not None:
        r = r[np.asarray(order, dtype=np.int64)]
    ncmd = r["n"].astype(np.int64)
    cmds = np.frombuffer(pool, dtype=np.uint8).reshape(-1, C.sizeof(mr_command))
    starts = np.repeat(r["off"].astype(np.int64), ncmd)
    within = np.arange(int(ncmd.sum()), dtype=np.int64) - np.repeat(np.cumsum(ncmd) - ncmd, ncmd)
    h = hashlib.sha256()
    for f in ("legs", "money", "time_s", "n", "status"):
        h.update(np.ascontiguousarray(r[f]).tobytes())
    h.update(cmds[starts + within].tobytes())
    return h.hexdigest()


def pin_host(arr) -> None:
    """mr_host_register: page-lock a host buffer (a ctypes array, e.g. of fetch_buffers)
    so mr_plan_fetch fills it by direct DMA; unpin_host(arr) before it is freed."""
    st = lib().mr_host_register(C.addressof(arr), C.sizeof(arr))
    if st != MR_OK:
        raise EngineError(st, last_error())


def unpin_host(arr) -> None:
    st = lib().mr_host_unregister(C.addressof(arr))
    if st != MR_OK:
        raise EngineError(st, last_error())


def fetch_buffers(n: int, max_cmds: int = 16):
    """Host buffers for Plan.fetch_raw(out=...) of plans of up to n queries with max_cmds
    command slots: (results, command pool: the slots + the overflow pool)."""
    cap = n * max_cmds + max(4096, n * 8)
    return _host_array(mr_result, max(n, 1)), _host_array(mr_command, cap)


class Plan:
    """Device-resident batch: inputs uploaded once, `run()` enqueues one pass."""

    def __init__(self, grid: MapGrid, params: Params, pairs: Sequence[Tuple[CellIndex, CellIndex]],
                 max_cmds: int = 0, query_array=None):
        """max_cmds: command slots per query in the device output (0 = the C default, 16);
        longer labels go through the plan's overflow pool.  query_array: the queries as
        a contiguous numpy array of mr_query records (16 B each) instead of `pairs`
        (millions of queries without one Python object each)."""
        self.grid = grid
        self.max_cmds = max_cmds or 16
        if query_array is not None:
            if query_array.dtype.itemsize != C.sizeof(mr_query) or not query_array.flags["C_CONTIGUOUS"]:
                raise EngineError(abi.MR_ERR_INVALID_ARG, "query array must be contiguous mr_query records")
            self.n = len(query_array)
            self._qarr = query_array
            self._qs = C.cast(query_array.ctypes.data, C.POINTER(mr_query))
        else:
            self.n = len(pairs)
            self._qs = queries_to_c(pairs)
        self._p = params.to_c()
        h = C.c_void_p()
        if max_cmds:
            st = lib().mr_plan_create_ex(grid.handle, C.byref(self._p), self._qs, self.n, max_cmds, C.byref(h))
        else:
            st = lib().mr_plan_create(grid.handle, C.byref(self._p), self._qs, self.n, C.byref(h))
        if st != MR_OK:
            raise EngineError(st, last_error())
        self.handle = h

    @property
    def num_sources(self) -> int:
        return lib().mr_plan_num_sources(self.handle)

    def record_queries(self) -> List[int]:
        """query_of_record[k]: the input query whose compact output is device record k
        (records are grouped by source; 0xFFFFFFFF past the valid queries)."""
        out = (C.c_uint32 * max(1, self.n))()
        st = lib().mr_plan_record_queries(self.handle, out, self.n)
        if st != MR_OK:
            raise EngineError(st, last_error())
        return list(out)[:self.n]

    def fallback_sources(self) -> List[CellIndex]:
        """The sources the last pass re-solved with the SSSP kernel (mr_plan_fallback_sources)."""
        n = C.c_uint32()
        st = lib().mr_plan_fallback_sources(self.handle, None, 0, C.byref(n))
        if st != MR_OK:
            raise EngineError(st, last_error())
        out = (mr_cell_index * max(1, n.value))()
        st = lib().mr_plan_fallback_sources(self.handle, out, n.value, C.byref(n))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return [CellIndex(c.kind, c.sub, c.x, c.y) for c in out[: n.value]]

    def handed_over_sources(self) -> List[Tuple[CellIndex, bool]]:
        """Every source the hub handed over in the last pass, with whether the certificate
        answered it (True) or the SSSP kernel solved it (mr_plan_handed_over_sources)."""
        n = C.c_uint32()
        st = lib().mr_plan_handed_over_sources(self.handle, None, None, 0, C.byref(n))
        if st != MR_OK:
            raise EngineError(st, last_error())
        out = (mr_cell_index * max(1, n.value))()
        cert = (C.c_uint8 * max(1, n.value))()
        st = lib().mr_plan_handed_over_sources(self.handle, out, cert, n.value, C.byref(n))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return [(CellIndex(c.kind, c.sub, c.x, c.y), bool(f)) for c, f in zip(out[: n.value], cert[: n.value])]

    def run(self, stream: int = 0) -> None:
        st = lib().mr_plan_run(self.handle, C.c_void_p(stream) if stream else None)
        if st != MR_OK:
            raise EngineError(st, last_error())

    def wait(self, stream: int = 0) -> None:
        """mr_plan_wait: `stream` (or, with 0, this thread) waits for every pass so far."""
        st = lib().mr_plan_wait(self.handle, C.c_void_p(stream) if stream else None)
        if st != MR_OK:
            raise EngineError(st, last_error())

    def stats(self) -> dict:
        st = mr_plan_stats()
        rc = lib().mr_plan_get_stats(self.handle, C.byref(st))
        if rc != MR_OK:
            raise EngineError(rc, last_error())
        d = {f: getattr(st, f) for f, _ in mr_plan_stats._fields_}
        d["solver"] = {0: "bucketed", 1: "levels", 2: "hub", 3: "hub_wide"}.get(st.solver, str(st.solver))
        d["fill_launch"] = {0: None, 1: "serial", 2: "streams", 3: "fused"}.get(st.fill_launch, str(st.fill_launch))
        return d

    def kernel_ms(self) -> Tuple[float, int]:
        n = C.c_uint32()
        ms = lib().mr_plan_kernel_ms(self.handle, C.byref(n))
        return ms, n.value

    def device_outputs(self):
        r, rb, c, cb = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        st = lib().mr_plan_device_outputs(self.handle, C.byref(r), C.byref(rb), C.byref(c), C.byref(cb))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return r.value, rb.value, c.value, cb.value

    def bind_outputs(self, d_results: int, d_commands: int, d_overflow: int = 0, overflow_cap: int = 0) -> None:
        """Caller device buffers for the compact outputs (and, with d_overflow, the
        overflow pool of overflow_cap commands): one collective then moves them all."""
        st = lib().mr_plan_bind_outputs_ex(self.handle, C.c_void_p(d_results), C.c_void_p(d_commands),
                                           C.c_void_p(d_overflow) if d_overflow else None, overflow_cap)
        if st != MR_OK:
            raise EngineError(st, last_error())

    def wire_records(self, d_rows: int, d_pool: int = 0, pool_cap: int = 0, stream=None) -> None:
        """Enqueues the wire encoding of the last pass (mr_plan_wire_records) into caller
        device memory: n rows of wire_row_words(max_cmds) words at d_rows and the pool of
        long labels (pool_cap commands, 8 B each) at d_pool — what a gather then moves."""
        st = lib().mr_plan_wire_records(self.handle, C.c_void_p(d_rows), C.c_void_p(d_pool) if d_pool else None,
                                        pool_cap, C.c_void_p(stream) if stream else None)
        if st != MR_OK:
            raise EngineError(st, last_error())

    def fetch_buffers(self):
        """Host buffers fetch_raw can fill (results, command pool), sized for this plan:
        a caller answering batch after batch allocates them once and passes them back."""
        return fetch_buffers(self.n, self.max_cmds)

    def fetch_raw(self, out=None):
        """(results, command pool) as ctypes arrays, no Python label objects.  The
        buffers are uninitialised host memory (mr_plan_fetch writes every result and
        the commands they point at; a zero-filled pool of n * (max_cmds + 8) commands
        costs seconds at millions of queries); `out` = buffers of fetch_buffers() (of
        this plan or a larger one) to fill instead of new ones."""
        res, pool = out if out is not None else self.fetch_buffers()
        cap = len(pool)
        if len(res) < max(self.n, 1):
            raise EngineError(abi.MR_ERR_INVALID_ARG, "fetch_raw: result buffer shorter than the batch")
        st = lib().mr_plan_fetch(self.handle, res, pool, cap)
        if st < 0 and st not in (abi.MR_ERR_INVALID_INDEX, MR_ERR_CAPACITY):
            raise EngineError(st, last_error())
        return res, pool

    def fetch(self) -> List[Optional[TotalCost]]:
        res = (mr_result * max(self.n, 1))()
        cap = self.n * self.max_cmds + max(4096, self.n * 8)  # slots + overflow pool
        pool = (mr_command * cap)()
        st = lib().mr_plan_fetch(self.handle, res, pool, cap)
        if st < 0 and st != abi.MR_ERR_INVALID_INDEX:
            raise EngineError(st, last_error())
        return [result_from_c(res[i], pool) for i in range(self.n)]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.mr_plan_destroy(h)
            self.handle = None


class SSSPPlan(Plan):
    """All destinations of each source: run() computes a record for
    every (source, cell) on the device; label(i, dst) rebuilds the full TotalCost."""

    def __init__(self, grid: MapGrid, params: Params, sources: Sequence[CellIndex]):
        self.grid = grid
        self.n = len(sources)
        self.sources = list(sources)
        arr = (mr_cell_index * max(self.n, 1))()
        for i, c in enumerate(sources):
            arr[i].kind, arr[i].sub, arr[i].x, arr[i].y = c.kind, c.sub, c.x, c.y
        self._p = params.to_c()
        h = C.c_void_p()
        st = lib().mr_sssp_plan_create(grid.handle, C.byref(self._p), arr, self.n, C.byref(h))
        if st != MR_OK:
            raise EngineError(st, last_error())
        self.handle = h

    def records(self, i: int):
        """(V, 4) uint32 array: legs, money, time, via — row-major cells."""
        import numpy as np
        V = self.grid.square_size ** 2
        out = np.empty((V, 4), dtype=np.uint32)
        st = lib().mr_sssp_records(self.handle, i, out.ctypes.data)
        if st != MR_OK:
            raise EngineError(st, last_error())
        return out

    def device_records(self):
        ptr, n = C.c_void_p(), C.c_uint64()
        st = lib().mr_sssp_device_records(self.handle, C.byref(ptr), C.byref(n))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return ptr.value, n.value

    def record_pitch(self) -> int:
        """Cell words per row of device_records() (rows padded to a multiple of 32)."""
        p = C.c_uint32()
        st = lib().mr_sssp_record_pitch(self.handle, C.byref(p))
        if st != MR_OK:
            raise EngineError(st, last_error())
        return p.value

    def label(self, i: int, dst: CellIndex) -> TotalCost:
        res = mr_result()
        cap = 64
        while True:
            cmds = (mr_command * cap)()
            st = lib().mr_sssp_label(self.handle, i, dst.to_c(), C.byref(res), cmds, cap)
            if st == MR_ERR_CAPACITY and res.n_commands > cap:
                cap = res.n_commands
                continue
            break
        if st != MR_OK:
            raise EngineError(st, last_error())
        res.command_offset = 0
        return result_from_c(res, cmds)

    def labels_raw(self, i: int):
        """Every cell's full label from source i (mr_sssp_labels): (mr_result array of
        V entries in row-major cell order, mr_command pool, commands used)."""
        V = self.grid.square_size ** 2
        res = (mr_result * V)()
        cap = V * 6
        while True:
            pool = (mr_command * cap)()
            st = lib().mr_sssp_labels(self.handle, i, res, pool, cap)
            if st == MR_ERR_CAPACITY:
                need = max(res[V - 1].command_offset + res[V - 1].n_commands, cap + 1)
                cap = need
                continue
            break
        if st != MR_OK:
            raise EngineError(st, last_error())
        used = res[V - 1].command_offset + res[V - 1].n_commands
        return res, pool, used

    def fill_ms(self) -> float:
        """Average fill-kernel time of the window the last kernel_ms() closed."""
        return lib().mr_plan_fill_ms(self.handle)

    def fetch(self):
        raise NotImplementedError("all-destinations plans: use records() / label()")
