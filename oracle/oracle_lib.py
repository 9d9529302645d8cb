"""ctypes loader for the C++ oracle — TEST INFRASTRUCTURE ONLY.

Used by tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() as the
checker; the product package (marshrutka_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from marshrutka_amd.abi import (MR_ERR_CAPACITY, MR_NOT_FOUND, MR_OK, CellIndex, Params, TotalCost,  # noqa: E402
                                cells_to_c, mr_cell, mr_cell_index, mr_command, mr_params,
                                mr_query, mr_result, queries_to_c, result_from_c)

LIB_PATH = os.path.join(HERE, "build", "libmr_oracle.so")


def build(quiet: bool = True) -> str:
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.mro_grid_create.argtypes = [C.POINTER(mr_cell), C.c_uint32, C.POINTER(C.c_void_p)]
        L.mro_grid_create.restype = C.c_int
        L.mro_grid_destroy.argtypes = [C.c_void_p]
        L.mro_grid_nearest_campfire.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(mr_cell_index)]
        L.mro_grid_nearest_campfire_direct.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32,
                                                       C.POINTER(mr_cell_index)]
        L.mro_find_path.argtypes = [C.c_void_p, C.POINTER(mr_params), mr_cell_index, mr_cell_index,
                                    C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint32]
        L.mro_find_path.restype = C.c_int
        L.mro_find_path_batch.argtypes = [C.c_void_p, C.POINTER(mr_params), C.POINTER(mr_query), C.c_uint32,
                                          C.POINTER(mr_result), C.POINTER(mr_command), C.c_uint64, C.c_uint32]
        L.mro_find_path_batch.restype = C.c_int
        L.mro_sssp_all.argtypes = [C.c_void_p, C.POINTER(mr_params), mr_cell_index, C.POINTER(mr_result),
                                   C.POINTER(mr_command), C.c_uint64]
        L.mro_sssp_all.restype = C.c_int
        vp = C.c_void_p
        L.mro_sssp_digest_batch.argtypes = [C.c_void_p, C.POINTER(mr_params), C.POINTER(mr_cell_index), C.c_uint32,
                                            C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.mro_sssp_digest_batch.restype = C.c_int
        L.mro_region_table_bfs.argtypes = [C.c_uint32, vp, vp, C.c_uint32, vp, C.c_uint32]
        L.mro_region_table_bfs.restype = C.c_int
        L.mro_duration_display.argtypes = [C.c_int64, C.c_char_p, C.c_uint32]
        L.mro_duration_display.restype = C.c_int
        _lib = L
    return _lib


class OracleGrid:
    def __init__(self, cells: Sequence[Tuple[CellIndex, int]]):
        self._cells = cells_to_c(cells)
        self._create(self._cells, len(cells))

    @classmethod
    def from_array(cls, arr) -> "OracleGrid":
        """From a numpy record array with mr_cell's layout (mapgen.SyntheticMap.cells_array)."""
        g = cls.__new__(cls)
        g._cells = arr
        g._create(C.cast(arr.ctypes.data, C.POINTER(mr_cell)), len(arr))
        return g

    def _create(self, ptr, n: int) -> None:
        self.n = n
        h = C.c_void_p()
        st = lib().mro_grid_create(ptr, n, C.byref(h))
        if st != MR_OK:
            raise ValueError(f"oracle grid create failed: {st}")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().mro_grid_destroy(self.h)
            self.h = None

    def nearest_campfire(self, i: int, homeland: int, direct: bool = False) -> Optional[CellIndex]:
        out = mr_cell_index()
        f = lib().mro_grid_nearest_campfire_direct if direct else lib().mro_grid_nearest_campfire
        return CellIndex.from_c(out) if f(self.h, i, homeland, C.byref(out)) else None

    def find_path(self, params: Params, src: CellIndex, dst: CellIndex) -> Optional[TotalCost]:
        p = params.to_c()
        res = mr_result()
        cap = 256
        cmds = (mr_command * cap)()
        st = lib().mro_find_path(self.h, C.byref(p), src.to_c(), dst.to_c(), C.byref(res), cmds, cap)
        if st == MR_NOT_FOUND:
            return None
        if st != MR_OK:
            raise ValueError(f"oracle find_path failed: {st}")
        res.command_offset = 0
        return result_from_c(res, cmds)

    def find_path_batch_raw(self, params: Params, queries, threads: int = 0):
        n = len(queries)
        qs = queries_to_c(queries)
        p = params.to_c()
        res = (mr_result * n)()
        cap = max(1, n * 24)
        pool = (mr_command * cap)()
        st = lib().mro_find_path_batch(self.h, C.byref(p), qs, n, res, pool, cap, threads)
        if st < 0:
            raise ValueError(f"oracle batch failed: {st}")
        return res, pool

    def find_path_batch(self, params: Params, queries, threads: int = 0) -> List[Optional[TotalCost]]:
        res, pool = self.find_path_batch_raw(params, queries, threads)
        return [result_from_c(res[i], pool) for i in range(len(queries))]


    def sssp_all(self, params: Params, src: CellIndex) -> List[Optional[TotalCost]]:
        """Every cell's label from src (the reference's Dijkstra without its early
        exit), in the grid's input order."""
        p = params.to_c()
        res = (mr_result * self.n)()
        cap = self.n * 24
        while True:
            pool = (mr_command * cap)()
            st = lib().mro_sssp_all(self.h, C.byref(p), src.to_c(), res, pool, cap)
            if st != MR_ERR_CAPACITY or cap > self.n * 4096:  # grow the pool
                break
            cap *= 4
        if st != MR_OK:
            raise ValueError(f"oracle sssp_all failed: {st}")
        return [result_from_c(res[i], pool) for i in range(self.n)]

    def sssp_digests(self, params: Params, sources, threads: int = 0) -> dict:
        """Every cell's label from each source (the reference's Dijkstra run to
        completion, sources spread over host threads) as numpy arrays of shape
        (len(sources), V) in row-major cell order: legs, money, time_s, n_commands,
        status and `digest`, the command-list digest of tests/label_digest.py."""
        import numpy as np
        n, V = len(sources), self.n
        out = {"legs": np.zeros((n, V), np.uint32), "money": np.zeros((n, V), np.uint32),
               "time_s": np.zeros((n, V), np.int64), "n_commands": np.zeros((n, V), np.uint32),
               "status": np.zeros((n, V), np.int32), "digest": np.zeros((n, V), np.uint64)}
        srcs = (mr_cell_index * max(n, 1))()
        for i, s in enumerate(sources):
            srcs[i] = s.to_c()
        p = params.to_c()
        st = lib().mro_sssp_digest_batch(self.h, C.byref(p), srcs, n, threads,
                                         *(out[k].ctypes.data for k in ("legs", "money", "time_s", "n_commands",
                                                                        "status", "digest")))
        if st != MR_OK:
            raise ValueError(f"oracle sssp_digests failed: {st}")
        return out


def region_table_bfs(S: int, rank, region, nreg: int, threads: int = 0):
    """mro_region_table_bfs: the SoE region table of a map (one BFS per region over the
    grid minus the Center) as a (S*S, nreg, 2) uint32 array {distance, rank}."""
    import numpy as np
    rank = np.ascontiguousarray(rank, dtype=np.uint32)
    region = np.ascontiguousarray(region, dtype=np.uint32)
    out = np.empty((S * S, nreg, 2), dtype=np.uint32)
    st = lib().mro_region_table_bfs(S, rank.ctypes.data, region.ctypes.data, nreg, out.ctypes.data, threads)
    if st != MR_OK:
        raise ValueError(f"oracle region_table_bfs failed: {st}")
    return out


def duration_display(seconds: int) -> str:
    buf = C.create_string_buffer(64)
    lib().mro_duration_display(seconds, buf, 64)
    return buf.value.decode()
