"""The SoE region table's inputs and a numpy model of its device build (test
infrastructure for tests/test_region_table.py and tests/test_gpu_region_table.py).

* cell_ranks: every cell's CellIndex rank (derived Ord, src/index.rs:41-46: variant,
  then homeland / border, then x, y), by a sort of the cells' (kind, sub, x, y).
* cell_regions: every cell's region = the index (CellIndex order) of its nearest
  Homeland-indexed campfire of `homeland`, by the direct argmin of the reference's key
  (Manhattan distance, |fx| != |fy|, |fx| + |fy|, |fx|, |fy|; src/grid.rs:297-325), the
  Center none; independent of the engine's multi-source BFS.
* transform_model: the three passes of marshrutka_amd/csrc/mr_k_region.hip in numpy.
"""
from __future__ import annotations

import numpy as np

from marshrutka_amd.abi import CELL_HOMELAND, POI_CAMPFIRE

NONE = np.uint32(0xFFFFFFFF)


def cell_ranks(arr) -> np.ndarray:
    order = np.lexsort((arr["y"], arr["x"], arr["sub"], arr["kind"]))
    rank = np.empty(len(arr), dtype=np.uint32)
    rank[order] = np.arange(len(arr), dtype=np.uint32)
    return rank


def cell_regions(arr, homeland: int, chunk: int = 1 << 20):
    """(regions per cell as uint32 with 0xFFFFFFFF for none, number of regions)."""
    V = len(arr)
    S = int(round(V ** 0.5))
    H = S // 2
    rank = cell_ranks(arr)
    cf = np.nonzero((arr["poi"] == POI_CAMPFIRE) & (arr["kind"] == CELL_HOMELAND) & (arr["sub"] == homeland))[0]
    cf = cf[np.argsort(rank[cf])]  # CellIndex order
    fx, fy = (cf % S).astype(np.int64) - H, (cf // S).astype(np.int64) - H
    ax, ay = np.abs(fx), np.abs(fy)
    tie = ((ax != ay).astype(np.int64) << 62) | ((ax + ay) << 40) | (ax << 20) | ay
    out = np.full(V, NONE, dtype=np.uint32)
    for lo in range(0, V, chunk):
        v = np.arange(lo, min(V, lo + chunk), dtype=np.int64)
        x, y = v % S - H, v // S - H
        d = np.abs(x[:, None] - fx[None, :]) + np.abs(y[:, None] - fy[None, :])
        # lexicographic (distance, tie key): distance < 2^20 here, tie key < 2^63
        best = np.zeros(len(v), dtype=np.int64)
        bd = d[:, 0].copy()
        bt = np.full(len(v), tie[0])
        for j in range(1, len(cf)):
            better = (d[:, j] < bd) | ((d[:, j] == bd) & (tie[j] < bt))
            best = np.where(better, j, best)
            bd = np.where(better, d[:, j], bd)
            bt = np.where(better, tie[j], bt)
        out[lo:lo + len(v)] = best.astype(np.uint32)
    out[H * S + H] = NONE
    return out, len(cf)


def _lex_min(a, b):
    """Elementwise lexicographic min of (..., 2) uint32 arrays."""
    take_b = (b[..., 0] < a[..., 0]) | ((b[..., 0] == a[..., 0]) & (b[..., 1] < a[..., 1]))
    return np.where(take_b[..., None], b, a)


def _plus1(a):
    out = a.copy()
    m = a[..., 0] != NONE
    out[..., 0][m] += 1
    return out


def _line_transform(region_line, rank_line, nreg, split_at=None):
    """Per region the nearest region cell along one line (left/right sweeps); with
    split_at the cell there separates the two halves (the Center)."""
    n = len(region_line)
    out = np.full((n, nreg, 2), NONE, dtype=np.uint32)
    for r in range(nreg):
        pos = np.nonzero(region_line == r)[0]
        for x in range(n):
            cands = pos if split_at is None else (pos[pos < split_at] if x < split_at else pos[pos > split_at])
            if x == split_at or cands.size == 0:
                continue
            d = np.abs(cands - x)
            k = np.lexsort((rank_line[cands], d))[0]
            out[x, r] = (d[k], rank_line[cands[k]])
    return out


def transform_model(S: int, rank, region, nreg: int) -> np.ndarray:
    """The device passes (rows, columns, axis lines) in numpy: (S*S, nreg, 2)."""
    H = S // 2
    reg = region.reshape(S, S)
    rk = rank.reshape(S, S)
    T = np.stack([_line_transform(reg[y], rk[y], nreg) for y in range(S)])  # (y, x, r, 2)
    axh = _line_transform(reg[H], rk[H], nreg, split_at=H)
    axv = _line_transform(reg[:, H], rk[:, H], nreg, split_at=H)
    f = np.full((S, nreg, 2), NONE, dtype=np.uint32)
    for y in range(S):  # down
        f = _lex_min(T[y], _plus1(f))
        T[y] = f
    b = np.full((S, nreg, 2), NONE, dtype=np.uint32)
    for y in range(S - 1, -1, -1):  # up
        b = _lex_min(T[y], _plus1(b))
        T[y] = b
    row_above, row_below = T[H - 1].copy(), T[H + 1].copy()
    col_left, col_right = T[:, H - 1].copy(), T[:, H + 1].copy()
    T[H] = _lex_min(axh, _lex_min(_plus1(row_above), _plus1(row_below)))
    T[:, H] = _lex_min(axv, _lex_min(_plus1(col_left), _plus1(col_right)))
    T[H, H] = NONE
    return T.reshape(S * S, nreg, 2)
