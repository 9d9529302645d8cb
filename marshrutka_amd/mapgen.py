"""Synthetic ChatWars-style maps.

The reference ships no map (it is fetched at runtime, src/app.rs:654-702), so
every workload is a synthetic map in the reference's own cell schema:

* odd side S = 2H+1, cell i at x = i % S - H, y = i // S - H (src/grid.rs:64-77);
* quadrants consistent with the index adjacency of src/pathfinder.rs:24-138 and
  src/homeland.rs:66-77:  Blue (x<0,y<0), Red (x<0,y>0), Green (x>0,y>0),
  Yellow (x>0,y<0); borders BR (y=0,x<0), RG (x=0,y>0), GY (y=0,x>0),
  YB (x=0,y<0); homeland pos = (|x|,|y|), border shift = |x|+|y|;
* campfires placed per homeland by a splitmix64 stream.

`to_html` writes the same map in the HTML schema MapGrid::parse reads
(src/grid.rs:47-120,337-369) so a real map and a synthetic one are
interchangeable inputs.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from .abi import (BLUE, BORDER_NAMES, BR, CELL_BORDER, CELL_CENTER, CELL_HOMELAND, GREEN, GY,
                  HOMELAND_ABBREV, POI_CAMPFIRE, POI_FORUM, POI_FOUNTAIN, POI_NONE, RED, RG,
                  YB, YELLOW, CellIndex)

MASK64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n


def geo_to_index(x: int, y: int) -> CellIndex:
    if x == 0 and y == 0:
        return CellIndex.center()
    if y == 0:
        return CellIndex.border(BR if x < 0 else GY, abs(x))
    if x == 0:
        return CellIndex.border(RG if y > 0 else YB, abs(y))
    if x < 0:
        return CellIndex.homeland(BLUE if y < 0 else RED, -x, abs(y))
    return CellIndex.homeland(GREEN if y > 0 else YELLOW, x, abs(y))


def index_to_geo(ci: CellIndex) -> Tuple[int, int]:
    if ci.kind == CELL_CENTER:
        return 0, 0
    if ci.kind == CELL_BORDER:
        s = ci.x
        return {BR: (-s, 0), GY: (s, 0), RG: (0, s), YB: (0, -s)}[ci.sub]
    sx = -1 if ci.sub in (BLUE, RED) else 1
    sy = -1 if ci.sub in (BLUE, YELLOW) else 1
    return sx * ci.x, sy * ci.y


def homeland_quadrant(h: int) -> Tuple[int, int]:
    return {BLUE: (-1, -1), RED: (-1, 1), GREEN: (1, 1), YELLOW: (1, -1)}[h]


class SyntheticMap:
    """Row-major list of (CellIndex, poi) for an odd S."""

    def __init__(self, size: int, campfires_per_homeland: int = 4, seed: int = 1,
                 clustered: bool = False, extra_campfires: Sequence[CellIndex] = (),
                 fountains: int = 1, forums: int = 1):
        if size < 3 or size % 2 == 0:
            raise ValueError("square size must be odd and >= 3 (SURVEY §8a A14)")
        self.size = size
        self.h = size // 2
        self.seed = seed
        rng = SplitMix64(seed)
        poi: Dict[Tuple[int, int], int] = {}
        H = self.h
        for hl in (BLUE, RED, GREEN, YELLOW):
            sx, sy = homeland_quadrant(hl)
            k = min(campfires_per_homeland, H * H)
            placed = 0
            misses = 0
            if clustered and k > 0:
                cx, cy = 1 + rng.below(H), 1 + rng.below(H)
                rad = max(1, H // 8)
            while placed < k:
                if clustered:
                    px = min(H, max(1, cx + rng.below(2 * rad + 1) - rad))
                    py = min(H, max(1, cy + rng.below(2 * rad + 1) - rad))
                else:
                    px, py = 1 + rng.below(H), 1 + rng.below(H)
                key = (sx * px, sy * py)
                if key in poi:
                    misses += 1
                    if clustered and misses > 8 * k:
                        rad, misses = rad + 1, 0
                    continue
                poi[key] = POI_CAMPFIRE
                placed += 1
        for ci in extra_campfires:
            poi[index_to_geo(ci)] = POI_CAMPFIRE
        # decorative PoIs (unused by the path, src/pathfinder.rs:177 targets Center)
        for kind, count in ((POI_FOUNTAIN, fountains), (POI_FORUM, forums)):
            for _ in range(count):
                for _try in range(64):
                    x, y = rng.below(size) - H, rng.below(size) - H
                    if (x, y) != (0, 0) and (x, y) not in poi:
                        poi[(x, y)] = kind
                        break
        self.poi = poi

    def cells(self) -> List[Tuple[CellIndex, int]]:
        H, S = self.h, self.size
        out = []
        for i in range(S * S):
            x, y = i % S - H, i // S - H
            out.append((geo_to_index(x, y), self.poi.get((x, y), POI_NONE)))
        return out

    def all_indices(self) -> List[CellIndex]:
        return [ci for ci, _ in self.cells()]

    def index_at(self, i: int) -> CellIndex:
        """CellIndex of row-major cell i (no list of all cells)."""
        return geo_to_index(i % self.size - self.h, i // self.size - self.h)

    def cells_array(self):
        """The cells as a numpy record array with mr_cell's layout (16 B per cell),
        vectorised for large maps (S = 4097: 16.8 M cells); same content as cells()."""
        import numpy as np
        S, H = self.size, self.h
        dt = np.dtype([("kind", "u1"), ("sub", "u1"), ("x", "<u2"), ("y", "<u2"), ("res", "<u2"),
                       ("poi", "u1"), ("pad", "u1", (7,))])
        out = np.zeros(S * S, dtype=dt)
        x = (np.arange(S, dtype=np.int32) - H)[None, :].repeat(S, 0).ravel()
        y = (np.arange(S, dtype=np.int32) - H)[:, None].repeat(S, 1).ravel()
        kind = np.full(S * S, CELL_HOMELAND, np.uint8)
        sub = np.where(x < 0, np.where(y < 0, BLUE, RED), np.where(y > 0, GREEN, YELLOW)).astype(np.uint8)
        ix, iy = np.abs(x), np.abs(y)
        on_y0, on_x0 = (y == 0) & (x != 0), (x == 0) & (y != 0)
        kind[on_y0 | on_x0] = CELL_BORDER
        sub[on_y0] = np.where(x[on_y0] < 0, BR, GY)
        sub[on_x0] = np.where(y[on_x0] > 0, RG, YB)
        bx = np.where(on_y0, ix, np.where(on_x0, iy, ix))
        by = np.where(on_y0 | on_x0, 0, iy)
        c = (x == 0) & (y == 0)
        kind[c], sub[c], bx[c], by[c] = CELL_CENTER, 0, 0, 0
        out["kind"], out["sub"], out["x"], out["y"] = kind, sub, bx, by
        for (px, py), p in self.poi.items():
            out["poi"][(py + H) * S + (px + H)] = p
        return out

    def query_array(self, src: Sequence[int], dst: Sequence[int], cells=None):
        """Queries (row-major cell src[i] -> cell dst[i]) as a numpy array with
        mr_query's 16 B layout (pathfinder.Plan(query_array=...)), vectorised;
        `cells` = this map's cells_array() when the caller already has it."""
        import numpy as np
        if cells is None:
            cells = self.cells_array()
        ix = np.dtype([("kind", "u1"), ("sub", "u1"), ("x", "<u2"), ("y", "<u2"), ("res", "<u2")])
        out = np.zeros(len(src), dtype=np.dtype([("from", ix), ("to", ix)]))
        for side, idx in (("from", np.asarray(src, dtype=np.int64)), ("to", np.asarray(dst, dtype=np.int64))):
            for f in ("kind", "sub", "x", "y"):
                out[side][f] = cells[f][idx]
        return out

    def cell_of(self, ci: CellIndex) -> int:
        """Row-major position of a cell (inverse of index_at)."""
        x, y = index_to_geo(ci)
        return (y + self.h) * self.size + (x + self.h)

    def campfires(self) -> List[CellIndex]:
        return sorted(geo_to_index(x, y) for (x, y), p in self.poi.items() if p == POI_CAMPFIRE)

    def to_json(self) -> dict:
        return {"size": self.size, "poi": [[x, y, p] for (x, y), p in sorted(self.poi.items())]}

    @staticmethod
    def from_json(d: dict) -> "SyntheticMap":
        m = SyntheticMap.__new__(SyntheticMap)
        m.size = d["size"]
        m.h = m.size // 2
        m.seed = None
        m.poi = {(x, y): p for x, y, p in d["poi"]}
        return m


# ---- HTML schema (src/grid.rs:47-120, 337-369; src/index.rs:419-431) --------
_POI_EMOJI = {POI_CAMPFIRE: "\U0001F525", POI_FOUNTAIN: "⛲", POI_FORUM: "\U0001F3DB"}
_HOMELAND_COLOURS = ["#3b82f6", "#ef4444", "#22c55e", "#eab308"]


def to_html(m: SyntheticMap) -> str:
    parts = ['<html><body><div class="map-grid">']
    for ci, poi in m.cells():
        if ci.kind == CELL_CENTER:
            br, tr, colour = None, "0#0", "#ffffff"
        elif ci.kind == CELL_HOMELAND:
            br, tr, colour = HOMELAND_ABBREV[ci.sub], f"{ci.x}#{ci.y}", _HOMELAND_COLOURS[ci.sub]
        else:
            br, tr, colour = BORDER_NAMES[ci.sub], str(ci.x), "#cccccc"
        cell = [f'<div class="map-cell" style="background-color:{colour}">']
        if poi in _POI_EMOJI:
            cell.append(_POI_EMOJI[poi])
        cell.append(f'<div class="top-right-text">{tr}</div>')
        if br is not None:
            cell.append(f'<div class="bottom-right-text">{br}</div>')
        cell.append("</div>")
        parts.append("".join(cell))
    parts.append("</div></body></html>")
    return "\n".join(parts)


def random_queries(m: SyntheticMap, n: int, seed: int) -> List[Tuple[CellIndex, CellIndex]]:
    rng = SplitMix64(seed ^ 0x5DEECE66D)
    V = m.size * m.size
    return [(m.index_at(rng.below(V)), m.index_at(rng.below(V))) for _ in range(n)]


def random_query_cells(m: SyntheticMap, n: int, seed: int):
    """random_queries as row-major cell numbers, vectorised: (src, dst) int64 arrays
    with src[i] / dst[i] the cells of random_queries(m, n, seed)[i] (the same
    splitmix64 stream: draw 2i is the source, 2i + 1 the destination)."""
    import numpy as np
    V = m.size * m.size
    with np.errstate(over="ignore"):
        s0 = np.uint64((seed ^ 0x5DEECE66D) & MASK64)
        z = s0 + np.arange(1, 2 * n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    cell = (z % np.uint64(V)).astype(np.int64)
    return cell[0::2], cell[1::2]


def random_sources_queries(m: SyntheticMap, n: int, n_sources: int, seed: int):
    """Queries drawn from a fixed pool of n_sources sources (SSSP-style batches)."""
    rng = SplitMix64(seed ^ 0x2545F4914F6CDD1D)
    idx = m.all_indices()
    V = len(idx)
    srcs = [idx[rng.below(V)] for _ in range(n_sources)]
    return [(srcs[rng.below(n_sources)], idx[rng.below(V)]) for _ in range(n)]
