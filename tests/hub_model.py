"""Pure-Python model of the engine's hub solver (csrc/mr_device.hpp, HubSolver)
— TEST INFRASTRUCTURE.  It restates the closed-form algorithm with full
reference labels (oracle/py_ref.py) so its exactness claim can be
checked against the oracle on CPU, independently of the GPU:

  plain v:  L(v) = min over boundaries b of walk(b, d_b(v))     (linear run time)
  specials: exact Dijkstra over walk / CentralMove / caravan / SoE edges,
            SoE from every region through the region cell nearest to each boundary.

Returns None for a source whose order-sensitive tie makes the closed form
inapplicable (the engine re-solves those with the SSSP kernel).
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import py_ref  # noqa: E402
from py_ref import CARAVAN, CENTER, CENTRAL, NOMOVE, SFM, SHQ, SOE, STANDARD  # noqa: E402


def walk_dist(a, b):
    (ax, ay), (bx, by) = a, b
    d = abs(ax - bx) + abs(ay - by)
    if (ay == 0 and by == 0 and ax != 0 and bx != 0 and (ax < 0) != (bx < 0)) or \
       (ax == 0 and bx == 0 and ay != 0 and by != 0 and (ay < 0) != (by < 0)):
        d += 2
    return d


class HubModel:
    def __init__(self, grid: py_ref.Grid, params: dict):
        self.g = grid
        self.f = py_ref.Finder(grid, params)
        self.p = params
        g = grid
        S = g.size
        self.specials = [CENTER] + [py_ref.bd(b, 1) for b in range(4)]
        for c in g.campfires:
            if c not in self.specials:
                self.specials.append(c)
        hq = self.f.hq
        if hq is not None and hq not in self.specials:
            self.specials.append(hq)
        self.home = params["homeland"]
        self.regions = sorted(c for c in g.campfires if c[0] == 1 and c[1] == self.home)
        # nearest region cell per (vertex, region): BFS over the grid minus the Center
        self.cells = list(g.pos.keys())
        self.near = {}
        rank = {c: i for i, c in enumerate(sorted(self.cells))}
        bypos = {v: k for k, v in g.pos.items()}
        for r in self.regions:
            src = [u for u in self.cells if u != CENTER and g.nearest[(u, self.home)] == r]
            dist = {u: (0, rank[u], u) for u in src}
            frontier = list(src)
            d = 0
            while frontier:
                nxt = {}
                for u in frontier:
                    x, y = g.pos[u]
                    for w in ((x - 1, y), (x + 1, y), (x, y - 1), (x, y + 1)):
                        wc = bypos.get(w)
                        if wc is None or wc == CENTER or wc in dist:
                            continue
                        cand = (d + 1, dist[u][1], dist[u][2])
                        if wc not in nxt or cand < nxt[wc]:
                            nxt[wc] = cand
                dist.update(nxt)
                frontier = list(nxt)
                d += 1
            for v, (dd, _, u) in dist.items():
                self.near[(v, r)] = (dd, u)

    def walk(self, blabel, bvert, k, v):
        """blabel extended by k StandardMoves ending at v (merged run)."""
        lab = blabel
        cur = bvert
        # k single steps; the target of intermediate steps does not matter once merged
        for i in range(k):
            lab = self.f.extend(lab, cur, v, STANDARD, None)
            cur = v
        return lab

    def solve(self, src, dsts):
        f = self.f
        key = f.key
        g = self.g
        start = (0, 0, 0, (((NOMOVE,), src, src),))
        lab = {}      # tentative labels of specials
        settled = {}
        best_walk = {}
        boundaries = [(src, start)] if src != CENTER else []

        def offer(t, cand, is_walk=False):
            if t in settled:
                return
            if is_walk:
                bw = best_walk.get(t)
                m = key(cand)[:3]
                if bw is None or m < bw:
                    best_walk[t] = m
            if t not in lab or key(cand) < key(lab[t]):
                lab[t] = cand

        def relax_boundary(b, blab):
            for t in self.specials:
                if t == CENTER or t == b:
                    continue
                d = walk_dist(g.pos[b], g.pos[t])
                offer(t, self.walk(blab, b, d, t), is_walk=True)
            if f.use_soe:
                for r in self.regions:
                    d, u = self.near.get((b, r), (None, None))
                    if d is None or (d == 0 and b != src):
                        continue
                    base = self.walk(blab, b, d, u) if d > 0 else blab
                    offer(r, f.extend(base, u, r, SOE, None))

        if src in self.specials:
            offer(src, start)
        if f.hq is not None:
            offer(f.hq, f.extend(start, src, f.hq, SHQ, None))
        if f.use_sfm:
            offer(CENTER, f.extend(start, src, CENTER, SFM, None))
        if src != CENTER:
            relax_boundary(src, start)
        tie = False
        while True:
            cands = [t for t in lab if t not in settled]
            if not cands:
                break
            s = min(cands, key=lambda t: key(lab[t]))
            L = lab[s]
            settled[s] = L
            last = L[3][-1][0][0]
            boundary = last not in (NOMOVE, STANDARD)
            if boundary and best_walk.get(s) == key(L)[:3]:
                tie = True
            for w, kind, car in f.edges(s):
                if kind in (CENTRAL, CARAVAN, SOE) and w in self.specials:
                    offer(w, f.extend(L, s, w, kind, car))
            if boundary and s != CENTER:
                boundaries.append((s, L))
                relax_boundary(s, L)
        if tie:
            return None
        out = {}
        for w in dsts:
            if w == src:
                out[w] = start
            elif w in self.specials:
                out[w] = settled[w]
            else:
                best = None
                for b, bl in boundaries:
                    c = self.walk(bl, b, walk_dist(g.pos[b], g.pos[w]), w)
                    if best is None or key(c) < key(best):
                        best = c
                out[w] = best
        return out
