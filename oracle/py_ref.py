"""py_ref.py — TEST INFRASTRUCTURE ONLY.

An independent pure-Python restatement of the reference pathfinder, written
separately from the C++ oracle (oracle/mr_oracle.cpp) so the two can
cross-check each other on small grids.  It is slow (pure-Python loops) and is
only run on grids with S <= ~21.  Its outputs are committed as golden vectors
under tests/golden/ (tests/golden/make_golden.py).

Followed, item by item:
  FindPath::eval                src/pathfinder.rs:199-248
  Inflight::edges               src/pathfinder.rs:24-180
  caravan_cost                  src/pathfinder.rs:251-273
  EdgeCost legs/money/time      src/cost.rs:35-74
  AggregatedCost (Ord, time..)  src/cost.rs:90-151
  From<EdgeCost..>              src/cost.rs:153-185
  TotalCost += (extension)      src/cost.rs:208-315
  comparator / eval_next        src/cost.rs:370-427
  CellIndex Ord / build         src/index.rs:41-46, 257-312
  Border/Homeland topology      src/index.rs:339-353, src/homeland.rs:57-96
  Skill::time                   src/skill.rs:21-71
  MapGrid / nearest_campfire    src/grid.rs:47-237, 297-325 (direct argmin form)
"""
from __future__ import annotations

import heapq
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

# CellIndex as a plain tuple (variant, a, b, c) ordered like the derived Ord:
#   Center          -> (0, 0, 0, 0)
#   Homeland{h,x,y} -> (1, h, x, y)
#   Border{b,s}     -> (2, b, s, 0)
CENTER = (0, 0, 0, 0)
BLUE, RED, GREEN, YELLOW = range(4)
BR, RG, GY, YB = range(4)

RG_TABLE = {0: Fraction(1), 1: Fraction(19, 24), 2: Fraction(7, 10), 3: Fraction(73, 120),
            4: Fraction(31, 60), 5: Fraction(51, 120)}
FF_TABLE = {0: Fraction(1), 1: Fraction(50, 53), 2: Fraction(100, 109), 3: Fraction(25, 28)}

NOMOVE, CENTRAL, STANDARD, CARAVAN, SOE, SHQ, SFM = range(7)
LEGS, TIME, MONEY = range(3)
U32 = (1 << 32) - 1


def hl(h, x, y):
    if x == 0 and y == 0:
        return CENTER
    if x == 0:
        return (2, YB if h in (YELLOW, BLUE) else RG, y, 0)
    if y == 0:
        return (2, BR if h in (BLUE, RED) else GY, x, 0)
    return (1, h, x, y)


def bd(b, s):
    return CENTER if s == 0 else (2, b, s, 0)


def skill(table, level, t):
    r = table.get(level)
    if r is None:
        return None
    if r == 1:
        return t
    v = r * t
    return -((-v.numerator) // v.denominator)  # ceil


class Grid:
    def __init__(self, cells):
        """cells: row-major list of (index tuple, poi)."""
        n = len(cells)
        s = int(round(n ** 0.5))
        assert s * s == n
        self.size = s
        H = s // 2
        self.pos = {}
        self.poi = {}
        for i, (ci, p) in enumerate(cells):
            self.pos[ci] = (i % s - H, i // s - H)
            self.poi[ci] = p
        self.campfires = sorted(c for c, p in self.poi.items() if p == 1)
        self.nearest = {}
        for h in range(4):
            cf = [c for c in self.campfires if c[0] == 1 and c[1] == h]
            for c in self.pos:
                if c in cf:
                    self.nearest[(c, h)] = c
                    continue
                best = None
                for f in cf:
                    fx, fy = self.pos[f]
                    ax, ay = abs(fx), abs(fy)
                    key = (self.dist(c, f), ax != ay, ax + ay, ax, ay)
                    if best is None or key < best[0]:
                        best = (key, f)
                self.nearest[(c, h)] = None if best is None else best[1]

    def dist(self, a, b):
        (ax, ay), (bx, by) = self.pos[a], self.pos[b]
        return abs(ax - bx) + abs(ay - by)


def agg_time(a):
    kind = a[0]
    if kind in (CENTRAL, CARAVAN):
        return a[1]
    if kind == STANDARD:
        t = skill(FF_TABLE, a[3], a[1])
        return a[1] if t is None else t
    return 0


def agg_money(a):
    kind = a[0]
    if kind == CARAVAN:
        return a[2]
    if kind in (SOE, SHQ, SFM):
        return a[1]
    return 0


def agg_legs(a):
    return a[2] if a[0] == STANDARD else 0


# AggregatedCost as tuples whose natural tuple order is the derived Ord:
#   NoMove (0,) ; Central (1, time) ; Standard (2, time, legs, ff)
#   Caravan (3, time, money) ; SoE/SHQ/SFm (k, money)
def agg_of_edge(kind, car, costs, ff):
    if kind == NOMOVE:
        return (NOMOVE,)
    if kind == CENTRAL:
        return (CENTRAL, 10)
    if kind == STANDARD:
        return (STANDARD, 180, 1, ff)
    if kind == CARAVAN:
        return (CARAVAN, car[0], car[1])
    return (kind, costs[kind])


class Finder:
    def __init__(self, grid: Grid, params: dict):
        self.g = grid
        p = params
        self.costs = {SOE: p["scroll_of_escape_cost"], SHQ: p["scroll_of_escape_hq_cost"],
                      SFM: p["scroll_of_escape_forum_cost"]}
        self.use_soe, self.use_sfm, self.use_caravans = p["use_soe"], p["use_sfm"], p["use_caravans"]
        self.hq = tuple(p["hq_position"]) if p.get("hq_position") is not None else None
        self.rg, self.ff = p["route_guru"], p["fleetfoot"]
        self.home = p["homeland"]
        c1, c2 = p["sort_by"]
        if c1 == c2:
            c2 = TIME if c1 == LEGS else LEGS
        c3 = ({LEGS, TIME, MONEY} - {c1, c2}).pop()
        self.order = (c1, c2, c3)

    def key(self, label):
        legs, money, time, cmds = label
        m = {LEGS: legs, MONEY: money, TIME: time}
        return (m[self.order[0]], m[self.order[1]], m[self.order[2]], len(cmds), cmds)

    def caravan(self, a, b):
        d = self.g.dist(a, b)
        if b == CENTER or (b[0] == 1 and b[1] == self.home):
            coef = 2
        else:
            coef = 5
        t = skill(RG_TABLE, self.rg, 240)
        t = 240 if t is None else t
        return (t * d, (coef * d) & U32)

    def edges(self, v):
        H = self.g.size // 2
        out = []
        if v == CENTER:
            out += [(bd(b, 1), CENTRAL, None) for b in range(4)]
        elif v[0] == 2:
            b, s = v[1], v[2]
            out.append((CENTER, CENTRAL, None) if s == 1 else (bd(b, s - 1), STANDARD, None))
            if s < H:
                out.append((bd(b, s + 1), STANDARD, None))
            nbs = {BR: (BLUE, RED), RG: (RED, GREEN), GY: (GREEN, YELLOW), YB: (YELLOW, BLUE)}[b]
            horizontal = b in (BR, GY)
            for h in nbs:
                out.append((hl(h, s, 1) if horizontal else hl(h, 1, s), STANDARD, None))
        else:
            h, x, y = v[1], v[2], v[3]
            vert = {BLUE: YB, RED: RG, GREEN: RG, YELLOW: YB}[h]
            hor = {BLUE: BR, RED: BR, GREEN: GY, YELLOW: GY}[h]
            out.append((bd(vert, y) if x == 1 else hl(h, x - 1, y), STANDARD, None))
            out.append((bd(hor, x) if y == 1 else hl(h, x, y - 1), STANDARD, None))
            if x < H:
                out.append((hl(h, x + 1, y), STANDARD, None))
            if y < H:
                out.append((hl(h, x, y + 1), STANDARD, None))
        if self.use_caravans and (v == CENTER or v in self.g.campfires):
            for t in [CENTER] + self.g.campfires:
                if t != v:
                    out.append((t, CARAVAN, self.caravan(v, t)))
        if self.use_soe:
            nc = self.g.nearest[(v, self.home)]
            if nc is not None:
                out.append((nc, SOE, None))
        if self.hq is not None:
            out.append((self.hq, SHQ, None))
        if self.use_sfm:
            out.append((CENTER, SFM, None))
        return out

    def extend(self, label, v, w, kind, car):
        cmds = list(label[3])
        last_agg, last_from, _ = cmds[-1]
        if last_agg[0] == NOMOVE:
            agg = agg_of_edge(kind, car, self.costs, self.ff)
            frm = last_from
            cmds.pop()
        elif last_agg[0] == STANDARD and kind == STANDARD:
            agg = (STANDARD, last_agg[1] + 180, last_agg[2] + 1, last_agg[3])
            frm = last_from
            cmds.pop()
        elif last_agg[0] == CENTRAL and kind == CENTRAL:
            agg = (CENTRAL, last_agg[1] + 10)
            frm = last_from
            cmds.pop()
        else:
            agg = agg_of_edge(kind, car, self.costs, self.ff)
            frm = v
        cmds.append((agg, frm, w))
        legs = sum(agg_legs(c[0]) for c in cmds) & U32
        money = sum(agg_money(c[0]) for c in cmds) & U32
        time = sum(agg_time(c[0]) for c in cmds)
        return (legs, money, time, tuple(cmds))

    def eval(self, src, dst):
        start = (0, 0, 0, (((NOMOVE,), src, src),))
        if src == dst:
            return start
        dist = {src: start}
        heap = [(self.key(start), start)]
        while heap:
            _, cost = heapq.heappop(heap)
            v = cost[3][-1][2]
            if v == dst:
                return cost
            if self.key(cost) > self.key(dist[v]):
                continue
            for w, kind, car in self.edges(v):
                nxt = self.extend(cost, v, w, kind, car)
                old = dist.get(w)
                if old is None or self.key(nxt) < self.key(old):
                    dist[w] = nxt
                    heapq.heappush(heap, (self.key(nxt), nxt))
        return None


def label_to_json(label) -> Optional[dict]:
    """Same field layout as mr_result/mr_command (agg fields flattened)."""
    if label is None:
        return None
    legs, money, time, cmds = label
    out = []
    for agg, frm, to in cmds:
        k = agg[0]
        c = {"kind": k, "time_s": 0, "legs": 0, "money": 0, "fleetfoot": 0}
        if k == CENTRAL:
            c["time_s"] = agg[1]
        elif k == STANDARD:
            c["time_s"], c["legs"], c["fleetfoot"] = agg[1], agg[2], agg[3]
        elif k == CARAVAN:
            c["time_s"], c["money"] = agg[1], agg[2]
        elif k in (SOE, SHQ, SFM):
            c["money"] = agg[1]
        c["from"] = list(frm)
        c["to"] = list(to)
        out.append(c)
    return {"legs": legs, "money": money, "time_s": time, "commands": out}


# ---- the app's command table (src/app.rs:481-561) — test-side restatement --------
FF_LEVEL_RATIO = {1: (50, 53), 2: (100, 109), 3: (25, 28)}   # src/skill.rs:65-71


def command_time(c: dict) -> int:
    """AggregatedCost::time (src/cost.rs:118-150) on a label_to_json command."""
    if c["kind"] in (CENTRAL, CARAVAN):
        return c["time_s"]
    if c["kind"] == STANDARD:
        r = FF_LEVEL_RATIO.get(c["fleetfoot"])
        return c["time_s"] if r is None else -(-c["time_s"] * r[0] // r[1])
    return 0


def duration_str(s: int) -> str:
    """time 0.3 Duration Display (src/pathfinder.rs:279-285 pins "1h3m10s")."""
    if s == 0:
        return "0s"
    a, out = abs(s), ("-" if s < 0 else "")
    for v, u in ((a // 86400, "d"), (a // 3600 % 24, "h"), (a // 60 % 60, "m"), (a % 60, "s")):
        if v:
            out += f"{v}{u}"
    return out


def command_suffix(ci) -> str:
    """CellIndexCommandSuffix (src/index.rs:378-390) on a (kind, sub, x, y) tuple."""
    kind, sub, x, y = ci
    if kind == 0:
        return "0_0"
    if kind == 1:
        return f"{'brgy'[sub]}_{x}_{y}"
    return f"{['br', 'rg', 'gy', 'yb'][sub]}_{x}"


def render_schedule(label_json: dict, arrive_at_s: int, pause_s: int):
    """Rows (command, duration, total, start) of the app's table (src/app.rs:481-561)."""
    cmds = [c for c in label_json["commands"] if c["kind"] != NOMOVE]
    times, acc = [], arrive_at_s
    for c in reversed(cmds):
        acc -= command_time(c) + pause_s
        times.append(acc)
    times.reverse()
    rows, total = [], 0
    names = {SOE: "/use_soe", SHQ: "/use_shq", SFM: "/use_sfm"}
    for c, at in zip(cmds, times):
        if c["kind"] in (CENTRAL, STANDARD):
            cmd = "/go_direct_" + command_suffix(tuple(c["to"]))
        elif c["kind"] == CARAVAN:
            cmd = "/car_" + command_suffix(tuple(c["to"]))
        else:
            cmd = names[c["kind"]]
        t = command_time(c)
        total += t + pause_s
        tod = at % 86400
        rows.append((cmd, duration_str(t), duration_str(total), f"{tod // 3600:02d}:{tod // 60 % 60:02d}:{tod % 60:02d}"))
    return rows
