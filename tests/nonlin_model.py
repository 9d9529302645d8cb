"""Pure-Python model of the hub solver's certification for non-linear run times
(Fleetfoot 1..3; csrc/mr_device.hpp near_tie / path_tie / walk_clear, DESIGN.md
section 3a'') — TEST INFRASTRUCTURE.  Labels come from the oracle; the model says
whether the closed form walk(b, d_b(v)) is certified, and the tests check that a
certified label is the oracle's."""
from __future__ import annotations

import math

from hub_model import walk_dist

FF_RATIO = {1: (50, 53), 2: (100, 109), 3: (25, 28)}  # src/skill.rs Fleetfoot ratios
LEGS, MONEY, TIME = 0, 1, 2  # metric indices as in the engine (Rec.m[])


def run_time(k: int, ff: int) -> int:
    n, d = FF_RATIO.get(ff, (1, 1))
    return -(-180 * k * n // d)


def perm_of(sort_by) -> tuple:
    """CostComparator::eval_next (src/cost.rs:387-405) in metric indices."""
    code = {0: LEGS, 1: TIME, 2: MONEY}  # SORT_LEGS, SORT_TIME, SORT_MONEY
    c1, c2 = sort_by
    if c2 == c1:
        c2 = {0: 1, 1: 0, 2: 0}[c1]
    c3 = ({0, 1, 2} - {c1, c2}).pop()
    return code[c1], code[c2], code[c3]


def metrics(lab):
    return (lab.legs, lab.money, lab.time_s)


def near_tie(mq, gq, mb, gb, gv, perm, ff) -> bool:
    n, d = FF_RATIO[ff]
    before = perm[:perm.index(TIME)]
    (qx, qy), (bx, by), (vx, vy) = gq, gb, gv
    mlo = abs(qx - vx) + abs(qy - vy) - abs(bx - vx) - abs(by - vy)
    mhi = abs(qx - bx) + abs(qy - by) + 2
    d0 = mq[TIME] - mb[TIME]
    if MONEY in before and mq[MONEY] != mb[MONEY]:
        return False

    def gap_hits(m):
        a = 180 * n * abs(m)
        lo, hi = a // d, -(-a // d)
        if m < 0:
            lo, hi = -hi, -lo
        return d0 + lo in (-1, 0) or d0 + hi in (-1, 0)
    if LEGS in before:
        m = mb[LEGS] - mq[LEGS]
        return m != 0 and mlo <= m <= mhi and gap_hits(m)
    m0 = math.floor((-2 - d0) * d / (180 * n))
    return any(m != 0 and mlo <= m <= mhi and gap_hits(m) for m in range(m0 - 1, m0 + 3))


def path_tie(mq, nq, gq, q_src, mb, nb, gb, b_src, gv, perm, ff, x_first, lists=0) -> bool:
    before = perm[:perm.index(TIME)]
    after = perm[perm.index(TIME) + 1:]
    if MONEY in before and mq[MONEY] != mb[MONEY]:
        return False
    (bx, by), (vx, vy) = gb, gv
    sx, sy = (1 if vx > bx else -1), (1 if vy > by else -1)
    K, kx = abs(vx - bx) + abs(vy - by), abs(vx - bx)

    def cell(k):
        if x_first:
            return (bx + sx * k, by) if k < kx else (vx, by + sy * (k - kx))
        ky = K - kx
        return (bx, by + sy * k) if k < ky else (bx + sx * (k - ky), vy)
    for k in range(K):
        u = cell(k)
        if u == (0, 0):
            return True
        dq, dqn = walk_dist(gq, u), walk_dist(gq, cell(k + 1))
        if LEGS in before and mq[LEGS] + dq != mb[LEGS] + k:
            continue
        if dqn <= dq:  # q gets nearer: it stays ahead
            continue
        delta = run_time(dqn, ff) - run_time(dq, ff) - (run_time(k + 1, ff) - run_time(k, ff))
        gap = mq[TIME] + run_time(dq, ff) - mb[TIME] - run_time(k, ff)
        if gap not in (-1, 0) or delta < 0:
            continue

        def tail(dqq, kk):  # -1: q ahead after Time, +1: b ahead, 0: undecided (command lists)
            # (two walks of equal length that both append a command are ordered by their
            # boundaries' own command lists, the same at every cell: `lists`)
            for c in after:
                a_ = mq[c] + (dqq if c == LEGS else 0)
                b_ = mb[c] + (kk if c == LEGS else 0)
                if a_ != b_:
                    return -1 if a_ < b_ else 1
            lq = 1 if q_src else nq + (1 if dqq > 0 else 0)
            lb = 1 if b_src else nb + (1 if kk > 0 else 0)
            if lq != lb:
                return (lq > lb) - (lq < lb)
            return lists if (dqq > 0 and kk > 0) else 0
        q_beats_u = gap == -1 or tail(dq, k) != 1
        gw = gap + delta
        b_beats_w = gw > 0 or (gw == 0 and tail(dqn, k + 1) != -1)
        if q_beats_u and b_beats_w:
            return True
    return False


def walk_certified(b, v, bnd, lab, geo, src_i, perm, ff) -> bool:
    """walk_certain: one L-path (x first or y first) clean for every boundary q."""
    (bx, by), (vx, vy) = geo[b], geo[v]
    if (by == 0 and vy == 0 and bx != 0 and vx != 0 and (bx < 0) != (vx < 0)) or \
       (bx == 0 and vx == 0 and by != 0 and vy != 0 and (by < 0) != (vy < 0)):
        return False
    mb, nb = metrics(lab[b]), len(lab[b].commands)
    clean = {True, False}  # the paths still clean for every q so far (x_first flags)
    for q in bnd:
        if q == b or geo[q] == (0, 0):
            continue
        mq, nq = metrics(lab[q]), len(lab[q].commands)
        if not near_tie(mq, geo[q], mb, geo[b], geo[v], perm, ff):
            continue
        lists = 0  # the order of q's and b's command lists when their walks' lengths tie
        if q != src_i and b != src_i and nq == nb:
            kq, kb = [c.key() for c in lab[q].commands], [c.key() for c in lab[b].commands]
            lists = (kq > kb) - (kq < kb)
        args = (mq, nq, geo[q], q == src_i, mb, nb, geo[b], b == src_i, geo[v], perm, ff)
        clean = {x for x in clean if not path_tie(*args, x, lists)}
        if not clean:
            return False
    return True
