"""Experiment (CPU, oracle only): how often does the closed form
L(v) = min_b walk(b, d_b(v)) differ from the reference's labels when the
StandardMove run time is non-linear (Fleetfoot 1..3), and how often would the
near-tie test of DESIGN.md (non-linear hub) flag a label?  Not product code."""
import random
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_lib  # noqa: E402
from marshrutka_amd.abi import CMD_NO_MOVE, CMD_STANDARD, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, index_to_geo  # noqa: E402
from hub_model import walk_dist  # noqa: E402

FF = {1: (50, 53), 2: (100, 109), 3: (25, 28)}


def f(k, ff):
    n, d = FF[ff]
    return -(-180 * k * n // d)


def danger(lp, gp, ls, gs, gv, sort, ff):
    """Can boundary p (label lp at gp) be a non-isotonic beater of the winner s
    (label ls at gs) on a shortest s-path to v (gv)?  (prefix metrics tie and the
    time difference in {-1, 0}, DESIGN.md non-linear hub)"""
    (sx, sy), (vx, vy) = gs, gv
    if (sy == 0 and vy == 0 and sx != 0 and vx != 0 and (sx < 0) != (vx < 0)) or \
       (sx == 0 and vx == 0 and sy != 0 and vy != 0 and (sy < 0) != (vy < 0)):
        return True  # shortest paths detour round the Center: not handled
    l1 = lambda a, b: abs(a[0] - b[0]) + abs(a[1] - b[1])  # noqa: E731
    mlo, mhi = l1(gp, gv) - l1(gs, gv), l1(gp, gs) + 2
    n, d = FF[ff]
    d0 = lp.time_s - ls.time_s
    o = order(sort)
    before = o[:o.index(1)]
    if 2 in before and lp.money != ls.money:
        return False
    if 0 in before:
        lp_legs = lp.legs
        ms = [ls.legs - lp_legs] if mlo <= ls.legs - lp_legs <= mhi and ls.legs != lp_legs else []
    else:
        # Delta0 + c m in (-2, 1), c = 180 n / d
        lo = (-2 - d0) * d / (180 * n)
        hi = (1 - d0) * d / (180 * n)
        import math
        ms = [m for m in range(math.floor(lo), math.ceil(hi) + 1) if mlo <= m <= mhi and m != 0]
    for m in ms:
        a = 180 * n * abs(m)
        g = (a // d, -(-a // d))
        g = g if m >= 0 else (-g[1], -g[0])
        if any(d0 + x in (-1, 0) for x in g):
            return True
    return False


def main(S=65, k=4, nsrc=6, seed=1):
    m = SyntheticMap(S, campfires_per_homeland=k, seed=seed)
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    geo = [index_to_geo(c) for c in cells]
    rng = random.Random(seed)
    for ff in (1, 2, 3):
        for sort in ((0, 1), (1, 2), (2, 0), (0, 2), (2, 1), (1, 0)):
            p = Params(fleetfoot=ff, sort_by=sort)
            perm = [sort[0], sort[1] if sort[1] != sort[0] else None]
            # eval_next: 3 metrics; map sort codes Legs=0 Time=1 Money=2 to metric tuple positions
            mis = tot = amb = flag = 0
            for src in rng.sample(cells, nsrc):
                lab = og.sssp_all(p, src)
                bnd = [i for i, t in enumerate(lab) if t.commands[-1].kind != CMD_STANDARD]
                for i, t in enumerate(lab):
                    if t.commands[-1].kind != CMD_STANDARD:
                        continue
                    best = None
                    ties = 0
                    for b in bnd:
                        d = walk_dist(geo[b], geo[i])
                        lb = lab[b]
                        met = {0: lb.legs + d, 1: lb.time_s - (0) + f(d, ff), 2: lb.money}
                        key = tuple(met[c] for c in order(sort)) + (len(lb.commands) + (0 if lb.commands[-1].kind == CMD_NO_MOVE else 1),)
                        if best is None or key < best[0]:
                            best, ties = (key, b), 0
                        elif key == best[0]:
                            ties += 1
                    if ties == 0:
                        bs = best[1]
                        nd = sum(danger(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff) for b in bnd if b != bs)
                        flag += nd > 0
                    dk = {0: t.legs, 1: t.time_s, 2: t.money}
                    dkey = tuple(dk[c] for c in order(sort))
                    tot += 1
                    amb += ties > 0
                    if dkey != best[0][:3]:
                        mis += 1
            print(f"S={S} ff={ff} sort={sort}: cells {tot}, closed-form metric mismatches {mis}, exact key ties {amb}, near-tie flagged {flag}",
                  flush=True)


def order(sort):
    # CostComparator::eval_next (src/cost.rs:387-405): Legs=0, Time=1, Money=2
    c1, c2 = sort
    if c2 == c1:
        c2 = {0: 1, 1: 0, 2: 0}[c1]
    c3 = ({0, 1, 2} - {c1, c2}).pop()
    return (c1, c2, c3)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))


def path_tie(lp, gp, ls, gs, gv, sort, ff, x_first):
    (bx, by), (vx, vy), (qx, qy) = gs, gv, gp
    o = order(sort)
    before = o[:o.index(1)]
    if 2 in before and lp.money != ls.money:
        return False
    sx, sy = (1 if vx > bx else -1), (1 if vy > by else -1)
    K, kx = abs(vx - bx) + abs(vy - by), abs(vx - bx)
    for k in range(K):
        if x_first:
            ux, uy = (bx + sx * k, by) if k < kx else (vx, by + sy * (k - kx))
        else:
            ky = K - kx
            ux, uy = (bx, by + sy * k) if k < ky else (bx + sx * (k - ky), vy)
        if ux == 0 and uy == 0:
            return True
        dq = walk_dist((qx, qy), (ux, uy))
        if 0 in before and lp.legs + dq != ls.legs + k:
            continue
        gap = lp.time_s + f(dq, ff) - ls.time_s - f(k, ff)
        if gap in (-1, 0) and f(dq + 1, ff) - f(dq, ff) > f(k + 1, ff) - f(k, ff):
            return True
    return False


def source_rates(S=65, nq=2000, ff=1, seed=2024):
    from marshrutka_amd.mapgen import random_queries
    m = SyntheticMap(S, campfires_per_homeland=4, seed=seed)
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    pos = {c: i for i, c in enumerate(cells)}
    geo = [index_to_geo(c) for c in cells]
    qs = random_queries(m, nq, 7)
    by_src = {}
    for s_, d_ in qs:
        by_src.setdefault(s_, []).append(d_)
    for sort in ((0, 2), (0, 1), (2, 0), (1, 2)):
        p = Params(fleetfoot=ff, sort_by=sort)
        nfb = ndanger = 0
        for src, dsts in list(by_src.items())[:300]:
            lab = og.sssp_all(p, src)
            bnd = [i for i, t in enumerate(lab) if t.commands[-1].kind != CMD_STANDARD and geo[i] != (0, 0)]
            fb = False
            for d_ in dsts:
                i = pos[d_]
                t = lab[i]
                if t.commands[-1].kind != CMD_STANDARD or d_ == src:
                    continue
                bs = pos[src] if t.commands[-1].from_ == src else pos[t.commands[-1].from_]
                for b in bnd:
                    if b == bs:
                        continue
                    if danger(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff):
                        ndanger += 1
                        if path_tie(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff, True) and \
                                path_tie(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff, False):
                            fb = True
            nfb += fb
        print(f"S={S} ff={ff} sort={sort}: sources {min(300, len(by_src))}, dest-check fallbacks {nfb}, "
              f"near-tie pairs {ndanger}", flush=True)


def path_flip(lp, gp, ls, gs, gv, sort, ff, x_first, q_is_source, b_is_source):
    """Refined path check: a cell u of the L-path where q beats walk(b) and the next
    leg flips the order (prefix tie, the real delta = +1, time gap and tail as below)."""
    (bx, by), (vx, vy), (qx, qy) = gs, gv, gp
    o = order(sort)
    ti = o.index(1)
    before, after = o[:ti], o[ti + 1:]
    if 2 in before and lp.money != ls.money:
        return False
    sx, sy = (1 if vx > bx else -1), (1 if vy > by else -1)
    K, kx = abs(vx - bx) + abs(vy - by), abs(vx - bx)

    def cell(k):
        if x_first:
            return (bx + sx * k, by) if k < kx else (vx, by + sy * (k - kx))
        ky = K - kx
        return (bx, by + sy * k) if k < ky else (bx + sx * (k - ky), vy)
    for k in range(K):
        ux, uy = cell(k)
        if ux == 0 and uy == 0:
            return True
        dq = walk_dist((qx, qy), (ux, uy))
        if 0 in before and lp.legs + dq != ls.legs + k:
            continue
        dqn = walk_dist((qx, qy), cell(k + 1))
        if dqn < dq:
            continue
        delta = f(dq + 1, ff) - f(dq, ff) - (f(k + 1, ff) - f(k, ff))
        if delta != 1:
            continue
        gap = lp.time_s + f(dq, ff) - ls.time_s - f(k, ff)
        if gap not in (-1, 0):
            continue
        # tail after time: the remaining metric, then the length
        tail = 0
        for c in after:
            a_ = {0: lp.legs + dq, 2: lp.money}[c]
            b_ = {0: ls.legs + k, 2: ls.money}[c]
            if a_ != b_:
                tail = -1 if a_ < b_ else 1
                break
        if tail == 0:
            lq = (1 if q_is_source else len(lp.commands) + (1 if dq > 0 else 0))
            lb = (1 if b_is_source else len(ls.commands) + (1 if k > 0 else 0))
            if lq != lb:
                tail = -1 if lq < lb else 1
        if gap == -1 and tail <= 0 and tail != -1:
            return True
        if gap == -1 and tail == 1:
            return True
        if gap == 0 and tail != 1:
            return True
    return False


def source_rates2(S=65, nq=2000, ff=1, seed=2024, nsrc=300):
    from marshrutka_amd.mapgen import random_queries
    m = SyntheticMap(S, campfires_per_homeland=4, seed=seed)
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    pos = {c: i for i, c in enumerate(cells)}
    geo = [index_to_geo(c) for c in cells]
    qs = random_queries(m, nq, 7)
    by_src = {}
    for s_, d_ in qs:
        by_src.setdefault(s_, []).append(d_)
    specials = [pos[c] for c in m.campfires()] + [i for i, g in enumerate(geo) if abs(g[0]) + abs(g[1]) == 1 and 0 in g]
    for sort in ((1, 0), (1, 2), (0, 1), (0, 2), (2, 1)):
        p = Params(fleetfoot=ff, sort_by=sort)
        res = {"coarse": 0, "refined": 0}
        for src, dsts in list(by_src.items())[:nsrc]:
            lab = og.sssp_all(p, src)
            si = pos[src]
            bnd = [i for i, t in enumerate(lab) if t.commands[-1].kind != CMD_STANDARD and geo[i] != (0, 0)]
            targets = [pos[d] for d in dsts] + specials
            fb_c = fb_r = False
            for i in targets:
                t = lab[i]
                if t.commands[-1].kind != CMD_STANDARD or i == si:
                    continue
                bs = pos[t.commands[-1].from_]
                for b in bnd:
                    if b == bs or not danger(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff):
                        continue
                    if path_tie(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff, True) and \
                            path_tie(lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff, False):
                        fb_c = True
                    args = (lab[b], geo[b], lab[bs], geo[bs], geo[i], sort, ff)
                    if path_flip(*args, True, b == si, bs == si) and path_flip(*args, False, b == si, bs == si):
                        fb_r = True
            res["coarse"] += fb_c
            res["refined"] += fb_r
        print(f"S={S} ff={ff} sort={sort}: sources {min(nsrc, len(by_src))} fallbacks {res}", flush=True)
