"""CPU experiment (oracle only, not product code): the fixed-point certificate for
non-linear run times.

For a source, C(v) = min over boundaries b of walk(b, d_b(v)) on every plain cell
(the closed form), the specials' labels taken from the oracle.  The Bellman check
asks, per plain cell v, whether C(v) equals the least extension of its neighbours'
C labels.  Labels with a leading metric below every failing cell's are certified
(DESIGN.md section 3a'''': an induction over the label order).  The probe reports
how many cells the closed form gets wrong, how many the check certifies, and
whether any certified cell is wrong (it must not be).

usage: python tools/cert_probe.py S ff sort1 sort2 nsrc [seed] [src_x src_y ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_lib  # noqa: E402
from label_digest import CMD_DT, Q, cell_keys, command_hashes  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, geo_to_index, index_to_geo  # noqa: E402
from nonlin_model import FF_RATIO, perm_of  # noqa: E402

STD = 2


def ci_t(c):
    return (c.kind, c.sub, c.x, c.y)


def cmd_key(c):
    return (c.kind, c.time_s, c.legs, c.money, c.fleetfoot, ci_t(c.from_), ci_t(c.to))


def lex_less(a, b):
    """a < b for tuples of equal-shaped arrays (lexicographic)."""
    lt = np.zeros(a[0].shape, bool)
    eq = np.ones(a[0].shape, bool)
    for x, y in zip(a, b):
        lt |= eq & (x < y)
        eq &= (x == y)
    return lt


def probe(m, og, prm, src_geo, verbose=True, repair=0):
    S, H = m.size, m.h
    V = S * S
    ff = prm.fleetfoot
    n, d = FF_RATIO.get(ff, (1, 1))
    perm = perm_of(prm.sort_by)
    idx = np.arange(V)
    X, Y = idx % S - H, idx // S - H
    keys = cell_keys(m.cells_array())
    src = geo_to_index(*src_geo)
    tr = og.sssp_digests(prm, [src], threads=8)
    tr = {k: v[0] for k, v in tr.items()}
    # specials and their oracle labels
    sp = [(0, 0), (-1, 0), (0, 1), (1, 0), (0, -1)]
    sp += sorted(g for g, p in m.poi.items() if p == 1)
    sp = list(dict.fromkeys(sp))
    if prm.hq_position is not None:
        sp.append(index_to_geo(prm.hq_position))
    labs = {g: og.find_path(prm, src, geo_to_index(*g)) for g in sp}
    # boundaries: the source (start label) and every special whose label does not end in a StandardMove
    bnd = [(src_geo, 0, 0, 0, 1, ((0, 0, 0, 0, 0, ci_t(src), ci_t(src)),))]
    walk_sp = {}
    for g, L in labs.items():
        if g == src_geo:
            continue
        if L.commands[-1].kind != STD:
            bnd.append((g, L.legs, L.money, L.time_s, len(L.commands), tuple(cmd_key(c) for c in L.commands)))
        else:
            walk_sp[g] = (index_to_geo(L.commands[-1].from_), L.commands[-1].legs)
    bnd.sort(key=lambda b: b[5])  # rank = list order
    bi = {b[0]: i for i, b in enumerate(bnd)}
    NB = len(bnd)
    Bm = np.array([[b[1], b[2], b[3]] for b in bnd], np.int64)  # legs, money, time
    Blen = np.array([b[4] for b in bnd], np.int64)
    Bsrc = np.array([b[0] == src_geo for b in bnd])
    cell_of = lambda g: (g[1] + H) * S + (g[0] + H)  # noqa: E731
    Bdig = np.array([0 if Bsrc[i] else int(tr["digest"][cell_of(b[0])]) for i, b in enumerate(bnd)], np.uint64)

    def ftime(k):
        return -(-(180 * k * n) // d)

    def walk_metrics(bidx, k):
        legs = Bm[bidx, 0] + k
        money = Bm[bidx, 1]
        time = Bm[bidx, 2] + ftime(k)
        ln = np.where(Bsrc[bidx], 1, Blen[bidx] + 1)
        met = {0: legs, 1: money, 2: time}
        return (met[perm[0]], met[perm[1]], met[perm[2]], ln, bidx)

    def wdist(gx, gy, vx, vy):
        dd = np.abs(gx - vx) + np.abs(gy - vy)
        det = ((gy == 0) & (vy == 0) & (gx != 0) & (vx != 0) & ((gx < 0) != (vx < 0))) | \
              ((gx == 0) & (vx == 0) & (gy != 0) & (vy != 0) & ((gy < 0) != (vy < 0)))
        return dd + 2 * det
    # closed form over every cell: (bidx, k)
    best = None
    for i, b in enumerate(bnd):
        k = wdist(b[0][0], b[0][1], X, Y)
        cand = walk_metrics(np.full(V, i), k)
        if best is None:
            best, bb, bk = cand, np.full(V, i), k
        else:
            lt = lex_less(cand, best)
            best = tuple(np.where(lt, c, o) for c, o in zip(cand, best))
            bb, bk = np.where(lt, i, bb), np.where(lt, k, bk)
    special = np.zeros(V, bool)
    for g in sp:
        special[cell_of(g)] = True
    center = cell_of((0, 0))
    # every cell's C label as (walk?, bidx, k): specials from the oracle
    own = np.zeros(V, bool)   # label is a boundary's own label (extension = walk(b, 1))
    ownb = np.zeros(V, np.int64)
    for g in sp:
        v = cell_of(g)
        if g in bi:
            own[v], ownb[v] = True, bi[g]
        elif g in walk_sp:
            bg, k = walk_sp[g]
            bb[v], bk[v] = bi[bg], k
    # closed form vs truth on plain cells (metrics, length, digest)
    legs_c = Bm[bb, 0] + bk
    money_c = Bm[bb, 1]
    time_c = Bm[bb, 2] + ftime(bk)
    len_c = np.where(Bsrc[bb], 1, Blen[bb] + 1)
    cm = np.zeros(V, CMD_DT)
    cm["kind"], cm["legs"], cm["fleetfoot"], cm["time_s"] = STD, bk, ff, 180 * bk
    cm["from"], cm["to"] = keys[np.array([cell_of(b[0]) for b in bnd])[bb]], keys
    h = command_hashes(cm.tobytes(), V)
    with np.errstate(over="ignore"):
        dig_c = np.where(Bsrc[bb], h, Bdig[bb] * Q + h)
    plain = ~special & (idx != cell_of(src_geo))
    wrong = plain & ((legs_c != tr["legs"]) | (money_c != tr["money"]) | (time_c != tr["time_s"]) |
                     (len_c != tr["n_commands"]) | (dig_c != tr["digest"]))
    # Bellman check on plain cells: C(v) == min over the 4 neighbours of ext(C(u))
    ext_b = np.where(own, ownb, bb)
    ext_k = np.where(own, 1, bk + 1)
    BIG = np.iinfo(np.int64).max // 4
    nbrs = []
    for dx, dy in ((1, 0), (-1, 0), (0, 1), (0, -1)):
        ux, uy = X - dx, Y - dy
        ok = (np.abs(ux) <= H) & (np.abs(uy) <= H)
        u = np.where(ok, (uy + H) * S + (ux + H), 0)
        ok &= u != center
        nbrs.append((u, ok))

    geo_only = os.environ.get("GEO", "0") == "1"
    DB = np.stack([wdist(b[0][0], b[0][1], X, Y) for b in bnd]) if geo_only else None

    def best4(ext_b, ext_k, geo=False):
        cb = None
        for u, ok in nbrs:
            cand = walk_metrics(ext_b[u], ext_k[u]) + (ext_k[u],)
            if geo:
                ok = ok & (ext_k[u] == DB[ext_b[u], idx])
            cand = tuple(np.where(ok, c, BIG) for c in cand)
            if cb is None:
                cb = cand
            else:
                lt = lex_less(cand[:5], cb[:5])
                cb = tuple(np.where(lt, c, o) for c, o in zip(cand, cb))
        return cb

    cb = best4(ext_b, ext_k)
    mine = walk_metrics(bb, bk)
    fail = plain & ~np.all(np.stack([a == b for a, b in zip(mine, cb[:5])]), axis=0)
    fkey = np.where(fail, np.minimum(mine[0], cb[0]), BIG)
    minfail = int(fkey.min())
    cert = plain & (mine[0] < minfail)
    unsound = int((cert & wrong).sum())
    sweep_rounds = int(os.environ.get("SWEEP", "0"))
    if sweep_rounds:
        # Sorted sweep: the failing cells' bounding box (+ margin), its plain cells in
        # order of their current lead metric (buckets of the least step), each bucket
        # recomputed from its neighbours' current labels; then the check again.
        lead = perm[0] if perm[0] != 1 else perm[1]
        W = 1 if lead == 0 else (180 * n) // d
        M = int(os.environ.get("MARGIN", "2"))
        win = np.zeros(V, bool)
        for rnd in range(sweep_rounds):
            if not fail.any():
                break
            fx, fy = X[fail], Y[fail]
            win |= plain & (X >= fx.min() - M) & (X <= fx.max() + M) & (Y >= fy.min() - M) & (Y <= fy.max() + M)
            cells = np.flatnonzero(win)
            lv = (Bm[bb[cells], 0] + bk[cells]) if lead == 0 else (Bm[bb[cells], 2] + ftime(bk[cells]))
            key = lv // W
            order = np.argsort(key, kind="stable")
            cells, key = cells[order], key[order]
            cuts = np.flatnonzero(np.diff(key)) + 1
            groups = np.split(cells, cuts)
            for g in groups:
                best = None
                for u_all, ok_all in nbrs:
                    u, ok = u_all[g], ok_all[g]
                    eb = np.where(own[u], ownb[u], bb[u])
                    ek = np.where(own[u], 1, bk[u] + 1)
                    cand = walk_metrics(eb, ek) + (ek,)
                    cand = tuple(np.where(ok, c, BIG) for c in cand)
                    if best is None:
                        best = cand
                    else:
                        lt = lex_less(cand[:5], best[:5])
                        best = tuple(np.where(lt, c, o) for c, o in zip(cand, best))
                bb[g], bk[g] = best[4], best[5]
            ext_b = np.where(own, ownb, bb)
            ext_k = np.where(own, 1, bk + 1)
            cb = best4(ext_b, ext_k)
            mine = walk_metrics(bb, bk)
            fail = plain & ~np.all(np.stack([a == b for a, b in zip(mine, cb[:5])]), axis=0)
            legs_c = Bm[bb, 0] + bk
            time_c = Bm[bb, 2] + ftime(bk)
            money_c = Bm[bb, 1]
            len_c = np.where(Bsrc[bb], 1, Blen[bb] + 1)
            cm["legs"], cm["time_s"] = bk, 180 * bk
            cm["from"] = keys[np.array([cell_of(b[0]) for b in bnd])[bb]]
            h = command_hashes(cm.tobytes(), V)
            with np.errstate(over="ignore"):
                dig_c = np.where(Bsrc[bb], h, Bdig[bb] * Q + h)
            wrong2 = plain & ((legs_c != tr["legs"]) | (money_c != tr["money"]) | (time_c != tr["time_s"]) |
                              (len_c != tr["n_commands"]) | (dig_c != tr["digest"]))
            print(f"  sweep round {rnd}: window {len(cells)} cells, {len(groups)} buckets; after: fail {int(fail.sum())} "
                  f"wrong {int(wrong2.sum())}", flush=True)
    if repair:
        # Jacobi repair of the plain cells (specials fixed): C <- min over neighbours of ext(C)
        it, hist = 0, []
        bb0 = bb.copy()
        if geo_only:
            cb = best4(ext_b, ext_k, True)
            cf = best4(ext_b, ext_k)
            none = cb[0] == BIG
            cb = tuple(np.where(none, f, c) for f, c in zip(cf, cb))
        while it < repair:
            upd = plain & ~np.all(np.stack([a == b for a, b in zip(walk_metrics(bb, bk), cb)]), axis=0)
            if os.environ.get("RISE", "0") == "1":  # only raise (the closed form is a lower bound)
                upd &= lex_less(walk_metrics(bb, bk), cb[:5])
            if os.environ.get("RB", "0") == "1":  # red-black: one colour per half step
                col = ((X + Y) & 1) == (it & 1)
                hist_any = int(upd.sum())
                upd &= col
                if hist_any and not upd.any():
                    upd = plain & ~np.all(np.stack([a == b for a, b in zip(walk_metrics(bb, bk), cb)]), axis=0)
            cnt = int(upd.sum())
            hist.append(cnt)
            if cnt == 0:
                break
            if it == 0:
                trace = np.flatnonzero(wrong)[::max(1, int(wrong.sum()) // 3)][:3]
                tr_hist = {int(v): [] for v in trace}
            for v in tr_hist:
                tr_hist[v].append((int(bb[v]), int(bk[v])))
            bb = np.where(upd, cb[4], bb)
            bk = np.where(upd, cb[5], bk)
            ext_b = np.where(own, ownb, bb)
            ext_k = np.where(own, 1, bk + 1)
            cb = best4(ext_b, ext_k, geo_only)
            if geo_only:  # no geodesic candidate: the full minimum
                cf = best4(ext_b, ext_k)
                none = cb[0] == BIG
                cb = tuple(np.where(none, f, c) for f, c in zip(cf, cb))
            it += 1
        legs_c = Bm[bb, 0] + bk
        time_c = Bm[bb, 2] + ftime(bk)
        money_c = Bm[bb, 1]
        len_c = np.where(Bsrc[bb], 1, Blen[bb] + 1)
        cm["legs"], cm["time_s"] = bk, 180 * bk
        cm["from"] = keys[np.array([cell_of(b[0]) for b in bnd])[bb]]
        h = command_hashes(cm.tobytes(), V)
        with np.errstate(over="ignore"):
            dig_c = np.where(Bsrc[bb], h, Bdig[bb] * Q + h)
        wrong2 = plain & ((legs_c != tr["legs"]) | (money_c != tr["money"]) | (time_c != tr["time_s"]) |
                          (len_c != tr["n_commands"]) | (dig_c != tr["digest"]))
        kgeo = np.zeros(V, np.int64)
        for i, b in enumerate(bnd):
            kk = wdist(b[0][0], b[0][1], X, Y)
            kgeo = np.where(bb == i, kk, kgeo)
        fixed = wrong
        print(f"  wrong cells: truth non-geodesic {int((fixed & (bk != kgeo)).sum())}, "
              f"boundaries closed form {sorted(set(np.unique(bb0[fixed]).tolist()))} -> truth {sorted(set(np.unique(bb[fixed]).tolist()))}; "
              f"bbox x {X[fixed].min()}..{X[fixed].max()} y {Y[fixed].min()}..{Y[fixed].max()}")
        for v, hh in tr_hist.items():
            comp = [hh[0]] + [hh[j] for j in range(1, len(hh)) if hh[j] != hh[j - 1]]
            print("   trace", (int(X[v]), int(Y[v])), "geo", [int(wdist(b[0][0], b[0][1], X[v], Y[v])) for b in bnd][:5], comp[:20], len(comp))
        for i, b in enumerate(bnd):
            print("   bnd", i, b[0], b[1:4], "len", b[4])
        print(f"  repair: {it} iterations, {sum(hist)} updates, changed per iteration {hist[:12]}...{hist[-3:]}, wrong after {int(wrong2.sum())}",
              flush=True)
    if verbose:
        print(f"src {src_geo}: plain {int(plain.sum())} wrong {int(wrong.sum())} fail {int(fail.sum())} "
              f"minfail c1 {minfail if minfail < BIG else None} certified {int(cert.sum())} "
              f"({cert.sum() / plain.sum():.3f}) UNSOUND {unsound}", flush=True)
    return {"wrong": wrong, "fail": fail, "cert": cert, "unsound": unsound, "c1": mine[0], "minfail": minfail,
            "plain": plain}


def main():
    a = sys.argv[1:]
    S, ff, s1, s2, nsrc = (int(x) for x in a[:5])
    seed = int(a[5]) if len(a) > 5 else 2024
    m = SyntheticMap(S, campfires_per_homeland=4, seed=seed)
    og = oracle_lib.OracleGrid.from_array(m.cells_array())
    prm = Params(fleetfoot=ff, sort_by=(s1, s2))
    rng = np.random.default_rng(seed)
    srcs = [(int(a[i]), int(a[i + 1])) for i in range(6, len(a) - 1, 2)]
    H = m.h
    while len(srcs) < nsrc:
        g = (int(rng.integers(-H, H + 1)), int(rng.integers(-H, H + 1)))
        if g != (0, 0):
            srcs.append(g)
    bad = 0
    for g in srcs:
        bad += probe(m, og, prm, g, repair=int(os.environ.get("REPAIR", "0")))["unsound"]
    print("UNSOUND total", bad)


if __name__ == "__main__":
    main()
