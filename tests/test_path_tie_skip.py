"""The non-linear certification's path scan with periodic skipping (csrc/mr_device.hpp
path_tie, DESIGN.md section 3a'') against the cell-by-cell scan of the Python model
(tests/nonlin_model.py path_tie) — CPU only, test infrastructure.

Along a run of steps on which boundary q moves away from the walk's cells (q's
distance grows by one a step, no axis crossed), every quantity the flip test reads
is constant or periodic in the step index with period den (the Fleetfoot ratio's
denominator: run_time(k + den) = run_time(k) + 180 num).  So once den consecutive
steps of such a run have been checked, the rest of the run can be skipped; the scan
resumes exactly at the first step that leaves the run; a run of at least den steps is
decided at its start by one period of the time gaps (every residue of k mod den occurs
on it) and skipped whole.  A stretch on which the walk
approaches q's column (row) is skipped whole: q's distance drops there,
and only a step on which it grows can flip.  `path_tie_skip` below is a line-by-line
restatement of the device loop; it must agree with the full scan."""
import random

import pytest

from nonlin_model import FF_RATIO, LEGS, MONEY, TIME, path_tie, run_time
from hub_model import walk_dist


def path_tie_skip(mq, nq, gq, q_src, mb, nb, gb, b_src, gv, perm, ff, x_first, lists=0):
    before = perm[:perm.index(TIME)]
    after = perm[perm.index(TIME) + 1:]
    if MONEY in before and mq[MONEY] != mb[MONEY]:
        return False
    den = FF_RATIO[ff][1]
    (bx, by), (vx, vy), (qx, qy) = gb, gv, gq
    sx, sy = (1 if vx > bx else -1), (1 if vy > by else -1)
    K, kx = abs(vx - bx) + abs(vy - by), abs(vx - bx)
    ky = K - kx

    def cell(k):
        if x_first:
            return (bx + sx * k, by) if k < kx else (vx, by + sy * (k - kx))
        return (bx, by + sy * k) if k < ky else (bx + sx * (k - ky), vy)

    def tail(dqq, kk):
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

    k, run = 0, 0
    u = cell(0)
    dq = walk_dist(gq, u)
    while k < K:
        if u == (0, 0):
            return True
        # Approach skip: moving along a segment towards q's column (row), q's distance drops
        # by one a step until the walk reaches it (or the step before the axis being
        # crossed: the Center detour's term stays constant), so no step of it can flip
        along_x = (k < kx) if x_first else (k >= ky)
        seg_end = (kx if x_first else K) if along_x else (K if x_first else ky)
        c0, qc, sd = (u[0], qx, sx) if along_x else (u[1], qy, sy)
        if sd * (c0 - qc) < 0:
            j = min(seg_end, k + abs(c0 - qc))
            if c0 * sd < 0:
                j = min(j, k + abs(c0) - 1)
            if j > k + 1:
                k, run = j, 0
                u = cell(k)
                dq = walk_dist(gq, u)
                continue
        w = cell(k + 1)
        dqn = walk_dist(gq, w)
        tie_before = not (LEGS in before and mq[LEGS] + dq != mb[LEGS] + k)
        if tie_before and dqn > dq:
            delta = run_time(dqn, ff) - run_time(dq, ff) - (run_time(k + 1, ff) - run_time(k, ff))
            gap = mq[TIME] + run_time(dq, ff) - mb[TIME] - run_time(k, ff)
            if gap in (-1, 0) and delta >= 0:
                q_beats_u = gap == -1 or tail(dq, k) != 1
                gw = gap + delta
                if q_beats_u and (gw > 0 or (gw == 0 and tail(dqn, k + 1) != -1)):
                    return True
        # a plain step: q's distance grows by one along the segment, no axis touched
        along_x = (k < kx) if x_first else (k >= ky)
        if along_x:
            plain = k >= 1 and u[0] != 0 and w[0] != 0 and sx * (u[0] - qx) >= 0
        else:
            plain = k >= 1 and u[1] != 0 and w[1] != 0 and sy * (u[1] - qy) >= 0
        seg_end = (kx if x_first else K) if along_x else (K if x_first else ky)
        run = run + 1 if plain else 0
        # the next step that is not plain: the segment's end, or the step before the one
        # whose cell lies on the axis being crossed
        j = seg_end
        if along_x:
            c0 = cell(k)[0]
            if c0 * sx < 0:  # the x = 0 axis ahead
                jz = k + abs(c0)  # the step index whose cell has x = 0
                j = min(j, jz - 1)
        else:
            c0 = cell(k)[1]
            if c0 * sy < 0:
                jz = k + abs(c0)
                j = min(j, jz - 1)
        # A plain run of at least den steps from here (q off the walk, so the tail below
        # is the run's): its steps see every residue of k mod den, and the time gaps at a
        # step and the next are d0 + F(r), d0 + F(r + 1) with F(r) = f(r + m) - f(r)
        # (m = dq - k, constant on the run, F periodic in r).  One period of F decides
        # whether some step of the run flips; the run is then skipped whole.
        if plain and tie_before and dq > 0 and j - k >= den:
            m, T, d0 = dq - k, tail(dq, k), mq[TIME] - mb[TIME]
            base = den * (-(-max(0, -m) // den))  # (r + m >= 0: f's argument)
            for i in range(den):
                r = base + i
                g = d0 + run_time(r + m, ff) - run_time(r, ff)
                gw = d0 + run_time(r + 1 + m, ff) - run_time(r + 1, ff)
                if g in (-1, 0) and gw >= g and (g == -1 or T != 1) and (gw > 0 or (gw == 0 and T != -1)):
                    return True
            k, run = j, 0
            u = cell(k)
            dq = walk_dist(gq, u)
            continue
        # (with Legs before Time the legs gap is constant on a plain run too: a run that
        # starts untied stays untied and is skipped at once)
        if run >= den or (plain and not tie_before):
            if j > k + 1:
                k, run = j, 0
                u = cell(k)
                dq = walk_dist(gq, u)
                continue
        k += 1
        u, dq = w, dqn
    return False


PERMS = [(LEGS, MONEY, TIME), (LEGS, TIME, MONEY), (MONEY, LEGS, TIME), (MONEY, TIME, LEGS),
         (TIME, LEGS, MONEY), (TIME, MONEY, LEGS)]


@pytest.mark.parametrize("ff", [1, 2, 3])
def test_skip_scan_matches_full_scan(ff):
    rng = random.Random(ff)
    H = 60
    hits = 0
    for trial in range(6000):
        perm = rng.choice(PERMS)
        gb = (rng.randint(-H, H), rng.randint(-H, H))
        gv = (rng.randint(-H, H), rng.randint(-H, H))
        gq = (rng.randint(-H, H), rng.randint(-H, H))
        if rng.random() < 0.2:  # on an axis now and then
            gq = (0, gq[1]) if rng.random() < 0.5 else (gq[0], 0)
        if rng.random() < 0.2:
            gb = (0, gb[1]) if rng.random() < 0.5 else (gb[0], 0)
        x_first = rng.random() < 0.5
        # metrics tuned so that the time gap passes -1 / 0 somewhere on the path
        K = abs(gv[0] - gb[0]) + abs(gv[1] - gb[1])
        k0 = rng.randint(0, max(0, K - 1))
        cells = (gb[0] + (k0 if gv[0] >= gb[0] else -k0), gb[1])
        dq0 = walk_dist(gq, cells)
        tb = rng.randint(0, 5000)
        tq = tb + run_time(k0, ff) - run_time(dq0, ff) + rng.choice([-2, -1, 0, 0, 1])
        lb = rng.randint(0, 50)
        lq = lb + k0 - dq0 if rng.random() < 0.7 else rng.randint(0, 50)
        mb_ = rng.choice([0, 50, 100])
        mq_ = mb_ if rng.random() < 0.8 else rng.choice([0, 50, 100])
        mq, mb = (lq, mq_, tq), (lb, mb_, tb)
        nq, nb = rng.randint(1, 6), rng.randint(1, 6)
        q_src, b_src = rng.random() < 0.1, rng.random() < 0.1
        lists = rng.choice([-1, 0, 1])
        want = path_tie(mq, nq, gq, q_src, mb, nb, gb, b_src, gv, perm, ff, x_first, lists)
        got = path_tie_skip(mq, nq, gq, q_src, mb, nb, gb, b_src, gv, perm, ff, x_first, lists)
        hits += want
        assert got == want, (trial, mq, nq, gq, q_src, mb, nb, gb, b_src, gv, perm, ff, x_first, lists)
    assert hits > 50  # the flip is found on a fair share of the cases
