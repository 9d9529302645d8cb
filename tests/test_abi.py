"""CPU-side checks of the C-ABI library: it builds, loads, exports every
function include/marshrutka_pf.h declares, validates grids on the host, and
fails loudly (MR_ERR_NO_DEVICE) instead of falling back to the CPU."""
import ctypes as C
import os
import re

import pytest

from marshrutka_amd import abi
from marshrutka_amd.abi import BLUE, CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap, to_html

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    return pathfinder


def declared_functions():
    names = []
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names += re.findall(r"^[A-Za-z_][\w \*]*?\b(mr_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_api():
    names = declared_functions()
    assert "mr_find_path" in names and "mr_find_path_batch" in names and "mr_grid_create" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol(eng):
    L = C.CDLL(eng.LIB_PATH)
    for name in declared_functions():
        assert hasattr(L, name), name
    assert sorted(declared_functions()) == sorted(eng.EXPORTED_SYMBOLS)


def test_abi_version_and_defaults(eng):
    L = eng.lib()
    assert L.mr_abi_version() == 7
    p = abi.mr_params()
    L.mr_params_default(C.byref(p))
    d = Params().to_c()
    for f, _ in abi.mr_params._fields_:
        if f in ("hq_position", "sort_by", "reserved"):
            continue
        assert getattr(p, f) == getattr(d, f), f
    assert list(p.sort_by) == [abi.SORT_LEGS, abi.SORT_MONEY]


def test_grid_validation_on_host(eng):
    m = SyntheticMap(9, campfires_per_homeland=2, seed=1)
    g = eng.MapGrid(m.cells())
    assert g.square_size == 9 and g.homeland_size() == 4
    cells = m.cells()
    # not square
    with pytest.raises(eng.EngineError, match="INVALID_GRID"):
        eng.MapGrid(cells[:-1])
    # duplicate index
    bad = list(cells)
    bad[0] = bad[1]
    with pytest.raises(eng.EngineError, match="INVALID_GRID"):
        eng.MapGrid(bad)
    # labels that are not a consistent 4-grid (two homeland cells swapped)
    bad = list(cells)
    bad[0], bad[10] = bad[10], bad[0]
    with pytest.raises(eng.EngineError, match="INVALID_GRID"):
        eng.MapGrid(bad)
    # a homeland without campfires: the reference panics (src/grid.rs:209)
    m2 = SyntheticMap(7, campfires_per_homeland=0, seed=0,
                      extra_campfires=[CellIndex.homeland(h, 3, 3) for h in range(3)])
    with pytest.raises(eng.EngineError, match="INVALID_GRID"):
        eng.MapGrid(m2.cells())


def test_rotated_layout_is_accepted(eng):
    # any orientation whose labels are consistent with the index adjacency is a valid map
    m = SyntheticMap(7, campfires_per_homeland=1, seed=4)
    S = 7
    cells = m.cells()
    rot = [cells[(S - 1 - (i % S)) * S + (i // S)] for i in range(S * S)]  # transpose + flip
    eng.MapGrid(rot)


def test_no_cpu_fallback_without_device(eng):
    if eng.device_available():
        pytest.skip("a device is visible")
    m = SyntheticMap(7, campfires_per_homeland=1, seed=4)
    g = eng.MapGrid(m.cells())
    fp = eng.FindPath(g)
    with pytest.raises(eng.EngineError, match="NO_DEVICE"):
        fp.eval(CellIndex.homeland(BLUE, 1, 1), CellIndex.center())


def test_html_writer_schema():
    m = SyntheticMap(5, campfires_per_homeland=1, seed=2)
    html = to_html(m)
    assert html.count('class="map-cell"') == 25
    assert '<div class="top-right-text">0#0</div>' in html


def _ranks(m):
    """CellIndex -> rank (position in the derived Ord, src/index.rs:41-46)."""
    cells = sorted(m.all_indices(), key=lambda c: (c.kind, c.sub, c.x, c.y))
    return {c: i for i, c in enumerate(cells)}


def test_decode_records_on_host(eng):
    """mr_decode_records: compact records as another rank gathers them (result
    record, command slots, overflow pool) decode to full labels without a device."""
    import numpy as np
    from marshrutka_amd.abi import GREEN, Command, TotalCost
    m = SyntheticMap(7, campfires_per_homeland=1, seed=4)
    g = eng.MapGrid(m.cells())
    rk = _ranks(m)
    b33, c, g33 = CellIndex.homeland(BLUE, 3, 3), CellIndex.center(), CellIndex.homeland(GREEN, 3, 3)
    car = lambda d, five: (3 << 29) | (d << 1) | five  # noqa: E731  Caravan payload: d << 1 | coef==5
    # (0, 42, 2880, [Caravan{1440,12} B3#3->0#0, Caravan{1440,30} 0#0->G3#3])
    want = TotalCost(0, 42, 2880, [Command(3, 1440, 0, 12, 0, b33, c), Command(3, 1440, 0, 30, 0, c, g33)])
    cmds = [[car(6, 0), rk[b33], rk[c], 0], [car(6, 1), rk[c], rk[g33], 0]]
    p = Params(route_guru=0)
    # three records, max_cmds 2: the label in its slots, a NOT_FOUND record, the label
    # again but tagged into the overflow pool at offset 3
    res = np.array([[0, 42, 2880, (16 << 16) | 2], [0, 0, 0, 17 << 16], [0, 42, 2880, ((16 + 64) << 16) | 2]],
                   dtype=np.uint32)
    slots = np.zeros((3, 2, 4), dtype=np.uint32)
    slots[0] = cmds
    slots[2, 0] = [0xFFFFFFFF, 3, 2, 0]
    pool = np.zeros((5, 4), dtype=np.uint32)
    pool[3:5] = cmds
    out = eng.decode_records(g, p, res, slots, 3, 2, pool)
    assert out[0].as_tuple() == want.as_tuple()
    assert out[1] is None
    assert out[2].as_tuple() == want.as_tuple()
    # a tag that points past the pool, and a command naming no cell, are errors
    with pytest.raises(eng.EngineError, match="DEVICE"):
        eng.decode_records(g, p, res, slots, 3, 2, pool[:4])
    bad = slots.copy()
    bad[0, 1, 2] = 49
    with pytest.raises(eng.EngineError, match="DEVICE"):
        eng.decode_records(g, p, res, bad, 3, 2, pool)


def test_decode_wire_on_host(eng):
    """mr_decode_wire: wire rows (first `from` rank | count, then {kind|payload, `to`}) with
    the metrics left out decode to the same full labels as the compact records."""
    import numpy as np
    from marshrutka_amd.abi import GREEN, Command, TotalCost
    m = SyntheticMap(7, campfires_per_homeland=1, seed=4)
    g = eng.MapGrid(m.cells())
    rk = _ranks(m)
    b33, c, g33 = CellIndex.homeland(BLUE, 3, 3), CellIndex.center(), CellIndex.homeland(GREEN, 3, 3)
    car = lambda d, five: (3 << 29) | (d << 1) | five  # noqa: E731
    want = TotalCost(0, 42, 2880, [Command(3, 1440, 0, 12, 0, b33, c), Command(3, 1440, 0, 30, 0, c, g33)])
    p = Params(route_guru=0)
    # max_cmds 2: the label in its slots, NOT_FOUND, the label in the pool at offset 3,
    # a capacity row (what the encoder writes for a label past the pool)
    st = lambda s_: (65 + 32 + s_) << 25  # noqa: E731
    rows = np.array([[rk[b33] | 2 << 25, car(6, 0), rk[c], car(6, 1), rk[g33]],
                     [st(1), 0, 0, 0, 0],
                     [rk[b33] | 64 << 25, 3, 2, 0, 0],
                     [st(-4), 0, 0, 0, 0]], dtype=np.uint32)
    pool = np.zeros((5, 2), dtype=np.uint32)
    pool[3:5] = [[car(6, 0), rk[c]], [car(6, 1), rk[g33]]]
    out, cmds = eng.decode_wire_raw(g, p, rows, 4, 2, pool)
    lab = [eng.result_from_c(out[k], cmds) if out[k].status == 0 else out[k].status for k in range(4)]
    assert lab[0].as_tuple() == want.as_tuple() and lab[2].as_tuple() == want.as_tuple()
    assert lab[1] == 1 and lab[3] == -4
    assert eng.wire_row_words(4) == 9  # 36 B a query at max_cmds 4
    with pytest.raises(eng.EngineError, match="DEVICE"):  # a pool reference past the pool
        eng.decode_wire_raw(g, p, rows, 4, 2, pool[:4])


@pytest.mark.parametrize("ff,rg", [(0, 0), (1, 3), (2, 5), (3, 1), (7, 2)])
def test_decode_wire_matches_decode_records(eng, ff, rg):
    """Random command chains of every kind: the wire decoder's recomputed metrics
    (Fleetfoot ceil per StandardMove run, caravan time and coefficient, scroll prices)
    and commands equal mr_decode_records over the same labels with the metrics given."""
    import random as _r
    from fractions import Fraction

    import numpy as np
    m = SyntheticMap(15, campfires_per_homeland=3, seed=ff + 11)
    g = eng.MapGrid(m.cells())
    V = len(m.all_indices())
    p = Params(fleetfoot=ff, route_guru=rg, scroll_of_escape_cost=7, scroll_of_escape_hq_cost=11,
               scroll_of_escape_forum_cost=13)
    ffr = {0: Fraction(1), 1: Fraction(50, 53), 2: Fraction(100, 109), 3: Fraction(25, 28)}.get(ff, Fraction(1))
    rgt = {0: 240, 1: 190, 2: 168, 3: 146, 4: 124, 5: 102}[rg]  # ceil(240 * RouteGuru ratio)
    rng = _r.Random(ff * 31 + rg)
    n, mc = 300, 3
    res = np.zeros((n, 4), dtype=np.uint32)
    slots = np.zeros((n, mc, 4), dtype=np.uint32)
    rows = np.zeros((n, 1 + 2 * mc), dtype=np.uint32)
    ovf, wpool = [], []
    for k in range(n):
        if rng.random() < 0.05:
            res[k, 3] = 17 << 16
            rows[k, 0] = (65 + 32 + 1) << 25
            continue
        nc = rng.randint(0, 6)
        at = rng.randrange(V)
        first = at
        legs = money = t = 0
        seq = []
        for _ in range(nc):
            kind = rng.randint(1, 6)
            if kind == 1:
                pay = rng.randint(1, 20)
                t += 10 * pay
            elif kind == 2:
                pay = rng.randint(1, 400)
                legs += pay
                t += -((-ffr * 180 * pay).numerator // (ffr * 180 * pay).denominator)
            elif kind == 3:
                d, five = rng.randint(1, 600), rng.randint(0, 1)
                pay = d << 1 | five
                t += rgt * d
                money += d * (5 if five else 2)
            else:
                pay = 0
                money += {4: 7, 5: 11, 6: 13}[kind]
            to = rng.randrange(V)
            seq.append([(kind << 29) | pay, at, to, 0])
            at = to
        res[k] = [legs, money, t, (16 << 16) | nc]
        if nc <= mc:
            slots[k, :nc] = seq if nc else 0
            rows[k, 0] = (first if nc else 0) | nc << 25
            for j, s_ in enumerate(seq):
                rows[k, 1 + 2 * j:3 + 2 * j] = [s_[0], s_[2]]
        else:
            res[k, 3] = (80 << 16) | nc
            slots[k, 0] = [0xFFFFFFFF, len(ovf), nc, 0]
            rows[k, 0] = first | 64 << 25
            rows[k, 1:3] = [len(ovf), nc]
            ovf += seq
            wpool += [[s_[0], s_[2]] for s_ in seq]
    ovf = np.array(ovf, dtype=np.uint32).reshape(-1, 4)
    wpool = np.array(wpool, dtype=np.uint32).reshape(-1, 2)
    a_out, a_pool = eng.decode_records_raw(g, p, res, slots, n, mc, ovf)
    b_out, b_pool = eng.decode_wire_raw(g, p, rows, n, mc, wpool)
    for k in range(n):
        fa = [getattr(a_out[k], f) for f, _ in a_out[k]._fields_]
        fb = [getattr(b_out[k], f) for f, _ in b_out[k]._fields_]
        assert fa == fb, k
    ncmd = sum(a_out[k].n_commands for k in range(n))
    assert bytes(memoryview(a_pool)[:ncmd]) == bytes(memoryview(b_pool)[:ncmd])


def test_labels_digest_follows_query_order(eng):
    """labels_digest (the N > 1 gather check): the same labels stored in another
    order hash alike once the order is given, and differently without it."""
    import numpy as np
    from marshrutka_amd.abi import mr_command, mr_result
    n, perm = 4, [2, 0, 3, 1]
    res, pool = (mr_result * n)(), (mr_command * (2 * n))()
    res2, pool2 = (mr_result * n)(), (mr_command * (2 * n))()
    for i in range(n):
        res[i].legs, res[i].n_commands, res[i].command_offset = i, 2, 2 * i
        for c in range(2):
            pool[2 * i + c].kind, pool[2 * i + c].money = c, 10 * i + c
    for k, i in enumerate(perm):  # record k holds query i
        res2[k].legs, res2[k].n_commands, res2[k].command_offset = i, 2, 2 * k
        for c in range(2):
            pool2[2 * k + c].kind, pool2[2 * k + c].money = c, 10 * i + c
    inv = np.empty(n, dtype=np.int64)
    inv[np.array(perm)] = np.arange(n)
    assert eng.labels_digest(res2, pool2, n, inv) == eng.labels_digest(res, pool, n)
    assert eng.labels_digest(res2, pool2, n) != eng.labels_digest(res, pool, n)
