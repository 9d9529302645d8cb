"""Known-answer tests of the CPU oracle (hand-derived from the
reference code) plus the one fixture the reference itself pins on this
boundary (Duration Display, src/pathfinder.rs:279-285)."""
import pytest

from marshrutka_amd.abi import (BLUE, BR, CMD_CARAVAN, CMD_CENTRAL, CMD_NO_MOVE, CMD_SFM,
                                CMD_STANDARD, GREEN, RG, SORT_LEGS, SORT_MONEY, CellIndex,
                                Params, duration_display)
from marshrutka_amd.mapgen import SyntheticMap

C = CellIndex


def corner_campfires(size):
    h = size // 2
    return tuple(C.homeland(k, h, h) for k in range(4))


def plain_map(size, campfires=None):
    # MapGrid::parse reaches unreachable!() (src/grid.rs:209) when a homeland has
    # no campfire, so every map carries at least one per homeland; the
    # "no teleports" KATs switch SoE and caravans off instead.
    if campfires is None:
        campfires = corner_campfires(size)
    return SyntheticMap(size, campfires_per_homeland=0, seed=0, extra_campfires=campfires,
                        fountains=0, forums=0)


NO_TELEPORTS = dict(use_soe=False, use_caravans=False)


def grid(ol, size, campfires=None):
    return ol.OracleGrid(plain_map(size, campfires).cells())


def cmd_tuple(c):
    return (c.kind, c.time_s, c.legs, c.money, c.fleetfoot, str(c.from_), str(c.to))


def test_duration_display_reference_fixture(oracle_lib):
    # src/pathfinder.rs:279-285: 63 min + 10 s displays as "1h3m10s"
    assert oracle_lib.duration_display(63 * 60 + 10) == "1h3m10s"
    assert duration_display(63 * 60 + 10) == "1h3m10s"
    assert duration_display(1100) == "18m20s"


def test_kat1_from_equals_to(oracle_lib):
    g = grid(oracle_lib, 5)
    r = g.find_path(Params(), C.homeland(BLUE, 1, 1), C.homeland(BLUE, 1, 1))
    assert (r.legs, r.money, r.time_s) == (0, 0, 0)
    assert [cmd_tuple(c) for c in r.commands] == [(CMD_NO_MOVE, 0, 0, 0, 0, "B 1#1", "B 1#1")]


def test_kat2_single_standard_move(oracle_lib):
    g = grid(oracle_lib, 5)
    r = g.find_path(Params(), C.parse("B 1#1"), C.parse("B 2#1"))
    assert (r.legs, r.money, r.time_s) == (1, 0, 180)
    assert [cmd_tuple(c) for c in r.commands] == [(CMD_STANDARD, 180, 1, 0, 0, "B 1#1", "B 2#1")]


def test_kat3_central_move(oracle_lib):
    g = grid(oracle_lib, 5)
    r = g.find_path(Params(), C.center(), C.parse("BR 1"))
    assert (r.legs, r.money, r.time_s) == (0, 0, 10)
    assert [cmd_tuple(c) for c in r.commands] == [(CMD_CENTRAL, 10, 0, 0, 0, "0#0", "BR 1")]


def test_kat4_central_moves_merge(oracle_lib):
    g = grid(oracle_lib, 5)
    r = g.find_path(Params(), C.parse("BR 1"), C.parse("RG 1"))
    assert (r.legs, r.money, r.time_s) == (0, 0, 20)
    assert [cmd_tuple(c) for c in r.commands] == [(CMD_CENTRAL, 20, 0, 0, 0, "BR 1", "RG 1")]


@pytest.mark.parametrize("ff,time", [(0, 1100), (1, 1040), (2, 1012), (3, 986)])
def test_kat5_tie_break_and_fleetfoot(oracle_lib, ff, time):
    g = grid(oracle_lib, 7)
    r = g.find_path(Params(fleetfoot=ff, **NO_TELEPORTS), C.parse("B 2#2"), C.parse("G 2#2"))
    assert (r.legs, r.money, r.time_s) == (6, 0, time)
    assert [cmd_tuple(c) for c in r.commands] == [
        (CMD_STANDARD, 540, 3, 0, ff, "B 2#2", "BR 1"),
        (CMD_CENTRAL, 20, 0, 0, 0, "BR 1", "RG 1"),
        (CMD_STANDARD, 540, 3, 0, ff, "RG 1", "G 2#2"),
    ]
    if ff == 0:
        assert duration_display(r.time_s) == "18m20s"


def test_kat6_forum_scroll_and_money_first(oracle_lib):
    g = grid(oracle_lib, 7)
    r = g.find_path(Params(use_sfm=True, **NO_TELEPORTS), C.parse("B 3#3"), C.center())
    assert (r.legs, r.money, r.time_s) == (0, 100, 0)
    assert [cmd_tuple(c) for c in r.commands] == [(CMD_SFM, 0, 0, 100, 0, "B 3#3", "0#0")]
    r = g.find_path(Params(use_sfm=True, sort_by=(SORT_MONEY, SORT_LEGS), **NO_TELEPORTS),
                    C.parse("B 3#3"), C.center())
    assert (r.legs, r.money, r.time_s) == (5, 0, 910)
    assert [cmd_tuple(c) for c in r.commands] == [
        (CMD_STANDARD, 900, 5, 0, 0, "B 3#3", "BR 1"),
        (CMD_CENTRAL, 10, 0, 0, 0, "BR 1", "0#0"),
    ]


def test_kat7_caravans_via_center(oracle_lib):
    g = grid(oracle_lib, 7)  # campfires at B/R/G/Y 3#3
    r = g.find_path(Params(), C.parse("B 3#3"), C.parse("G 3#3"))
    assert (r.legs, r.money, r.time_s) == (0, 42, 2880)
    assert [cmd_tuple(c) for c in r.commands] == [
        (CMD_CARAVAN, 1440, 0, 12, 0, "B 3#3", "0#0"),
        (CMD_CARAVAN, 1440, 0, 30, 0, "0#0", "G 3#3"),
    ]


def test_nearest_campfire_projection_equals_argmin(oracle_lib):
    # src/grid.rs:155-230 computes nearest campfires via border/centre
    # projections; SURVEY §8a A13 claims this equals the direct argmin.
    for seed in range(4):
        m = SyntheticMap(15, campfires_per_homeland=3, seed=seed)
        g = oracle_lib.OracleGrid(m.cells())
        for i in range(15 * 15):
            for h in range(4):
                assert g.nearest_campfire(i, h) == g.nearest_campfire(i, h, direct=True)


def test_invalid_inputs(oracle_lib):
    from marshrutka_amd.abi import MR_ERR_INVALID_INDEX
    g = grid(oracle_lib, 5)
    with pytest.raises(ValueError, match=str(MR_ERR_INVALID_INDEX)):
        g.find_path(Params(), C.parse("B 3#1"), C.center())  # outside a 5x5 grid


def test_homeland_without_campfire_is_rejected(oracle_lib):
    # the reference panics (unreachable!(), src/grid.rs:209); we return an error
    m = SyntheticMap(7, campfires_per_homeland=0, seed=0, extra_campfires=corner_campfires(7)[:3])
    with pytest.raises(ValueError, match="-2"):
        oracle_lib.OracleGrid(m.cells())


@pytest.mark.parametrize("size,k,seed", [(15, 3, 1), (21, 4, 2)])
def test_sssp_all_equals_per_query_eval(oracle_lib, size, k, seed):
    """The all-destinations oracle (Dijkstra without the early exit) gives, for every
    cell, exactly the label a separate eval(src, cell) returns."""
    import random
    from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, Params
    from marshrutka_amd.mapgen import SyntheticMap
    m = SyntheticMap(size, campfires_per_homeland=k, seed=seed, clustered=seed % 2 == 0)
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    rng = random.Random(seed)
    key = lambda t: None if t is None else t.as_tuple()  # noqa: E731
    for params in (Params(), Params(sort_by=(SORT_TIME, SORT_MONEY), fleetfoot=2, use_sfm=True)):
        for src in rng.sample(cells, 2):
            full = og.sssp_all(params, src)
            each = og.find_path_batch(params, [(src, d) for d in cells])
            assert [key(a) for a in full] == [key(b) for b in each]
