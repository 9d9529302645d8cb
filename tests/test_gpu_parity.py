"""Parity of the HIP engine (through the C ABI) with the CPU oracle and the
committed golden vectors.  Integer/index work: the bar is bit-exact equality of
(legs, money, time, every command)."""
import os
import random

import pytest

from golden_util import as_expected, fixture_names, load
from marshrutka_amd.abi import (BLUE, GREEN, RED, SORT_LEGS, SORT_MONEY, SORT_TIME, YELLOW,
                                CellIndex, Params)
from marshrutka_amd.mapgen import SyntheticMap, random_queries

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


@pytest.fixture(params=["auto-lds", "auto-hbm", "lane-lds", "lanenl-lds", "lanetab-lds", "group-lds", "group16-lds", "group32-lds", "hub1-lds", "hub2-lds", "wide-lds", "widescan-lds", "fallback-lds", "fallback-hbm", "fbsssp-lds",
                        "sssp-lds", "sssp-hbm", "generic-lds", "generic-hbm"])
def grid_state(request, monkeypatch):
    """Every solver path x both grid-state regimes:
    auto     — hub solver when the run time is linear (one source per lane when the
               table fits 22 entries, a source has <= 32 queries and the plan has
               enough such sources to fill the GPU, else one source per 16 or 32 lanes when
               the table fits 32 entries, else two sources per wave when the specials
               fit 32 lanes), else the SSSP solvers
    group    — auto with one source per group of 8 lanes (hub_group_kernel) wherever it
               applies, the lane kernel's plans included (MR_HUB_GROUP_FORCE=1)
    group16  — the same with groups of 16 lanes
    group32  — the same with groups of 32 lanes (the last round through ds_swizzle)
    lane     — auto with the lane kernel whenever it applies (MR_HUB_LANE=1); on the
               standard layout it computes ranks and looks up specials itself
    lanenl   — the same (Fleetfoot 1..3 on the lane kernel is the default; the mode
               keeps the name of the switch, MR_LANE_NONLIN=1)
    lanetab  — the same reading every cell's {sinfo, rank} record (MR_RANK_TABLE=1)
    hub1     — hub solver with one source per wave (no lane or group kernel)
    hub2     — hub solver with two sources per wave (no lane or group kernel)
    wide     — the wide hub solver (several specials per lane) even where the
               narrow one applies
    widescan — the same with each source's region row scanned from the regions'
               boundary cells instead of read from the grid's region table
    fallback — hub solver handing every source over: 64 a pass through the
               certificate (fill, check, repair sweep), the
               rest (and any the certificate cannot answer) to the SSSP kernel
    fbsssp   — the same with the certificate off: every source on the SSSP kernel
    sssp     — no hub solver (level-synchronous solver for Legs-first orders)
    generic  — the bucketed solver for every order."""
    algo, state = request.param.split("-")
    monkeypatch.setenv("MR_GRID_STATE", state)
    monkeypatch.delenv("MR_ALGO", raising=False)
    monkeypatch.delenv("MR_HUB_FALLBACK_ALL", raising=False)
    monkeypatch.delenv("MR_HUB_SPW", raising=False)
    monkeypatch.delenv("MR_HUB_WIDE", raising=False)
    monkeypatch.delenv("MR_HUB_LANE", raising=False)
    monkeypatch.delenv("MR_CERT", raising=False)
    monkeypatch.delenv("MR_CERT_SLOTS", raising=False)
    monkeypatch.delenv("MR_RANK_TABLE", raising=False)
    monkeypatch.delenv("MR_HUB_GROUP", raising=False)
    monkeypatch.delenv("MR_HUB_GROUP_FORCE", raising=False)
    monkeypatch.delenv("MR_LANE_NONLIN", raising=False)
    if algo == "lanenl":
        monkeypatch.setenv("MR_LANE_NONLIN", "1")
        algo = "lane"
    if algo in ("group", "group16", "group32"):
        monkeypatch.setenv("MR_HUB_GROUP_FORCE", "1")
        monkeypatch.setenv("MR_HUB_GROUP", algo[5:] or "8")
    if algo == "lanetab":
        monkeypatch.setenv("MR_RANK_TABLE", "1")
        algo = "lane"
    if algo in ("hub1", "hub2"):
        monkeypatch.setenv("MR_HUB_LANE", "0")
        monkeypatch.setenv("MR_HUB_GROUP", "0")
    if algo == "lane":
        monkeypatch.setenv("MR_HUB_LANE", "1")
    if algo == "wide":
        monkeypatch.setenv("MR_HUB_WIDE", "1")
    if algo == "widescan":
        monkeypatch.setenv("MR_HUB_WIDE", "scan")
    if algo == "hub1":
        monkeypatch.setenv("MR_HUB_SPW", "1")
    if algo in ("sssp", "generic"):
        monkeypatch.setenv("MR_ALGO", algo)
    if algo in ("fallback", "fbsssp"):
        monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    if algo == "fallback":
        monkeypatch.setenv("MR_CERT_SLOTS", "64")
    if algo == "fbsssp":
        monkeypatch.setenv("MR_CERT", "0")
    return request.param


def check(eng, oracle_lib, m, params, queries, label=""):
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    got = eng.FindPath.with_params(g, params).eval_batch(queries)
    exp = og.find_path_batch(params, queries, threads=0)
    bad = [(q, e, r) for q, e, r in zip(queries, exp, got) if as_expected(e) != as_expected(r)]
    assert not bad, f"{label}: {len(bad)}/{len(queries)} mismatches; first: {bad[0]}"


@pytest.mark.parametrize("name", fixture_names())
def test_golden(eng, grid_state, name):
    m, queries, runs = load(name)
    g = eng.MapGrid(m.cells())
    for params, expected in runs:
        got = eng.FindPath.with_params(g, params).eval_batch(queries)
        bad = [(q, e, as_expected(r)) for q, e, r in zip(queries, expected, got) if as_expected(r) != e]
        assert not bad, f"{name} {params}: {len(bad)} mismatches; first {bad[0]}"


def test_kat_single_query_api(eng, oracle_lib):
    # KAT5 through the single-query entry point (src/pathfinder.rs:199)
    m = SyntheticMap(7, campfires_per_homeland=0, seed=0, fountains=0, forums=0,
                     extra_campfires=[CellIndex.homeland(h, 3, 3) for h in range(4)])
    g = eng.MapGrid(m.cells())
    r = eng.FindPath(g, use_soe=False, use_caravans=False, fleetfoot=2).eval(
        CellIndex.parse("B 2#2"), CellIndex.parse("G 2#2"))
    assert (r.legs, r.money, r.time_s) == (6, 0, 1012)
    assert [str(c.to) for c in r.commands] == ["BR 1", "RG 1", "G 2#2"]
    r = eng.FindPath(g).eval(CellIndex.parse("B 3#3"), CellIndex.parse("G 3#3"))
    assert (r.legs, r.money, r.time_s) == (0, 42, 2880)
    r = eng.FindPath(g).eval(CellIndex.center(), CellIndex.center())
    assert (r.legs, r.money, r.time_s, len(r.commands)) == (0, 0, 0, 1)


SORTS = [(a, b) for a in (SORT_LEGS, SORT_TIME, SORT_MONEY) for b in (SORT_LEGS, SORT_TIME, SORT_MONEY)]


def random_params(rng, m):
    hq = None
    if rng.random() < 0.3:
        hq = rng.choice(m.all_indices())
    return Params(scroll_of_escape_cost=rng.choice([0, 1, 50, 500]),
                  scroll_of_escape_hq_cost=rng.choice([0, 75, 3]),
                  scroll_of_escape_forum_cost=rng.choice([0, 100, 7]),
                  use_soe=rng.random() < 0.8, use_sfm=rng.random() < 0.3,
                  use_caravans=rng.random() < 0.8, hq_position=hq,
                  route_guru=rng.choice([0, 1, 2, 3, 4, 5, 6]), fleetfoot=rng.choice([0, 1, 2, 3, 4]),
                  sort_by=rng.choice(SORTS), homeland=rng.choice([BLUE, RED, GREEN, YELLOW]))


@pytest.mark.parametrize("size,k,clustered", [(5, 1, False), (7, 2, False), (11, 3, False),
                                              (15, 4, False), (21, 6, True), (33, 4, False),
                                              (65, 4, False)])
def test_random_params_vs_oracle(eng, oracle_lib, grid_state, size, k, clustered):
    rng = random.Random(size * 1000 + k)
    for trial in range(4):
        m = SyntheticMap(size, campfires_per_homeland=k, seed=rng.randrange(1 << 30), clustered=clustered)
        params = random_params(rng, m)
        queries = random_queries(m, 200 if size <= 33 else 120, rng.randrange(1 << 30))
        check(eng, oracle_lib, m, params, queries, f"S={size} trial={trial} {params}")


def test_default_params_c2_sample(eng, oracle_lib):
    # configs[1]: 64x64 -> odd S = 65, uniform queries, default (app) parameters
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
    check(eng, oracle_lib, m, Params(), random_queries(m, 400, 7), "c2 sample")


def test_c2_full_batch(eng, oracle_lib):
    """configs[1] at its stated size: bench.py's whole c2 batch (10 000 uniform queries
    on the 65x65 map, default parameters) through one plan, every label against the
    oracle's FindPath::eval (src/pathfinder.rs:199-248)."""
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)  # bench.py c2
    qs = random_queries(m, 10_000, 2024 + 17)
    check(eng, oracle_lib, m, Params(), qs, "c2 full batch")


@pytest.mark.parametrize("group", [8, 16, 32])
def test_c2_full_batch_group_kernel(eng, oracle_lib, monkeypatch, group):
    """configs[1]'s whole batch on hub_group_kernel at each group size (MR_HUB_GROUP),
    the plan stats proving which kernel answered, every label against the oracle's
    FindPath::eval (src/pathfinder.rs:199-248)."""
    for v in ("MR_HUB_LANE", "MR_HUB_FALLBACK_ALL", "MR_ALGO", "MR_HUB_WIDE", "MR_HUB_SPW"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("MR_HUB_GROUP", str(group))
    monkeypatch.setenv("MR_HUB_GROUP_FORCE", "1")
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)  # bench.py c2
    qs = random_queries(m, 10_000, 2024 + 17)
    g = eng.MapGrid(m.cells())
    plan = eng.Plan(g, Params(), qs)
    plan.run()
    st = plan.stats()
    # lanes_per_source = G: every source of the plan ran on hub_group_kernel
    assert st["solver"] == "hub" and st["lanes_per_source"] == group and st["fallback_sources"] == 0, st
    got = plan.fetch()
    exp = oracle_lib.OracleGrid(m.cells()).find_path_batch(Params(), qs, threads=0)
    bad = [(q, e, r) for q, e, r in zip(qs, exp, got) if as_expected(e) != as_expected(r)]
    assert not bad, f"G={group}: {len(bad)}/{len(qs)} mismatches; first: {bad[0]}"


@pytest.mark.parametrize("max_cmds", [1, 3, 16])
def test_certificate_sfm_fleetfoot_vs_oracle(eng, oracle_lib, monkeypatch, max_cmds):
    """The scenario whose two plans once disagreed (tools/plan_diff.py; DESIGN.md
    section 3d): 65x65, 5 campfires per homeland, Fleetfoot 2, (Time, Money), the
    Scroll of the Forum, few command slots.  Every source is handed to the certificate
    (MR_HUB_FALLBACK_ALL, 64 slots), in plans of at most 64 sources so that each one
    goes through a slot, and every label is compared with the oracle (SoE / SFm
    src/pathfinder.rs:162-178, the Fleetfoot ceil per run src/cost.rs:122-124).  A
    second run of each plan must give the same bytes (slots are given in source
    order, never by arrival)."""
    import ctypes as C
    from marshrutka_amd.abi import mr_command, mr_result, result_from_c
    from marshrutka_amd import pathfinder as pf
    monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    monkeypatch.setenv("MR_CERT_SLOTS", "64")
    monkeypatch.delenv("MR_CERT", raising=False)
    monkeypatch.delenv("MR_HUB_LANE", raising=False)
    m = SyntheticMap(65, campfires_per_homeland=5, seed=11)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    params = Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True)
    qs = random_queries(m, 3000, 12)
    exp = og.find_path_batch(params, qs, threads=0)
    by_src = {}
    for i, (a, _) in enumerate(qs):
        by_src.setdefault(a, []).append(i)
    groups = list(by_src.values())
    certified = 0
    for lo in range(0, len(groups), 64):
        idx = [i for grp in groups[lo:lo + 64] for i in grp]
        sub = [qs[i] for i in idx]
        plan = eng.Plan(g, params, sub, max_cmds=max_cmds)
        outs = []
        for _ in range(2):
            plan.run()
            cap = len(sub) * 24
            res, pool = (mr_result * len(sub))(), (mr_command * cap)()
            st = pf.lib().mr_plan_fetch(plan.handle, res, pool, cap)
            assert st == 0, st
            outs.append((bytes(res), bytes(pool)))
        assert outs[0] == outs[1], "two runs of one plan differ"
        stats = plan.stats()
        certified += stats["certified_sources"]
        assert stats["fallback_sources"] == len(groups[lo:lo + 64])
        # the sources left to the SSSP kernel: the ones the certificate did not answer
        assert len(plan.fallback_sources()) == stats["fallback_sources"] - stats["certified_sources"]
        got = [result_from_c(res[k], pool) for k in range(len(sub))]
        bad = [(sub[k], exp[i]) for k, i in enumerate(idx) if as_expected(got[k]) != as_expected(exp[i])]
        assert not bad, f"max_cmds={max_cmds}: {len(bad)}/{len(sub)} mismatches; first {bad[0]}"
    assert certified > 0


def test_hbm_regime_mid_grid(eng, oracle_lib):
    m = SyntheticMap(129, campfires_per_homeland=4, seed=77)
    for params in (Params(), Params(fleetfoot=3, sort_by=(SORT_TIME, SORT_MONEY)),
                   Params(sort_by=(SORT_MONEY, SORT_LEGS), use_sfm=True)):
        check(eng, oracle_lib, m, params, random_queries(m, 60, 3), f"S=129 {params}")


def test_edge_cases(eng, oracle_lib):
    m = SyntheticMap(9, campfires_per_homeland=2, seed=3)
    cf = m.campfires()
    specials = [CellIndex.center()] + [CellIndex.border(b, 1) for b in range(4)] + cf
    qs = [(a, b) for a in specials for b in specials]
    qs += [(a, a) for a in m.all_indices()[:20]]
    for params in (Params(), Params(hq_position=cf[0], use_sfm=True),
                   Params(scroll_of_escape_cost=0, hq_position=CellIndex.center(), use_sfm=True,
                          scroll_of_escape_forum_cost=0, scroll_of_escape_hq_cost=0),
                   Params(sort_by=(SORT_TIME, SORT_TIME), fleetfoot=1)):
        check(eng, oracle_lib, m, params, qs, f"edges {params}")


@pytest.mark.parametrize("n_dst", [1, 31, 33, 225])
def test_destinations_per_source(eng, oracle_lib, grid_state, n_dst):
    """The hub solver reads destinations off one query at a time (few per source)
    or one lane per query (many per source); both against the oracle."""
    m = SyntheticMap(15, campfires_per_homeland=3, seed=11, clustered=True)
    cells = m.all_indices()
    rng = random.Random(n_dst)
    srcs = rng.sample(cells, 6)
    qs = [(a, b) for a in srcs for b in (cells if n_dst >= len(cells) else rng.sample(cells, n_dst))]
    for params in (Params(), Params(sort_by=(SORT_TIME, SORT_LEGS)), Params(sort_by=(SORT_MONEY, SORT_TIME))):
        check(eng, oracle_lib, m, params, qs, f"n_dst={n_dst} {params}")


def test_lane_kernel_selection(eng, oracle_lib, monkeypatch):
    """hub_lane_kernel takes a plan's few-query sources when there are enough of them
    to fill the GPU (MR_HUB_LANE_MIN, default half a wave per SIMD), always with
    MR_HUB_LANE=1, never with MR_HUB_LANE=0; the table layout it needs (region
    campfires in entries 6..11) comes from the host's special order.  A plan the lane
    kernel does not take runs one source per group of lanes (hub_group_kernel: 32 for
    plans of at most 1024 sources, else 16) unless MR_HUB_GROUP=0.  Results are the oracle's either way."""
    m = SyntheticMap(33, campfires_per_homeland=4, seed=5)
    qs = random_queries(m, 400, 6)
    g = eng.MapGrid(m.cells())
    lanes, per = {}, {}
    for mode, env in (("default", {}), ("force", {"MR_HUB_LANE": "1"}), ("off", {"MR_HUB_LANE": "0"}),
                      ("min1", {"MR_HUB_LANE_MIN": "1"}), ("nogroup", {"MR_HUB_GROUP": "0"}),
                      ("g16", {"MR_HUB_GROUP": "16"})):
        for k in ("MR_HUB_LANE", "MR_HUB_LANE_MIN", "MR_HUB_GROUP", "MR_HUB_GROUP_FORCE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        pl = eng.Plan(g, Params(), qs)
        st = pl.stats()
        lanes[mode], per[mode] = st["lane_sources"], st["lanes_per_source"]
        check(eng, oracle_lib, m, Params(), qs, f"lane mode {mode}")
    n_src = len({a for a, _ in qs})
    assert lanes["default"] == 0 and lanes["off"] == 0, lanes  # 400 sources < half a wave per SIMD
    assert lanes["force"] == n_src and lanes["min1"] == n_src, lanes
    assert per == {"default": 32, "force": 1, "off": 32, "min1": 1, "nogroup": 0, "g16": 16}, per


@pytest.mark.parametrize("k,hq,tm", [(4, True, 24), (5, False, 32), (6, True, 32)])
def test_lane_kernel_wide_tables(eng, oracle_lib, monkeypatch, k, hq, tm):
    """hub_lane_kernel with the 24- and 32-entry tables (one wave per SIMD): maps with
    k campfires per homeland (+ HQ) put NS = 5 + 4k (+1) specials in registers; every
    comparator order, against the oracle."""
    monkeypatch.setenv("MR_HUB_LANE", "1")
    m = SyntheticMap(41, campfires_per_homeland=k, seed=40 + k)
    qs = random_queries(m, 300, k)
    g = eng.MapGrid(m.cells())
    extra = {"hq_position": m.campfires()[-1]} if hq else {}
    for sort_by in ((0, 2), (1, 2), (2, 0), (1, 0)):
        params = Params(sort_by=sort_by, **extra)
        pl = eng.Plan(g, params, qs)
        st = pl.stats()
        assert st["num_specials"] + 1 <= tm and st["lane_sources"] == st["num_sources"], st
        check(eng, oracle_lib, m, params, qs, f"k={k} hq={hq} {sort_by}")


def test_fallback_sources_reported(eng, oracle_lib, monkeypatch):
    """mr_plan_fallback_sources: the sources a pass re-solved with the SSSP kernel —
    none on a plain hub pass; with MR_HUB_FALLBACK_ALL=1 every source is handed over,
    and the list holds exactly those the certificate did not answer (the certified
    ones cost no search: the cost signal shard.SourceCosts learns from).  The
    certificate's slots go to the least source indices, so with the certificate off
    the list is every source, and with 8 slots it is the same set every run."""
    m = SyntheticMap(25, campfires_per_homeland=3, seed=4)
    qs = random_queries(m, 120, 8)
    g = eng.MapGrid(m.cells())
    pl = eng.Plan(g, Params(), qs)
    pl.run()
    assert pl.stats()["solver"] == "hub" and pl.fallback_sources() == []
    monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    monkeypatch.setenv("MR_CERT", "0")
    pl = eng.Plan(g, Params(), qs)
    pl.run()
    got = pl.fallback_sources()
    assert len(got) == pl.stats()["fallback_sources"] == pl.num_sources
    assert set(got) == {a for a, _ in qs}
    monkeypatch.delenv("MR_CERT")
    monkeypatch.setenv("MR_CERT_SLOTS", "8")  # (the default on this grid size is 64: more than its sources)
    runs = []
    for _ in range(2):
        pl = eng.Plan(g, Params(), qs)
        pl.run()
        st = pl.stats()
        got = pl.fallback_sources()
        assert st["fallback_sources"] == pl.num_sources and 0 < st["certified_sources"] <= 8, st
        assert len(got) == st["fallback_sources"] - st["certified_sources"]
        runs.append(got)
    assert runs[0] == runs[1]
    check(eng, oracle_lib, m, Params(), qs, "all sources re-solved")


def test_invalid_queries_report_errors(eng):
    from marshrutka_amd.abi import MR_ERR_INVALID_INDEX, MR_OK
    m = SyntheticMap(7, campfires_per_homeland=1, seed=3)
    g = eng.MapGrid(m.cells())
    fp = eng.FindPath(g)
    res, _ = fp.eval_batch_raw([(CellIndex.center(), CellIndex.homeland(BLUE, 9, 9)),
                                (CellIndex.center(), CellIndex.homeland(BLUE, 1, 1))])
    assert res[0].status == MR_ERR_INVALID_INDEX and res[1].status == MR_OK
    with pytest.raises(eng.EngineError, match="INVALID_INDEX"):
        fp.eval(CellIndex.homeland(BLUE, 0, 4), CellIndex.center())  # non-canonical


def test_plan_rerun_is_identical(eng):
    m = SyntheticMap(33, campfires_per_homeland=3, seed=5)
    g = eng.MapGrid(m.cells())
    qs = random_queries(m, 300, 9)
    plan = eng.Plan(g, Params(), qs)
    plan.run()
    a = [as_expected(r) for r in plan.fetch()]
    plan.run()
    plan.run()
    b = [as_expected(r) for r in plan.fetch()]
    assert a == b
    ms, n = plan.kernel_ms()
    assert n == 3 and ms > 0


def test_many_passes_without_timing_reads(eng):
    """A plan run far past the pending-event window (mr_plan_run folds the oldest
    timing events itself) still reports every pass in kernel_ms and keeps its
    results; the same for an all-destinations plan (its fill timing too)."""
    m = SyntheticMap(33, campfires_per_homeland=3, seed=6)
    g = eng.MapGrid(m.cells())
    plan = eng.Plan(g, Params(), random_queries(m, 200, 4))
    plan.run()
    a = [as_expected(r) for r in plan.fetch()]
    plan.kernel_ms()
    for _ in range(1300):
        plan.run()
    ms, n = plan.kernel_ms()
    assert n == 1300 and ms > 0
    assert [as_expected(r) for r in plan.fetch()] == a
    sp = eng.SSSPPlan(g, Params(), [CellIndex.center(), m.campfires()[0]])
    sp.run()
    rec = sp.records(1).copy()
    sp.kernel_ms()
    for _ in range(1100):
        sp.run()
    ms, n = sp.kernel_ms()
    assert n == 1100 and ms > 0 and sp.fill_ms() > 0
    assert (sp.records(1) == rec).all()
    del sp, plan  # destroys plans right after their last pass


def test_plan_rerun_with_fallback_sources(eng, oracle_lib):
    """A hub plan whose sources partly fall back (clustered map, Time first) keeps
    both launches on every pass; a plan without any skips the empty fallback launch
    once a pass has shown it empty.  Results stay identical and exact either way."""
    m = SyntheticMap(21, campfires_per_homeland=6, seed=5, clustered=True)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    for params in (Params(sort_by=(SORT_TIME, SORT_MONEY)), Params()):
        qs = random_queries(m, 300, 13)
        exp = [as_expected(e) for e in og.find_path_batch(params, qs, threads=0)]
        plan = eng.Plan(g, params, qs)
        for _ in range(3):
            plan.run()
            assert [as_expected(r) for r in plan.fetch()] == exp
        st = plan.stats()
        assert st["solver"] == "hub"
        if params.sort_by[0] == SORT_TIME:
            assert st["fallback_sources"] > 0


def _sweep():
    """Every FindPath dimension over its whole range, one at a time:
    the 9 sort_by inputs (src/cost.rs:387-405), Fleetfoot 0..3 and out of range,
    RouteGuru 0..5 and out of range, each scroll/caravan toggle, zero and odd costs."""
    sorts = [(a, b) for a in (SORT_LEGS, SORT_TIME, SORT_MONEY) for b in (SORT_LEGS, SORT_TIME, SORT_MONEY)]
    out = [Params(sort_by=s) for s in sorts]
    out += [Params(fleetfoot=f, sort_by=(SORT_TIME, SORT_LEGS)) for f in range(6)]
    out += [Params(route_guru=r, sort_by=(SORT_TIME, SORT_MONEY)) for r in range(8)]
    out += [Params(use_soe=False), Params(use_caravans=False), Params(use_sfm=True),
            Params(use_sfm=True, scroll_of_escape_forum_cost=0),
            Params(scroll_of_escape_cost=0), Params(scroll_of_escape_cost=7, sort_by=(SORT_MONEY, SORT_TIME))]
    return out


@pytest.mark.parametrize("params", _sweep(), ids=lambda p: f"sort{p.sort_by}-ff{p.fleetfoot}-rg{p.route_guru}-"
                         f"soe{int(p.use_soe)}{p.scroll_of_escape_cost}-sfm{int(p.use_sfm)}-car{int(p.use_caravans)}")
def test_parameter_sweep(eng, oracle_lib, params):
    for size, k, clustered, seed in ((15, 3, False, 21), (21, 5, True, 22)):
        m = SyntheticMap(size, campfires_per_homeland=k, seed=seed, clustered=clustered)
        hq = m.campfires()[-1]
        for p in (params, Params(**{**params.__dict__, "hq_position": hq})):
            check(eng, oracle_lib, m, p, random_queries(m, 150, seed + 1), f"S={size} {p}")


@pytest.mark.parametrize("k,clustered", [(16, False), (40, True), (64, True)])
def test_many_campfires(eng, oracle_lib, grid_state, k, clustered):
    """More than 63 specials (SURVEY c5 has 64 clustered campfires per homeland): the
    wide hub solver (2 or 5 specials per lane) with linear run times, the SSSP kernel
    (LDS argmin over the specials) otherwise; Time- and Money-first orders as c5
    prescribes."""
    m = SyntheticMap(41, campfires_per_homeland=k, seed=k, clustered=clustered)
    for params in (Params(), Params(sort_by=(SORT_TIME, SORT_LEGS)), Params(sort_by=(SORT_MONEY, SORT_TIME)),
                   Params(sort_by=(SORT_TIME, SORT_MONEY), fleetfoot=2, route_guru=4)):
        check(eng, oracle_lib, m, params, random_queries(m, 150, k + 1), f"k={k} {params}")
    if grid_state.startswith("auto"):
        st = eng.Plan(eng.MapGrid(m.cells()), Params(), random_queries(m, 10, 1)).stats()
        assert st["solver"] == "hub_wide" and st["specials_per_lane"] == (2 if k == 16 else 5)


@pytest.mark.parametrize("max_cmds", [1, 2, 3])
def test_overflow_pool(eng, oracle_lib, grid_state, max_cmds):
    """Labels longer than the plan's command slots go through the overflow pool
    (mr_plan_create_ex); with 1-3 slots most labels do, and every one must still
    come back whole.  Reruns reuse the pool (its allocator resets per pass)."""
    m = SyntheticMap(25, campfires_per_homeland=6, seed=9, clustered=True)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    for params in (Params(), Params(sort_by=(SORT_TIME, SORT_MONEY))):
        qs = random_queries(m, 200, 3 + max_cmds)
        exp = [as_expected(e) for e in og.find_path_batch(params, qs, threads=0)]
        plan = eng.Plan(g, params, qs, max_cmds=max_cmds)
        for _ in range(2):
            plan.run()
            assert [as_expected(r) for r in plan.fetch()] == exp
        assert any(len(e[3]) > max_cmds for e in exp)


def test_overflow_pool_bound_in_record_order(eng, oracle_lib, grid_state):
    """Outputs bound to one caller buffer with an overflow pool (what the N > 1 gather
    moves raw, mr_plan_bind_outputs_ex): every pass leaves the pool in record order
    (ovf_order_kernel). Each overflowing record's tag points at the prefix sum of
    the command counts of the overflowing records before it. So the raw bytes are the
    same from pass to pass and from plan to plan, and they decode to the oracle's labels."""
    import ctypes as C

    import numpy as np
    # device buffers from the HIP runtime the engine library runs on (torch's wheel carries
    # a runtime of its own, which cannot start once this one holds the device)
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    m = SyntheticMap(25, campfires_per_homeland=6, seed=9, clustered=True)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    mc = 2
    for params in (Params(), Params(sort_by=(SORT_TIME, SORT_MONEY))):
        qs = random_queries(m, 300, 17)
        exp = [as_expected(e) for e in og.find_path_batch(params, qs, threads=0)]
        n, rw, cw, ovf_cap = len(qs), 4, 4 * mc, 8 * len(qs)
        snaps = []
        for _plan in range(2):
            plan = eng.Plan(g, params, qs, max_cmds=mc)
            nw = n * (rw + cw) + ovf_cap * 4
            dbuf = C.c_void_p()
            assert hip.hipMalloc(C.byref(dbuf), nw * 4) == 0 and hip.hipMemset(dbuf, 0, nw * 4) == 0
            p0 = dbuf.value
            plan.bind_outputs(p0, p0 + n * rw * 4, p0 + n * (rw + cw) * 4, ovf_cap)
            for _pass in range(2):
                plan.run()
                plan.wait()
                host = np.zeros(nw, dtype=np.uint32)
                assert hip.hipMemcpy(host.ctypes.data, dbuf, nw * 4, 2) == 0  # device to host
                snaps.append(host)
            words = snaps[-1]
            res = words[: n * rw].reshape(n, rw)
            slots = words[n * rw: n * (rw + cw)].reshape(n, mc, 4)
            st, ln = res[:, 3] >> 16, res[:, 3] & 0xFFFF
            ov = st == 80
            assert ov.sum() >= 20
            offs = np.concatenate([[0], np.cumsum(ln[ov])[:-1]]).astype(np.uint32)
            assert (slots[ov, 0, 0] == 0xFFFFFFFF).all() and (slots[ov, 0, 2] == ln[ov]).all()
            assert (slots[ov, 0, 1] == offs).all(), "overflow offsets not in record order"
            labels = eng.decode_records(g, params, res, slots, n, mc, words[n * (rw + cw):])
            q_of = plan.record_queries()
            got = [None] * n
            for k in range(n):
                got[q_of[k]] = as_expected(labels[k])
            assert got == exp
            assert [as_expected(r) for r in plan.fetch()] == exp
            del plan
            hip.hipFree(dbuf)
        assert all((s == snaps[0]).all() for s in snaps), "raw outputs differ between passes / plans"


@pytest.mark.parametrize("mc,ff,sort_by", [(2, 0, (SORT_LEGS, SORT_MONEY)), (4, 2, (SORT_TIME, SORT_MONEY)),
                                            (3, 3, (SORT_MONEY, SORT_TIME)), (16, 1, (SORT_TIME, SORT_LEGS))])
def test_wire_records_match_oracle(eng, oracle_lib, grid_state, mc, ff, sort_by):
    """mr_plan_wire_records (what the N > 1 gather moves, 4 + 8 max_cmds bytes a query)
    decoded on the host by mr_decode_wire: every label equals the oracle's and the plan's
    own fetch — metrics recomputed from the commands, `from` cells from the chain, long
    labels through the wire pool, rows past the records (invalid queries) INVALID_INDEX."""
    import ctypes as C

    import numpy as np
    from marshrutka_amd.abi import MR_ERR_INVALID_INDEX
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    m = SyntheticMap(33, campfires_per_homeland=5, seed=21 + mc, clustered=True)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    params = Params(fleetfoot=ff, sort_by=sort_by, use_sfm=mc == 3, route_guru=mc % 6)
    qs = random_queries(m, 400, 5 + mc)
    exp = [as_expected(e) for e in og.find_path_batch(params, qs, threads=0)]
    qs_all = qs + [(CellIndex.center(), CellIndex.homeland(BLUE, 99, 99))] * 3
    n, rw, pcap = len(qs_all), eng.wire_row_words(mc), 4 * len(qs_all)
    nw = n * rw + 2 * pcap
    dbuf = C.c_void_p()
    assert hip.hipMalloc(C.byref(dbuf), nw * 4) == 0 and hip.hipMemset(dbuf, 0, nw * 4) == 0
    try:
        plan = eng.Plan(g, params, qs_all, max_cmds=mc)
        for _pass in range(2):
            plan.run()
            plan.wire_records(dbuf.value, dbuf.value + n * rw * 4, pcap)
            plan.wait()
            host = np.zeros(nw, dtype=np.uint32)
            assert hip.hipMemcpy(host.ctypes.data, dbuf, nw * 4, 2) == 0
            out, cmds = eng.decode_wire_raw(g, params, host[: n * rw], n, mc, host[n * rw:])
            q_of = plan.record_queries()
            got = [None] * len(qs)
            for k in range(n):
                if k >= len(qs):
                    assert out[k].status == MR_ERR_INVALID_INDEX and q_of[k] == 0xFFFFFFFF
                    continue
                got[q_of[k]] = as_expected(eng.result_from_c(out[k], cmds)) if out[k].status == 0 else None
            assert got == exp
        assert mc != 2 or any(len(e[3]) > mc for e in exp if e)
        assert [as_expected(r) for r in plan.fetch()[: len(qs)]] == exp
        del plan
    finally:
        hip.hipFree(dbuf)


@pytest.mark.parametrize("kernel", ["hub", "lane", "group8", "group32"])
@pytest.mark.parametrize("ff", [1, 2, 3])
@pytest.mark.parametrize("sort_by", [(SORT_LEGS, SORT_MONEY), (SORT_LEGS, SORT_TIME), (SORT_MONEY, SORT_LEGS),
                                     (SORT_MONEY, SORT_TIME), (SORT_TIME, SORT_LEGS), (SORT_TIME, SORT_MONEY)])
def test_fleetfoot_hub(eng, oracle_lib, monkeypatch, ff, sort_by, kernel):
    """Non-linear run times (Fleetfoot 1..3) through the hub solver: every closed-form
    label certified against near-ties of the time gap, uncertain sources re-solved by
    the SSSP kernel.  Bit-exact against the oracle, with both one and many
    destinations per source, and most sources answered by the hub itself.  kernel:
    hub_kernel alone, the lane kernel's Fleetfoot instantiation for every source with at
    most 32 queries (MR_HUB_LANE=1, MR_LANE_NONLIN=1; 22- and 32-entry tables), or the
    group kernel's with 8 / 32 lanes a source (MR_HUB_GROUP_FORCE=1)."""
    for v in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_HUB_SPW", "MR_HUB_WIDE", "MR_HUB_NONLIN", "MR_GRID_STATE",
              "MR_HUB_GROUP", "MR_HUB_GROUP_FORCE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("MR_HUB_LANE", "1" if kernel == "lane" else "0")
    monkeypatch.setenv("MR_LANE_NONLIN", "0" if kernel == "hub" else "1")
    if kernel.startswith("group"):
        monkeypatch.setenv("MR_HUB_LANE", "0")
        monkeypatch.setenv("MR_HUB_GROUP_FORCE", "1")
        monkeypatch.setenv("MR_HUB_GROUP", kernel[5:])
    for size, k, clustered, seed in ((33, 4, False, 31), (65, 6, True, 32), (129, 4, False, 33)):
        m = SyntheticMap(size, campfires_per_homeland=k, seed=seed + ff, clustered=clustered)
        params = Params(fleetfoot=ff, sort_by=sort_by, route_guru=ff, hq_position=m.campfires()[2])
        rng = random.Random(seed * 7 + ff)
        cells = m.all_indices()
        qs = random_queries(m, 400, seed + ff)
        src = rng.choice(cells)
        qs += [(src, d) for d in rng.sample(cells, 120)]  # many destinations for one source
        g = eng.MapGrid(m.cells())
        og = oracle_lib.OracleGrid(m.cells())
        plan = eng.Plan(g, params, qs)
        plan.run()
        got = plan.fetch()
        exp = og.find_path_batch(params, qs, threads=0)
        bad = [(q, e, r) for q, e, r in zip(qs, exp, got) if as_expected(e) != as_expected(r)]
        assert not bad, f"S={size} {params}: {len(bad)}/{len(qs)} mismatches; first: {bad[0]}"
        st = plan.stats()
        assert st["solver"] == "hub"
        assert st["fallback_sources"] <= st["num_sources"] // 4, st
        if kernel == "lane":
            assert st["lane_sources"] == st["num_sources"] - 1 and st["lanes_per_source"] == 1, st
        elif kernel == "hub":
            assert st["lane_sources"] == 0 and st["lanes_per_source"] == 0, st
        else:
            assert st["lanes_per_source"] == int(kernel[5:]), st


@pytest.mark.parametrize("kernel", ["lane", "group16"])
@pytest.mark.parametrize("ff", [1, 2, 3])
def test_fleetfoot_random_257(eng, oracle_lib, monkeypatch, ff, kernel):
    """The Fleetfoot lane / group kernels on 257^2 maps (6 campfires a homeland: a 32-entry
    table, or 4 clustered: 22 entries; SoE / SFm / caravans toggled; Route Guru; HQ on a campfire or none), every
    order, against the oracle: 6 orders x 2 maps x 240 queries per case, each source with
    at most a few queries, so the lane kernel answers all of them (or relists them for
    hub_kernel)."""
    for v in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_HUB_SPW", "MR_HUB_WIDE", "MR_HUB_NONLIN", "MR_GRID_STATE",
              "MR_HUB_GROUP", "MR_HUB_GROUP_FORCE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("MR_LANE_NONLIN", "1")
    if kernel == "lane":
        monkeypatch.setenv("MR_HUB_LANE", "1")
    else:
        monkeypatch.setenv("MR_HUB_LANE", "0")
        monkeypatch.setenv("MR_HUB_GROUP_FORCE", "1")
        monkeypatch.setenv("MR_HUB_GROUP", "16")
    rng = random.Random(257 + ff)
    for clustered in (False, True):
        m = SyntheticMap(257, campfires_per_homeland=6 if not clustered else 4, seed=900 + ff + 10 * clustered,
                         clustered=clustered)
        g = eng.MapGrid(m.cells())
        og = oracle_lib.OracleGrid(m.cells())
        qs = random_queries(m, 240, 31 * ff + clustered)
        for sort_by in SORTS:
            if sort_by[0] == sort_by[1]:
                continue
            params = Params(fleetfoot=ff, sort_by=sort_by, route_guru=rng.choice([0, 2, 5]),
                            use_soe=rng.random() < 0.8, use_sfm=rng.random() < 0.5, use_caravans=rng.random() < 0.8,
                            hq_position=m.campfires()[rng.randrange(len(m.campfires()))] if rng.random() < 0.5 else None)
            plan = eng.Plan(g, params, qs)
            plan.run()
            got = plan.fetch()
            st = plan.stats()
            assert st["solver"] == "hub", st
            assert st["lanes_per_source"] == (1 if kernel == "lane" else 16), st
            exp = og.find_path_batch(params, qs, threads=0)
            bad = [(q, e, r) for q, e, r in zip(qs, exp, got) if as_expected(e) != as_expected(r)]
            assert not bad, f"{kernel} ff={ff} {params}: {len(bad)}/{len(qs)} mismatches; first: {bad[0]}"


def test_device_records_grouped_by_source(eng):
    """The compact device records (what the multi-GPU gather moves) are grouped by
    source; mr_plan_record_queries maps record k back to its query, and each record's
    metrics equal the fetched result of that query."""
    m = SyntheticMap(33, campfires_per_homeland=3, seed=8)
    g = eng.MapGrid(m.cells())
    qs = random_queries(m, 500, 4) + [(CellIndex.homeland(BLUE, 200, 1), m.campfires()[0])]  # one invalid
    plan = eng.Plan(g, Params(), qs)
    plan.run()
    got = plan.fetch()
    d_res, rb, _, _ = plan.device_outputs()
    words = _device_words(d_res, rb)
    qmap = plan.record_queries()
    valid = [k for k in range(len(qs)) if qmap[k] != 0xFFFFFFFF]
    assert len(valid) == len(qs) - 1 and sorted(qmap[k] for k in valid) == list(range(len(qs) - 1))
    srcs = [qs[qmap[k]][0] for k in valid]  # each source's records contiguous
    assert all(srcs[i] == srcs[i - 1] or srcs[i] not in srcs[:i] for i in range(1, len(srcs)))
    for k in valid:
        r = got[qmap[k]]
        assert (int(words[4 * k]), int(words[4 * k + 1]), int(words[4 * k + 2])) == (r.legs, r.money, r.time_s)


def _device_words(ptr: int, nbytes: int):
    """Copies nbytes of device memory at ptr into a host numpy uint32 array (hipMemcpy)."""
    import ctypes as C
    import numpy as np
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    out = np.empty(nbytes // 4, dtype=np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, C.c_void_p(ptr), nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


@pytest.mark.parametrize("max_cmds", [1, 3, 16])
def test_device_fetch_matches_host_decode(eng, monkeypatch, max_cmds):
    """mr_plan_fetch expands the records on the device (mr_k_decode.hip) and copies the
    ABI arrays once; MR_HOST_DECODE=1 keeps the host decoder.  Both must write the same
    bytes: invalid queries, labels in the overflow pool (few command slots), Time-first
    Fleetfoot labels, and a caller pool too short for every label (MR_ERR_CAPACITY).
    "pinned": the device path into page-locked caller arrays (mr_host_register: direct
    DMA, no stage)."""
    import ctypes as C
    from marshrutka_amd.abi import MR_ERR_CAPACITY, mr_command, mr_query, mr_result
    from marshrutka_amd import pathfinder as pf
    m = SyntheticMap(65, campfires_per_homeland=5, seed=11)
    g = eng.MapGrid(m.cells())
    qs = random_queries(m, 3000, 12)
    qs[5] = (CellIndex(1, 0, 999, 999), qs[5][1])  # not a cell of the grid
    qs[77] = (qs[77][0], CellIndex(2, 1, 999, 0))
    for params in (Params(), Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True)):
        out = {}
        for mode in ("device", "pinned", "wire", "host"):
            if mode == "host":
                monkeypatch.setenv("MR_HOST_DECODE", "1")
            else:
                monkeypatch.delenv("MR_HOST_DECODE", raising=False)
            # "wire" (the default): rows re-encoded on the device, decoded on the host
            # pool; "device" / "pinned": the device decoder (MR_FETCH_WIRE=0)
            monkeypatch.setenv("MR_FETCH_WIRE", "1" if mode == "wire" else "0")
            plan = eng.Plan(g, params, qs, max_cmds=max_cmds)
            plan.run()
            for cap in (len(qs) * 24, 500):
                res = (mr_result * len(qs))()
                pool = (mr_command * cap)()
                if mode == "pinned":
                    pf.pin_host(res)
                    pf.pin_host(pool)
                st = pf.lib().mr_plan_fetch(plan.handle, res, pool, cap)
                if mode == "pinned":
                    pf.unpin_host(res)
                    pf.unpin_host(pool)
                out[(mode, cap)] = (st, bytes(res), bytes(pool))
        for cap in (len(qs) * 24, 500):
            for mode in ("device", "pinned", "wire"):
                d, h = out[(mode, cap)], out[("host", cap)]
                assert d[0] == h[0], (mode, cap, d[0], h[0])
                assert d[1] == h[1], (mode, cap)
                assert d[2] == h[2], (mode, cap)
        assert out[("device", 500)][0] == MR_ERR_CAPACITY or out[("device", 500)][0] < 0
