"""Parity at the BASELINE sizes (configs[2], [3], [4]) through the C ABI.

The oracle's Dijkstra run to completion (oracle/mr_oracle.cpp mro_sssp_digest_batch,
the reference's FindPath::eval loop src/pathfinder.rs:219-246 without its early exit)
gives every cell's label from a source; labels are compared whole (metrics, command
count and a digest of the command list, tests/label_digest.py) with numpy.

* configs[3] (c4): the bench's whole 1M-query batch on the 1025^2 map plus 1000
  destinations for each of 32 sources (16 of every kind: Center, border-1 cells,
  campfires, on-axis and random cells; 16 of the batch's own), one Plan as the bench
  runs it.  Every label of the batch is property-checked; every label of the 32
  sources is compared with the oracle, and 64 batch queries with the oracle's
  single-query eval.
* configs[2] (c3): every one of the 1 050 625 cells of 4 sources at 1025^2 through the
  all-destinations plan (hub + fill), two comparator orders.
* configs[4] (c5): every one of the 16.8 M cells of 3 sources at 4097^2 (64 clustered
  campfires per homeland, Time and Money first) through the wide hub solver's query
  path, and a 2000-query batch.  The oracle needs minutes and ~13 GB per solve at
  that size, so its answers are committed fixtures (tests/golden/make_full_scale.py).
"""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest

import label_digest as ld
from golden_util import as_expected
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, CellIndex, Params, mr_command, mr_result
from marshrutka_amd.mapgen import SyntheticMap, random_queries, random_query_cells

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16  # the GPU box's CPU share
FF_RATIO = {1: (50, 53), 2: (100, 109), 3: (25, 28)}  # Fleetfoot run-time ratios (src/skill.rs:65-71)
C5_FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_scale", "c5.json")


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    for v in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_HUB_SPW", "MR_HUB_WIDE", "MR_HUB_NONLIN", "MR_GRID_STATE",
              "MR_FILL_GX", "MR_DBG_FLAGS", "MR_FILL_OVERLAP", "MR_FILL_FUSED", "MR_FILL_SLOTS"):
        os.environ.pop(v, None)
    return pathfinder


@pytest.fixture(scope="module")
def c4_map():
    m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)  # bench.py c3/c4
    return m, m.cells_array()


def _sources_of_every_kind(m, rng):
    H = m.h
    cf = m.campfires()
    srcs = [CellIndex.center()] + [CellIndex.border(b, 1) for b in range(4)]
    srcs += [cf[0], cf[len(cf) // 3], cf[-1]]
    srcs += [CellIndex.border(0, H), CellIndex.border(1, H // 2), CellIndex.border(3, 2)]  # on the axes
    srcs += [CellIndex.homeland(2, 1, 1), CellIndex.homeland(0, H, H)]  # next to the Center, a corner
    while len(srcs) < 16:
        c = m.index_at(rng.randrange(m.size * m.size))
        if c not in srcs:
            srcs.append(c)
    return srcs


@pytest.fixture(scope="module")
def c4_batch(c4_map):
    """bench.py's configs[3] batch: 1M uniform queries on the 1025^2 map (645k sources),
    as row-major cells and as mr_query records."""
    m, arr = c4_map
    uni_src, uni_dst = random_query_cells(m, 1_000_000, 4096 + 17)
    return uni_src, uni_dst, m.query_array(uni_src, uni_dst, arr)


@pytest.fixture(scope="module")
def c4_sources(c4_map, c4_batch):
    """32 sources with 1 000 destinations each and the oracle's Dijkstra from each of
    them (mro_sssp_digest_batch: every cell's label, src/pathfinder.rs:219-246 run to
    completion): 16 of every kind (Center, border-1 cells, campfires, on-axis, random)
    and the 16 batch sources with the most queries."""
    import oracle_lib
    oracle_lib.build()
    m, arr = c4_map
    uni_src, _, _ = c4_batch
    V = m.size * m.size
    rng = random.Random(4096)
    srcs = _sources_of_every_kind(m, rng)
    cnt = np.bincount(uni_src, minlength=V)
    for c in np.argsort(-cnt, kind="stable"):
        if len(srcs) == 32:
            break
        ci = m.index_at(int(c))
        if ci not in srcs:
            srcs.append(ci)
    cf_cells = [m.cell_of(c) for c in m.campfires()]
    dsts = []
    for s in srcs:
        dsts.append(np.array(rng.sample(range(V), 1000 - len(cf_cells) - 2) + cf_cells +
                             [m.cell_of(CellIndex.center()), m.cell_of(s)], dtype=np.int64))
    og = oracle_lib.OracleGrid.from_array(arr)
    want = og.sssp_digests(Params(), srcs, threads=ORACLE_THREADS)
    return srcs, dsts, want, og


def _tail_digests(res, pool, n_total: int, first: int):
    """label_digest fields of records first..n_total-1 of a fetch (no work on the rest)."""
    raw = np.frombuffer(res, dtype=np.uint8, count=n_total * C.sizeof(mr_result))
    return ld.digests(raw[first * C.sizeof(mr_result):], pool, n_total - first)


def test_c4_full_scale(eng, c4_map, c4_batch, c4_sources):
    """configs[3] at its stated size: the bench's whole 1M-query batch on one GPU (645k
    unique sources) as the bench runs it.  Every source runs on hub_lane_kernel (plan
    stats), every label is property-checked, and the batch's own queries are compared
    with the oracle: >= 2 000 of them through the oracle's Dijkstra from the busiest
    batch sources (whole label: metrics, command count, command-list digest), and 64
    random ones through the oracle's single-query FindPath::eval."""
    m, arr = c4_map
    uni_src, uni_dst, qarr = c4_batch
    _, _, _, og = c4_sources
    V = m.size * m.size
    keys = ld.cell_keys(arr)
    n = len(uni_src)
    g = eng.MapGrid.from_array(arr)
    plan = eng.Plan(g, Params(), None, max_cmds=6, query_array=qarr)
    plan.run()
    plan.run()  # the bench's steady state: a rerun of the same plan
    res, pool = plan.fetch_raw()
    # the same fetch into page-locked arrays (mr_host_register: direct DMA) writes the same bytes
    pres, ppool = plan.fetch_buffers()
    for b in (pres, ppool):
        eng.pin_host(b)
    plan.fetch_raw((pres, ppool))
    for b in (pres, ppool):
        eng.unpin_host(b)
    assert np.array_equal(np.frombuffer(pres, dtype=np.uint8), np.frombuffer(res, dtype=np.uint8))
    nb_cmd = int(np.frombuffer(res, dtype=np.uint32).reshape(n, 8)[:, 4].astype(np.int64).sum()) * C.sizeof(mr_command)
    assert np.array_equal(np.frombuffer(ppool, dtype=np.uint8, count=nb_cmd), np.frombuffer(pool, dtype=np.uint8, count=nb_cmd))
    st = plan.stats()
    assert st["solver"] == "hub" and st["num_sources"] >= 645_000, st
    # the headline kernel answered every source of the batch
    assert st["lanes_per_source"] == 1 and st["lane_sources"] == st["num_sources"], st
    assert st["fallback_sources"] == 0, st
    props = ld.label_properties(res, pool, n, keys[uni_src], keys[uni_dst])
    assert all(v == 0 for v in props.values()), props
    got = ld.digests(res, pool, n)
    # >= 2 000 batch queries: every query of the busiest batch sources, one oracle
    # Dijkstra per source, 32 sources at a time (33 MB of digests per source)
    cnt = np.bincount(uni_src, minlength=V)
    busiest = np.argsort(-cnt, kind="stable")
    take = int(np.searchsorted(np.cumsum(cnt[busiest]), 2000)) + 1
    checked = 0
    for lo in range(0, take, 32):
        chunk = busiest[lo:lo + 32]
        want = og.sssp_digests(Params(), [m.index_at(int(c)) for c in chunk], threads=ORACLE_THREADS)
        for i, c in enumerate(chunk):
            mine = np.nonzero(uni_src == c)[0]
            bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=mine, idx_exp=uni_dst[mine])
            assert bad.size == 0, (str(m.index_at(int(c))), len(bad), [str(m.index_at(int(uni_dst[mine][j]))) for j in bad[:4]])
            checked += mine.size
        del want
    assert checked >= 2000, checked
    # uniform batch queries from random sources: the oracle's own single-query eval
    rng = random.Random(4097)
    sample = rng.sample(range(n), 64)
    pairs = [(m.index_at(int(uni_src[i])), m.index_at(int(uni_dst[i]))) for i in sample]
    eres, epool = og.find_path_batch_raw(Params(), pairs, threads=ORACLE_THREADS)
    ed = ld.digests(eres, epool, len(sample))
    bad = ld.mismatches(got, ed, idx_got=np.array(sample))
    assert bad.size == 0, [pairs[j] for j in bad[:4]]


def test_c4_lane_kernel_vs_oracle(eng, c4_map, c4_batch, c4_sources):
    """hub_lane_kernel itself against the oracle at configs[3]: 32 sources x 1 000
    destinations (32 000 labels), each plan the bench's whole 1M batch plus every one
    of the 32 sources with at most 32 queries in all (kLaneMaxQ: a source with more
    runs on hub_kernel), so each compared label is the lane kernel's read-off; the plan
    stats prove that every source of every plan ran on it."""
    m, arr = c4_map
    uni_src, uni_dst, qarr = c4_batch
    srcs, dsts, want, _ = c4_sources
    V = m.size * m.size
    nb = len(uni_src)
    cnt = np.bincount(uni_src, minlength=V)
    caps = [32 - int(cnt[m.cell_of(s)]) for s in srcs]
    assert min(caps) >= 16, caps
    n_plans = max(-(-len(d) // c) for d, c in zip(dsts, caps))
    g = eng.MapGrid.from_array(arr)
    bufs = None
    compared = 0
    for p in range(n_plans):
        ex_src, ex_dst, owner = [], [], []
        for i, (s, d, c) in enumerate(zip(srcs, dsts, caps)):
            piece = d[p * c:(p + 1) * c]
            ex_src.append(np.full(len(piece), m.cell_of(s), dtype=np.int64))
            ex_dst.append(piece)
            owner.append(np.full(len(piece), i, dtype=np.int64))
        ex_src, ex_dst, owner = np.concatenate(ex_src), np.concatenate(ex_dst), np.concatenate(owner)
        q = np.concatenate([qarr, m.query_array(ex_src, ex_dst, arr)])
        plan = eng.Plan(g, Params(), None, max_cmds=6, query_array=q)
        plan.run()
        st = plan.stats()
        assert st["solver"] == "hub" and st["lanes_per_source"] == 1, st
        assert st["lane_sources"] == st["num_sources"] and st["fallback_sources"] == 0, st
        if bufs is None:
            bufs = eng.fetch_buffers(len(q) + 1024, 6)
        res, pool = plan.fetch_raw(bufs)
        got = _tail_digests(res, pool, len(q), nb)
        for i in range(len(srcs)):
            sel = np.nonzero(owner == i)[0]
            if sel.size == 0:
                continue
            bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=ex_dst[sel])
            assert bad.size == 0, (p, str(srcs[i]), len(bad), [str(m.index_at(int(ex_dst[sel][j]))) for j in bad[:4]])
            compared += sel.size
        del plan
    assert compared == sum(len(d) for d in dsts) >= 32_000, compared


def test_c4_busy_sources_hub_kernel(eng, c4_map, c4_batch, c4_sources):
    """The same 32 sources with all 1 000 destinations each in one plan beside the 1M
    batch: sources with more than 32 queries leave the lane kernel for hub_kernel (a
    lane per query), so this compares hub_kernel's read-off at configs[3]'s size."""
    m, arr = c4_map
    uni_src, uni_dst, qarr = c4_batch
    srcs, dsts, want, _ = c4_sources
    nb = len(uni_src)
    ex_src = np.concatenate([np.full(len(d), m.cell_of(s), dtype=np.int64) for s, d in zip(srcs, dsts)])
    ex_dst = np.concatenate(dsts)
    q = np.concatenate([qarr, m.query_array(ex_src, ex_dst, arr)])
    g = eng.MapGrid.from_array(arr)
    plan = eng.Plan(g, Params(), None, max_cmds=6, query_array=q)
    plan.run()
    st = plan.stats()
    assert st["solver"] == "hub" and st["lane_sources"] == st["num_sources"] - len(srcs), st
    res, pool = plan.fetch_raw()
    got = _tail_digests(res, pool, len(q), nb)
    for i, s in enumerate(srcs):
        sel = np.arange(i * 1000, (i + 1) * 1000)
        bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=ex_dst[sel])
        assert bad.size == 0, (str(s), len(bad), [str(m.index_at(int(ex_dst[sel][j]))) for j in bad[:4]])


@pytest.mark.parametrize("ff", [1, 2, 3])
def test_fleetfoot_time_first_1025(eng, oracle_lib, c4_map, ff):
    """Non-linear run times (Fleetfoot 1, 2, 3) with Time first at configs[3]'s size: the
    certified hub path (DESIGN.md section 3a'') plus the SSSP kernel for the sources it
    hands over.  A 20k-query batch property-checked in full (the time of a StandardMove
    run through the Fleetfoot ceil), and every destination of 8 sources x 1 000 against
    the oracle's Dijkstra from each source (mro_sssp_digest_batch)."""
    m, arr = c4_map
    V = m.size * m.size
    keys = ld.cell_keys(arr)
    rng = random.Random(ff)
    params = Params(fleetfoot=ff, sort_by=(SORT_TIME, SORT_MONEY))
    uni = random_queries(m, 20_000, 77 + ff)
    srcs = _sources_of_every_kind(m, rng)[::2]
    cf_cells = [m.cell_of(c) for c in m.campfires()]
    extra_src, extra_dst = [], []
    for s in srcs:
        d = rng.sample(range(V), 1000 - len(cf_cells)) + cf_cells
        extra_src += [m.cell_of(s)] * len(d)
        extra_dst += d
    q_src = np.concatenate([np.array([m.cell_of(a) for a, _ in uni]), np.array(extra_src)])
    q_dst = np.concatenate([np.array([m.cell_of(b) for _, b in uni]), np.array(extra_dst)])
    n = len(q_src)
    g = eng.MapGrid.from_array(arr)
    plan = eng.Plan(g, params, None, max_cmds=8, query_array=m.query_array(q_src, q_dst, arr))
    plan.run()
    res, pool = plan.fetch_raw()
    st = plan.stats()
    assert st["solver"] == "hub" and st["fallback_sources"] <= 8, st
    props = ld.label_properties(res, pool, n, keys[q_src], keys[q_dst], fleetfoot_ratio=FF_RATIO[ff])
    assert all(v == 0 for v in props.values()), props
    got = ld.digests(res, pool, n)
    want = oracle_lib.OracleGrid.from_array(arr).sssp_digests(params, srcs, threads=ORACLE_THREADS)
    off = len(uni)
    for i, s in enumerate(srcs):
        sel = np.arange(off + i * 1000, off + (i + 1) * 1000)
        bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=q_dst[sel])
        assert bad.size == 0, (str(s), len(bad), [str(m.index_at(int(q_dst[sel][j]))) for j in bad[:4]])


# sources the hub hands over, of a 125k Time-first batch on configs[3]'s map, that the
# certificate still leaves to the SSSP kernel: at Fleetfoot 3, sources whose repaired words
# still fail at border-1 cells (a border-1 cell's label is not
# demoted).  A source is emitted from its slot when every label asked of it lies below the
# failing key, so with 1 000 destinations (the forced plan) both such sources need the
# SSSP kernel, and with the batch's few destinations one of them does not.
C4_MAP_SSSP_MAX = {1: 0, 2: 0, 3: 1}
C4_MAP_SSSP_MAX_1000 = {1: 0, 2: 0, 3: 2}


@pytest.mark.parametrize("ff", [1, 2, 3])
def test_c4_map_time_first_handed_over(eng, oracle_lib, c4_map, ff):
    """configs[3]'s own map (seed 4096), a 125k-query Time-first batch at Fleetfoot 1-3
    (tools/r06/ff_c4map.py): the hub hands over tens of sources (42 / 10 / 3).  Per source,
    mr_plan_handed_over_sources says which path answered it (certificate or SSSP kernel),
    consistent with the plan stats, and the certificate must answer all but
    C4_MAP_SSSP_MAX of them.  Every handed-over source's own queries of the batch are
    compared with the oracle, and so are >= 1 000 destinations of each, in a second plan
    that sends every source through a certificate slot (MR_HUB_FALLBACK_ALL): the label of
    every compared cell is the certificate's (or, where it still fails, the SSSP kernel's)."""
    m, arr = c4_map
    V = m.size * m.size
    params = Params(fleetfoot=ff, sort_by=(SORT_TIME, SORT_LEGS))
    src, dst = random_query_cells(m, 125_000, 5001)
    g = eng.MapGrid.from_array(arr)
    plan = eng.Plan(g, params, None, max_cmds=8, query_array=m.query_array(src, dst, arr))
    plan.run()
    plan.run()  # (a second pass: the path a source takes does not change)
    st = plan.stats()
    handed = plan.handed_over_sources()
    assert st["solver"] == "hub" and len(handed) == st["fallback_sources"] > 0, (st, len(handed))
    n_cert = sum(1 for _, c in handed if c)
    assert n_cert == st["certified_sources"], (st, n_cert)
    assert len(handed) - n_cert <= C4_MAP_SSSP_MAX[ff], (ff, [str(s) for s, c in handed if not c])
    sssp = {str(s) for s in plan.fallback_sources()}
    assert sssp == {str(s) for s, c in handed if not c}
    srcs = [s for s, _ in handed]
    og = oracle_lib.OracleGrid.from_array(arr)
    want = og.sssp_digests(params, srcs, threads=ORACLE_THREADS)
    # the batch's own queries of those sources
    res, pool = plan.fetch_raw()
    got = ld.digests(res, pool, len(src))
    for i, s in enumerate(srcs):
        sel = np.flatnonzero(src == m.cell_of(s))
        assert sel.size > 0
        bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=dst[sel])
        assert bad.size == 0, (str(s), len(bad))
    # >= 1 000 destinations each, every source through a certificate slot
    rng = random.Random(ff)
    cf_cells = [m.cell_of(c) for c in m.campfires()]
    q_src, q_dst = [], []
    for s in srcs:
        d = rng.sample(range(V), 1000) + cf_cells
        q_src += [m.cell_of(s)] * len(d)
        q_dst += d
    q_src, q_dst = np.array(q_src, dtype=np.int64), np.array(q_dst, dtype=np.int64)
    os.environ["MR_HUB_FALLBACK_ALL"] = "1"
    try:
        p2 = eng.Plan(g, params, None, max_cmds=8, query_array=m.query_array(q_src, q_dst, arr))
        p2.run()
        st2 = p2.stats()
        h2 = p2.handed_over_sources()
        res2, pool2 = p2.fetch_raw()
    finally:
        os.environ.pop("MR_HUB_FALLBACK_ALL", None)
    assert len(h2) == len(srcs) and st2["certified_sources"] >= len(srcs) - C4_MAP_SSSP_MAX_1000[ff], st2
    got2 = ld.digests(res2, pool2, len(q_src))
    per = 1000 + len(cf_cells)
    for i, s in enumerate(srcs):
        sel = np.arange(i * per, (i + 1) * per)
        bad = ld.mismatches(got2, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=q_dst[sel])
        assert bad.size == 0, (str(s), len(bad), [str(m.index_at(int(q_dst[sel][j]))) for j in bad[:4]])


@pytest.mark.parametrize("ff,sort_by", [(2, (SORT_LEGS, SORT_MONEY)), (1, (SORT_MONEY, SORT_TIME)),
                                        (3, (SORT_TIME, SORT_MONEY)), (1, (SORT_TIME, SORT_LEGS))],
                         ids=["ff2_legs_money", "ff1_money_time", "ff3_time_money", "ff1_time_legs"])
def test_c4_lane_kernel_fleetfoot_vs_oracle(eng, c4_map, ff, sort_by):
    """hub_lane_kernel's Fleetfoot instantiation (DESIGN.md section 3a'') against the
    oracle at configs[3]'s map: 16 sources of every kind x 512 destinations (8 192 labels),
    spread over plans of a 125k-query batch (lane-kernel size) plus at most 32 queries a
    source, so every compared label is the lane kernel's read-off, or, for a source it
    cannot certify, hub_kernel's after the relist (the certificate / SSSP kernel behind
    it).  The plan stats prove every source ran on the lane kernel."""
    import oracle_lib
    oracle_lib.build()
    m, arr = c4_map
    V = m.size * m.size
    params = Params(fleetfoot=ff, sort_by=sort_by)
    uni_src, uni_dst = random_query_cells(m, 125_000, 5000 + ff)
    qarr = m.query_array(uni_src, uni_dst, arr)
    rng = random.Random(77 + ff)
    srcs = _sources_of_every_kind(m, rng)
    cf_cells = [m.cell_of(c) for c in m.campfires()]
    dsts = [np.array(rng.sample(range(V), 512 - len(cf_cells)) + cf_cells, dtype=np.int64) for _ in srcs]
    want = oracle_lib.OracleGrid.from_array(arr).sssp_digests(params, srcs, threads=ORACLE_THREADS)
    cnt = np.bincount(uni_src, minlength=V)
    caps = [32 - int(cnt[m.cell_of(s)]) for s in srcs]
    assert min(caps) >= 16, caps
    n_plans = max(-(-len(d) // c) for d, c in zip(dsts, caps))
    g = eng.MapGrid.from_array(arr)
    nb = len(uni_src)
    compared = 0
    for p in range(n_plans):
        ex_src, ex_dst, owner = [], [], []
        for i, (s, d, c) in enumerate(zip(srcs, dsts, caps)):
            piece = d[p * c:(p + 1) * c]
            ex_src.append(np.full(len(piece), m.cell_of(s), dtype=np.int64))
            ex_dst.append(piece)
            owner.append(np.full(len(piece), i, dtype=np.int64))
        ex_src, ex_dst, owner = np.concatenate(ex_src), np.concatenate(ex_dst), np.concatenate(owner)
        q = np.concatenate([qarr, m.query_array(ex_src, ex_dst, arr)])
        plan = eng.Plan(g, params, None, max_cmds=6, query_array=q)
        plan.run()
        st = plan.stats()
        assert st["solver"] == "hub" and st["lanes_per_source"] == 1, st
        assert st["lane_sources"] == st["num_sources"], st  # (Time first hands over tens of sources here)
        res, pool = plan.fetch_raw()
        got = _tail_digests(res, pool, len(q), nb)
        for i in range(len(srcs)):
            sel = np.nonzero(owner == i)[0]
            if sel.size == 0:
                continue
            bad = ld.mismatches(got, {f: want[f][i] for f in want}, idx_got=sel, idx_exp=ex_dst[sel])
            assert bad.size == 0, (p, str(srcs[i]), len(bad), [str(m.index_at(int(ex_dst[sel][j]))) for j in bad[:4]])
            compared += sel.size
        del plan
    assert compared == sum(len(d) for d in dsts) >= 8_000, compared


@pytest.mark.parametrize("params", [Params(), Params(sort_by=(SORT_TIME, SORT_MONEY), route_guru=2)],
                         ids=["legs_money", "time_money_rg2"])
def test_c3_every_cell_1025(eng, oracle_lib, c4_map, params):
    m, arr = c4_map
    V = m.size * m.size
    rng = random.Random(33)
    srcs = [CellIndex.center(), m.campfires()[5], m.index_at(rng.randrange(V)), CellIndex.border(2, 300)]
    g = eng.MapGrid.from_array(arr)
    plan = eng.SSSPPlan(g, params, srcs)
    plan.run()
    plan.run()
    assert plan.stats()["solver"] == "hub"
    og = oracle_lib.OracleGrid.from_array(arr)
    want = og.sssp_digests(params, srcs, threads=ORACLE_THREADS)
    keys = ld.cell_keys(arr)
    for i, s in enumerate(srcs):
        res, pool, used = plan.labels_raw(i)
        got = ld.digests(res, pool, V, pool_len=used)
        bad = ld.mismatches(got, {f: want[f][i] for f in want})
        assert bad.size == 0, (str(s), len(bad), [str(m.index_at(int(j))) for j in bad[:4]])
        props = ld.label_properties(res, pool, V, np.full(V, keys[m.cell_of(s)]), keys)
        assert all(v == 0 for v in props.values()), props


@pytest.fixture(scope="module")
def c5(eng):
    """bench.py's c5 map and the oracle's answers on it (tests/golden/make_full_scale.py)."""
    with open(C5_FIXTURE) as f:
        fx = json.load(f)
    m = SyntheticMap(**fx["map"])
    arr = m.cells_array()
    return m, arr, eng.MapGrid.from_array(arr), fx


def _labels_of_source(eng, m, arr, g, params, sv, chunk=1 << 21, max_cmds=24):
    """Every cell's label from row-major cell sv through query plans of `chunk`
    destinations (one source, so one wave solves it and reads them all off), as
    label_digest fields over the V cells, plus the batch's property violations.
    max_cmds 24: c5's labels run to 22 commands (Time first), and the plan's
    overflow pool (8 commands per query) would not hold most of them beyond 8 slots
    (MR_ERR_CAPACITY records, the documented behaviour)."""
    V = m.size * m.size
    keys = ld.cell_keys(arr)
    out = {f: [] for f in ld.FIELDS}
    props = {}
    for lo in range(0, V, chunk):
        dst = np.arange(lo, min(V, lo + chunk), dtype=np.int64)
        plan = eng.Plan(g, params, None, max_cmds=max_cmds, query_array=m.query_array(np.full(len(dst), sv), dst, arr))
        plan.run()
        res, pool = plan.fetch_raw()
        assert plan.stats()["solver"] == "hub_wide"
        d = ld.digests(res, pool, len(dst))
        for f in ld.FIELDS:
            out[f].append(d[f])
        for k, v in ld.label_properties(res, pool, len(dst), np.full(len(dst), keys[sv]), keys[dst]).items():
            props[k] = props.get(k, 0) + v
        del plan, res, pool
    return {f: np.concatenate(v) for f, v in out.items()}, props


def test_c5_every_destination_4097(eng, c5):
    """configs[4] at full size: every one of the 16.8 M cells of 3 sources (two orders)
    through the wide hub solver's query path, against the oracle's labels of every
    cell (one checksum per grid row, committed: tests/golden/full_scale/c5.json)."""
    m, arr, g, fx = c5
    assert len(fx["sources"]) >= 3
    for src in fx["sources"]:
        params = Params.from_json(src["params"])
        got, props = _labels_of_source(eng, m, arr, g, params, src["cell"])
        assert props["not_ok"] == 0, (src["spec"], props)
        assert all(v == 0 for v in props.values()), (src["spec"], props)
        rows = ld.row_checksums(got, m.size)
        want = np.array([int(x, 16) for x in src["rows"]], dtype=np.uint64)
        bad = np.nonzero(rows != want)[0]
        assert bad.size == 0, (src["spec"], params.sort_by, f"{bad.size} of {m.size} rows differ", bad[:8].tolist())


def test_c5_full_scale_sample(eng, c5):
    """configs[4]/c5 at full size: S = 4097 (16.8 M cells), 64 clustered campfires per
    homeland (NS = 261), Time first (SURVEY 8d option a) and Money first (option b).
    The wide hub solver answers a 2000-query batch (2000 sources in one launch); 8 of
    them against the oracle's FindPath::eval (committed fixture), and every label of
    the batch against properties that hold at any size."""
    m, arr, g, fx = c5
    keys = ld.cell_keys(arr)
    for run in fx["sample"]:
        params = Params.from_json(run["params"])
        qs = random_queries(m, *run["batch"])
        plan = eng.Plan(g, params, qs)
        plan.run()
        got = plan.fetch()
        assert plan.stats()["solver"] == "hub_wide"
        for i, e in zip(run["index"], run["expected"]):
            assert as_expected(got[i]) == e, (params.sort_by, qs[i])
        res, pool = plan.fetch_raw()
        src = np.array([m.cell_of(a) for a, _ in qs])
        dst = np.array([m.cell_of(b) for _, b in qs])
        props = ld.label_properties(res, pool, len(qs), keys[src], keys[dst])
        assert all(v == 0 for v in props.values()), (params.sort_by, props)
