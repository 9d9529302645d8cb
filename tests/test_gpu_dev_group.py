"""Query batches grouped by source on the device (mr_k_groupq.hip)
against the host grouping of the same batch: the same records in the same order, the
same decoded labels, the same record order and fallback sources, every solver path the
plan picks.  MR_DEV_GROUP=1 groups any batch on the device, =0 none (the default is
device grouping from 32 768 queries).  The labels themselves are checked against the
oracle by the parity suite; here both groupings must agree bit for bit."""
import ctypes as C

import numpy as np
import pytest

from marshrutka_amd.abi import (MR_ERR_INVALID_INDEX, MR_OK, SORT_LEGS, SORT_MONEY, SORT_TIME, CellIndex, Params,
                                mr_query)
from marshrutka_amd.mapgen import SyntheticMap, random_queries, random_query_cells

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


def _run(eng, monkeypatch, dev, g, params, qarr, max_cmds=8, env=()):
    monkeypatch.setenv("MR_DEV_GROUP", "1" if dev else "0")
    for k, v in env:
        monkeypatch.setenv(k, v)
    plan = eng.Plan(g, params, None, max_cmds=max_cmds, query_array=qarr)
    plan.run()
    res, pool = plan.fetch_raw()
    n = len(qarr)
    r = np.frombuffer(res, dtype=np.uint8, count=n * 32).copy()
    ncmd = int(np.frombuffer(res, dtype=np.uint32, count=n * 8).reshape(n, 8)[:, 4].astype(np.int64).sum())
    p = np.frombuffer(pool, dtype=np.uint8, count=ncmd * 40).copy()
    _, rb, _, cb = plan.device_outputs()
    out = {"res": r, "pool": p, "order": plan.record_queries(), "fallback": [str(c) for c in plan.fallback_sources()],
           "stats": plan.stats()}
    return out


def _same(a, b):
    assert np.array_equal(a["res"], b["res"])
    assert np.array_equal(a["pool"], b["pool"])
    assert a["order"] == b["order"]
    assert a["fallback"] == b["fallback"]
    for k in ("solver", "num_sources", "lane_sources", "lanes_per_source", "fallback_sources"):
        assert a["stats"][k] == b["stats"][k], (k, a["stats"][k], b["stats"][k])


def _with_invalid(m, q, every=97):
    """Every `every`-th query gets a CellIndex that is not a grid cell (alternately as
    source and destination)."""
    q = q.copy()
    bad = np.arange(0, len(q), every)
    for j, i in enumerate(bad):
        side = "from" if j % 2 == 0 else "to"
        q[side]["kind"][i] = 1
        q[side]["sub"][i] = 0
        q[side]["x"][i] = m.h + 3  # past the homeland size
        q[side]["y"][i] = 1
    return q, bad


@pytest.mark.parametrize("case", ["c2_group", "lane_forced", "hub_nonlinear", "time_first", "busy_sources"])
def test_device_grouping_matches_host(eng, monkeypatch, case):
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
    arr = m.cells_array()
    g = eng.MapGrid.from_array(arr)
    src, dst = random_query_cells(m, 10_000, 77)
    params, env = Params(), ()
    if case == "lane_forced":
        env = (("MR_HUB_LANE", "1"),)
    elif case == "hub_nonlinear":
        params = Params(fleetfoot=2, sort_by=(SORT_LEGS, SORT_TIME))
    elif case == "time_first":
        params = Params(sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True, route_guru=3)
    elif case == "busy_sources":  # sources with more than 32 queries (the lane kernel's partition)
        src = np.where(np.arange(len(src)) % 5 == 0, src[:7].repeat(len(src) // 7 + 1)[: len(src)], src)
        env = (("MR_HUB_LANE", "1"),)
    q, bad = _with_invalid(m, m.query_array(src, dst, arr))
    a = _run(eng, monkeypatch, True, g, params, q, env=env)
    b = _run(eng, monkeypatch, False, g, params, q, env=env)
    _same(a, b)
    st = np.frombuffer(a["res"].tobytes(), dtype=np.int32).reshape(len(q), 8)[:, 6]
    assert np.all(st[bad] == MR_ERR_INVALID_INDEX) and np.all(np.delete(st, bad) == MR_OK)


def test_device_grouping_edge_batches(eng, monkeypatch):
    """A one-query batch, every query invalid, one source for every query, src == dst."""
    m = SyntheticMap(33, campfires_per_homeland=3, seed=5)
    arr = m.cells_array()
    g = eng.MapGrid.from_array(arr)
    V = m.size * m.size
    batches = [m.query_array(np.array([5]), np.array([700]), arr),
               _with_invalid(m, m.query_array(np.arange(50), np.arange(50) + 1, arr), every=1)[0],
               m.query_array(np.full(3000, 17), np.arange(3000) % V, arr),
               m.query_array(np.arange(V), np.arange(V), arr)]
    for q in batches:
        monkeypatch.delenv("MR_HUB_LANE", raising=False)
        _same(_run(eng, monkeypatch, True, g, Params(), q), _run(eng, monkeypatch, False, g, Params(), q))
        _same(_run(eng, monkeypatch, True, g, Params(), q, env=(("MR_HUB_LANE", "1"),)),
              _run(eng, monkeypatch, False, g, Params(), q, env=(("MR_HUB_LANE", "1"),)))


def test_device_grouping_c4_batch(eng, monkeypatch):
    """configs[3]'s whole 1M batch (the default: grouped on the device) against the host
    grouping of the same batch, and the page-locked input path (mr_host_register)."""
    m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
    arr = m.cells_array()
    g = eng.MapGrid.from_array(arr)
    src, dst = random_query_cells(m, 1_000_000, 4096 + 17)
    q = m.query_array(src, dst, arr)
    monkeypatch.delenv("MR_DEV_GROUP", raising=False)
    plan = eng.Plan(g, Params(), None, max_cmds=6, query_array=q)
    plan.run()
    assert plan.stats()["lanes_per_source"] == 1
    a = _run(eng, monkeypatch, True, g, Params(), q, max_cmds=6)
    b = _run(eng, monkeypatch, False, g, Params(), q, max_cmds=6)
    _same(a, b)
    # the raw queries straight from page-locked caller memory
    buf = (mr_query * len(q)).from_buffer(q)
    eng.pin_host(buf)
    try:
        c = _run(eng, monkeypatch, True, g, Params(), q, max_cmds=6)
    finally:
        eng.unpin_host(buf)
    _same(a, c)


@pytest.mark.parametrize("every", [1, 2])
def test_device_grouping_many_invalid(eng, monkeypatch, every):
    """More than 4 096 invalid queries in a device-grouped batch: the plan
    copies every grouped id back and rebuilds the invalid list on the host
    (group_on_device's long path).  Statuses, records and labels equal the host grouping's."""
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
    arr = m.cells_array()
    g = eng.MapGrid.from_array(arr)
    src, dst = random_query_cells(m, 12_000, 91)
    q, bad = _with_invalid(m, m.query_array(src, dst, arr), every=every)
    assert len(bad) > 4096
    a = _run(eng, monkeypatch, True, g, Params(), q)
    b = _run(eng, monkeypatch, False, g, Params(), q)
    _same(a, b)
    st = np.frombuffer(a["res"].tobytes(), dtype=np.int32).reshape(len(q), 8)[:, 6]
    assert np.all(st[bad] == MR_ERR_INVALID_INDEX) and np.all(np.delete(st, bad) == MR_OK)
