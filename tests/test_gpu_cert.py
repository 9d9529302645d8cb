"""The certified fallback on the GPU, through the C ABI.

A hub source whose closed form the hub kernel cannot certify goes to a certificate
slot: the fill writes every cell's closed-form word, the fixed-point check finds the
cells whose word is not the least extension of their neighbours', one sorted sweep
recomputes their box in order of the leading metric, and the check runs again.  Labels
below the least failing leading metric are emitted from the slot; the others go to the
SSSP kernel.

* The two sources the hub hands over at Fleetfoot 1 and 2 with Time first in the
  ff_rates batch (1025^2, seed 2024; found by tools/ff_dump.py on an MI355X).  Their
  closed form is wrong on 5.7k / 75k cells (a band where the ceil makes two
  boundaries' walks alternate); after the sweep every label is the reference's.
  2000 destinations each (plus every campfire and the handed-over query) against the
  oracle's Dijkstra from the source, with the certificate answering the source.
* Every source handed over (MR_HUB_FALLBACK_ALL) with 64 slots a pass, small maps,
  every order and Fleetfoot level, against the oracle's single-query eval; and the
  same with the certificate off (every source on the SSSP kernel).
"""
import random

import numpy as np
import pytest

import label_digest as ld
from golden_util import as_expected
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap, random_queries

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16
FF_RATIO = {1: (50, 53), 2: (100, 109), 3: (25, 28)}
# (Fleetfoot, handed-over source, its query's destination) in the ff_rates.py batch
FLAGGED = {1: (CellIndex(1, 3, 361, 241), CellIndex(1, 0, 408, 426)),
           2: (CellIndex(1, 0, 402, 209), CellIndex(1, 1, 221, 482))}


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


@pytest.fixture(autouse=True)
def clean_env(monkeypatch):
    for v in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_HUB_SPW", "MR_HUB_WIDE", "MR_HUB_NONLIN", "MR_GRID_STATE",
              "MR_CERT", "MR_CERT_SLOTS", "MR_HUB_LANE"):
        monkeypatch.delenv(v, raising=False)


@pytest.fixture(scope="module")
def ff_map():
    m = SyntheticMap(1025, campfires_per_homeland=4, seed=2024)  # tools/ff_rates.py
    return m, m.cells_array()


@pytest.mark.parametrize("ff", [1, 2])
@pytest.mark.parametrize("sort_by", [(SORT_TIME, SORT_LEGS), (SORT_TIME, SORT_MONEY)], ids=["time_legs", "time_money"])
def test_flagged_source_certified_1025(eng, oracle_lib, ff_map, ff, sort_by):
    m, arr = ff_map
    V = m.size * m.size
    src, dst = FLAGGED[ff]
    rng = random.Random(ff)
    d = rng.sample(range(V), 2000) + [m.cell_of(c) for c in m.campfires()] + [m.cell_of(dst)]
    q_src = np.full(len(d), m.cell_of(src), dtype=np.int64)
    q_dst = np.array(d, dtype=np.int64)
    params = Params(fleetfoot=ff, sort_by=sort_by)
    g = eng.MapGrid.from_array(arr)
    plan = eng.Plan(g, params, None, max_cmds=8, query_array=m.query_array(q_src, q_dst, arr))
    plan.run()
    res, pool = plan.fetch_raw()
    st = plan.stats()
    assert st["solver"] == "hub" and st["fallback_sources"] == 1, st
    assert st["certified_sources"] == 1, st  # the sweep repaired the closed form: no SSSP solve
    keys = ld.cell_keys(arr)
    props = ld.label_properties(res, pool, len(d), keys[q_src], keys[q_dst], fleetfoot_ratio=FF_RATIO[ff])
    assert all(v == 0 for v in props.values()), props
    got = ld.digests(res, pool, len(d))
    want = oracle_lib.OracleGrid.from_array(arr).sssp_digests(params, [src], threads=ORACLE_THREADS)
    bad = ld.mismatches(got, {f: want[f][0] for f in want}, idx_exp=q_dst)
    assert bad.size == 0, (len(bad), [str(m.index_at(int(q_dst[j]))) for j in bad[:4]])


@pytest.mark.parametrize("cert", ["slots64", "off"])
@pytest.mark.parametrize("size,k,seed", [(33, 3, 5), (65, 4, 2024), (41, 9, 8)])
def test_every_source_handed_over(eng, oracle_lib, monkeypatch, cert, size, k, seed):
    monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    if cert == "off":
        monkeypatch.setenv("MR_CERT", "0")
    else:
        monkeypatch.setenv("MR_CERT_SLOTS", "64")
    m = SyntheticMap(size, campfires_per_homeland=k, seed=seed)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    qs = random_queries(m, 300, seed + 1)
    # a few sources with many destinations (hub_kernel's one lane per query)
    for s in (CellIndex.center(), m.campfires()[0], m.index_at(7)):
        qs += [(s, m.index_at(i)) for i in random.Random(seed).sample(range(size * size), 40)]
    for ff in (0, 1, 2, 3):
        for sort_by in ((SORT_LEGS, SORT_MONEY), (SORT_TIME, SORT_LEGS), (SORT_MONEY, SORT_TIME), (SORT_TIME, SORT_MONEY)):
            params = Params(fleetfoot=ff, sort_by=sort_by)
            plan = eng.Plan(g, params, qs)
            plan.run()
            got = plan.fetch()
            st = plan.stats()
            exp = og.find_path_batch(params, qs, threads=0)
            bad = [(q, e, r) for q, e, r in zip(qs, exp, got) if as_expected(e) != as_expected(r)]
            assert not bad, (ff, sort_by, len(bad), bad[0])
            if st["solver"] == "hub":
                assert st["fallback_sources"] == st["num_sources"], st
                if cert == "off":
                    assert st["certified_sources"] == 0, st
                else:  # slots for the first 64 a pass; a few may still need the SSSP kernel
                    assert st["certified_sources"] >= min(64, st["num_sources"]) // 2, st


def test_more_fallbacks_than_the_staging(eng, oracle_lib, monkeypatch):
    """A pass that hands over more sources than the certificate's staging holds (4 096
    entries, kCertStageMax) gives no slots at all: which entries were staged would depend
    on arrival order, so every handed-over source goes to the SSSP kernel instead
    (the throughput cliff).  Every source of the 65^2
    map (4 225 > 4 096) handed over; the labels are still the oracle's."""
    monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    monkeypatch.setenv("MR_CERT_SLOTS", "64")
    monkeypatch.delenv("MR_CERT", raising=False)
    m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
    V = m.size * m.size
    rng = random.Random(65)
    qs = [(m.index_at(v), m.index_at(rng.randrange(V))) for v in range(V)]
    g = eng.MapGrid(m.cells())
    params = Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY))
    plan = eng.Plan(g, params, qs)
    plan.run()
    got = plan.fetch()
    st = plan.stats()
    assert st["solver"] == "hub" and st["num_sources"] == V > 4096, st
    assert st["fallback_sources"] == V and st["certified_sources"] == 0, st
    sample = rng.sample(range(V), 400)
    exp = oracle_lib.OracleGrid(m.cells()).find_path_batch(params, [qs[i] for i in sample], threads=0)
    bad = [(qs[i], e, got[i]) for i, e in zip(sample, exp) if as_expected(e) != as_expected(got[i])]
    assert not bad, (len(bad), bad[0])
