"""All destinations of a source through the C ABI: every cell's
label rebuilt from its device record must equal the oracle's FindPath::eval,
for the hub path (fill kernel), sources handed to the SSSP kernel, and the SSSP
kernel alone (non-linear run times)."""
import random

import pytest

from golden_util import as_expected
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


@pytest.fixture(params=["auto", "fallback", "sssp"])
def mode(request, monkeypatch):
    monkeypatch.delenv("MR_ALGO", raising=False)
    monkeypatch.delenv("MR_HUB_FALLBACK_ALL", raising=False)
    if request.param == "fallback":
        monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    if request.param == "sssp":
        monkeypatch.setenv("MR_ALGO", "sssp")
    return request.param


PARAMS = [Params(), Params(sort_by=(SORT_TIME, SORT_MONEY)), Params(sort_by=(SORT_MONEY, SORT_LEGS), use_sfm=True),
          Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_LEGS)), Params(route_guru=3, use_soe=False)]


def all_labels_match(eng, oracle_lib, m, params, sources):
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    plan = eng.SSSPPlan(g, params, sources)
    plan.run()
    for i, s in enumerate(sources):
        exp = og.find_path_batch(params, [(s, d) for d in cells], threads=0)
        rec = plan.records(i)
        pos = {c: j for j, (c, _) in enumerate(m.cells())}
        for d, e in zip(cells, exp):
            got = plan.label(i, d)
            assert as_expected(got) == as_expected(e), (params, s, d)
            r = rec[pos[d]]
            assert (int(r[0]), int(r[1]), int(r[2])) == (e.legs, e.money, e.time_s)


@pytest.mark.parametrize("size,k,clustered", [(9, 2, False), (21, 5, True), (33, 4, False)])
@pytest.mark.parametrize("pi", range(len(PARAMS)))
def test_every_cell_matches_oracle(eng, oracle_lib, mode, size, k, clustered, pi):
    m = SyntheticMap(size, campfires_per_homeland=k, seed=size + pi, clustered=clustered)
    rng = random.Random(size * 10 + pi)
    cells = m.all_indices()
    sources = [CellIndex.center(), m.campfires()[0]] + rng.sample(cells, 2)
    all_labels_match(eng, oracle_lib, m, PARAMS[pi], sources)


def test_repeated_sources_and_reruns(eng, oracle_lib):
    m = SyntheticMap(15, campfires_per_homeland=3, seed=4)
    s = m.all_indices()[7]
    g = eng.MapGrid(m.cells())
    plan = eng.SSSPPlan(g, Params(), [s, s, m.campfires()[1]])
    plan.run()
    a = plan.records(0).copy()
    plan.run()
    plan.run()
    assert (plan.records(1) == a).all() and (plan.records(0) == a).all()
    assert plan.stats()["num_sources"] == 2


def test_c3_sample_1025(eng, oracle_lib):
    """configs[2]/c3: S = 1025, single source -> all 1 050 625 cells; a sample of
    destinations against the oracle (one CPU Dijkstra over 1M cells each)."""
    m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    cells = m.all_indices()
    rng = random.Random(3)
    sources = rng.sample(cells, 2)
    plan = eng.SSSPPlan(g, Params(), sources)
    plan.run()
    for i, s in enumerate(sources):
        dsts = rng.sample(cells, 24) + m.campfires()[:2]
        exp = og.find_path_batch(Params(), [(s, d) for d in dsts], threads=0)
        for d, e in zip(dsts, exp):
            assert as_expected(plan.label(i, d)) == as_expected(e), (s, d)


# Maps wide enough for 64x16 fill tiles away from the axes through the Center (the
# packed-key fast path), with the tile pruning and the key packing each switched off
# in turn (MR_DBG_FLAGS bit 0 / bit 1), and a small fill grid (MR_FILL_GX) so each
# wave walks many tiles and several sources.  Every cell's full label (commands
# included) against the oracle's Dijkstra run to completion.
FILL_PARAMS = [Params(), Params(sort_by=(SORT_TIME, SORT_MONEY)),
               Params(sort_by=(SORT_MONEY, SORT_LEGS), use_sfm=True, route_guru=2),
               Params(sort_by=(SORT_LEGS, SORT_TIME), use_soe=False),
               Params(sort_by=(SORT_TIME, SORT_LEGS), hq_position=CellIndex.homeland(2, 3, 5), fleetfoot=7),
               Params(sort_by=(SORT_MONEY, SORT_TIME), scroll_of_escape_cost=0, homeland=3)]


@pytest.mark.parametrize("flags,gx", [("", None), ("1", None), ("2", None), ("", "3")])
@pytest.mark.parametrize("size,k,clustered,pi", [(129, 4, False, 0), (129, 9, True, 1), (161, 6, False, 2),
                                                  (129, 5, True, 3), (193, 4, False, 4), (161, 7, True, 5)])
def test_fill_tiles_every_cell(eng, oracle_lib, monkeypatch, flags, gx, size, k, clustered, pi):
    monkeypatch.delenv("MR_ALGO", raising=False)
    monkeypatch.delenv("MR_HUB_FALLBACK_ALL", raising=False)
    monkeypatch.setenv("MR_DBG_FLAGS", flags or "0")
    if gx:
        monkeypatch.setenv("MR_FILL_GX", gx)
    else:
        monkeypatch.delenv("MR_FILL_GX", raising=False)
    params = FILL_PARAMS[pi]
    m = SyntheticMap(size, campfires_per_homeland=k, seed=size * 7 + pi, clustered=clustered)
    rng = random.Random(size + pi)
    cells = m.all_indices()
    sources = [m.campfires()[1], CellIndex.center()] + rng.sample(cells, 3)
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    plan = eng.SSSPPlan(g, params, sources)
    plan.run()
    assert plan.stats()["solver"] == "hub"
    for i, s in enumerate(sources):
        exp = og.sssp_all(params, s)
        rec = plan.records(i)
        bad = []
        for j, (d, e) in enumerate(zip(cells, exp)):
            r = rec[j]
            if (int(r[0]), int(r[1]), int(r[2])) != (e.legs, e.money, e.time_s) or \
                    as_expected(plan.label(i, d)) != as_expected(e):
                bad.append(d)
        assert not bad, (params, s, len(bad), bad[:4])


@pytest.mark.parametrize("flags,pi", [("", 0), ("2", 1), ("", 2)])
def test_fill_ragged_last_tile_column(eng, oracle_lib, monkeypatch, flags, pi):
    """S = 2^k + 1 (every BASELINE side): the last tile column of the fill is one cell
    wide, on the packed-key path and (MR_DBG_FLAGS=2) the wide-metric launch.  Every
    cell of 257^2 against the oracle, full labels on the last column."""
    monkeypatch.delenv("MR_ALGO", raising=False)
    monkeypatch.delenv("MR_HUB_FALLBACK_ALL", raising=False)
    monkeypatch.delenv("MR_FILL_GX", raising=False)
    monkeypatch.setenv("MR_DBG_FLAGS", flags or "0")
    params = FILL_PARAMS[pi]
    m = SyntheticMap(257, campfires_per_homeland=4, seed=257 + pi)
    rng = random.Random(pi)
    cells = m.all_indices()
    # a source on the last column, and one anywhere
    from marshrutka_amd.mapgen import index_to_geo
    sources = [rng.choice([c for c in cells if index_to_geo(c)[0] == 128]), rng.choice(cells)]
    g = eng.MapGrid(m.cells())
    og = oracle_lib.OracleGrid(m.cells())
    plan = eng.SSSPPlan(g, params, sources)
    plan.run()
    assert plan.stats()["solver"] == "hub"
    for i, s in enumerate(sources):
        exp = og.sssp_all(params, s)
        rec = plan.records(i)
        bad = [j for j, e in enumerate(exp) if (int(rec[j][0]), int(rec[j][1]), int(rec[j][2])) != (e.legs, e.money, e.time_s)]
        assert not bad, (params, s, len(bad), [cells[j] for j in bad[:4]])
        for j in range(256, len(cells), 257):  # the last column's full labels
            assert as_expected(plan.label(i, cells[j])) == as_expected(exp[j]), (s, cells[j])


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("fb,slots", [(False, 2), (True, 2), (False, 3), (True, 3)])
def test_overlapped_passes_match_serial(eng, oracle_lib, monkeypatch, fb, slots, fused):
    """All-destinations passes take slots of label tables round robin, the specials'
    solve of pass k + 1 running beside the fill of pass k (mr_plan_run): in the same
    launch (fused, the default) or on a stream of the plan's own (MR_FILL_FUSED=0).
    Back-to-back passes (no host sync between them) must leave the records and
    labels of one serial pass (MR_FILL_OVERLAP=0), after every count of passes up to
    a wrap round the slots, with and without sources handed to the SSSP kernel."""
    monkeypatch.setenv("MR_FILL_SLOTS", str(slots))
    monkeypatch.setenv("MR_FILL_FUSED", fused)
    monkeypatch.delenv("MR_ALGO", raising=False)
    monkeypatch.delenv("MR_FILL_GX", raising=False)
    monkeypatch.delenv("MR_DBG_FLAGS", raising=False)
    if fb:
        monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")
    else:
        monkeypatch.delenv("MR_HUB_FALLBACK_ALL", raising=False)
    m = SyntheticMap(129, campfires_per_homeland=5, seed=77)
    rng = random.Random(8)
    cells = m.all_indices()
    sources = [CellIndex.center(), m.campfires()[2]] + rng.sample(cells, 6)
    g = eng.MapGrid(m.cells())
    monkeypatch.setenv("MR_FILL_OVERLAP", "0")
    ref = eng.SSSPPlan(g, Params(), sources)
    ref.run()
    want = [ref.records(i) for i in range(len(sources))]
    assert ref.stats()["fill_launch"] == "serial"
    monkeypatch.delenv("MR_FILL_OVERLAP")
    plan = eng.SSSPPlan(g, Params(), sources)
    assert plan.stats()["solver"] == "hub"
    assert plan.stats()["fill_launch"] == ("fused" if fused == "1" else "streams")
    dsts = rng.sample(cells, 12)
    for passes in (1, 2, 3, 4):
        for _ in range(passes):
            plan.run()
        for i in range(len(sources)):
            assert (plan.records(i) == want[i]).all(), (passes, i)
            for d in dsts[:4]:
                assert as_expected(plan.label(i, d)) == as_expected(ref.label(i, d)), (passes, i, d)


@pytest.mark.parametrize("inject_slot,passes", [(0, 2), (1, 3), (2, 4), (0, 5)])
def test_overlap_error_of_either_slot_is_reported(eng, monkeypatch, inject_slot, passes):
    """A device error flag raised by a pass whose slot is not the current one (an
    earlier overlap slot) must still be reported, then collected."""
    for k in ("MR_ALGO", "MR_FILL_GX", "MR_DBG_FLAGS", "MR_HUB_FALLBACK_ALL", "MR_FILL_OVERLAP", "MR_FILL_FUSED"):
        monkeypatch.delenv(k, raising=False)
    nslots = 3
    monkeypatch.setenv("MR_FILL_SLOTS", str(nslots))
    m = SyntheticMap(33, campfires_per_homeland=3, seed=5)
    sources = m.all_indices()[:4]
    g = eng.MapGrid(m.cells())
    monkeypatch.setenv("MR_DBG_INJECT_SLOT", str(inject_slot))
    plan = eng.SSSPPlan(g, Params(), sources)
    monkeypatch.delenv("MR_DBG_INJECT_SLOT")
    # pass p (1-based) runs in slot (p - 1) % nslots; after `passes` passes the current
    # slot is (passes - 1) % nslots, and the injected slot ran an earlier pass
    assert (passes - 1) % nslots != inject_slot and passes > inject_slot
    for _ in range(passes):
        plan.run()
    with pytest.raises(eng.EngineError):
        plan.records(0)
    # collected: both slots' flags were cleared by the report
    plan.records(0)


@pytest.mark.parametrize("size,mode_env", [(33, None), (65, None), (33, "fallback")])
def test_device_records_padded_rows(eng, monkeypatch, size, mode_env):
    """The device cell words sit in rows padded to mr_sssp_record_pitch cells (a
    multiple of 32: whole 128 B lines): word y * pitch + x of each source is cell (x, y)'s word, and it
    names the same boundary / special / source as the expanded record."""
    import ctypes as C

    import numpy as np
    if mode_env == "fallback":
        monkeypatch.setenv("MR_HUB_FALLBACK_ALL", "1")  # the SSSP kernel's writes
    m = SyntheticMap(size, campfires_per_homeland=3, seed=size)
    g = eng.MapGrid(m.cells())
    cells = m.all_indices()
    sources = [cells[0], cells[len(cells) // 2], cells[-1], cells[size + 3]]
    plan = eng.SSSPPlan(g, Params(), sources)
    plan.run()
    via = [plan.records(i)[:, 3] for i in range(len(sources))]  # (waits for the plan's passes)
    pitch = plan.record_pitch()
    assert pitch % 32 == 0 and size <= pitch < size + 32
    ptr, nbytes = plan.device_records()
    assert nbytes == plan.num_sources * size * pitch * 4
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    words = np.empty(nbytes // 4, dtype=np.uint32)
    assert hip.hipMemcpy(words.ctypes.data, C.c_void_p(ptr), nbytes, 2) == 0
    words = words.reshape(plan.num_sources, size, pitch)[:, :, :size].reshape(plan.num_sources, -1)
    # plan sources are the distinct sources in row-major cell order
    order = sorted(set(range(len(sources))), key=lambda i: cells.index(sources[i]))
    for ps, i in enumerate(order):
        w = words[ps]
        plain = (w & 0x80000000) == 0
        assert np.array_equal(w[plain] >> 20, via[i][plain])
        assert np.array_equal(w[~plain], via[i][~plain])


def test_many_sources_per_pass_match_single_source_plans(eng):
    """More sources in one pass than the fill has wave groups (every cell of a 41x41
    map: 1 681 sources, so groups take several sources one after another): each
    sampled source's records equal those of a plan holding that source alone, and
    every source's own cell holds the source word."""
    import numpy as np
    m = SyntheticMap(41, campfires_per_homeland=4, seed=41)
    g = eng.MapGrid(m.cells())
    cells = m.all_indices()
    plan = eng.SSSPPlan(g, Params(), cells)
    plan.run()
    assert plan.num_sources == len(cells)
    rng = random.Random(3)
    for i in sorted(rng.sample(range(len(cells)), 12)) + [0, len(cells) - 1]:
        one = eng.SSSPPlan(g, Params(), [cells[i]])
        one.run()
        got, exp = plan.records(i), one.records(0)
        assert np.array_equal(got, exp), (i, cells[i])
        assert got[i, 3] == 0xFFFFFFFF


def _hip():
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipStreamDestroy.argtypes = [C.c_void_p]
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    return hip


def _raw_words(hip, ptr, nbytes):
    import ctypes as C

    import numpy as np
    out = np.empty(nbytes // 4, dtype=np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, C.c_void_p(ptr), nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


def test_raw_device_pointers_right_after_run(eng, monkeypatch):
    """The device-output getters wait for the passes enqueued so far (the header's
    contract), so a raw hipMemcpy of the returned pointer, issued right after
    mr_plan_run with no other sync, reads finished words: an all-destinations plan
    whose pass takes a while (512 sources on 257^2) and a query plan."""
    import numpy as np
    for k in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_FILL_GX", "MR_DBG_FLAGS", "MR_FILL_OVERLAP", "MR_FILL_FUSED"):
        monkeypatch.delenv(k, raising=False)
    hip = _hip()
    m = SyntheticMap(257, campfires_per_homeland=4, seed=257)
    g = eng.MapGrid(m.cells())
    cells = m.all_indices()
    sources = random.Random(5).sample(cells, 512)
    ref = eng.SSSPPlan(g, Params(), sources)
    ref.run()
    ref.records(0)  # synced
    ptr, nbytes = ref.device_records()
    want = _raw_words(hip, ptr, nbytes)
    plan = eng.SSSPPlan(g, Params(), sources)
    for passes in (1, 2):
        for _ in range(passes):
            plan.run()
        ptr, nbytes = plan.device_records()  # straight after the runs
        got = _raw_words(hip, ptr, nbytes)
        pitch = plan.record_pitch()
        cols = np.arange(got.size) % pitch < 257  # pad words are unspecified
        assert np.array_equal(got[cols], want[cols]), passes
    qs = [(random.Random(i).choice(cells), random.Random(i + 7).choice(cells)) for i in range(20000)]
    qp = eng.Plan(g, Params(), qs)
    qp.run()
    want_res = [(r.legs, r.money, r.time_s) if r else None for r in qp.fetch()]
    order = qp.record_queries()
    qp.run()
    d_res, rb, _, _ = qp.device_outputs()
    words = _raw_words(hip, d_res, rb).reshape(-1, 4)
    for k in range(0, len(qs), 97):
        q = order[k]
        assert (int(words[k, 0]), int(words[k, 1]), int(words[k, 2])) == want_res[q], k


@pytest.mark.parametrize("mode", ["fused", "streams", "query"])
def test_passes_on_alternating_streams_match_serial(eng, monkeypatch, mode):
    """mr_plan_run on a different stream every pass: passes still run in
    submission order (a pass on a new stream waits for the previous pass), so the
    look-ahead tables, slots and counters they hand over are finished; the records
    equal one serial pass's."""
    import ctypes as C

    import numpy as np
    for k in ("MR_ALGO", "MR_HUB_FALLBACK_ALL", "MR_FILL_GX", "MR_DBG_FLAGS", "MR_FILL_OVERLAP", "MR_FILL_SLOTS"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MR_FILL_FUSED", "0" if mode == "streams" else "1")
    hip = _hip()
    streams = [C.c_void_p(), C.c_void_p()]
    for s in streams:
        assert hip.hipStreamCreate(C.byref(s)) == 0
    try:
        m = SyntheticMap(193, campfires_per_homeland=5, seed=19)
        g = eng.MapGrid(m.cells())
        cells = m.all_indices()
        if mode == "query":
            qs = [(random.Random(i).choice(cells), random.Random(i + 3).choice(cells)) for i in range(30000)]
            ref = eng.Plan(g, Params(), qs)
            ref.run()
            want = np.frombuffer(ref.fetch_raw()[0], dtype=np.uint32).copy()
            plan = eng.Plan(g, Params(), qs)
        else:
            sources = random.Random(6).sample(cells, 256)
            monkeypatch.setenv("MR_FILL_OVERLAP", "0")
            ref = eng.SSSPPlan(g, Params(), sources)
            ref.run()
            want = [ref.records(i) for i in range(0, 256, 17)]
            monkeypatch.delenv("MR_FILL_OVERLAP")
            plan = eng.SSSPPlan(g, Params(), sources)
            assert plan.stats()["fill_launch"] == mode
        for p in range(7):
            plan.run(streams[p % 2].value)
        if mode == "query":
            got = np.frombuffer(plan.fetch_raw()[0], dtype=np.uint32)
            assert np.array_equal(got, want)
        else:
            for j, i in enumerate(range(0, 256, 17)):
                assert np.array_equal(plan.records(i), want[j]), i
        del plan, ref
    finally:
        for s in streams:
            hip.hipStreamSynchronize(s)
            hip.hipStreamDestroy(s)
