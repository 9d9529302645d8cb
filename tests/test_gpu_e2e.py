"""The path end to end on the GPU: the reference's HTML map (MapGrid::parse,
src/grid.rs:47-237) -> mr_grid_from_html -> the device solve (FindPath::eval,
src/pathfinder.rs:199-248) -> the app's command table (src/app.rs:481-561,
src/index.rs:378-390) through mr_render_schedule.

The oracle grid is built from the cells the same HTML parses to, so parse, grid
construction (nearest campfires, regions), solve and rendering are all exercised
on one input; every label is compared with the oracle's and every rendered table
with the test-side restatement (oracle/py_ref.py) of the oracle's label."""
import random

import pytest

import py_ref
from golden_util import as_expected
from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap, random_queries, to_html

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


def _messy(html: str) -> str:
    """The same map as a browser-saved page would carry it: a doctype, comments, a
    script, other classes on the grid, single-quoted and reordered attributes, a
    variation selector on the fountain."""
    html = html.replace('<div class="map-grid">',
                        '<!DOCTYPE html><head><script>var s = "<div class=\\"map-cell\\">";</script></head>'
                        '<!-- <div class="map-grid"> --><DIV id="g" CLASS="map map-grid">', 1)
    html = html.replace('<div class="map-cell" style="background-color:#cccccc">',
                        "<div style='background-color: #CCCCCC' class='map-cell'>")
    return html.replace("⛲", "⛲️")


def _label_json(label):
    return {"commands": [{"kind": c.kind, "time_s": c.time_s, "legs": c.legs, "money": c.money,
                          "fleetfoot": c.fleetfoot, "from": [c.from_.kind, c.from_.sub, c.from_.x, c.from_.y],
                          "to": [c.to.kind, c.to.sub, c.to.x, c.to.y]} for c in label.commands]}


@pytest.mark.parametrize("size,k,clustered,params", [
    (33, 4, False, Params()),
    (65, 6, True, Params(sort_by=(SORT_TIME, SORT_MONEY), fleetfoot=2, route_guru=3)),
    (129, 4, False, Params(sort_by=(SORT_MONEY, SORT_TIME), use_sfm=True, homeland=2)),
], ids=["s33-default", "s65-time-ff2", "s129-money-sfm"])
def test_html_to_gpu_to_render(eng, oracle_lib, size, k, clustered, params):
    m = SyntheticMap(size, campfires_per_homeland=k, seed=size + k, clustered=clustered, fountains=3, forums=2)
    html = _messy(to_html(m))
    cells = eng.parse_map_html(html)
    assert cells == list(m.cells())
    g = eng.MapGrid.from_html(html)  # mr_grid_from_html: parse + grid in one call
    og = oracle_lib.OracleGrid(cells)
    if params.homeland == 2:
        params = Params(**{**params.__dict__, "hq_position": m.campfires()[1]})
    rng = random.Random(size)
    qs = random_queries(m, 300, size) + [(CellIndex.center(), c) for c in m.campfires()[:4]]
    qs += [(rng.choice(m.campfires()), rng.choice(m.all_indices())) for _ in range(20)]
    got = eng.FindPath.with_params(g, params).eval_batch(qs)
    exp = og.find_path_batch(params, qs, threads=0)
    bad = [(q, e, r) for q, e, r in zip(qs, exp, got) if as_expected(e) != as_expected(r)]
    assert not bad, f"{len(bad)}/{len(qs)} labels differ; first {bad[0]}"
    for q, lab in zip(qs, got):
        for arrive, pause in ((9 * 3600, 0), (125, 3)):  # the second wraps past midnight
            rows = eng.render_schedule(lab, arrive, pause)
            assert rows == py_ref.render_schedule(_label_json(lab), arrive, pause), q
            assert len(rows) == sum(1 for c in lab.commands if c.kind != 0)
    # the single-query entry point the app calls (update_path, src/app.rs:704-731)
    a, b = qs[7]
    one = eng.FindPath.with_params(g, params).eval(a, b)
    assert as_expected(one) == as_expected(exp[7])
