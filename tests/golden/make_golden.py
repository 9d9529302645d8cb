"""Generates tests/golden/*.json — golden (inputs, expected outputs) vectors.

Expected outputs come from oracle/py_ref.py, the independent pure-Python
restatement of the reference pathfinder (the Rust reference itself cannot be
built or run here).  tests/test_golden.py then checks the C++
oracle against these files, and tests/test_gpu_parity.py checks the HIP engine.

Run from the repo root:  python tests/golden/make_golden.py
"""
import itertools
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import py_ref  # noqa: E402
from marshrutka_amd.abi import (BLUE, GREEN, RED, SORT_LEGS, SORT_MONEY, SORT_TIME,  # noqa: E402
                                YELLOW, CellIndex, Params)
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402


def t4(c):
    return [c.kind, c.sub, c.x, c.y]


def case(name, m, params_list, nq, qseed):
    cells = m.cells()
    pg = py_ref.Grid([((c.kind, c.sub, c.x, c.y), p) for c, p in cells])
    qs = random_queries(m, nq, qseed)
    runs = []
    for p in params_list:
        f = py_ref.Finder(pg, p.to_json())
        exp = []
        for a, b in qs:
            lab = f.eval((a.kind, a.sub, a.x, a.y), (b.kind, b.sub, b.x, b.y))
            j = py_ref.label_to_json(lab)
            if j is None:
                exp.append(None)
            else:
                exp.append([j["legs"], j["money"], j["time_s"],
                            [[c["kind"], c["time_s"], c["legs"], c["money"], c["fleetfoot"],
                              c["from"], c["to"]] for c in j["commands"]]])
        runs.append({"params": p.to_json(), "expected": exp})
    return {"name": name, "map": m.to_json(), "queries": [[t4(a), t4(b)] for a, b in qs],
            "runs": runs}


def main():
    out = []
    # 1) every sort_by pair (9 inputs -> 6 orders, src/cost.rs:387-405) on a small map
    m5 = SyntheticMap(5, campfires_per_homeland=1, seed=11)
    sorts = [Params(sort_by=s) for s in itertools.product((SORT_LEGS, SORT_TIME, SORT_MONEY), repeat=2)]
    out.append(case("s5_all_sorts", m5, sorts, 120, 1))
    # 2) skills (in and out of range), toggles, HQ, homelands, zero-cost scrolls
    m9 = SyntheticMap(9, campfires_per_homeland=2, seed=5)
    variants = [
        Params(),
        Params(fleetfoot=1), Params(fleetfoot=2), Params(fleetfoot=3), Params(fleetfoot=7),
        Params(route_guru=1), Params(route_guru=3), Params(route_guru=5), Params(route_guru=9),
        Params(use_soe=False), Params(use_caravans=False), Params(use_sfm=True),
        Params(use_soe=False, use_caravans=False, use_sfm=True),
        Params(hq_position=CellIndex.homeland(RED, 3, 2)),
        Params(hq_position=CellIndex.center(), use_sfm=True),
        Params(homeland=RED), Params(homeland=GREEN), Params(homeland=YELLOW),
        Params(scroll_of_escape_cost=0), Params(scroll_of_escape_cost=0, scroll_of_escape_hq_cost=0,
                                                scroll_of_escape_forum_cost=0, use_sfm=True,
                                                hq_position=CellIndex.homeland(GREEN, 4, 4)),
        Params(sort_by=(SORT_TIME, SORT_MONEY), fleetfoot=3, route_guru=2),
        Params(sort_by=(SORT_MONEY, SORT_TIME), fleetfoot=1, use_sfm=True),
        Params(sort_by=(SORT_TIME, SORT_LEGS), fleetfoot=2, hq_position=CellIndex.homeland(BLUE, 1, 4)),
        Params(sort_by=(SORT_MONEY, SORT_LEGS), scroll_of_escape_cost=0, homeland=YELLOW),
    ]
    out.append(case("s9_variants", m9, variants, 60, 2))
    # 3) a mid-size map with several campfires per homeland
    m15 = SyntheticMap(15, campfires_per_homeland=3, seed=7)
    out.append(case("s15_mixed", m15, [Params(), Params(fleetfoot=3, route_guru=4),
                                       Params(sort_by=(SORT_TIME, SORT_TIME), fleetfoot=1),
                                       Params(sort_by=(SORT_MONEY, SORT_MONEY), use_sfm=True,
                                              scroll_of_escape_cost=0)], 150, 3))
    # 4) clustered campfires (the c5 "skew" map family) at small scale
    m21 = SyntheticMap(21, campfires_per_homeland=5, seed=9, clustered=True)
    out.append(case("s21_clustered", m21, [Params(), Params(fleetfoot=2),
                                           Params(sort_by=(SORT_TIME, SORT_MONEY))], 100, 4))
    for c in out:
        path = os.path.join(HERE, f"{c['name']}.json")
        with open(path, "w") as f:
            json.dump(c, f, separators=(",", ":"))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
