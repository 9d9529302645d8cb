"""GPU probe: the ff2 / max_cmds=1 batch of plan_diff.py under the certificate off, 64
slots and the default, three plans each; query 1084 against the oracle's label.  Not
product code."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, CellIndex, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

m = SyntheticMap(65, campfires_per_homeland=5, seed=11)
g = pf.MapGrid(m.cells())
qs = random_queries(m, 3000, 12)
qs[5] = (CellIndex(1, 0, 999, 999), qs[5][1])
qs[77] = (qs[77][0], CellIndex(2, 1, 999, 0))
params = Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True)
src = qs[1084][0]
for mode in ("off", "64", "default", "default", "off"):
    os.environ.pop("MR_CERT", None)
    os.environ.pop("MR_CERT_SLOTS", None)
    if mode == "off":
        os.environ["MR_CERT"] = "0"
    elif mode == "64":
        os.environ["MR_CERT_SLOTS"] = "64"
    for mc in (1, 16):
        plan = pf.Plan(g, params, qs, max_cmds=mc)
        plan.run()
        got = plan.fetch()
        fb = plan.fallback_sources()
        st = plan.stats()
        lab = got[1084]
        print(mode, "mc", mc, "label", (lab.legs, lab.money, lab.time_s, len(lab.commands)), "src handed over",
              src in fb, "certified", st["certified_sources"], "of", st["fallback_sources"], flush=True)
        del plan
