"""GPU probe: two plans of the same batch, one after the other (the second reuses the
first's cached device blocks), compared record by record.  Not product code."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, CellIndex, Params, mr_command, mr_result  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402
from label_digest import RESULT_DT  # noqa: E402

m = SyntheticMap(65, campfires_per_homeland=5, seed=11)
g = pf.MapGrid(m.cells())
qs = random_queries(m, 3000, 12)
qs[5] = (CellIndex(1, 0, 999, 999), qs[5][1])
qs[77] = (qs[77][0], CellIndex(2, 1, 999, 0))
os.environ["MR_HOST_DECODE"] = "1"
for mc in (1, 3, 16):
    for params in (Params(), Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True)):
        outs = []
        for rep in range(3):
            plan = pf.Plan(g, params, qs, max_cmds=mc)
            plan.run()
            cap = len(qs) * 24
            res = (mr_result * len(qs))()
            pool = (mr_command * cap)()
            st = pf.lib().mr_plan_fetch(plan.handle, res, pool, cap)
            outs.append((st, np.frombuffer(bytes(res), dtype=RESULT_DT), bytes(pool), plan.stats()))
            del plan
        for rep in (1, 2):
            bad = np.flatnonzero(outs[0][1] != outs[rep][1])
            print("mc", mc, "ff", params.fleetfoot, "rep", rep, "status", outs[0][0], outs[rep][0], "bad", len(bad),
                  "pool equal", outs[0][2] == outs[rep][2], flush=True)
            for i in bad[:3]:
                print("  q", i, qs[i], outs[0][1][i], outs[rep][1][i], flush=True)
        print("  stats", {k: outs[0][3][k] for k in ("solver", "fallback_sources", "certified_sources", "num_sources")}, flush=True)
