"""GPU probe: device vs host decode of one plan's records, first differences.  Not
product code."""
import ctypes as C
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
for params in (Params(), Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_MONEY), use_sfm=True)):
    plan = pf.Plan(g, params, qs, max_cmds=1)
    plan.run()
    out = {}
    for mode in ("device", "host"):
        if mode == "host":
            os.environ["MR_HOST_DECODE"] = "1"
        else:
            os.environ.pop("MR_HOST_DECODE", None)
        cap = len(qs) * 24
        res = (mr_result * len(qs))()
        pool = (mr_command * cap)()
        st = pf.lib().mr_plan_fetch(plan.handle, res, pool, cap)
        out[mode] = (st, np.frombuffer(bytes(res), dtype=RESULT_DT), bytes(pool))
    d, h = out["device"], out["host"]
    bad = np.flatnonzero(d[1] != h[1])
    print("params", params.fleetfoot, "status", d[0], h[0], "bad results", len(bad), flush=True)
    for i in bad[:5]:
        print(" q", i, "dev", d[1][i], "host", h[1][i], flush=True)
    print(" pool equal", d[2] == h[2], flush=True)
