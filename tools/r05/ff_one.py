"""GPU probe (not product code): one Fleetfoot configuration of tools/ff_rates.py's batch
(1025^2, 125k queries), a few passes, for a kernel trace of the certified fallback.
usage: python tools/r05/ff_one.py FF SORT1 SORT2 [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_query_cells  # noqa: E402

ff, s1, s2 = (int(x) for x in sys.argv[1:4])
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
m = SyntheticMap(1025, campfires_per_homeland=4, seed=2024)
arr = m.cells_array()
g = pf.MapGrid.from_array(arr)
src, dst = random_query_cells(m, 125000, 7)
plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=(s1, s2)), None, max_cmds=8, query_array=m.query_array(src, dst, arr))
for _ in range(steps):
    plan.run()
plan.fetch_raw()
ms, n = plan.kernel_ms()
st = plan.stats()
print(f"ff={ff} sort=({s1},{s2}) fallback {st['fallback_sources']} certified {st['certified_sources']} pass {ms:.3f} ms")
