"""GPU probe (not product code): a 125k Time-first batch on c4's own map (seed 4096) at
Fleetfoot 1-3: handed-over, certified and SSSP-solved sources and the pass rate.
usage: python tools/r06/ff_c4map.py [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_query_cells  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
m = SyntheticMap(1025, campfires_per_homeland=4, seed=seed)
arr = m.cells_array()
g = pf.MapGrid.from_array(arr)
src, dst = random_query_cells(m, 125000, 5001)
for ff in (1, 2, 3):
    for sort in ((1, 0), (1, 2)):
        plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=sort), None, max_cmds=8, query_array=m.query_array(src, dst, arr))
        plan.run()
        plan.kernel_ms()
        for _ in range(3):
            plan.run()
        ms, _ = plan.kernel_ms()
        st = plan.stats()
        print(f"seed {seed} ff={ff} sort={sort}: handed over {st['fallback_sources']} certified {st['certified_sources']} "
              f"SSSP {st['fallback_sources'] - st['certified_sources']}  pass {ms:.2f} ms  {125000 / ms / 1e3:.1f} M q/s",
              flush=True)
