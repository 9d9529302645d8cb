"""GPU probe (not product code): the lane kernel against the group kernel (8 / 16 / 32
lanes a source) on c4's map at 125k and 250k queries (the crossover
of the selection rule).  Kernel time of a pass after a first untimed one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_query_cells  # noqa: E402

m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
arr = m.cells_array()
g = pf.MapGrid.from_array(arr)
for nq in (60_000, 125_000, 250_000):
    src, dst = random_query_cells(m, nq, 4096 + 17)
    qa = m.query_array(src, dst, arr)
    row = [f"{nq} queries:"]
    for tag, env in (("lane", {"MR_HUB_LANE": "1"}), ("G8", {"MR_HUB_GROUP_FORCE": "1", "MR_HUB_GROUP": "8"}),
                     ("G16", {"MR_HUB_GROUP_FORCE": "1", "MR_HUB_GROUP": "16"}),
                     ("G32", {"MR_HUB_GROUP_FORCE": "1", "MR_HUB_GROUP": "32"})):
        for k, v in env.items():
            os.environ[k] = v
        plan = pf.Plan(g, Params(), None, max_cmds=6, query_array=qa)
        for k in env:
            del os.environ[k]
        plan.run()
        plan.kernel_ms()
        for _ in range(10):
            plan.run()
        ms, _ = plan.kernel_ms()
        st = plan.stats()
        row.append(f"{tag} {ms * 1e3:.0f} us (sources {st['num_sources']}, lanes/src {st['lanes_per_source']})")
        del plan
    print("  ".join(row), flush=True)
