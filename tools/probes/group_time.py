"""Kernel time of one plan's passes (mr_plan_kernel_ms) under the current environment:
bench.py's c2 batch by default; timing experiments (MR_DBG_FLAGS) do not fetch results.
    python tools/probes/group_time.py [size queries campfires seed]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from marshrutka_amd import pathfinder as eng  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

size, nq, k, seed = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (65, 10000, 4, 2024)))
m = SyntheticMap(size, campfires_per_homeland=k, seed=seed)
g = eng.MapGrid(m.cells())
qs = random_queries(m, nq, seed + 17)
pl = eng.Plan(g, Params(), qs, max_cmds=6)
for _ in range(3):
    pl.run()
pl.stats()  # (a pass without fallback sources is known: later passes are the hub launch alone)
pl.kernel_ms()
for _ in range(20):
    pl.run()
ms, n = pl.kernel_ms()
st = pl.stats()
print(f"S={size} q={nq} flags={os.environ.get('MR_DBG_FLAGS', '0')} group={os.environ.get('MR_HUB_GROUP', '8')} "
      f"lanes/src={st['lanes_per_source']} sources={st['num_sources']} kernel {ms * 1000:.1f} us ({n} passes)", flush=True)
del pl  # (MR_STAMPS builds print their phase cycles when the plan is destroyed)
