"""Histogram of label lengths (commands per result) over a bench workload's batch: how
many command slots the records need (bench.py max_cmds; the N > 1 gather moves them)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_query_cells  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c4"
wl = bench.WORKLOADS[w]
m = SyntheticMap(wl["size"], campfires_per_homeland=wl["campfires"], seed=wl["seed"], clustered=wl.get("clustered", False))
g = pathfinder.MapGrid(m.cells())
n = wl.get("queries_total", wl.get("queries_per_gpu"))
q_src, q_dst = random_query_cells(m, n, wl["seed"] + 17)
qa = m.query_array(q_src, q_dst, m.cells_array())
params = Params(sort_by=wl["sort"]) if "sort" in wl else Params()
plan = pathfinder.Plan(g, params, None, max_cmds=16, query_array=qa)
plan.run()
res, _ = plan.fetch_raw()
words = np.frombuffer(res, dtype=np.uint32).reshape(-1, 8)[: plan.n]
ncmd = words[:, 4].astype(np.int64)
print(w, "queries", plan.n, "max commands", int(ncmd.max()), "histogram", np.bincount(ncmd).tolist(), flush=True)
