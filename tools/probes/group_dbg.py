"""Diagnostics for hub_group_kernel: the golden fixtures through the group kernel
(MR_HUB_GROUP_FORCE=1) with device flags reported instead of raised, each label against
the fixture; prints the first mismatches with their command lists."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ["MR_HUB_GROUP_FORCE"] = "1"
os.environ["MR_DEBUG_FLAGS_OK"] = "1"
if len(sys.argv) > 2:
    os.environ["MR_HUB_GROUP"] = sys.argv[2]
from golden_util import as_expected, load  # noqa: E402
from marshrutka_amd import pathfinder as eng  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "s15_mixed"
m, queries, runs = load(name)
g = eng.MapGrid(m.cells())
shown = 0
for params, expected in runs:
    pl = eng.Plan(g, params, queries)
    print(params, pl.stats()["lanes_per_source"], flush=True)
    got = eng.FindPath.with_params(g, params).eval_batch(queries)
    bad = [(q, e, as_expected(r)) for q, e, r in zip(queries, expected, got) if as_expected(r) != e]
    print(f"  {len(bad)} / {len(queries)} mismatches", flush=True)
    for q, e, r in bad[:3]:
        if shown < 8:
            print("   query", q, "\n    want", e, "\n    got ", r, flush=True)
            shown += 1
