"""Generates tests/golden/shard_records.npz on an MI355X: the device records of a
two-rank split of a query batch, each rank's shard solved by its own plan into one
flat buffer laid out as bench.py's N > 1 path lays it out (result records, command
slots, overflow pool; marshrutka_amd/shard.py), the same passes as wire rows
(mr_plan_wire_records, what bench.py gathers), plus the one-rank labels of the
whole batch.  tests/test_shard_dist.py gathers these buffers over gloo and decodes
them with mr_decode_records on the host.  Run: python tests/golden/make_shard_records.py
(a GPU box; the fixture is data, committed)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from golden_util import as_expected  # noqa: E402
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402
from marshrutka_amd.shard import shard_by_source  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shard_records.npz")
WORLD = 2
MAP = dict(size=33, campfires_per_homeland=3, seed=5, clustered=True)
RUNS = [(Params(), 3), (Params(sort_by=(SORT_TIME, SORT_MONEY), route_guru=2), 16)]


def source_key(c):
    return (c.kind << 40) | (c.sub << 32) | (c.x << 16) | c.y


def main():
    m = SyntheticMap(**MAP)
    g = pathfinder.MapGrid(m.cells())
    qs = random_queries(m, 400, 21)
    keys = [source_key(a) for a, _ in qs]
    shards = shard_by_source(keys, WORLD)
    arrays, meta = {}, {"map": MAP, "queries": [[[a.kind, a.sub, a.x, a.y], [b.kind, b.sub, b.x, b.y]] for a, b in qs],
                        "world": WORLD, "shards": shards, "runs": []}
    for j, (params, max_cmds) in enumerate(RUNS):
        counts = [len(s) for s in shards]
        rows = max(counts)
        run = {"params": params.to_json(), "max_cmds": max_cmds, "counts": counts, "orders": []}
        for r in range(WORLD):
            mine = [qs[i] for i in shards[r]]
            plan = pathfinder.Plan(g, params, mine, max_cmds=max_cmds)
            _, rbytes, _, cbytes = plan.device_outputs()
            nq = max(1, len(mine))
            rw, cw = rbytes // nq // 4, cbytes // nq // 4
            ovf_cap = max(1024, rows // 8)
            buf = torch.zeros(rows * (rw + cw) + ovf_cap * 4, dtype=torch.int32, device="cuda")
            p0 = buf.data_ptr()
            plan.bind_outputs(p0, p0 + rows * rw * 4, p0 + rows * (rw + cw) * 4, ovf_cap)
            plan.run()
            plan.wait()
            torch.cuda.synchronize()
            arrays[f"run{j}_rank{r}"] = buf.cpu().numpy()
            # the same pass as wire rows (what bench.py gathers since round 6):
            # mr_plan_wire_records, then the pool of long labels
            wrw = pathfinder.wire_row_words(max_cmds)
            wpool_cap = max(1024, rows // 8)
            wbuf = torch.zeros(rows * wrw + wpool_cap * 2, dtype=torch.int32, device="cuda")
            plan.wire_records(wbuf.data_ptr(), wbuf.data_ptr() + rows * wrw * 4, wpool_cap)
            plan.wait()
            torch.cuda.synchronize()
            arrays[f"run{j}_rank{r}_wire"] = wbuf.cpu().numpy()
            run["orders"].append(plan.record_queries())
            run.update(rows=rows, rw=rw, cw=cw, ovf_cap=ovf_cap, wrw=wrw, wpool_cap=wpool_cap)
        pl = pathfinder.Plan(g, params, qs, max_cmds=16)  # the one-rank run of the whole batch
        pl.run()
        whole = pl.fetch()
        run["expected"] = [as_expected(x) for x in whole]
        meta["runs"].append(run)
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
