"""The N>1 path on CPU: world_size-2 gloo processes shard a batch by source
and gather fixed-size result rows to rank 0 (the RCCL gather of bench.py)."""
import os
import socket

import pytest

from marshrutka_amd.mapgen import SyntheticMap, random_queries
from marshrutka_amd.shard import shard_by_source


def test_shard_by_source_partitions_and_balances():
    m = SyntheticMap(33, campfires_per_homeland=2, seed=1)
    qs = random_queries(m, 5000, 3)
    keys = [hash((a.kind, a.sub, a.x, a.y)) for a, _ in qs]
    for world in (1, 2, 3, 8):
        shards = shard_by_source(keys, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(qs)))
        # every source lives on exactly one rank
        owner = {}
        for r, s in enumerate(shards):
            for i in s:
                assert owner.setdefault(keys[i], r) == r
        sizes = [len(s) for s in shards]
        assert max(sizes) - min(sizes) <= max(8, len(qs) // 100)
    assert shard_by_source(keys, 4) == shard_by_source(keys, 4)  # deterministic


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, ret):
    import torch
    import torch.distributed as dist
    from marshrutka_amd.shard import gather_rows_to_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts = [3, 5]
        local = torch.full((5, 4), -1, dtype=torch.int32)
        local[: counts[rank]] = torch.arange(counts[rank] * 4, dtype=torch.int32).view(-1, 4) + 100 * rank
        out = gather_rows_to_root(local, counts, rank, world)
        if rank == 0:
            ret.put(out.tolist())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gather_rows_to_root_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ret)) for r in range(2)]
    for p in procs:
        p.start()
    out = ret.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(out) == 8
    assert out[0] == [0, 1, 2, 3] and out[3] == [100, 101, 102, 103]
    assert out[-1] == [116, 117, 118, 119]


def _pipe_worker(rank, world, port, ret):
    import torch
    import torch.distributed as dist
    from marshrutka_amd.shard import PipelinedGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts, rw = [2, 3], 4
        bufs = [torch.full((3 * rw + 6,), -1, dtype=torch.int32) for _ in range(2)]
        pg = PipelinedGather(bufs, rank, world)
        seen = []
        for step in range(5):
            k = step % 2
            pg.reuse(k)
            if rank == 0 and step >= 2:
                seen.append([r.tolist() for r in pg.rows(k, counts, rw)])
            b = bufs[k]
            b.fill_(-1)
            b[: counts[rank] * rw] = torch.arange(counts[rank] * rw, dtype=torch.int32) + 1000 * step + 100 * rank
            pg.issue(k)
        pg.drain()
        if rank == 0:
            seen.append([r.tolist() for r in pg.rows(1, counts, rw)])
            seen.append([r.tolist() for r in pg.rows(0, counts, rw)])
            ret.put(seen)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_pipelined_gather_gloo_world2():
    """Double-buffered gathers: every batch's rows arrive intact at rank 0 even
    though a buffer is rewritten two steps later."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, ret)) for r in range(2)]
    for p in procs:
        p.start()
    seen = ret.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # batches 0, 1, 2 read back before reuse, then 3 and 4 after the drain
    for step, got in zip([0, 1, 2, 3, 4], seen):
        assert got[0] == [[1000 * step + j * 4 + c for c in range(4)] for j in range(2)]
        assert got[1] == [[1000 * step + 100 + j * 4 + c for c in range(4)] for j in range(3)]


def test_cost_aware_lpt_spreads_fallback_sources():
    """SourceCosts: the sources a pass re-solved with the SSSP kernel are dealt out
    first, one per rank, and the hub work goes to the other ranks."""
    from marshrutka_amd.shard import SourceCosts
    keys = [i % 50 for i in range(1000)]
    costs = SourceCosts()
    costs.observe([3, 7])
    shards = shard_by_source(keys, 4, costs())
    owner = {keys[i]: r for r, s in enumerate(shards) for i in s}
    assert owner[3] != owner[7]
    heavy = {owner[3], owner[7]}
    for r, s in enumerate(shards):
        if r in heavy:  # only the fallback source's own queries
            assert {keys[i] for i in s} <= {3, 7}
    light = [len(s) for r, s in enumerate(shards) if r not in heavy]
    assert max(light) - min(light) <= 20 and sum(light) == 960
    assert shard_by_source(keys, 4) == shard_by_source(keys, 4, {})  # no costs: the query-count LPT


FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "shard_records.npz")


def _records_worker(rank, world, port, ret, wire=False):
    import json
    import numpy as np
    import torch.distributed as dist
    import torch
    from golden_util import as_expected
    from marshrutka_amd import pathfinder
    from marshrutka_amd.abi import Params
    from marshrutka_amd.mapgen import SyntheticMap
    from marshrutka_amd.shard import PipelinedGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(FIX)
        meta = json.loads(str(z["meta"]))
        summary = []
        for j, run in enumerate(meta["runs"]):
            key = f"run{j}_rank{rank}" + ("_wire" if wire else "")
            pg = PipelinedGather([torch.from_numpy(z[key].copy())], rank, world, host_staging=True)
            pg.issue(0)
            pg.drain()
            if rank != 0:
                continue
            m = SyntheticMap(**meta["map"])
            g = pathfinder.MapGrid(m.cells())
            params = Params.from_json(run["params"])
            rows, rw, cw, ovf_cap = run["rows"], run["rw"], run["cw"], run["ovf_cap"]
            got = [None] * len(meta["queries"])
            covered = 0
            for r, buf in enumerate(pg.out[0]):
                words = buf.numpy().view(np.uint32)
                n = run["counts"][r]
                if wire:
                    wrw = run["wrw"]
                    out, cmds = pathfinder.decode_wire_raw(g, params, words[: n * wrw], n, run["max_cmds"],
                                                           words[rows * wrw: rows * wrw + run["wpool_cap"] * 2])
                    labs = [None if out[k].status == 1 else pathfinder.result_from_c(out[k], cmds) for k in range(n)]
                    assert all(out[k].status in (0, 1) for k in range(n))
                else:
                    res = words[: n * rw]
                    slots = words[rows * rw: rows * rw + n * cw]
                    ovf = words[rows * (rw + cw): rows * (rw + cw) + ovf_cap * 4]
                    labs = pathfinder.decode_records(g, params, res, slots, n, cw // 4, ovf)
                for k, lab in enumerate(labs):
                    q = meta["shards"][r][run["orders"][r][k]]
                    got[q] = as_expected(lab)
                    covered += 1
            bad = sum(1 for a, b in zip(got, run["expected"]) if a != b)
            summary.append((covered, bad))
        if rank == 0:
            ret.put(summary)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_engine_records_gather_gloo_world2():
    """The N > 1 result path with real engine output: each rank's buffer holds the
    device records of its shard as its own plan wrote them on an MI355X (fixture:
    tests/golden/make_shard_records.py, bench.py's buffer layout: records, command
    slots, overflow pool); rank 0 gathers both over gloo (PipelinedGather), decodes
    them on the host (mr_decode_records) and maps record k of rank r back to its
    query.  Every label equals the one-rank run of the whole batch, including labels
    longer than the 3 command slots (overflow pool)."""
    import torch.multiprocessing as mp
    assert os.path.exists(FIX), "tests/golden/shard_records.npz (make_shard_records.py on a GPU box)"
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_records_worker, args=(r, 2, port, ret)) for r in range(2)]
    for p in procs:
        p.start()
    summary = ret.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(summary) == 2
    for covered, bad in summary:
        assert covered == 400 and bad == 0, summary


def test_engine_wire_gather_gloo_world2():
    """The same with the wire rows bench.py gathers (mr_plan_wire_records on the MI355X:
    4 + 8 max_cmds bytes a query, then the pool of long labels), decoded on rank 0 by
    mr_decode_wire: every label equals the one-rank run, labels longer than 3 commands
    (wire pool) included."""
    import numpy as np
    import torch.multiprocessing as mp
    assert "run0_rank0_wire" in np.load(FIX).files, "regenerate tests/golden/shard_records.npz"
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_records_worker, args=(r, 2, port, ret, True)) for r in range(2)]
    for p in procs:
        p.start()
    summary = ret.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(summary) == 2
    for covered, bad in summary:
        assert covered == 400 and bad == 0, summary


def _lpt_heap(src_keys, world, extra_cost=None):
    """The plain LPT (a heap of rank loads, source by source) that shard_by_source vectorises."""
    import heapq
    groups = {}
    for i, s in enumerate(src_keys):
        groups.setdefault(s, []).append(i)
    extra = extra_cost or {}
    cost = {k: len(v) + float(extra.get(k, 0.0)) for k, v in groups.items()}
    heap = [(0.0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for key, idxs in sorted(groups.items(), key=lambda kv: (-cost[kv[0]], kv[0])):
        load, r = heapq.heappop(heap)
        out[r].extend(idxs)
        heapq.heappush(heap, (load + cost[key], r))
    return [sorted(o) for o in out]


def test_shard_by_source_equals_heap_lpt():
    import random
    rng = random.Random(5)
    for trial in range(40):
        world = rng.choice([1, 2, 3, 4, 7, 8])
        n = rng.choice([0, 1, 5, 100, 3000])
        keys = [rng.randrange(max(1, n // rng.choice([1, 2, 5]))) for _ in range(n)]
        extra = {k: rng.choice([1e7, 3.0, 250.0]) for k in rng.sample(sorted(set(keys)), min(len(set(keys)), 3))}
        for ex in (None, extra):
            assert shard_by_source(keys, world, ex) == _lpt_heap(keys, world, ex), (trial, world, n)


def test_shard_by_source_1m_is_fast():
    import time
    import numpy as np
    keys = np.random.default_rng(1).integers(0, 1_050_625, 1_000_000)
    t0 = time.perf_counter()
    shards = shard_by_source(keys, 8)
    assert time.perf_counter() - t0 < 5.0
    assert sum(len(s) for s in shards) == 1_000_000
