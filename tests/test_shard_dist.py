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
