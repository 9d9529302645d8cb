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
