"""Multi-GPU sharding of a query batch.

Queries are independent and the grid is read-only, so a batch shards by
*source*: all queries of one source go to the same rank (one single-source
solve answers all of them).  Sources are dealt to ranks by a deterministic
longest-processing-time greedy on their estimated cost: the query count, plus
what a source is known to cost beyond that (SourceCosts: a source the hub solver
hands to the SSSP kernel costs a full single-source search, ~10^4 times a hub
source).  The only collective is the final gather of the fixed-size result
records to rank 0 (RCCL over xGMI on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Mapping, Optional, Sequence


def shard_by_source(src_keys: Sequence[int], world: int,
                    extra_cost: Optional[Mapping[int, float]] = None) -> List[List[int]]:
    """Returns, per rank, the (ascending) query indices it owns.  A source's cost is
    its query count plus extra_cost.get(source key, 0) (in query units).

    Longest processing time first: the costliest sources first, ties by source key, each
    to the least-loaded rank (ties by rank).  Vectorised by cost class: within a run of
    sources of one cost c, rank r is picked at loads L_r, L_r + c, L_r + 2c, ... so the
    picks are the run's length smallest (load, rank) pairs of those sequences, in order
    (the same assignment as a heap popping the least-loaded rank source by source; costs
    are integers, so the loads are exact)."""
    import numpy as np
    keys = np.asarray(src_keys, dtype=np.int64)
    if keys.size == 0:
        return [[] for _ in range(world)]
    uniq, inv, counts = np.unique(keys, return_inverse=True, return_counts=True)
    cost = counts.astype(np.float64)
    for k, e in (extra_cost or {}).items():
        i = int(np.searchsorted(uniq, k))
        if i < uniq.size and uniq[i] == k:
            cost[i] += float(e)
    order = np.lexsort((uniq, -cost))
    cs = cost[order]
    runs = np.concatenate([[0], np.flatnonzero(np.diff(cs)) + 1, [cs.size]])
    load = np.zeros(world, dtype=np.float64)
    rank_of = np.empty(uniq.size, dtype=np.int64)
    ranks = np.arange(world, dtype=np.int64)
    for a, b in zip(runs[:-1], runs[1:]):
        m, c = int(b - a), float(cs[a])
        # at most m picks per rank
        t = np.arange(m, dtype=np.float64)
        cand_load = (load[:, None] + t[None, :] * c).ravel()
        cand_rank = np.repeat(ranks, m)
        pick = np.lexsort((cand_rank, cand_load))[:m]
        got = cand_rank[pick]
        rank_of[order[a:b]] = got
        load += c * np.bincount(got, minlength=world)
    rq = rank_of[inv]
    return [np.flatnonzero(rq == r).tolist() for r in range(world)]


class SourceCosts:
    """Per-source costs learned from passes, for shard_by_source's extra_cost.

    observe(keys) records the sources a pass re-solved with the SSSP kernel
    (Plan.fallback_sources(), mr_plan_fallback_sources): the closed form is not
    certain for them, and the same source with the same parameters falls back again
    on the next batch.  Such a source costs `fallback_cost` queries more: one full
    search, ~16-25 ms at 1025^2 (DESIGN.md section 3a''), against ~1.8 ns per query
    of the lane hub kernel (c4: 0.224 ms per 125k) -> ~10^7.  LPT then deals the
    fallback sources out first, one per rank while they last, and the hub work goes
    to the ranks without one: the ranks that pay a search get nothing else to do."""

    def __init__(self, fallback_cost: float = 1e7):
        self.fallback_cost = float(fallback_cost)
        self.extra: Dict[int, float] = {}

    def observe(self, fallback_keys: Iterable[int]) -> None:
        for k in fallback_keys:
            self.extra[k] = self.fallback_cost

    def __call__(self) -> Dict[int, float]:
        return dict(self.extra)


def gather_rows_to_root(local, counts: Sequence[int], rank: int, world: int, group=None):
    """Gathers each rank's first counts[rank] rows of `local` (a tensor padded to
    max(counts) rows) to rank 0.  Returns the concatenation on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local[: counts[0]]
    if rank == 0:
        bufs = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local, gather_list=bufs, dst=0, group=group)
        return torch.cat([b[: counts[r]] for r, b in enumerate(bufs)], dim=0)
    dist.gather(local, dst=0, group=group)
    return None


class PipelinedGather:
    """Double-buffered result gather for a stream of batches (bench.py at N > 1).

    Each rank owns `depth` flat device buffers (result records followed by command
    slots, padded to the largest shard).  `issue(k)` starts an asynchronous gather
    of buffer k to rank 0 — on RCCL the collective runs on the process group's
    own stream, ordered after the kernels already enqueued on the caller's stream
    — so the gather of batch i overlaps the solve of batch i+1.  `reuse(k)` makes
    the caller's stream wait for the previous gather of buffer k before a new
    solve overwrites it; `drain()` waits for every gather still in flight."""

    def __init__(self, bufs, rank: int, world: int, group=None, host_staging: bool = False):
        """host_staging: gather host copies (a gloo rehearsal of the RCCL path on one GPU)."""
        import torch
        self.bufs, self.rank, self.world, self.group = list(bufs), rank, world, group
        self.host = host_staging
        self.pending = [None] * len(self.bufs)
        dev = "cpu" if host_staging else None
        self.out = ([[torch.empty_like(b, device=dev) for _ in range(world)] for b in self.bufs]
                    if rank == 0 else None)

    def issue(self, k: int) -> None:
        import torch.distributed as dist
        src = self.bufs[k].cpu() if self.host else self.bufs[k]
        self.pending[k] = dist.gather(src, gather_list=self.out[k] if self.rank == 0 else None, dst=0,
                                      group=self.group, async_op=True)

    def reuse(self, k: int) -> None:
        w, self.pending[k] = self.pending[k], None
        if w is not None:
            w.wait()

    def drain(self) -> None:
        for k in range(len(self.pending)):
            self.reuse(k)

    def rows(self, k: int, counts: Sequence[int], row_words: int):
        """Rank 0: the gathered rows of buffer k, per rank, as views [counts[r], row_words]
        of the region that starts the buffer (the caller's layout)."""
        return [b[: counts[r] * row_words].view(counts[r], row_words) for r, b in enumerate(self.out[k])]
