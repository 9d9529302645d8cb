#!/usr/bin/env python3
"""bench.py — queries/sec of the gfx950 pathfinder hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]

One "step" = one pass of the hot path over one batch: every query of the
rank's shard is answered (one single-source solve per unique source, all
destinations of that source read off it) and, for N > 1, the fixed-size
result records are gathered to rank 0 over RCCL.  Inputs are resident in HBM
before the timed region starts.

Workloads (BASELINE.json configs; odd sides per SURVEY.md §8a A14):
  c1           one query on a 15x15 game-like map (configs[0]: plumbing; latency of
               one query through the device path)
  c4 (default) configs[3]: one batch of 1M uniform queries on the 1025x1025 map,
               its sources sharded over the N ranks (1M on one GPU, 125k per rank
               at N=8; strong scaling: the north-star target, >= 1e6 q/s on a
               1024x1024 grid at 8 GPUs, is quoted on this batch)
  c2           10k uniform (src,dst) queries per GPU on a 65x65 synthetic map
               (configs[1]: "10k random (src,dst) batch on 64x64")
  c3           1024 sources per GPU, every destination of each on 1025x1025
               (configs[2]: single-source -> all-destinations; V queries per source)
  c5           10k uniform queries per GPU on a 4097x4097 map with 64 clustered
               campfires per homeland (261 specials), Time first (configs[4],
               SURVEY 8d c5 option a)

N>1 is launched by the driver as
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
one process per GPU; each rank owns the sources of its shard (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "shortest-path queries/sec on N×N weighted grid; bit-exact vs CPU pathfinder"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: Chip-level parameters)
BYTES_PER_VERTEX_SOLVE = 20  # per full single-source solve, V x 20 B

WORKLOADS = {
    "c1": dict(size=15, queries_per_gpu=1, campfires=4, seed=15, max_cmds=16,
               desc="configs[0]: one (src,dst) query on a 15x15 game-like synthetic map (no game map ships with "
                    "the reference, SURVEY 8c), default FindPath params; a step is one whole query through the "
                    "device path (the reference runs it on the CPU)"),
    # max_cmds: command slots per query record (what the N > 1 gather moves); the app's
    # default orders give labels of at most 4 commands on these maps (c4's 1M batch:
    # 52k / 47k / 302k / 599k labels of 1 / 2 / 3 / 4, tools/probes/cmd_hist.py), the
    # Time-first c5 up to 14+; a longer label goes to the rank's overflow pool (its slot
    # is tagged)
    "c2": dict(size=65, queries_per_gpu=10_000, campfires=4, seed=2024, max_cmds=4,
               desc="configs[1]: 10k uniform (src,dst) per GPU on a 65x65 synthetic map (64x64 -> odd 65), "
                    "default FindPath params"),
    # c3: 1024 sources a pass (4.5 GB of cell words), far past the 256 MiB Infinity Cache,
    # so the stores are priced at HBM (64 sources, 269 MB, were partly absorbed by it)
    "c3": dict(size=1025, queries_per_gpu=1024, campfires=4, seed=4096, all_destinations=True,
               desc="configs[2]: single source -> all 1 050 625 cells of the 1025x1025 synthetic map, 1024 "
                    "sources per GPU per pass; a step answers V queries per source (SURVEY 8d c3)"),
    # c4: one 1M-query batch for the whole job (strong scaling), split by source over
    # the ranks: N = 1 answers all of configs[3] on one GPU
    "c4": dict(size=1025, queries_total=1_000_000, campfires=4, seed=4096, max_cmds=4,
               desc="configs[3]: one batch of 1M uniform (src,dst) queries on a 1025x1025 synthetic map "
                    "(1024 -> odd 1025), default FindPath params, its sources sharded over the GPUs"),
    "c5": dict(size=4097, queries_per_gpu=10_000, campfires=64, clustered=True, seed=4097, sort=(1, 2), max_cmds=16,
               desc="configs[4]: 10k uniform (src,dst) per GPU on a 4097x4097 synthetic map (4096 -> odd 4097) "
                    "with 64 clustered campfires per homeland (261 specials); sort_by (Time, Money), so caravan "
                    "edges span 102 s .. 240 s x 2S (SURVEY 8d c5 option a)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--queries", type=int, default=0,
                    help="override queries per GPU (c4: the whole batch is this x N)")
    ap.add_argument("--cpu-seconds", type=float, default=24.0,
                    help="CPU-baseline budget (wall seconds, split between the 1-thread and all-threads legs)")
    ap.add_argument("--e2e-reps", type=int, default=3, help="fresh batches timed end to end (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default="", help="JSON with PMC-derived HBM bytes per launch (profiles/)")
    return ap.parse_args()


def host_cores():
    """(cores this process may run on, threads the baseline uses).  The first is the
    affinity mask; the second is capped by the cgroup CPU quota when one is set (a GPU
    box's share of a 256-thread host is 16 CPUs: more threads than the quota only
    time-slice) and by MR_CPU_THREADS."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    use = cores
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            use = min(use, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    if os.environ.get("MR_CPU_THREADS"):
        use = min(use, max(1, int(os.environ["MR_CPU_THREADS"])))
    return cores, use


def cpu_baseline_leg(m, params, queries, gpu_results, budget_s):
    """Oracle (C++ restatement of the reference, oracle/) on host cores over a
    bounded sample of the same workload, once on one thread and once on every thread
    the host gives this process; also checks the sample's GPU
    results.  Each leg runs ~budget_s / 2 of wall time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib
    oracle_lib.build()
    og = oracle_lib.OracleGrid.from_array(m.cells_array())
    cores, threads = host_cores()
    leg_s = max(1.0, budget_s / 2)
    # one thread: queries in order until the leg's time is spent
    t0 = time.perf_counter()
    n1 = 0
    while n1 < len(queries) and (n1 == 0 or time.perf_counter() - t0 < leg_s):
        og.find_path_batch_raw(params, queries[n1:n1 + 1], threads=1)
        n1 += 1
    wall1 = time.perf_counter() - t0
    per_q = wall1 / n1
    # every thread: a sample sized to ~leg_s of wall (at least one query per thread)
    n = int(min(len(queries), max(threads, threads * leg_s / per_q)))
    sample = queries[:n]
    t0 = time.perf_counter()
    labels = og.find_path_batch(params, sample, threads=threads)
    wall = time.perf_counter() - t0
    mism = sum(1 for e, g in zip(labels, gpu_results[:n]) if as_expected(e) != as_expected(g))
    return ({"value": n / wall, "unit": "queries/s", "cores": threads, "kind": "port",
             "value_all_cores": n / wall, "value_1thread": n1 / wall1, "cores_all": cores,
             "sample": f"first {n} queries of the rank-0 batch on {threads} threads ({wall:.1f} s wall) and the first "
                       f"{n1} on 1 thread ({wall1:.1f} s), oracle/mr_oracle.cpp (binary heap of full labels + hash map, "
                       f"as the reference); cpu model: {cpu_model()}; {cores} cores in the affinity mask, "
                       f"os.cpu_count() {os.cpu_count()}"},
            {"checked": n, "mismatches": mism})


def cpu_baseline_all(m, params, plan, sources, budget_s):
    """Oracle single-source solves to the cell farthest from each source (a full
    Dijkstra over the grid, as the reference would need for every destination), on
    host threads; value = cells answered per second.  The sampled labels are also
    checked against the GPU's records."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib
    oracle_lib.build()
    og = oracle_lib.OracleGrid.from_array(m.cells_array())
    cores, threads = host_cores()
    H = m.size // 2
    V = m.size * m.size

    cells = m.all_indices()
    pos = {c: (j % m.size - H, j // m.size - H) for j, c in enumerate(cells)}

    def far(s):
        # the opposite corner of the map from the source's quadrant
        x, y = pos[s]
        tx, ty = (-H if x >= 0 else H), (-H if y >= 0 else H)
        return cells[(ty + H) * m.size + (tx + H)]

    t0 = time.perf_counter()
    og.find_path_batch_raw(params, [(sources[0], far(sources[0]))], threads=1)
    per = max(time.perf_counter() - t0, 1e-3)
    n = int(max(1, min(len(sources), threads * max(1, budget_s / per / threads))))
    sample = [(s, far(s)) for s in sources[:n]]
    t0 = time.perf_counter()
    labels = og.find_path_batch(params, sample, threads=threads)
    wall = time.perf_counter() - t0
    mism = sum(1 for i, ((s, d), e) in enumerate(zip(sample, labels)) if as_expected(plan.label(i, d)) != as_expected(e))
    return ({"value": n * V / wall, "unit": "queries/s", "cores": threads, "kind": "port", "cores_all": cores,
             "value_all_cores": n * V / wall, "value_1thread": V / per,
             "sample": f"{n} single-source solves to the farthest cell (~all {V} cells settled each), "
                       f"oracle/mr_oracle.cpp on {threads} host threads, {wall:.2f} s wall, cells/s; the 1-thread "
                       f"figure is the first solve alone ({per:.2f} s); cpu model: {cpu_model()}; {cores} cores in "
                       f"the affinity mask"},
            {"checked": n, "mismatches": mism})


def algorithmic_bytes(plan, stats, V):
    """Bytes one launch must move.

    SSSP kernel: V x 20 B per unique source (4 B per-cell record
    read + 16 B final label write).  Hub solver: it never touches the grid, so
    its bytes are what it reads and writes per query (destination 4 B,
    destination static word 4 B, result record 16 B, 16 B per command slot
    written; records go out in grouped order, so no query id is read), per source (source vertex + range 8 B, its region row
    8 B x regions), plus the SSSP figure for every source it hands to the
    fallback.  Returns (bytes, kernel name, SURVEY-8d-equivalent bytes)."""
    n_src = stats["num_sources"]
    survey = float(n_src) * V * BYTES_PER_VERTEX_SOLVE
    if stats["solver"] not in ("hub", "hub_wide"):
        return survey, "sssp_kernel", survey
    import numpy as np
    res, _ = plan.fetch_raw()
    words = np.frombuffer(res, dtype=np.uint32).reshape(-1, 8)[: plan.n]
    ok = words[:, 6].view(np.int32) == 0
    n_cmds = int(words[ok, 4].astype(np.int64).sum())
    nq = plan.n
    b = nq * (4 + 4 + 16) + 16 * n_cmds + n_src * (8 + 8 * stats["num_regions"])
    b += 8 * stats["region_boundary_cells"]  # wide solver: the regions' boundary cells, read once (L2-resident)
    b += stats["fallback_sources"] * V * BYTES_PER_VERTEX_SOLVE
    if stats["solver"] == "hub_wide":
        kern = "hub_wide_kernel"
    elif stats.get("lanes_per_source", 0) > 1:  # one source per group of 8 / 16 / 32 lanes
        kern = "hub_group_kernel"
    elif stats.get("lane_sources", 0) == 0:
        kern = "hub_kernel"
    else:  # one source per lane; sources with many queries stay on hub_kernel
        kern = "hub_lane_kernel" + (" + hub_kernel" if stats["lane_sources"] < n_src else "")
    name = kern + (" + sssp_kernel (fallback)" if stats["fallback_sources"] else "")
    return float(b), name, survey


def check_gather(pipe, plan, k, grid, params, shards, orders, counts, rows, rw, wpool_cap, rank, world):
    """After the timed region (N > 1): rank 0 decodes every wire row of the last batch as
    gathered (rows, then the pool of long labels, of each rank) on the host
    (mr_decode_wire), puts row j of rank r at its query shards[r][orders[r][j]], and
    compares the labels with each rank's own fetch of that batch (mr_plan_fetch, in the
    rank's query order): one digest per rank.  Returns the check's summary on rank 0."""
    import numpy as np
    import torch.distributed as dist
    from marshrutka_amd import pathfinder
    res, pool = plan.fetch_raw()  # this rank's labels, in its local query order
    digests = [None] * world
    dist.all_gather_object(digests, pathfinder.labels_digest(res, pool, counts[rank]))
    if rank != 0:
        return None
    bad_status, mismatched, seen = 0, 0, np.zeros(sum(counts), dtype=bool)
    mc = (rw - 1) // 2
    for r, buf in enumerate(pipe.out[k]):
        words = buf.to("cpu").numpy().view("uint32")
        n = counts[r]
        out, opool = pathfinder.decode_wire_raw(grid, params, words[: n * rw], n, mc,
                                                words[rows * rw: rows * rw + wpool_cap * 2])
        st = np.array([out[j].status for j in range(n)])
        bad_status += int(((st != 0) & (st != 1)).sum())
        order = np.asarray(orders[r][:n], dtype=np.int64)  # row j answers local query order[j]
        inv = np.empty(n, dtype=np.int64)
        inv[order] = np.arange(n)  # local query i is row inv[i]
        seen[np.asarray(shards[r], dtype=np.int64)[order]] = True
        if pathfinder.labels_digest(out, opool, n, inv) != digests[r]:
            mismatched += 1
    return {"rows": sum(counts), "bad_status": bad_status, "queries_covered": int(seen.sum()),
            "ranks_matching_own_fetch": world - mismatched, "ranks": world,
            "wire_bytes_per_query": rw * 4 + wpool_cap * 8 / max(1, rows)}


def as_expected(label):
    if label is None:
        return None
    return (label.legs, label.money, label.time_s, tuple(c.as_tuple() for c in label.commands))


def end_to_end(m, grid, params, qpg, seed, max_cmds, reps, pinned=False):
    """Whole-call throughput of fresh batches: plan creation (host grouping by source,
    the per-plan tables, the uploads), one pass, the device->host copy and decode of
    every label (mr_plan_fetch), synchronised.  The queries are built as a numpy
    mr_query array beforehand (the caller's input).  Median over `reps` batches.
    pinned: the output arrays page-locked once (mr_host_register), as a serving caller
    reusing them would: the fetch DMAs straight into them."""
    import numpy as np
    import torch
    from marshrutka_amd import pathfinder
    V = m.size * m.size
    rows = []
    # the caller's output arrays, allocated (and touched) once and reused by every batch
    bufs = pathfinder.fetch_buffers(qpg, max_cmds)
    for b in bufs:
        np.frombuffer(b, dtype=np.uint8).fill(0)
    if pinned:
        for b in bufs:
            pathfinder.pin_host(b)
    # one batch before the timed ones: the first also pays one-time setup (the pinned
    # staging buffers, the sort's first call); it is reported as cold_ms, never in the median
    for r in range(reps + 1):
        rng = np.random.default_rng(seed + 1000 + r)
        src = rng.integers(0, V, qpg, dtype=np.int64)
        dst = rng.integers(0, V, qpg, dtype=np.int64)
        qa = m.query_array(src, dst)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plan = pathfinder.Plan(grid, params, None, max_cmds=max_cmds, query_array=qa)
        t1 = time.perf_counter()
        plan.run()
        plan.wait()
        t2 = time.perf_counter()
        plan.fetch_raw(bufs)
        t3 = time.perf_counter()
        del plan
        rows.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2))
    if pinned:
        for b in bufs:
            pathfinder.unpin_host(b)
    cold = rows.pop(0)
    rows.sort()
    tot, cr, run, fe = rows[len(rows) // 2]
    return {"e2e_queries_per_s": qpg / tot, "cold_ms": cold[0] * 1e3, "output_arrays": "page-locked" if pinned else "pageable", "queries": qpg, "ms": tot * 1e3, "plan_create_ms": cr * 1e3,
            "run_ms": run * 1e3, "fetch_ms": fe * 1e3, "reps": reps,
            "what": "fresh batch: Plan create (host grouping, tables, H2D) + one pass + mr_plan_fetch (D2H and "
                    "decode of every label) into the caller's output arrays (allocated once, reused across batches), "
                    "median of reps after one untimed batch (cold_ms: its time)"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    # stdout carries the one JSON line only: native libraries that print to fd 1 (RCCL's
    # version banner at communicator creation) go to stderr instead
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    from marshrutka_amd import build, pathfinder
    from marshrutka_amd.abi import Params
    from marshrutka_amd.mapgen import SyntheticMap, random_queries, random_query_cells
    from marshrutka_amd.shard import PipelinedGather, SourceCosts, shard_by_source

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # MR_BENCH_BACKEND=gloo: a rehearsal of the N>1 path with every rank on the one
    # visible GPU and the gather staged through host memory (RCCL needs a GPU per rank)
    backend = os.environ.get("MR_BENCH_BACKEND", "nccl")
    # MR_BENCH_DIST=1: the N > 1 code path (process group, double-buffered RCCL gather,
    # gather check) at world size 1 too, to exercise it on a one-GPU box
    dist_on = world > 1 or os.environ.get("MR_BENCH_DIST") == "1"
    device = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(device)
    # a dedicated stream: the solve kernel and the RCCL gather are ordered on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", device))
    build.build()
    if not pathfinder.device_available():
        raise SystemExit("no gfx950 device visible: the engine has no CPU fallback")

    wl = dict(WORKLOADS[args.workload])
    # strong-scaling workloads (c4) split one batch of queries_total over the ranks
    strong = "queries_total" in wl and not args.queries
    qpg = args.queries or (-(-wl["queries_total"] // world) if strong else wl["queries_per_gpu"])
    total_q = wl["queries_total"] if strong else qpg * world
    m = SyntheticMap(wl["size"], campfires_per_homeland=wl["campfires"], seed=wl["seed"],
                     clustered=bool(wl.get("clustered")))
    # the app's defaults (src/app.rs:782-811), with the workload's sort order
    params = Params(sort_by=wl["sort"]) if "sort" in wl else Params()
    all_dst = bool(wl.get("all_destinations"))
    cells_in = m.cells_array()
    tg = time.perf_counter()
    grid = pathfinder.MapGrid.from_array(cells_in)
    grid_ms = (time.perf_counter() - tg) * 1e3
    # grid preprocessing the hub plans need: the query homeland's region table, built on
    # the device (mr_grid_region_table); timed here, before the first plan would build it
    nreg, region_ms, _ = grid.region_table(params.homeland, fetch=False)
    grid_load = {"grid_create_ms": grid_ms, "region_table_ms": region_ms, "regions": nreg,
                 "note": "mr_grid_create on the host (layout check, ranks, nearest campfires) and the "
                         "device build of the V x regions table (DESIGN.md section 4), once per map"}
    fb_total_probe = None  # N > 1 query batches: sources the probe pass saw re-solved
    if all_dst:
        # distinct sources, a contiguous block per rank; no cross-rank data path
        cells = m.all_indices()
        pick = random_queries(m, 4 * qpg * world, wl["seed"] + 17)
        srcs = list(dict.fromkeys(a for a, _ in pick))[: qpg * world]
        mine = srcs[rank * qpg:(rank + 1) * qpg]
        counts = [qpg * len(cells)] * world  # V queries answered per source
        plan = pathfinder.SSSPPlan(grid, params, mine)
        n_src = plan.num_sources
    else:
        import numpy as np
        # the batch as row-major cells (random_queries' stream, vectorised: 1M queries
        # need no Python object each); a source's key is its cell
        q_src, q_dst = random_query_cells(m, total_q, wl["seed"] + 17)
        cells_arr = m.cells_array()
        keys = q_src
        ts = time.perf_counter()
        shards = shard_by_source(keys, world)
        shard_ms = (time.perf_counter() - ts) * 1e3

        def my_queries(sh):
            idx = np.asarray(sh, dtype=np.int64)
            return m.query_array(q_src[idx], q_dst[idx], cells_arr)

        mine = my_queries(shards[rank])
        if dist_on:
            # cost-aware split (shard.SourceCosts): one untimed probe pass per rank names
            # the sources the hub solver hands to the SSSP kernel; the batch is re-dealt
            # with their cost, so they land one per rank and the hub work goes elsewhere
            probe = pathfinder.Plan(grid, params, None, max_cmds=wl.get("max_cmds", 16), query_array=mine)
            probe.run()
            fb_keys = [m.cell_of(c) for c in probe.fallback_sources()]
            del probe
            every = [None] * world
            dist.all_gather_object(every, fb_keys)
            costs = SourceCosts()
            costs.observe(k for ks in every for k in ks)
            fb_total_probe = len(costs.extra)
            if fb_total_probe:
                shards = shard_by_source(keys, world, costs())
                mine = my_queries(shards[rank])
        counts = [len(s) for s in shards]
        # N > 1: two plans over the same shard, so the result gather of one batch
        # overlaps the solve of the next (double buffering, shard.PipelinedGather)
        depth = 2 if dist_on else 1
        plans = [pathfinder.Plan(grid, params, None, max_cmds=wl.get("max_cmds", 16), query_array=mine)
                 for _ in range(depth)]
        plan = plans[0]
        n_src = plan.num_sources
    pipe = None
    if dist_on and not all_dst:
        # each pass re-encoded as wire rows (mr_plan_wire_records: 4 + 8 max_cmds bytes a
        # query, the metrics left to the decoder) and the pool of long labels, in one flat
        # torch-owned device buffer per plan, padded to the largest shard: one RCCL gather
        # per batch moves every label of the batch with all its commands
        rows = max(counts)
        rw = pathfinder.wire_row_words(plan.max_cmds)
        wpool_cap = max(1024, rows // 8)  # commands (8 B) of labels longer than the slots
        bufs = [torch.zeros(rows * rw + wpool_cap * 2, dtype=torch.int32, device="cuda") for _ in plans]
        pipe = PipelinedGather(bufs, rank, world, host_staging=backend == "gloo")
        # record k of rank r's buffer answers query shards[r][order_r[k]]: the grouping
        # order is fixed per plan, so it crosses once, outside the timed region
        orders = [None] * world
        dist.all_gather_object(orders, plan.record_queries())
    elif all_dst:
        plans = [plan]
    it = [0]

    # N > 1: the wire encoding and the gather of batch i run on a stream of their own, so
    # that they overlap the pass of batch i+1 (the other plan); the plan's next pass waits
    # for its encoding (mr_plan_wire_records)
    wstream = torch.cuda.Stream() if pipe is not None else None

    def step():
        k = it[0] % len(plans)
        it[0] += 1
        plans[k].run(stream.cuda_stream)
        if pipe is not None:
            b = bufs[k].data_ptr()
            with torch.cuda.stream(wstream):
                pipe.reuse(k)  # wstream waits until batch k-2's gather has read this buffer
                plans[k].wire_records(b, b + rows * rw * 4, wpool_cap, wstream.cuda_stream)
                pipe.issue(k)

    for _ in range(args.warmup):
        step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize()
    # the counters of a finished pass: a plan whose pass handed no source to the fallback
    # ends its later passes with the hub launch (the certificate and SSSP launches would
    # only exit at once), as a serving caller's plan does after its first fetch
    for p_ in plans:
        p_.stats()
    for p_ in plans:
        p_.kernel_ms()  # reset the per-launch event window to the timed region
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if pipe is not None:
        pipe.drain()  # every batch's results are at rank 0 inside the timed region
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gather_check = None
    if pipe is not None:
        gather_check = check_gather(pipe, plans[(it[0] - 1) % len(plans)], (it[0] - 1) % len(plans), grid, params,
                                    shards, orders, counts, rows, rw, wpool_cap, rank, world)
    kn = [p_.kernel_ms() for p_ in plans]
    nl = sum(n for _, n in kn)
    kms = sum(ms * n for ms, n in kn) / nl if nl else 0.0
    if dist_on:
        rdev = "cpu" if backend == "gloo" else "cuda"
        t = torch.tensor([elapsed, kms], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kms = float(t[0]), float(t[1])
        tot_src = torch.tensor([n_src], dtype=torch.int64, device=rdev)
        dist.all_reduce(tot_src)
        tot_src = int(tot_src)
    else:
        tot_src = n_src

    total_queries = sum(counts) * args.steps
    value = total_queries / elapsed
    V = wl["size"] ** 2
    stats = plan.stats()
    if all_dst:
        # V x 20 B per solve (the 4 B per-cell word read, the 16 B record written),
        # over the dominant kernel: the fill launch (hub plans) or the whole SSSP pass.  The
        # fill kernel reads no per-cell word (the specials come from the source's table) and
        # writes one 4 B cell word per cell (the label's walk over the source's table), so
        # its own bytes are V x 4 B plus the table: per entry the 44 B label, its 4 B rank
        # and the special's 32 B static record
        alg_bytes = survey_bytes = float(n_src) * V * BYTES_PER_VERTEX_SOLVE
        fms = plan.fill_ms()
        if stats["solver"] == "hub" and fms > 0:
            alg_bytes = float(n_src) * (V * 4 + (stats["num_specials"] + 1) * 80)
            # fused: the launch also solves the next pass's specials (priced as the fill's alone)
            kernel_name = "hub_fill_kernel" if stats["fill_launch"] == "fused" else "fill_kernel"
            pass_ms, kms = kms, fms
        else:
            kernel_name, pass_ms = "sssp_kernel", kms
    else:
        alg_bytes, kernel_name, survey_bytes = algorithmic_bytes(plan, stats, V)
    if dist_on:
        t = torch.tensor([alg_bytes, survey_bytes, stats["fallback_sources"]], dtype=torch.float64,
                         device="cpu" if backend == "gloo" else "cuda")
        dist.all_reduce(t)
        alg_bytes, survey_bytes, fb_total = float(t[0]), float(t[1]), int(t[2])
    else:
        fb_total = stats["fallback_sources"]
    # roofline: algorithmic bytes per launch (see algorithmic_bytes) over the solve's
    # average launch time (HIP events on its stream); with N ranks, the aggregate
    # bytes over the slowest rank's launch time
    achieved = alg_bytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    traffic = None
    pmc_path = args.pmc or os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("workload") == args.workload and pm.get("queries_per_gpu") == qpg:
                # one rank's PMC bytes per launch (profiled at N=1); the aggregate over
                # the N ranks, like alg_bytes
                traffic = pm.get("hbm_bytes_per_launch")
                if traffic is not None:
                    traffic *= world
        except (OSError, ValueError):
            traffic = None

    # the issue side of the roofline (the hub kernels are instruction-bound, DESIGN.md
    # section 5): SQ instruction counts per launch from a committed SQ pass of the same
    # workload, VALU busy = VALU wave-instructions x 2 cycles (wave64 on a SIMD-32)
    # over 1 024 SIMDs x the kernel's time at the 2.4 GHz peak clock
    issue = None
    sq_path = os.path.join(ROOT, "profiles", f"sq_{args.workload}.json")
    if os.path.exists(sq_path) and kms > 0:
        try:
            with open(sq_path) as f:
                sqf = json.load(f)
            # counters of another batch size describe another launch: not this one's
            if sqf.get("workload") != args.workload or sqf.get("queries_per_gpu") != qpg:
                raise ValueError("SQ counters of another workload or batch size")
            sq = sqf["per_launch"]
            busy = sq["SQ_INSTS_VALU"] * 2.0 / (1024 * kms * 1e-3 * 2.4e9)
            issue = {"valu_per_launch": sq["SQ_INSTS_VALU"], "salu_per_launch": sq["SQ_INSTS_SALU"],
                     "lds_per_launch": sq["SQ_INSTS_LDS"], "valu_busy_frac_at_2_4GHz": busy,
                     "source": os.path.relpath(sq_path, ROOT)}
        except (OSError, ValueError, KeyError):
            issue = None
    out = {
        "metric": METRIC, "value": value, "unit": "queries/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": wl["desc"], "grid": f"{wl['size']}x{wl['size']}", "queries_per_gpu": qpg,
                   "queries_per_step": sum(counts),
                   "campfires_per_homeland": wl["campfires"], "unique_sources_per_step": tot_src,
                   "params": "FindPath defaults: sort " + ("(Time,Money)" if wl.get("sort") == (1, 2) else
                                                           "(Legs,Money)") + ", SoE 50, caravans, skills 0, homeland Blue",
                   "solver": stats["solver"], "fallback_sources_per_step": fb_total,
                   "cost_aware_split": None if fb_total_probe is None else
                   {"fallback_sources_seen_by_probe": fb_total_probe},
                   "specials": stats["num_specials"],
                   "parallelism": f"sources sharded over {world} GPU(s), RCCL gather of results to rank 0 "
                                  "(double-buffered: overlaps the next batch's solve)"
                                  if world > 1 else "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kernel_name, "kernel_ms": kms, "launches": nl,
                     "pass_ms": pass_ms if all_dst else kms,
                     "alg_bytes_per_launch": alg_bytes, "issue": issue,
                     "survey_8d_bytes_per_launch": survey_bytes,
                     "note": ("all destinations: fill kernel, V x 4 B per source (the cell word written; no per-cell "
                              "read) + 80 B per table entry; survey_8d_bytes_per_launch is SURVEY 8d's V x 20 B; "
                              "kernel_ms spans the fill's two launches; pass_ms is the caller-stream span of a pass (the specials' "
                              "solve runs beside the previous pass's fill, DESIGN.md 3b)" if all_dst else
                              "hub solver: instruction-issue bound Dijkstra over the specials (one source per lane: "
                              "hub_lane_kernel; per group of lanes: hub_group_kernel; per wave: hub_kernel; see "
                              "roofline.issue); bytes = "
                              "queries in, results and command slots out, per-source region rows, plus V*20 B "
                              "per SSSP fallback source (DESIGN.md section 4)")
                     if stats["solver"] in ("hub", "hub_wide") else
                     "SSSP kernel: SURVEY 8d bytes, V*20 B per unique source"},
    }
    out["grid_load"] = grid_load
    if not all_dst and world > 1:
        out["config"]["shard_ms"] = shard_ms  # shard_by_source over the whole batch (host, untimed)
    if gather_check is not None:
        out["gather_check"] = gather_check
    if rank == 0 and not all_dst and args.e2e_reps > 0:
        out["end_to_end"] = end_to_end(m, grid, params, qpg, wl["seed"], wl.get("max_cmds", 16), args.e2e_reps)
        # the same with the output arrays page-locked once (mr_host_register)
        out["end_to_end_pinned"] = end_to_end(m, grid, params, qpg, wl["seed"], wl.get("max_cmds", 16), args.e2e_reps,
                                              pinned=True)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and all_dst:
        cb, parity = cpu_baseline_all(m, params, plan, mine, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["parity"] = parity
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the oracle's sample is a prefix of the batch (a few hundred queries at 1025^2):
        # only that prefix becomes Python objects
        from marshrutka_amd.abi import CellIndex, result_from_c
        head = min(len(mine), 50_000)
        qs = mine[:head]
        pairs = [(CellIndex(int(a["kind"]), int(a["sub"]), int(a["x"]), int(a["y"])),
                  CellIndex(int(b["kind"]), int(b["sub"]), int(b["x"]), int(b["y"])))
                 for a, b in zip(qs["from"], qs["to"])]
        res, pool = plan.fetch_raw()
        gpu_res = [result_from_c(res[i], pool) for i in range(head)]
        cb, parity = cpu_baseline_leg(m, params, pairs, gpu_res, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["parity"] = parity
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
