#!/usr/bin/env python3
"""All-sources SSSP on the 1025x1025 map: configs[2] taken literally, every one of the
1 050 625 cells as a source (1.1e12 labels), through all-destinations plans of
--per-plan sources each.

Per plan: one pass (the plan's own HIP-event time), then checks on the device words
(pad columns excluded):
  * every source's own cell holds the source word (0xFFFFFFFF) and no other cell does;
  * each source has exactly one word per special holding that special's own label
    (0x80000000 | t), none where the source itself is the special;
  * --check sampled (source, destination) labels rebuilt from the words
    (mr_sssp_label) equal the query path's labels (mr_plan_run on the same pairs:
    the hub solver's records), two independent device paths;
  * and, for the first plan, --oracle of those pairs against oracle/mr_oracle.cpp.
A wrapping int32 sum of all words is printed as a checksum of checksums.

    python tools/all_sources.py [--per-plan 2048] [--max-plans 0] [--out gpurun_out/all_sources.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _DevWords:
    """A device buffer as int32 words for torch.as_tensor (no copy)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i4", "data": (ptr, False), "version": 3,
                                         "strides": None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1025)
    ap.add_argument("--per-plan", type=int, default=2048)
    ap.add_argument("--max-plans", type=int, default=0)
    ap.add_argument("--check", type=int, default=32, help="sampled pairs per plan checked against the query path")
    ap.add_argument("--oracle", type=int, default=2, help="sampled pairs of the first plan checked against the oracle")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch

    from marshrutka_amd import build, pathfinder
    from marshrutka_amd.abi import Params
    from marshrutka_amd.mapgen import SyntheticMap
    build.build()
    if not pathfinder.device_available():
        raise SystemExit("no gfx950 device visible: the engine has no CPU fallback")
    S = args.size
    V = S * S
    m = SyntheticMap(S, campfires_per_homeland=4, seed=4096)
    grid = pathfinder.MapGrid.from_array(m.cells_array())
    cells = m.all_indices()
    params = Params()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rng = random.Random(7)
    key = lambda t: None if t is None else (t.legs, t.money, t.time_s, tuple(c.as_tuple() for c in t.commands))  # noqa: E731

    tot = dict(sources=0, pass_ms=0.0, fill_ms=0.0, create_s=0.0, check_s=0.0, checked=0, mismatches=0,
               oracle_checked=0, oracle_mismatches=0, fallback_sources=0, checksum=0)
    t_all = time.perf_counter()
    starts = list(range(0, V, args.per_plan))
    if args.max_plans:
        starts = starts[: args.max_plans]
    for k, start in enumerate(starts):
        srcs = cells[start:start + args.per_plan]
        t0 = time.perf_counter()
        plan = pathfinder.SSSPPlan(grid, params, srcs)
        tot["create_s"] += time.perf_counter() - t0
        plan.kernel_ms()  # open the timing window
        plan.run(stream.cuda_stream)
        stream.synchronize()
        ms, n = plan.kernel_ms()
        tot["pass_ms"] += ms * n
        tot["fill_ms"] += plan.fill_ms()
        st = plan.stats()
        ns = st["num_specials"]
        tot["fallback_sources"] += st["fallback_sources"]
        t1 = time.perf_counter()
        # ---- device checks on the words (plan sources: the distinct sources, row-major)
        ptr, nbytes = plan.device_records()
        pitch = plan.record_pitch()
        nsrc = plan.num_sources
        assert nsrc == len(srcs), (nsrc, len(srcs))
        words = torch.as_tensor(_DevWords(ptr, nbytes // 4), device="cuda").view(nsrc, S, pitch)[:, :, :S]
        src_words, csum, cnt = 0, 0, []
        for a in range(0, nsrc, 256):
            w = words[a:a + 256]
            src_words += int((w == -1).sum())
            cnt.append((w < -1).sum(dim=(1, 2)))
            csum += int(w.sum(dtype=torch.int64))
        cnt = torch.cat(cnt)
        # every source: its own cell (and only it); every special but the source: its
        # own label, so NS such words a source, NS - 1 for a source that is a special
        ok_src = src_words == nsrc
        v = torch.arange(start, start + nsrc, device="cuda", dtype=torch.int64)  # sources are cells start..
        own = words[torch.arange(nsrc, device="cuda"), v // S, v % S]
        ok_own = bool((own == -1).all())
        n_sp_src = int((cnt == ns - 1).sum())
        ok_spec = bool(((cnt == ns) | (cnt == ns - 1)).all()) and n_sp_src <= ns
        spec_words, exp_spec = int(cnt.sum()), nsrc * ns - n_sp_src
        tot["checksum"] = (tot["checksum"] + csum) & 0xFFFFFFFFFFFFFFFF
        # ---- sampled labels: the words (mr_sssp_label) against the query path
        pick = [(rng.randrange(nsrc), cells[rng.randrange(V)]) for _ in range(args.check)]
        qplan = pathfinder.Plan(grid, params, [(srcs[i], d) for i, d in pick])
        qplan.run(stream.cuda_stream)
        got_q = qplan.fetch()
        bad = sum(1 for (i, d), q in zip(pick, got_q) if key(plan.label(i, d)) != key(q))
        tot["checked"] += len(pick)
        tot["mismatches"] += bad
        if k == 0 and args.oracle:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle_lib
            oracle_lib.build()
            og = oracle_lib.OracleGrid.from_array(m.cells_array())
            sample = pick[: args.oracle]
            exp = og.find_path_batch(params, [(srcs[i], d) for i, d in sample], threads=min(16, os.cpu_count() or 1))
            tot["oracle_checked"] += len(sample)
            tot["oracle_mismatches"] += sum(1 for (i, d), e in zip(sample, exp) if key(plan.label(i, d)) != key(e))
        tot["check_s"] += time.perf_counter() - t1
        tot["sources"] += nsrc
        print(f"plan {k + 1}/{len(starts)}: {nsrc} sources, pass {ms:.2f} ms, fill {plan.fill_ms():.2f} ms, "
              f"fallback {st['fallback_sources']}, source words ok {ok_src and ok_own}, special words "
              f"{spec_words}/{exp_spec}, sampled {len(pick) - bad}/{len(pick)} ok", flush=True)
        if not (ok_src and ok_own and ok_spec) or bad:
            raise SystemExit(f"plan {k}: device words fail the checks")
        del qplan, plan, words, own
    wall = time.perf_counter() - t_all
    cells_total = tot["sources"] * V
    out = dict(grid=f"{S}x{S}", sources=tot["sources"], labels=cells_total, per_plan=args.per_plan,
               plans=len(starts), gpu_pass_s=tot["pass_ms"] / 1e3, gpu_fill_s=tot["fill_ms"] / 1e3,
               labels_per_s_gpu=cells_total / (tot["pass_ms"] / 1e3) if tot["pass_ms"] else None,
               plan_create_s=tot["create_s"], check_s=tot["check_s"], wall_s=wall,
               fallback_sources=tot["fallback_sources"], sampled_checked=tot["checked"],
               sampled_mismatches=tot["mismatches"], oracle_checked=tot["oracle_checked"],
               oracle_mismatches=tot["oracle_mismatches"], checksum_of_words=tot["checksum"])
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
