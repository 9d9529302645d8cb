"""Generates tests/golden/full_scale/c5.json: oracle answers on the configs[4] map
(S = 4097, 64 clustered campfires per homeland, bench.py's c5), which the oracle
needs ~70 s to build and ~100 s and ~13 GB per single-source solve for — too slow to
run inside the GPU suite, so they are computed here once (test infrastructure, CPU):

* `sources`: for 3 sources, every cell's label from the oracle's Dijkstra run to
  completion (mro_sssp_digest_batch), kept as one checksum per grid row
  (tests/label_digest.py row_checksums: 4097 u64 per source);
* `sample`: the labels of 8 queries of test_c5_full_scale_sample's 2000-query
  batch per comparator order (the oracle's FindPath::eval, early exit and all).

Usage: python tests/golden/make_full_scale.py [--threads 2]   (about 15 min, 30 GB)
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import label_digest as ld  # noqa: E402
import oracle_lib  # noqa: E402
from golden_util import as_expected  # noqa: E402
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

OUT = os.path.join(HERE, "full_scale", "c5.json")
C5 = dict(size=4097, campfires_per_homeland=64, seed=4097, clustered=True)
# (params, row-major source cells): a random cell and a campfire for the c5 order, one
# cell for Money first (SURVEY 8d c5 options a and b)
SOURCE_RUNS = [(Params(sort_by=(SORT_TIME, SORT_MONEY)), ["random:4097", "campfire:100"]),
               (Params(sort_by=(SORT_MONEY, SORT_LEGS)), ["random:5"])]
SAMPLE_RUNS = [Params(sort_by=(SORT_TIME, SORT_MONEY)), Params(sort_by=(SORT_MONEY, SORT_LEGS))]
SAMPLE_BATCH = (2000, 45)  # test_c5_full_scale_sample's batch: random_queries(m, 2000, 45)
SAMPLE_IDX = list(range(0, 2000, 250))


def resolve(m, spec):
    import random
    kind, arg = spec.split(":")
    if kind == "campfire":
        return m.cell_of(m.campfires()[int(arg)])
    return random.Random(int(arg)).randrange(m.size * m.size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=2, help="concurrent oracle solves (~13 GB each)")
    args = ap.parse_args()
    t0 = time.time()
    m = SyntheticMap(**C5)
    arr = m.cells_array()
    og = oracle_lib.OracleGrid.from_array(arr)
    print(f"oracle grid {time.time() - t0:.0f} s", flush=True)
    out = {"map": C5, "checksum": "label_digest.row_checksums over label_digest.FIELDS", "sources": [],
           "sample": []}
    for params, specs in SOURCE_RUNS:
        cells = [resolve(m, s) for s in specs]
        for lo in range(0, len(cells), args.threads):
            part = cells[lo:lo + args.threads]
            d = og.sssp_digests(params, [m.index_at(c) for c in part], threads=len(part))
            for i, c in enumerate(part):
                rows = ld.row_checksums({f: d[f][i] for f in d}, m.size)
                out["sources"].append({"params": params.to_json(), "spec": specs[lo + i], "cell": c,
                                       "rows": [f"{int(x):016x}" for x in rows]})
            print(f"sources {specs[lo:lo + len(part)]} {time.time() - t0:.0f} s", flush=True)
    qs = random_queries(m, *SAMPLE_BATCH)
    for params in SAMPLE_RUNS:
        labels = og.find_path_batch(params, [qs[i] for i in SAMPLE_IDX], threads=args.threads)
        out["sample"].append({"params": params.to_json(), "batch": list(SAMPLE_BATCH), "index": SAMPLE_IDX,
                              "expected": [as_expected(e) for e in labels]})
        print(f"sample {params.sort_by} {time.time() - t0:.0f} s", flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {OUT} in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
