"""The numpy label digest (tests/label_digest.py) equals the oracle's C++ one, and the
oracle's all-destinations batch equals its own single-query FindPath::eval: the two
facts the full-size GPU parity tests (test_gpu_full_scale.py) rest on.  CPU only."""
import random

import numpy as np

import label_digest as ld
from marshrutka_amd.abi import SORT_MONEY, SORT_TIME, CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap


def test_numpy_digest_equals_oracle_digest(oracle_lib):
    for size, k, params in ((15, 3, Params()), (21, 5, Params(sort_by=(SORT_TIME, SORT_MONEY), fleetfoot=2)),
                            (17, 4, Params(sort_by=(SORT_MONEY, SORT_TIME), use_sfm=True,
                                           hq_position=CellIndex.homeland(2, 3, 3)))):
        m = SyntheticMap(size, campfires_per_homeland=k, seed=size, clustered=size == 21)
        og = oracle_lib.OracleGrid.from_array(m.cells_array())
        cells = m.all_indices()
        rng = random.Random(size)
        sources = [CellIndex.center(), m.campfires()[0]] + rng.sample(cells, 2)
        want = og.sssp_digests(params, sources, threads=4)
        for i, s in enumerate(sources):
            res, pool = og.find_path_batch_raw(params, [(s, d) for d in cells], threads=4)
            got = ld.digests(res, pool, len(cells))
            row = {f: want[f][i] for f in want}
            bad = ld.mismatches(got, row)
            assert bad.size == 0, (size, s, [cells[j] for j in bad[:4]])
            assert (got["n_commands"] > 0).all() and len(np.unique(got["digest"])) > len(cells) // 2


def test_digest_sees_every_command_field(oracle_lib):
    """Changing any one field of one command changes the label's digest."""
    m = SyntheticMap(11, campfires_per_homeland=2, seed=3)
    og = oracle_lib.OracleGrid.from_array(m.cells_array())
    res, pool = og.find_path_batch_raw(Params(), [(CellIndex.parse("B 3#3"), CellIndex.parse("G 4#2"))], threads=1)
    base = ld.digests(res, pool, 1)["digest"][0]
    n = res[0].n_commands
    assert n >= 2
    raw = bytearray(bytes(pool)[: 40 * n])
    for off in (0, 4, 8, 12, 16, 24, 26, 28, 32, 34, 36):  # kind legs money ff time from.* to.*
        mod = bytearray(raw)
        mod[40 * (n - 1) + off] ^= 1
        assert ld.digests(res, bytes(mod), 1, pool_len=n)["digest"][0] != base, off
    swapped = raw[40:80] + raw[:40] + raw[80:]
    assert ld.digests(res, bytes(swapped), 1, pool_len=n)["digest"][0] != base
