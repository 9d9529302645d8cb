"""The grid's SoE region table built on the device (mr_grid_region_table,
marshrutka_amd/csrc/mr_k_region.hip) against the oracle's BFS per region
(oracle mro_region_table_bfs), every cell of the configs[3] map (1025^2, every homeland)
and of the configs[4] map (4097^2, 64 clustered campfires a homeland: 16.8 M cells x 64
regions).  The regions come from the direct argmin of the reference's nearest-campfire
key (src/grid.rs:297-325, tests/region_util.py), not from the engine."""
import json
import os

import numpy as np
import pytest

from marshrutka_amd.mapgen import SyntheticMap
from region_util import cell_ranks, cell_regions

pytestmark = pytest.mark.gpu

C5_FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_scale", "c5.json")


@pytest.fixture(scope="module")
def eng():
    from marshrutka_amd import build, pathfinder
    build.build()
    if not pathfinder.device_available():
        pytest.fail("no gfx950 device visible to the GPU tests")
    return pathfinder


def _check(eng, oracle_lib, m, homelands):
    arr = m.cells_array()
    g = eng.MapGrid.from_array(arr)
    rank = cell_ranks(arr)
    for h in homelands:
        region, nreg = cell_regions(arr, h)
        want = oracle_lib.region_table_bfs(m.size, rank, region, nreg, threads=16)
        n, ms, got = g.region_table(h)
        assert n == nreg and got.shape == want.shape, (n, nreg, got.shape, want.shape)
        bad = np.nonzero(np.any(got != want, axis=(1, 2)))[0]
        assert bad.size == 0, (h, bad.size, [(int(v), got[v].tolist(), want[v].tolist()) for v in bad[:2]])
        del want, got
        # the second call reuses the table (no rebuild)
        n2, ms2, _ = g.region_table(h, fetch=False)
        assert (n2, ms2) == (n, ms) and ms > 0


def test_region_table_1025_every_cell(eng, oracle_lib):
    _check(eng, oracle_lib, SyntheticMap(1025, campfires_per_homeland=4, seed=4096), range(4))


def test_region_table_small_maps(eng, oracle_lib):
    for size, k, clustered, seed in ((3, 1, False, 1), (5, 1, False, 2), (21, 6, True, 5), (41, 8, True, 7),
                                     (65, 4, False, 2024), (129, 16, True, 9)):
        _check(eng, oracle_lib, SyntheticMap(size, campfires_per_homeland=k, seed=seed, clustered=clustered), range(4))


def test_region_table_4097_every_cell(eng, oracle_lib):
    with open(C5_FIXTURE) as f:
        fx = json.load(f)
    _check(eng, oracle_lib, SyntheticMap(**fx["map"]), [0])
