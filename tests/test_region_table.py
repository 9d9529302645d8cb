"""The region table's separable transform (marshrutka_amd/csrc/mr_k_region.hip, DESIGN.md
section 4) restated in numpy (tests/region_util.py) against the oracle's BFS per region
(oracle mro_region_table_bfs) on small maps, every cell, every homeland.  CPU only: it
checks the algorithm the device kernels run; tests/test_gpu_region_table.py checks the
kernels themselves."""
import pytest

from marshrutka_amd.mapgen import SyntheticMap
from region_util import cell_ranks, cell_regions, transform_model


@pytest.mark.parametrize("size,k,clustered,seed", [(3, 1, False, 1), (5, 1, False, 2), (7, 2, False, 3),
                                                   (11, 3, False, 4), (21, 6, True, 5), (33, 4, False, 6),
                                                   (41, 8, True, 7)])
def test_transform_matches_bfs(oracle_lib, size, k, clustered, seed):
    import numpy as np
    m = SyntheticMap(size, campfires_per_homeland=k, seed=seed, clustered=clustered)
    arr = m.cells_array()
    rank = cell_ranks(arr)
    for h in range(4):
        region, nreg = cell_regions(arr, h)
        want = oracle_lib.region_table_bfs(size, rank, region, nreg)
        got = transform_model(size, rank, region, nreg)
        bad = np.argwhere(np.any(got != want, axis=2))
        assert bad.size == 0, (h, bad[:4].tolist(), got[tuple(bad[0])].tolist(), want[tuple(bad[0])].tolist())
