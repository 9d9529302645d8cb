#!/bin/bash
# round 4: group kernel with one meta column per group (smaller LDS): parity, crossover, c2/c4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04zj
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/parity.log 2>&1 || exit 1
for q in 5000 20000 40000; do
  for env in "MR_HUB_LANE=1" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=8" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=16"; do
    tag=$(echo $env | tr ' =' '__')
    env $env timeout -k 10 200 python bench.py --queries $q --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/b_${q}_$tag.json 2> $O/b_${q}_$tag.err || exit 1
  done
done
timeout -k 10 120 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 3 > $O/b_c2.json 2> $O/b_c2.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 2 > $O/b_c4.json 2> $O/b_c4.err
