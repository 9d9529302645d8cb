#!/bin/bash
# round 4: lane vs group kernel crossover (c4 map; 5k .. 60k queries)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04zi
mkdir -p $O
for q in 5000 10000 20000 40000 60000; do
  for env in "MR_HUB_LANE=1" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=8" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=16" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=32"; do
    tag=$(echo $env | tr ' =' '__')
    env $env timeout -k 10 200 python bench.py --queries $q --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/b_${q}_$tag.json 2> $O/b_${q}_$tag.err || exit 1
  done
done
