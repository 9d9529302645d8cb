#!/bin/bash
# round 4: lane vs group kernel on the c4 map at 125k queries (the N = 8 shard) and at 1M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04zh
mkdir -p $O
for q in 125000 250000; do
  for env in "X=0" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=8" "MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=16"; do
    tag=$(echo $env | tr ' =' '__')
    env $env timeout -k 10 200 python bench.py --queries $q --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/b_${q}_$tag.json 2> $O/b_${q}_$tag.err || exit 1
  done
done
MR_HUB_GROUP_FORCE=1 MR_HUB_GROUP=8 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-reps 0 > $O/b_1m_g8.json 2> $O/b_1m_g8.err
