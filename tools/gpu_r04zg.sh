#!/bin/bash
# round 4 (late): lane prefetch distance A/B on c4; N>1 rehearsals (gloo, 2 ranks on one GPU;
# the RCCL gather path at world 1) on c4 and c2 with the group kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04zg
mkdir -p $O
for i in 1 2; do
  for v in main pf2 pf0; do
    if [ $v = main ]; then LP=""; else LP=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so; fi
    MR_LIB_PATH=$LP timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/b_c4_$v$i.json 2> $O/b_c4_$v$i.err || exit 1
  done
done
for W in c4 c2; do
  MR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --workload $W > $O/bench_n2_$W.json 2> $O/bench_n2_$W.err || { tail -20 $O/bench_n2_$W.err; exit 1; }
  MR_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/rccl1_$W.json 2> $O/rccl1_$W.err || { tail -20 $O/rccl1_$W.err; exit 1; }
done
