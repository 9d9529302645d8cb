# Final checks of the round: full-scale parity, smoke(), the gloo N=2 rehearsal of the
# bench, and the c2 / c3 / c5 bench lines on the final tree
set -o pipefail
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_scale.py -x -q --timeout 600 --timeout-method thread > $O/full_scale.log 2>&1 && echo fullscale-ok || { tail -30 $O/full_scale.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || { tail -20 $O/smoke.log; exit 1; }
MR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err && echo n2-ok || { tail -20 $O/bench_n2.err; exit 1; }
for W in c2 c3 c5; do
  ST=20; [ $W = c5 ] && ST=3
  timeout -k 10 400 python bench.py --workload $W --steps $ST --warmup 2 > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
  echo "$W ok"
done
