# Quick GPU check: chosen tests (TESTS, default the overlap/fill tests), then the
# gloo rehearsal of the N=2 bench path for c2 and c4, then the default bench line
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_sssp.py} -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || { tail -30 $O/pytest.log; exit 1; }
for W in c2 c4; do
  MR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --workload $W > $O/bench_n2_$W.json 2> $O/bench_n2_$W.err && echo n2-$W-ok || { tail -20 $O/bench_n2_$W.err; exit 1; }
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo bench-ok
