# Full GPU test suite, then a gloo rehearsal of the N=2 bench path on the one GPU
set -o pipefail
O=gpurun_out/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || exit 1
MR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err && echo n2-ok
