set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v1/pytest.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python bench.py > gpurun_out/v1/bench_c2.json 2> gpurun_out/v1/bench_c2.err && echo c2-ok &&
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/v1/bench_c5.json 2> gpurun_out/v1/bench_c5.err && echo c5-ok
