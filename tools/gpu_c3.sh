set -o pipefail
mkdir -p gpurun_out/c3
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sssp.py -x -q -k "${K:-fill or every_cell or c3}" --timeout 300 --timeout-method thread > gpurun_out/c3/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/c3/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c3/bench_c3.json 2> gpurun_out/c3/bench_c3.err && echo bench-ok
