# Quick check after a host change: parity + e2e + sssp tests, the default bench line, timing
set -o pipefail
O=gpurun_out/quick2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_cert.py tests/test_gpu_sssp.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || { tail -30 $O/pytest.log; exit 1; }
MR_TIMING=1 timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo bench-ok
