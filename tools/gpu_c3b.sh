# c3 after a fill/record change: the all-destinations tests, then the c3 profiling recipe
set -o pipefail
mkdir -p gpurun_out/c3b
timeout -k 10 700 python -u -m pytest tests/test_gpu_sssp.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c3b/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/c3b/pytest.log; exit 1; }
bash tools/profile_round.sh r02 c3
