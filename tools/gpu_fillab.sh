# fill changes: the fill / every-cell / overlap tests, then a c3 A/B against variants
# usage: bash tools/gpu_fillab.sh variant1 [variant2 ...]
set -o pipefail
mkdir -p gpurun_out/fillab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sssp.py -x -q -k "fill_tiles or ragged or overlapped or c3" --timeout 300 --timeout-method thread > gpurun_out/fillab/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/fillab/pytest.log; exit 1; }
bash tools/ab_bench.sh "--workload c3 --steps 20 --warmup 3" "$@" && MR_FILL_OVERLAP=0 bash tools/ab_bench.sh "--workload c3 --steps 20 --warmup 3" "$@"
