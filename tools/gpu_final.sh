# Round-end validation: smoke, every gpu test, the default bench line, the profiling
# recipe for every workload (bench lines + kernel traces + PMC passes)
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo bench-ok || exit 1
bash tools/profile_round.sh r01 "c4 c2 c3 c5"
