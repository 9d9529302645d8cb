# round validation: smoke, every gpu test, the default bench line
set -o pipefail
O=gpurun_out/val
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo bench-ok || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
