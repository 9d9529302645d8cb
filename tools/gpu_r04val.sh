# Round 4 validation box (late): the whole GPU suite, smoke(), then the profiles of every
# workload (bench line, kernel trace, PMC, SQ) under gpurun_out/prof_r04/
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 && echo tests-ok || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || { tail -20 $O/smoke.log; exit 1; }
bash tools/profile_round.sh r04v "c4 c2 c3 c5" || exit 1
bash tools/gpu_sq_wait.sh c4 gpurun_out/prof_r04v/sqw_c4 && echo sqw-ok
