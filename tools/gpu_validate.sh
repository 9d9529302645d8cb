# Full GPU validation: every gpu test, then each workload's bench line (wall time logged)
set -o pipefail
O=gpurun_out/v2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || exit 1
for W in c2 c4 c3 c5; do
  S=$(date +%s.%N)
  ST=20; [ $W = c5 ] && ST=3; [ $W = c4 ] && ST=10
  timeout -k 10 400 python bench.py --workload $W --steps $ST --warmup 2 > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
  echo "$W wall $(python3 -c "import time;print(round(time.time()-$S,1))") s"
done
