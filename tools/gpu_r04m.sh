# lane kernel special lookup by LDS hash: lane parity, A/B against the per-cell record
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" tests/test_gpu_full_scale.py -k "lane or c4_full" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in std tab std tab; do
  E=""; [ $v = tab ] && E="MR_RANK_TABLE=1"
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/ab_$v.json 2> $O/ab_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
done
