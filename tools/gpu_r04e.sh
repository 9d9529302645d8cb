# lane kernel A/B: pair-table prefetch distance (MR_LANE_PF 0..3), configs[3] at 1M
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
for v in main pf0 pf2 pf3 main pf0 pf2 pf3; do
  L=""; [ $v != main ] && L=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so
  MR_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/ab_$v.json 2> $O/ab_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
done
MR_TIMING=1 timeout -k 10 300 python bench.py --queries 125000 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 3 > $O/bench_125k.json 2> $O/bench_125k.err && echo ok125
grep MR_TIMING $O/bench_125k.err | tail -4
python3 -c "import json;print(json.load(open('$O/bench_125k.json'))['end_to_end'])"
