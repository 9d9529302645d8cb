# lane kernel: parity (every lane-mode case + the 1M configs[3] test) and an A/B of the
# fused compare-select against the classic form (MR_LANE_CLASSIC), configs[3] at 1M
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" tests/test_gpu_full_scale.py::test_c4_full_scale -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in main classic main classic; do
  L=""; [ $v != main ] && L=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so
  MR_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/ab_$v.json 2> $O/ab_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
done
