# lane kernel A/B: scheduling fences every 1 (main), 2, 4 entries or none (with / without
# the pair-table prefetch)
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
for v in main f0 f0pf0 f2 f4 main f0 f0pf0 f2 f4; do
  L=""; [ $v != main ] && L=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so
  MR_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/ab_$v.json 2> $O/ab_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
done
