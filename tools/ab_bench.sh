# A/B: the same bench with the in-tree library and with experiment variants
# usage: bash tools/ab_bench.sh "<bench args>" variant1 [variant2 ...]
set -o pipefail
ARGS=$1; shift
mkdir -p gpurun_out/ab
timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > gpurun_out/ab/main.json 2> gpurun_out/ab/main.err || exit 1
echo "main $(python3 -c "import json;d=json.load(open('gpurun_out/ab/main.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])")"
for v in "$@"; do
  MR_LIB_PATH=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])")"
done
