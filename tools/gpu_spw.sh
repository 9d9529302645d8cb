# c2: sources per wave A/B (MR_HUB_SPW=1 vs the default 2)
set -o pipefail
mkdir -p gpurun_out/spw
for i in 1 2; do
  for v in 2 1; do
    MR_HUB_SPW=$v timeout -k 10 200 python bench.py --workload ${W:-c2} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/spw/$v.json 2> gpurun_out/spw/$v.err || exit 1
    echo "spw=$v $(python3 -c "import json;d=json.load(open('gpurun_out/spw/$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
  done
done
