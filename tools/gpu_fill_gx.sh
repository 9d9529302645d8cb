set -o pipefail
mkdir -p gpurun_out/gx
for g in default 1280 1024 768 2048; do
  if [ $g = default ]; then unset MR_FILL_GX; else export MR_FILL_GX=$g; fi
  timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gx/$g.json 2> gpurun_out/gx/$g.err || exit 1
  echo "$g $(python3 -c "import json;d=json.load(open('gpurun_out/gx/$g.json'));r=d['roofline'];print(d['ms_per_step'],r['kernel_ms'],r['frac'])")"
done
