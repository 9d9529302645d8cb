# c3: the fill with parts switched off (MR_DBG_FLAGS 64: no stores, 128: no boundary loop)
set -o pipefail
mkdir -p gpurun_out/parts
for i in 1 2; do
for f in ${FL:-0 64 128 192}; do
  MR_FILL_FUSED=0 MR_DBG_FLAGS=$f timeout -k 10 200 python bench.py --workload c3 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/parts/$f.json 2> gpurun_out/parts/$f.err || exit 1
  echo "flags=$f $(python3 -c "import json;d=json.load(open('gpurun_out/parts/$f.json'));r=d['roofline'];print(d['ms_per_step'],r['kernel_ms'])")"
done
done
