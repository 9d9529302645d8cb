# c3: the all-destinations tests, then the bench line per overlap slot count
set -o pipefail
mkdir -p gpurun_out/slots
timeout -k 10 700 python -u -m pytest tests/test_gpu_sssp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/slots/pytest.log 2>&1 && echo tests-ok || { tail -20 gpurun_out/slots/pytest.log; exit 1; }
for n in 2 3 4 3 2; do
  MR_FILL_SLOTS=$n timeout -k 10 300 python bench.py --workload c3 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/slots/s$n.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/slots/s$n.json'));r=d['roofline'];print('slots $n', round(d['value']/1e9,1), 'G cells/s', round(d['ms_per_step'],4), 'ms/pass', 'fill', round(r['kernel_ms'],4))"
done
