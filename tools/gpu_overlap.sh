set -o pipefail
mkdir -p gpurun_out/ov
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sssp.py -x -q -k "overlapped or fill_tiles or ragged or c3 or reruns or every_cell" --timeout 300 --timeout-method thread > gpurun_out/ov/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/ov/pytest.log; exit 1; }
for i in 1 2; do
timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ov/on$i.json 2> gpurun_out/ov/on$i.err || exit 1
MR_FILL_OVERLAP=0 timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ov/off$i.json 2> gpurun_out/ov/off$i.err || exit 1
done
for f in on1 off1 on2 off2; do echo "$f $(python3 -c "import json;d=json.load(open('gpurun_out/ov/$f.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['pass_ms'])")"; done
