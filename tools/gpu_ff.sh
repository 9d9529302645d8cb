mkdir -p gpurun_out/ff
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fleetfoot_hub" --timeout 300 --timeout-method thread > gpurun_out/ff/pytest_ff.log 2>&1; echo ff-tests $?
timeout -k 10 300 python -u tools/ff_rates.py 65 10000 3 > gpurun_out/ff/rates65.log 2>&1; echo rates65 $?
timeout -k 10 300 python -u tools/ff_rates.py 1025 125000 2 > gpurun_out/ff/rates1025.log 2>&1; echo rates1025 $?
