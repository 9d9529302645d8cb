# non-linear certification with the periodic path skip: the Fleetfoot parity tests, the
# certificate tests, and the Fleetfoot rates at 1025^2 / 125k queries (before: r03 log)
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "fleetfoot or random_params or hbm_regime or certificate" tests/test_gpu_cert.py tests/test_gpu_full_scale.py::test_fleetfoot_time_first_1025 -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python tools/ff_rates.py 1025 125000 3 > $O/ff_rates.log 2>&1 && echo rates-ok
cat $O/ff_rates.log
