# Certified fallback after the SoE check: its tests, the hand-over/Fleetfoot parity and
# the device-fetch tests, the repeated-plan probe, the Time-first rates
set -o pipefail
O=gpurun_out/cert3
mkdir -p $O
timeout -k 10 300 python -u tools/plan_diff2.py > $O/plan_diff2.log 2>&1 && echo diff-ok || { tail -20 $O/plan_diff2.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_cert.py -x -v --timeout 300 --timeout-method thread > $O/cert.log 2>&1 && echo cert-ok || { tail -40 $O/cert.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py -x -q -k "fallback or fbsssp or leetfoot or device_fetch" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && echo parity-ok || { tail -40 $O/parity.log; exit 1; }
timeout -k 10 600 python -u tools/ff_rates.py 1025 125000 3 > $O/ff_rates.log 2>&1 && echo ff-ok
