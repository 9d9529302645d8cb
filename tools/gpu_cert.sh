# Certified fallback on the GPU: its tests, the parity suite's hand-over modes, the
# Time-first Fleetfoot rates (tools/ff_rates.py)
set -o pipefail
O=gpurun_out/cert
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cert.py -x -v --timeout 300 --timeout-method thread > $O/cert.log 2>&1 && echo cert-ok || { tail -40 $O/cert.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fallback or fbsssp" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && echo parity-ok || { tail -40 $O/parity.log; exit 1; }
timeout -k 10 600 python -u tools/ff_rates.py 1025 125000 3 > $O/ff_rates.log 2>&1 && echo ff-ok
