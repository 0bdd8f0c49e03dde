set -u
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lowering.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -15
