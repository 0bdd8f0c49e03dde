set -u
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_parity.py::test_medium_first_fallback_stays_exact" -q -x --timeout 500 --timeout-method thread 2>&1 | tail -25
