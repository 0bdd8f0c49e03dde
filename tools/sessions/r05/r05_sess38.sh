set -u
timeout -k 10 900 python3 -u -m pytest "tests/test_gpu_parity.py::test_traversal_audit_full_frame" "tests/test_gpu_parity.py::test_sphere_pretest_audit_c2" tests/test_gpu_exec_join.py -q -x --timeout 600 --timeout-method thread 2>&1 | tail -5
