set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
