set -u
mkdir -p gpurun_out/tests; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests/gpu.log 2>&1; rc=$?; tail -5 gpurun_out/tests/gpu.log; exit $rc
