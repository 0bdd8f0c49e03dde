set -u
mkdir -p gpurun_out/r02d; export TMPDIR=/tmp
O=gpurun_out/r02d
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.log
