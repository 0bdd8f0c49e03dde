set -u
mkdir -p gpurun_out/r02e; export TMPDIR=/tmp
O=gpurun_out/r02e
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
RT_LAUNCH_LOG=1 timeout -k 10 300 python3 tools/render_once.py --config C4 --reps 1 > $O/c4_full.log 2>&1; rc=$?; echo "c4 rc=$rc"; cat $O/c4_full.log
