set -u
mkdir -p gpurun_out/mlate2; export TMPDIR=/tmp
O=gpurun_out/mlate2
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd_mlate.so $L/librtamd.so $L/librtamd_mlate.so $L/librtamd.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
