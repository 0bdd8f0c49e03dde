set -u
mkdir -p gpurun_out/r02g; export TMPDIR=/tmp
O=gpurun_out/r02g
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_suspall0.so $L/librtamd_suspall16.so $L/librtamd.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C5 --spp 200 --reps 2 $L/librtamd.so $L/librtamd_suspall0.so > $O/ab_c5.log 2>&1; rc=$?; echo "ab c5 rc=$rc"; grep -v amdgpu $O/ab_c5.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
