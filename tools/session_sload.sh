set -u
mkdir -p gpurun_out/sload; export TMPDIR=/tmp
O=gpurun_out/sload
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_sload.so $L/librtamd.so $L/librtamd_sload.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd.so $L/librtamd_sload.so > $O/ab_c2.log 2>&1; rc=$?; echo "ab c2 rc=$rc"; grep -v amdgpu $O/ab_c2.log
timeout -k 10 300 python3 tools/ab_time.py --config C5 --spp 200 --reps 2 $L/librtamd.so $L/librtamd_sload.so > $O/ab_c5.log 2>&1; rc=$?; echo "ab c5 rc=$rc"; grep -v amdgpu $O/ab_c5.log
timeout -k 10 300 python3 tools/ab_time.py --config C4 --spp 50 --reps 2 $L/librtamd.so $L/librtamd_sload.so > $O/ab_c4.log 2>&1; rc=$?; echo "ab c4 rc=$rc"; grep -v amdgpu $O/ab_c4.log
RT_LIBRARY=$L/librtamd_sload.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
