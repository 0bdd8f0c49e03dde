set -u
mkdir -p gpurun_out/susp; export TMPDIR=/tmp
O=gpurun_out/susp
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_susp8.so $L/librtamd_susp4.so $L/librtamd_susp16.so $L/librtamd.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; cat $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C4 --spp 50 --reps 2 $L/librtamd.so $L/librtamd_susp8.so > $O/ab_c4.log 2>&1; rc=$?; echo "ab c4 rc=$rc"; cat $O/ab_c4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C1 --reps 3 $L/librtamd.so $L/librtamd_susp8.so > $O/ab_c1.log 2>&1; rc=$?; echo "ab c1 rc=$rc"; cat $O/ab_c1.log
RT_LIBRARY=$L/librtamd_susp8.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_susp8.log 2>&1; rc=$?; echo "tests susp8 rc=$rc"; tail -3 $O/tests_susp8.log
