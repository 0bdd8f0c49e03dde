set -u
mkdir -p gpurun_out/susp2; export TMPDIR=/tmp
O=gpurun_out/susp2
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_s4m8.so $L/librtamd_s8m6.so $L/librtamd_s2m12.so $L/librtamd.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; cat $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C4 --spp 50 --reps 2 $L/librtamd.so $L/librtamd_susp8.so $L/librtamd_s16m2.so $L/librtamd_s12m4.so > $O/ab_c4.log 2>&1; rc=$?; echo "ab c4 rc=$rc"; cat $O/ab_c4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C5 --spp 200 --reps 2 $L/librtamd.so $L/librtamd_susp8.so > $O/ab_c5.log 2>&1; rc=$?; echo "ab c5 rc=$rc"; cat $O/ab_c5.log
